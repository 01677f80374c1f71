// compressor.hip — the 3-band multiband compressor (AME:207-210) on CDNA4.
//
// pydub compress_dynamic_range per band (restated in SURVEY.md Appendix A):
//   rms_i  = audioop.rms over frames [max(chunk0, i-look), i)  (excludes i)
//   M_i    = (1 - 1/ratio) * max(20 log10(rms_i / thr), 0)       (host table, exact)
//   att_i  = (rms_i > thr && att <= M_i) ? min(att + M_i/A, M_i) : max(att - M_i/R, 0)
//   out_i  = floor(x_i * 10^(-att_i/20))  if att_i != 0
// audioop.rms = (unsigned)sqrt(S/n) equals isqrt(S div n) for integer S and the n
// seen here (tests/test_oracle.py), so rms is computed exactly with
// integers.  M_i == 0 exactly when rms_i <= thr ("hold": att unchanged), and
// rms_i > thr <=> rms_i >= r0 (M is monotone in rms), r0 from the host table.
//
// The att recurrence is sequential and non-linear.  It is solved EXACTLY:
//  1. comp_rms     per tile: rms -> uint16 r (tile-major) + active-frame counts;
//  2. comp_offsets per chunk: exclusive scan of the counts (compacted offsets);
//  3. comp_compact per tile: M of every active frame, scattered into a compacted,
//     super-tile-major array (hold frames are identity, so they vanish);
//  4. comp_pass0   per super-tile (U active frames): speculative walk warmed up
//     over the previous super-tile from att = 0; the first of a chunk is exact;
//  5. comp_fix     Jacobi sweeps: a super-tile whose start differs from its
//     predecessor's end re-runs from it; at the fixed point every start is the
//     true state (induction from the exact chunk start);
//  6. comp_record  one more walk from the converged starts overwrites the
//     compacted M with the exact att after every active frame;
//  7. comp_tstart  per tile: att at its first frame (gathered from step 6);
//  8. comp_apply   per tile: exact att from there, gains, audioop.mul, overlay.
#include "common.h"

namespace mm {

__device__ __forceinline__ int32_t frame_energy(short2 v) {
    return (int32_t)v.x * v.x + (int32_t)v.y * v.y;
}

// largest r with n*r*r <= S (== trunc(sqrt(S/n)) computed in doubles)
__device__ __forceinline__ uint32_t rms_exact(int64_t S, int64_t n, float inv_n) {
    int64_t r = (int64_t)__fsqrt_rn((float)S * inv_n);
    r -= (r > 0 && n * r * r > S);
    r += (n * (r + 1) * (r + 1) <= S);
    return n > 0 ? (uint32_t)r : 0u;
}

// tile-major address of timeline frame f
__device__ __forceinline__ int64_t tm_index(int64_t f, int T, int64_t G) {
    int64_t g = f / T;
    return (f - g * T) * G + g;
}

// 1. rms per frame (uint16 r, tile-major) and active counts per tile.
// grid: (ceil(G/256), 3 bands)
__global__ void __launch_bounds__(256) comp_rms_kernel(CompArgs a) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (g >= a.G) return;
    const short2 *x = a.band[b];
    const int look = a.look[b];
    const uint32_t r0 = a.r0[b];
    const int T = a.T;
    const int64_t G = a.G;
    const int64_t f0 = g * T;
    const int64_t chunk0 = (g / a.K) * a.K * T;
    const int len = (int)min((int64_t)T, a.N_proc - f0);
    const int ch = a.ch;
    const int64_t lo0 = max(chunk0, f0 - look);
    const int wl = (int)(f0 - lo0);
    int64_t S = 0;
    stream<8, 2, short2>(
        wl, [&](int i) { return x[tm_index(lo0 + min(i, wl - 1), T, G)]; },
        [&](short2 v) { S += frame_energy(v); });
    uint16_t *R = a.r16[b];
    int64_t cnt_frames = f0 - lo0;
    float inv = cnt_frames > 0 ? 1.0f / (float)(cnt_frames * ch) : 0.f;
    int64_t pf = f0;
    int active = 0;
    struct Pair {
        short2 in, drop;
    };
    stream<8, 3, Pair>(
        len,
        [&](int i) {
            const int64_t f = f0 + min(i, len - 1);
            const int64_t fd = max(f - look, chunk0);  // clamped; unused when < chunk0
            Pair p;
            p.in = x[tm_index(f, T, G)];
            p.drop = x[tm_index(fd, T, G)];
            return p;
        },
        [&](Pair p) {
            const uint32_t r = rms_exact(S, cnt_frames * ch, inv);
            R[(pf - f0) * G + g] = (uint16_t)r;
            active += r >= r0;
            S += frame_energy(p.in);
            const bool full = pf - look >= chunk0;
            S -= full ? frame_energy(p.drop) : 0;
            if (!full) {
                ++cnt_frames;
                inv = 1.0f / (float)(cnt_frames * ch);
            }
            ++pf;
        });
    a.cnt[b][g] = active;
}

// 2. per (chunk, band): exclusive scan of active counts -> off; chunk totals.
__global__ void __launch_bounds__(1024) comp_offsets_kernel(CompArgs a) {
    __shared__ int32_t buf[1024];
    const int b = blockIdx.y;
    const int64_t t0 = (int64_t)blockIdx.x * a.K;
    const int64_t n = min((int64_t)a.K, a.G - t0);
    const int64_t c = (n + 1023) / 1024;
    const int tid = threadIdx.x;
    const int64_t b0 = tid * c, b1 = min(b0 + c, n);
    int32_t sum = 0;
    for (int64_t m = b0; m < b1; ++m) sum += a.cnt[b][t0 + m];
    buf[tid] = sum;
    __syncthreads();
    int32_t v = sum;
    for (int d = 1; d < 1024; d <<= 1) {
        int32_t o = tid >= d ? buf[tid - d] : 0;
        __syncthreads();
        v += o;
        buf[tid] = v;
        __syncthreads();
    }
    int32_t run = tid > 0 ? buf[tid - 1] : 0;
    for (int64_t m = b0; m < b1; ++m) {
        a.off[b][t0 + m] = run;
        run += a.cnt[b][t0 + m];
    }
    if (tid == 1023) a.total[b][blockIdx.x] = buf[1023];
}

// compacted index p of chunk c -> element address in the super-tile-major array
__device__ __forceinline__ int64_t cm_index(const CompArgs &a, int64_t c, int32_t p) {
    const int32_t k = p / a.U, o = p - k * a.U;
    return (int64_t)o * a.GS + c * a.SPC + k;
}

// 3. scatter M of active frames into the compacted array.  grid (ceil(G/256), 3)
__global__ void __launch_bounds__(256) comp_compact_kernel(CompArgs a) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (g >= a.G) return;
    if (a.cnt[b][g] == 0) return;
    const uint16_t *R = a.r16[b];
    const double *lut = a.max_att[b];
    const uint32_t r0 = a.r0[b];
    const int64_t c = g / a.K;
    const int len = (int)min((int64_t)a.T, a.N_proc - g * a.T);
    int32_t p = a.off[b][g];
    double *Mc = a.Mc[b];
    // inactive frames store into this lane's own padding slot (row U of the
    // array), so every store is unconditional and the pipeline stays counted
    double *dummy = Mc + (int64_t)a.U * a.GS + g % a.GS;
    stream2<8, 2, uint16_t, double>(
        len, [&](int i) { return R[(int64_t)min(i, len - 1) * a.G + g]; },
        [&](uint16_t r) { return lut[r]; },
        [&](uint16_t r, double m) {
            const bool act = r >= r0;
            double *dst = act ? Mc + cm_index(a, c, p) : dummy;
            *dst = m;
            p += act;
        });
}

// correctly rounded m / d given rd = RN(1/d) (Markstein; tests/test_oracle.py)
__device__ __forceinline__ double div_cr(double m, double d, double rd) {
    double q = m * rd;
    double rem = fma(-q, d, m);
    return fma(rem, rd, q);
}

struct BandStep {
    double A, R, rA, rR;
};

__device__ __forceinline__ BandStep band_step(const CompArgs &a, int b) {
    BandStep s;
    s.A = a.attack_frames[b];
    s.R = a.release_frames[b];
    s.rA = a.rcp_attack[b];
    s.rR = a.rcp_release[b];
    return s;
}

// one envelope step; M == 0 (hold) leaves att unchanged exactly
__device__ __forceinline__ double comp_step(double att, double M, const BandStep &bs) {
    const double inc = div_cr(M, bs.A, bs.rA);  // off the att critical path
    const double dec = div_cr(M, bs.R, bs.rR);
    double up = att + inc;
    up = (M < up) ? M : up;
    double dn = att - dec;
    dn = (0.0 > dn) ? 0.0 : dn;
    return (M != 0.0 && att <= M) ? up : dn;
}

struct Super {
    int64_t c;        // chunk
    int32_t p0, len;  // compacted range [p0, p0+len)
};

__device__ __forceinline__ Super super_of(const CompArgs &a, int b, int64_t s) {
    Super r;
    r.c = s / a.SPC;
    const int64_t k = s - r.c * a.SPC;
    const int32_t L = a.total[b][r.c];
    r.p0 = (int32_t)(k * a.U);
    r.len = (int32_t)max((int64_t)0, min((int64_t)a.U, (int64_t)L - r.p0));
    return r;
}

// Walk the envelope over a super-tile's compacted frames (branch-free stream).
// With STORE, overwrite each compacted M with the att after that frame.
template <bool STORE>
__device__ __forceinline__ double comp_walk(double att, const CompArgs &a, int b, int64_t s, int len,
                                            const BandStep &bs) {
    double *Mc = a.Mc[b];
    int o = 0;
    stream<8, 4, double>(
        len, [&](int i) { return Mc[(int64_t)min(i, len - 1) * a.GS + s]; },
        [&](double m) {
            att = comp_step(att, m, bs);
            if (STORE) Mc[(int64_t)(o++) * a.GS + s] = att;
        });
    return att;
}

// 4. speculative pass.  grid: (ceil(GS/256), 3)
__global__ void __launch_bounds__(256) comp_pass0_kernel(CompArgs a) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (s >= a.GS) return;
    const Super st = super_of(a, b, s);
    if (st.len == 0) return;
    const BandStep bs = band_step(a, b);
    double att = 0.0;
    if (a.warmup > 0 && st.p0 > 0) att = comp_walk<false>(att, a, b, s - 1, a.U, bs);
    a.start[b][s] = att;
    a.end_out[b][s] = comp_walk<false>(att, a, b, s, st.len, bs);
}

// 5. one Jacobi sweep (exits at once if the previous sweep changed nothing).
__global__ void __launch_bounds__(256) comp_fix_kernel(CompArgs a, const unsigned int *prev_changed) {
    if (prev_changed && *prev_changed == 0u) return;
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (s >= a.GS) return;
    const Super st = super_of(a, b, s);
    if (st.len == 0) return;
    const double *end_in = a.end_in[b];
    double e = end_in[s];
    if (st.p0 > 0) {
        const double want = end_in[s - 1];
        const double have = a.start[b][s];
        if (__double_as_longlong(want) != __double_as_longlong(have)) {
            e = comp_walk<false>(want, a, b, s, st.len, band_step(a, b));
            a.start[b][s] = want;
            *a.changed = 1u;  // benign race: every writer stores 1
        }
    }
    a.end_out[b][s] = e;
}

// 6. exact att after every active frame (Mc is overwritten in place).
__global__ void __launch_bounds__(256) comp_record_kernel(CompArgs a) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (s >= a.GS) return;
    const Super st = super_of(a, b, s);
    if (st.len == 0) return;
    comp_walk<true>(st.p0 > 0 ? a.start[b][s] : 0.0, a, b, s, st.len, band_step(a, b));
}

// 7. per tile: att at its first frame = att after compacted frame off-1 (0 if
// the chunk had no active frame before it).  grid (ceil(G/256), 3)
__global__ void __launch_bounds__(256) comp_tstart_kernel(CompArgs a) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (g >= a.G) return;
    const int32_t p = a.off[b][g];
    a.tstart[b][g] = p > 0 ? a.Mc[b][cm_index(a, g / a.K, p - 1)] : 0.0;
}

// 8. per tile: exact trajectory from tstart; gains on the three band samples
// (audioop.mul floor), overlay sat16(sat16(lo+mid)+hi) (AME:210) -> q2.
__global__ void __launch_bounds__(256) comp_apply_kernel(CompArgs a) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.G) return;
    BandStep bs[3];
    double att[3];
    const double *lut[3];
    uint32_t r0[3];
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        bs[b] = band_step(a, b);
        att[b] = a.tstart[b][g];
        lut[b] = a.max_att[b];
        r0[b] = a.r0[b];
    }
    const int64_t G = a.G;
    const int len = (int)min((int64_t)a.T, a.N_proc - g * a.T);
    struct Fr {
        uint16_t r[3];
        short2 v[3];
    };
    struct Ms {
        double m[3];
    };
    int pn = 0;
    stream2<4, 2, Fr, Ms>(
        len,
        [&](int i) {
            Fr f;
            const int64_t idx = (int64_t)min(i, len - 1) * G + g;
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                f.r[b] = a.r16[b][idx];
                f.v[b] = a.band[b][idx];
            }
            return f;
        },
        [&](const Fr &f) {
            Ms s;
#pragma unroll
            for (int b = 0; b < 3; ++b) s.m[b] = lut[b][f.r[b]];  // lut[r] == 0 for r < r0 (hold)
            return s;
        },
        [&](const Fr &f, const Ms &ms) {
            int32_t accl = 0, accr = 0;
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                att[b] = comp_step(att[b], ms.m[b], bs[b]);
                short2 s = f.v[b];
                if (att[b] != 0.0) {
                    const double gain = exp10(-att[b] / 20.0);
                    s.x = audioop_mul(s.x, gain);
                    s.y = audioop_mul(s.y, gain);
                }
                if (b == 0) {
                    accl = s.x;
                    accr = s.y;
                } else {
                    accl = sat16(accl + s.x);
                    accr = sat16(accr + s.y);
                }
            }
            a.q_out[(int64_t)(pn++) * G + g] =
                make_short2((int16_t)accl, a.ch == 2 ? (int16_t)accr : (int16_t)0);
        });
}

}  // namespace mm
