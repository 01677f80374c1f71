// compressor.hip — the 3-band multiband compressor (AME:207-210) on CDNA4.
//
// pydub compress_dynamic_range per band (restated in SURVEY.md Appendix A):
//   rms_i  = audioop.rms over frames [max(chunk0, i-look), i)  (excludes i)
//   M_i    = (1 - 1/ratio) * max(20 log10(rms_i / thr), 0)
//   att_i  = (rms_i > thr && att <= M_i) ? min(att + M_i/A, M_i) : max(att - M_i/R, 0)
//   out_i  = floor(x_i * 10^(-att_i/20))  if att_i != 0
// audioop.rms = (unsigned)sqrt(S/n) equals isqrt(S div n) for integer S and the n
// seen here (tests/test_oracle.py), so rms is computed exactly with integers.
// M depends on the integer rms only: the host tabulates it with Python's own
// float expressions (design.max_att_table); M/A and M/R are correctly rounded
// Markstein divisions on the device.  M == 0 exactly when rms <= thr (then att
// is held).
//
// Frames with M == 0 are identities, so the recurrence only "sees" the active
// frames; it is solved EXACTLY per (chunk, band) over the compacted sequence of
// active frames, cut into super-tiles of U active frames:
//  1. comp_rms     per (tile, band): uint16 rms per frame (tile-major) and the
//                  tile's active-frame count;
//  2. comp_offsets per (chunk, band): exclusive scan of the counts;
//  3. comp_compact per (tile, band): M of every active frame, scattered into
//                  the compacted super-tile-major array Mc[U][GS];
//  4. comp_pass0   per super-tile: warm-up walk over the previous super-tile
//                  from att = 0, then its own walk -> start, end (exact for the
//                  first super-tile of a chunk, where att starts at 0);
//  5. comp_fix     Jacobi sweeps: a super-tile whose start differs from its
//                  predecessor's end re-walks from it; at the fixed point every
//                  start is the true state (induction from the chunk start);
//     Every walk that OWNS a super-tile (pass 0's own walks, the sweeps'
//     re-walks) stores a checkpoint: the state on entry to every Q-th compacted
//     frame.  The last walk of a super-tile starts from its converged start, so
//     at the fixed point every checkpoint is exact;
//  6. comp_apply   per (tile, band): the tile's starting state from the
//                  checkpoint at or before its first compacted frame plus < Q
//                  steps, then the exact trajectory, gains, audioop.mul, overlay
//                  through LDS.
// Sparse bands (the high band is active on ~0.1 % of pink-noise frames) thus
// cost a few super-tiles per chunk, and dense ones ~frames/U.
#include "common.h"

namespace mm {

// x^2 + y^2 of one frame: at most 2 * 32768^2 = 2^31, exact in uint32
__device__ __forceinline__ uint32_t frame_energy(short2 v) {
    return (uint32_t)((int32_t)v.x * v.x) + (uint32_t)((int32_t)v.y * v.y);
}

// largest r with n*r*r <= S (== isqrt(S div n) == trunc(sqrt(S/n)) computed in
// doubles, tests/test_oracle.py).  S and n*r*r are integers below 2^53, so the
// f64 products and compares are exact; the f32 estimate is within 1 of r.
__device__ __forceinline__ uint32_t rms_exact(double S, double n, float inv_n) {
    int32_t r = (int32_t)__fsqrt_rn((float)S * inv_n);
    double rd = (double)r;
    r -= (n * rd * rd > S) ? 1 : 0;
    rd = (double)(r + 1);
    r += (n * rd * rd <= S) ? 1 : 0;
    return n > 0.0 ? (uint32_t)r : 0u;
}

// 1. rms per frame (uint16 r, tile-major).  grid: (ceil(G/256), 3 bands).  The
// window [max(chunk0, f-look), f) slides one frame per step: + frame f-1 (this
// lane's own previous frame), - frame f-1-look (up to ~4 tiles back: another
// lane's data, coalesced across the wave).  The window sum is an exact integer
// held in a double; element indices fit 32 bits (frames < 2^31).
__global__ void __launch_bounds__(256) comp_rms_kernel(CompArgs a) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (g >= a.G) return;
    const short2 *x = a.band[b];
    const int look = a.look[b];
    const int T = a.T;
    const uint32_t G = (uint32_t)a.G, g32 = (uint32_t)g;
    const int64_t f0 = g * T;
    const int64_t chunk0 = (g / a.K) * a.K * T;
    const int len = (int)min((int64_t)T, a.N_proc - f0);
    // S over [lo0, f0): the look / T whole tiles before this one plus the last
    // look % T frames of the one before them, from the crossover's per-tile sums
    // (tiles never straddle a chunk start, so the chunk clamp is per tile)
    const int64_t lo0 = max(chunk0, f0 - look);
    double S = 0.0;
    {
        const int kf = look / T;
        for (int t = 1; t <= kf; ++t)
            if ((g - t) * T >= chunk0) S += a.E[b][g - t];
        if (look % T != 0 && (g - kf - 1) * T >= chunk0) S += a.tail[b][g - kf - 1];
    }
    // drop frames: d = f - look for f >= chunk0 + look; the first `skip` frames drop nothing
    const int64_t d_first = max(f0 - look, chunk0);
    const int skip = (int)(d_first - (f0 - look));
    const uint32_t gd = (uint32_t)(d_first / T);
    const int nd = (int)(d_first - (int64_t)gd * T);
    uint16_t *R = a.r16[b];
    const int ch = a.ch;
    double n = (double)((f0 - lo0) * ch);
    float inv = n > 0.0 ? 1.0f / (float)n : 0.f;
    const uint32_t r0 = a.r0[b];
    int i_proc = 0, active = 0;
    struct Pair {
        short2 in, drop;
    };
    stream<8, 3, Pair>(
        len,
        [&](int i) {
            i = min(i, len - 1);
            Pair p;
            p.in = x[(uint32_t)i * G + g32];
            int k = nd + max(i - skip, 0);  // < 2T
            const int wrap = k >= T ? 1 : 0;
            k -= wrap * T;
            p.drop = x[(uint32_t)k * G + gd + (uint32_t)wrap];
            return p;
        },
        [&](Pair p) {
            const uint32_t r = rms_exact(S, n, inv);
            R[(uint32_t)i_proc * G + g32] = (uint16_t)r;
            active += r >= r0 ? 1 : 0;
            const bool drops = i_proc >= skip;
            S += (double)frame_energy(p.in) - (drops ? (double)frame_energy(p.drop) : 0.0);
            if (!drops) {  // window still growing (first `look` frames of a chunk only)
                n += ch;
                inv = 1.0f / (float)n;
            }
            ++i_proc;
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

// Column of super-tile s in Mc / ck: pass-0 lane j owns super-tiles j*own ..
// j*own + own-1, so super-tile j*own + t lives in column t*ocols + j and the 64
// lanes of a wave touch 64 consecutive columns (512 contiguous bytes) at every
// step of every walk, whatever `own` is.
__device__ __forceinline__ int64_t cm_col(const CompArgs &a, int64_t s) {
    return (s % a.own) * a.ocols + s / a.own;
}

// 3. scatter M of active frames into the compacted array.  grid (ceil(G/256), 3)
// Inactive frames store into this lane's own padding slot (row U of the array),
// so every store is unconditional; the element index is 32-bit and advanced
// with selects (no per-frame branch), keeping the load pipeline counted.
__global__ void __launch_bounds__(256) comp_compact_kernel(CompArgs a) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (g >= a.G) return;
    if (a.cnt[b][g] == 0) return;
    const uint32_t G32 = (uint32_t)a.G, g32 = (uint32_t)g, RS = (uint32_t)a.RS, U = (uint32_t)a.U;
    const uint32_t own = (uint32_t)a.own, ocols = (uint32_t)a.ocols;
    const uint16_t *R = a.r16[b] + g32;
    const double *lut = a.lut[b];
    const uint32_t r0 = a.r0[b];
    const int len = (int)min((int64_t)a.T, a.N_proc - g * a.T);
    const uint32_t p = (uint32_t)a.off[b][g];
    uint32_t k = p / U, o = p - k * U;  // super-tile and row of the next active frame
    const uint32_t base = (uint32_t)(g / a.K) * (uint32_t)a.SPC;
    uint32_t sg = base + k, t = sg % own, col = t * ocols + sg / own;  // its super-tile, column
    uint32_t idx = o * RS + col;  // its element
    const uint32_t dummy = U * RS + g32 % RS;
    double *Mc = a.Mc[b];
    stream2<8, 2, uint16_t, double>(
        len, [&](int i) { return R[(uint32_t)min(i, len - 1) * G32]; },
        [&](uint16_t r) { return lut[r]; },
        [&](uint16_t r, double m) {
            // mask arithmetic: the compiler would turn selects into exec-mask branches
            const uint32_t act = (uint32_t)r >= r0 ? 1u : 0u, amask = 0u - act;
            Mc[(idx & amask) | (dummy & ~amask)] = m;
            const uint32_t o1 = o + act;
            const uint32_t wmask = 0u - (o1 == U ? 1u : 0u);  // the super-tile is full
            // next super-tile's column: +ocols within a lane's group, else the next lane's first
            const uint32_t tw = 0u - (t + 1u == own ? 1u : 0u);
            const uint32_t ncol = ((col + ocols) & ~tw) | ((col - t * ocols + 1u) & tw);
            idx = ((idx + (RS & amask)) & ~wmask) | (ncol & wmask);
            col = (col & ~wmask) | (ncol & wmask);
            t = (t & ~wmask) | (((t + 1u) & ~tw) & wmask);
            o = o1 & ~wmask;
        });
}

// correctly rounded m / d given rd = RN(1/d) (Markstein; tests/test_oracle.py)
__device__ __forceinline__ double div_cr(double m, double d, double rd) {
    const double q = m * rd;
    const double rem = fma(-q, d, m);
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

// One envelope step, exactly pydub's
//   if rms > thr and att <= M: att = min(att + M/A, M)
//   else:                      att = max(att - M/R, 0)
// M == 0 (rms <= thr) leaves att unchanged (inc = dec = 0); M != 0 implies
// rms > thr, so the rms test folds away.  min/max are v_min_f64/v_max_f64
// (equal operands and signed zeros give the same observable att); the
// divisions are correctly rounded and off the att chain.
__device__ __forceinline__ double comp_step(double att, double M, const BandStep &bs) {
    const double inc = div_cr(M, bs.A, bs.rA);
    const double dec = div_cr(M, bs.R, bs.rR);
    const double up = fmin(att + inc, M);
    const double dn = fmax(att - dec, 0.0);
    return att <= M ? up : dn;
}

struct Super {
    int64_t c;        // chunk
    int32_t p0, len;  // compacted range [p0, p0+len)
    bool last;        // last super-tile holding frames of its chunk
};

__device__ __forceinline__ Super super_of(const CompArgs &a, int b, int64_t s) {
    Super r;
    r.c = s / a.SPC;
    const int64_t k = s - r.c * a.SPC;
    const int32_t L = a.total[b][r.c];
    r.p0 = (int32_t)(k * a.U);
    r.len = (int32_t)max((int64_t)0, min((int64_t)a.U, (int64_t)L - r.p0));
    r.last = r.p0 + r.len == L;
    return r;
}

// v_min_f64 / v_max_f64 without the operand canonicalisation fmin/fmax add
// (operands here are never NaN; equal operands and signed zeros give the same
// observable att)
__device__ __forceinline__ double vmin(double x, double y) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
__device__ __forceinline__ double vmax0(double x) {
    double r;
    asm("v_max_f64 %0, %1, 0" : "=v"(r) : "v"(x));
    return r;
}

// the step given M and its (precomputed) increments
__device__ __forceinline__ double lean_step(double att, double m, double inc, double dec) {
    const double up = vmin(att + inc, m);
    const double dn = vmax0(att - dec);
    return att <= m ? up : dn;
}

// Walk the envelope over a super-tile's compacted frames.  M streams WB frames
// ahead in registers; the two divisions run WP frames ahead of the step that
// uses them, so they issue while the att chain of earlier frames is in flight
// (in-order issue: tools/micro/walk2_bench.hip, 136 -> 98 cycles per step).
// With CK (an owning walk), store the state on entry to every CK_Q-th frame.
constexpr int WALK_WB = 32;  // M values in flight per walker
constexpr int WALK_PAD = WALK_WB;  // padding rows after the compacted array (prefetch past a super-tile's end)
constexpr int CK_Q = 8;      // checkpoint stride (compacted frames); divides WALK_WB, FIX_CHUNK and U

template <bool CK>
__device__ __forceinline__ double comp_walk(double att, const CompArgs &a, int b, int64_t s, int len,
                                            const BandStep &bs) {
    constexpr int WB = WALK_WB, WP = 4;
    if (len <= 0) return att;
    // column s, rows GS apart; loads run up to WB rows past the end (padding rows)
    const size_t GS = (size_t)a.RS;  // row stride
    const int64_t cs = cm_col(a, s);
    const double *pl = a.Mc[b] + cs;
    double *pc = CK ? a.ck[b] + cs : nullptr;  // checkpoint rows, one row stride apart
    double buf[WB], inc[WP], dec[WP];
#pragma unroll
    for (int k = 0; k < WB; ++k) {
        buf[k] = *pl;
        pl += GS;
    }
#pragma unroll
    for (int k = 0; k < WP; ++k) {
        inc[k] = div_cr(buf[k], bs.A, bs.rA);
        dec[k] = div_cr(buf[k], bs.R, bs.rR);
    }
    int i = 0;
    for (; i + WB <= len; i += WB) {
#pragma unroll
        for (int k = 0; k < WB; ++k) {
            const double m = buf[k], ik = inc[k % WP], dk = dec[k % WP];
            const double mn = buf[(k + WP) % WB];  // frame i+k+WP (already reloaded when k+WP >= WB)
            inc[k % WP] = div_cr(mn, bs.A, bs.rA);
            dec[k % WP] = div_cr(mn, bs.R, bs.rR);
            if (CK && k % CK_Q == 0) {
                *pc = att;
                pc += GS;
            }
            att = lean_step(att, m, ik, dk);
            buf[k] = *pl;
            pl += GS;
        }
    }
    const int rem = len - i;
#pragma unroll
    for (int k = 0; k < WB; ++k) {
        if (k < rem) {
            const double m = buf[k], ik = inc[k % WP], dk = dec[k % WP];
            const double mn = buf[(k + WP) % WB];
            inc[k % WP] = div_cr(mn, bs.A, bs.rA);
            dec[k % WP] = div_cr(mn, bs.R, bs.rR);
            if (CK && k % CK_Q == 0) {
                *pc = att;
                pc += GS;
            }
            att = lean_step(att, m, ik, dk);
        }
    }
    return att;
}

// Compact streamed owning walk (checkpoints) for the fix kernel's lane path,
// where the register budget is shared with the LDS-staged path.
__device__ __forceinline__ double comp_walk_lean(double att, const CompArgs &a, int b, int64_t s, int len,
                                                 const BandStep &bs) {
    const int64_t cs = cm_col(a, s);
    const double *col = a.Mc[b] + cs;
    double *ck = a.ck[b] + cs;
    const uint32_t GS = (uint32_t)a.RS;
    int i = 0;
    stream<8, 4, double>(
        len, [&](int k) { return col[(uint32_t)min(k, len - 1) * GS]; },
        [&](double m) {
            if (i % CK_Q == 0) ck[(uint32_t)(i / CK_Q) * GS] = att;
            att = comp_step(att, m, bs);
            ++i;
        });
    return att;
}

// 4. speculative pass.  grid: (ceil(GS/(own*BLOCK)), 3).  Each lane walks `own`
// consecutive super-tiles.  The start of the first is guessed by walking the
// `warmup` previous super-tiles of its chunk, from the M of the first warm-up
// frame (the state tracks M closely: this coalesces with the true trajectory far
// more often than a start at 0; tools/ studies); the later ones start from the
// end of the one before (a longer warm-up for free).  own > 1 divides the
// warm-up walks (and their M re-reads) by own; the host raises it with the
// problem size (more super-tiles than the chip needs lanes).
#ifndef MM_PASS0_BLOCK
#define MM_PASS0_BLOCK 64
#endif
constexpr int PASS0_BLOCK = MM_PASS0_BLOCK;

__global__ void __launch_bounds__(PASS0_BLOCK) comp_pass0_kernel(CompArgs a) {
    const int64_t s0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * a.own;
    const int b = blockIdx.y;
    if (s0 >= a.GS) return;
    const BandStep bs = band_step(a, b);
    double att = 0.0;
    bool warm = false;
    for (int64_t s = s0; s < min(s0 + a.own, a.GS); ++s) {
        const Super st = super_of(a, b, s);
        if (st.len == 0) {
            warm = false;
            continue;
        }
        if (st.p0 == 0) {  // chunk start: exact
            att = 0.0;
        } else if (!warm && a.warmup > 0) {
            const int64_t k = st.p0 / a.U;  // index of s within its chunk
            const int64_t w0 = s - min((int64_t)a.warmup, k);
            att = a.Mc[b][cm_col(a, w0)];  // row 0 of super-tile w0
            for (int64_t w = w0; w < s; ++w) att = comp_walk<false>(att, a, b, w, a.U, bs);
        } else if (!warm) {
            att = 0.0;
        }
        a.start[b][s] = att;
        att = comp_walk<true>(att, a, b, s, st.len, bs);
        a.end_out[b][s] = att;
        warm = true;
    }
}

// 5. one Jacobi sweep (exits at once if the previous sweep changed nothing).
// grid: (ceil(GS/64), 3), one wave per block, lane = super-tile.  A lane whose
// start changed re-walks its super-tile.  When at most FIX_SLOTS lanes of the
// wave walk (every sweep once the warm-up guesses are good), the wave serves
// them together: chunk by chunk, all 64 lanes load the walkers' next M values
// (prefetched one chunk ahead) and compute M/A and M/R into LDS, then every
// walker runs the lean step (add, min, select: ~50 cycles instead of ~130 for a
// lone lane that also divides; tools/micro/step_bench.hip) from LDS.
constexpr int FIX_SLOTS = 16;   // walkers per wave served from LDS
constexpr int FIX_CHUNK = 64;   // frames per walker per staging round
constexpr int FIX_MAX_U = 8192; // cap on frames per super-tile (slot lengths are int)

__global__ void __launch_bounds__(64) comp_fix_kernel(CompArgs a, const unsigned int *prev_changed) {
    __shared__ double sm[FIX_SLOTS][FIX_CHUNK + 1], si[FIX_SLOTS][FIX_CHUNK + 1], sd[FIX_SLOTS][FIX_CHUNK + 1];
    __shared__ int slot_lane[FIX_SLOTS], slot_len[FIX_SLOTS];
    __shared__ int64_t slot_col[FIX_SLOTS];
    if (prev_changed && *prev_changed == 0u) return;
    const int lane = threadIdx.x;
    const int64_t s = (int64_t)blockIdx.x * 64 + lane;
    const int b = blockIdx.y;
    const bool valid = s < a.GS;
    const Super st = valid ? super_of(a, b, s) : Super{0, 0, 0, false};
    const bool live = valid && st.len > 0;
    const double *end_in = a.end_in[b];
    double e = live ? end_in[s] : 0.0;
    double want = 0.0;
    bool need = false;
    if (live && st.p0 > 0) {
        want = end_in[s - 1];
        need = __double_as_longlong(want) != __double_as_longlong(a.start[b][s]);
    }
    const BandStep bs = band_step(a, b);
    const unsigned long long m = __ballot(need);
    const int k = __popcll(m);
    if (k > FIX_SLOTS) {
        if (need) e = comp_walk_lean(want, a, b, s, st.len, bs);
    } else if (k > 0) {
        const int slot = __popcll(m & ((1ull << lane) - 1));
        if (need) {
            slot_lane[slot] = lane;
            slot_len[slot] = st.len;
            slot_col[slot] = cm_col(a, s);
        }
        __syncthreads();
        int maxlen = 0;
        for (int w = 0; w < k; ++w) maxlen = max(maxlen, slot_len[w]);
        const double *Mc = a.Mc[b];
        const int64_t col0 = (int64_t)blockIdx.x * 64;
        double pre[FIX_SLOTS];  // lane = frame offset in the chunk, r = walker slot
        auto load_chunk = [&](int base) {
#pragma unroll
            for (int r = 0; r < FIX_SLOTS; ++r) {
                if (r < k) {
                    const int i = base + lane;
                    pre[r] = i < slot_len[r] ? Mc[(int64_t)i * a.RS + slot_col[r]] : 0.0;
                }
            }
        };
        load_chunk(0);
        double att = want;
        for (int base = 0; base < maxlen; base += FIX_CHUNK) {
#pragma unroll
            for (int r = 0; r < FIX_SLOTS; ++r) {
                if (r < k) {
                    const double mv = pre[r];
                    sm[r][lane] = mv;
                    si[r][lane] = div_cr(mv, bs.A, bs.rA);
                    sd[r][lane] = div_cr(mv, bs.R, bs.rR);
                }
            }
            __syncthreads();
            if (base + FIX_CHUNK < maxlen) load_chunk(base + FIX_CHUNK);
            if (need) {
                const int lim = min(FIX_CHUNK, st.len - base);
                const double *pm = sm[slot], *pi = si[slot], *pd = sd[slot];
                double *ck = a.ck[b] + slot_col[slot] + (int64_t)(base / CK_Q) * a.RS;
#pragma unroll 8
                for (int f = 0; f < lim; ++f) {
                    if (f % CK_Q == 0) ck[(int64_t)(f / CK_Q) * a.RS] = att;  // base is a multiple of CK_Q
                    const double up = fmin(att + pi[f], pm[f]);
                    const double dn = fmax(att - pd[f], 0.0);
                    att = att <= pm[f] ? up : dn;
                }
            }
            __syncthreads();
        }
        if (need) e = att;
    }
    if (need) {
        a.start[b][s] = want;
        *a.changed = 1u;  // benign race: every writer stores 1
        atomicAdd(a.walked, (unsigned long long)st.len);
    }
    if (live) a.end_out[b][s] = e;
}

// compacted index p of chunk c -> element address in the super-tile-major array
__device__ __forceinline__ int64_t cm_index(const CompArgs &a, int64_t c, int32_t p) {
    const int32_t k = p / a.U, o = p - k * a.U;
    return (int64_t)o * a.RS + cm_col(a, c * a.SPC + k);
}

// State on entry to compacted frame p of chunk c (the start of the tile whose
// first active frame is p): the checkpoint at or before p, then < CK_Q steps.
// p == total active frames of the chunk (a tile after its last active frame)
// uses the checkpoint before it (the one at p itself belongs to no walk).
__device__ __forceinline__ double comp_state_at(const CompArgs &a, int b, int64_t c, int32_t p, const BandStep &bs) {
    if (p <= 0) return 0.0;
    const int32_t L = a.total[b][c];
    int32_t q = p - p % CK_Q;
    if (q >= L) q -= CK_Q;
    const int32_t k = q / a.U, o = q - k * a.U;
    double att = a.ck[b][(int64_t)(o / CK_Q) * a.RS + cm_col(a, c * a.SPC + k)];
    for (int32_t i = q; i < p; ++i) att = comp_step(att, a.Mc[b][cm_index(a, c, i)], bs);
    return att;
}

// 7. gains + overlay.  A block = 64 tiles x 3 bands: wave w runs band w's exact
// trajectory from tstart for its 64 tiles (audioop.mul floor on both channels),
// 8 frames at a time into LDS; then all 192 threads overlay
// sat16(sat16(lo + mid) + hi) (AME:210) and store q2 coalesced.
#ifndef MM_APPLY_STEP
#define MM_APPLY_STEP 8
#endif
constexpr int APPLY_TILES = 64, APPLY_STEP = MM_APPLY_STEP;

// -att / 20, correctly rounded (Markstein with RN(1/20) = 0.05; checked
// exhaustively on the attenuation range in tests/test_oracle.py)
__device__ __forceinline__ double neg_div20(double att) {
    const double q = -att * 0.05;
    const double rem = fma(-q, 20.0, -att);
    return fma(rem, 0.05, q);
}

__global__ void __launch_bounds__(192) comp_apply_kernel(CompArgs a) {
    __shared__ short2 lds[3][APPLY_STEP][APPLY_TILES];
    const int b = threadIdx.x / APPLY_TILES;
    const int lane = threadIdx.x % APPLY_TILES;
    const int64_t G = a.G;
    const int64_t g0 = (int64_t)blockIdx.x * APPLY_TILES;
    const int64_t g = g0 + lane;
    const bool valid = g < G;
    const int T = a.T;
    const int len = valid ? (int)min((int64_t)T, a.N_proc - g * T) : 0;
    const double *lut = a.lut[b];
    const BandStep bs = band_step(a, b);
    const uint16_t *R = a.r16[b];
    const short2 *X = a.band[b];
    double att = valid ? comp_state_at(a, b, g / a.K, a.off[b][g], bs) : 0.0;
    double gain = 1.0, gain_att = -1.0;  // gain = db_to_float(-gain_att); att >= 0 never equals -1
    uint16_t rn[APPLY_STEP];
    short2 vn[APPLY_STEP];
    auto prefetch = [&](int n0) {
#pragma unroll
        for (int j = 0; j < APPLY_STEP; ++j) {
            const int n = min(n0 + j, max(len - 1, 0));
            const int64_t idx = (int64_t)n * G + (valid ? g : 0);
            rn[j] = R[idx];
            vn[j] = X[idx];
        }
    };
    prefetch(0);
    for (int n0 = 0; n0 < T; n0 += APPLY_STEP) {
        short2 v[APPLY_STEP];
        double m[APPLY_STEP];
#pragma unroll
        for (int j = 0; j < APPLY_STEP; ++j) {
            v[j] = vn[j];
            m[j] = lut[rn[j]];
        }
        if (n0 + APPLY_STEP < T) prefetch(n0 + APPLY_STEP);
#pragma unroll
        for (int j = 0; j < APPLY_STEP; ++j) {
            if (n0 + j < len) {
                // M == 0 (rms <= threshold) is the identity step, and the gain only
                // changes with att: the sparse band's wave skips both almost always
                if (m[j] != 0.0) att = comp_step(att, m[j], bs);
                short2 s = v[j];
                if (att != 0.0) {
                    if (att != gain_att) {
                        gain = exp10(neg_div20(att));  // db_to_float(-att)
                        gain_att = att;
                    }
                    s.x = audioop_mul(s.x, gain);
                    s.y = audioop_mul(s.y, gain);
                }
                lds[b][j][lane] = s;
            }
        }
        lds_barrier();
        for (int p = threadIdx.x; p < APPLY_STEP * APPLY_TILES; p += 3 * APPLY_TILES) {
            const int j = p / APPLY_TILES, tl = p % APPLY_TILES;
            const int64_t gt = g0 + tl;
            const int n = n0 + j;
            if (gt < G && n < (int)min((int64_t)T, a.N_proc - gt * T)) {
                const short2 lo = lds[0][j][tl], mi = lds[1][j][tl], hi = lds[2][j][tl];
                const int16_t l = sat16(sat16((int32_t)lo.x + mi.x) + hi.x);
                const int16_t rr = sat16(sat16((int32_t)lo.y + mi.y) + hi.y);
                a.q_out[(int64_t)n * G + gt] = make_short2(l, a.ch == 2 ? rr : (int16_t)0);
            }
        }
        lds_barrier();
    }
}

}  // namespace mm
