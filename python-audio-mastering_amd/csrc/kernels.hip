// kernels.hip — CDNA4 (gfx950) kernels of the mastering chain.
//
// Layout: a track's processed timeline (AME:48-54 chunking) is cut into tiles of
// T frames; every 30 s chunk is a whole number of tiles (T | chunk frames), so a
// chunk never shares a tile.  One lane owns one tile and walks it sequentially
// (the IIR / envelope recurrences are sequential in time); lanes of a wave own
// consecutive tiles.  Intermediates are stored TILE-MAJOR: element (tile g,
// frame n) lives at n*G + g, so at every step a wave's 64 lanes touch 64
// consecutive elements -> fully coalesced HBM/L2 traffic for every pass after
// ingest.  Linear recurrences (EQ, crossover, K-weighting) use the two-pass block
// method: pass 1 = zero-state end state per tile, a scan of affine state maps
// across tiles (scan.hip), pass 2 = exact re-run from the carried state.
//
// Every per-lane walk is a software-pipelined stream (stream<> below): NB blocks
// of B frames are in flight in registers while the recurrence consumes the
// oldest block, which hides HBM/Infinity-Cache latency behind a single lane's
// dependent f64 chain (there are only ~1-2 waves per SIMD at C2 sizes).
#include "common.h"

namespace mm {

// ---------------------------------------------------------------- pointwise

// float_array_to_audio_segment (AME:123-126): clip to [-1,1] (NaN propagates),
// * 32768, astype(int16) == trunc to int32 then wrap to 16 bits; NaN -> 0.
__device__ __forceinline__ int16_t quantize(double v) {
    if (v != v) return 0;
    v = v > 1.0 ? 1.0 : v;
    v = v < -1.0 ? -1.0 : v;
    int32_t i = (int32_t)(v * 32768.0);
    return (int16_t)i;
}

// apply_saturation (AME:128-134), f32 throughout; no FMA contraction so the
// rounding sequence matches numpy: keep*x + mix*tanh(x*drive).
__device__ __forceinline__ float saturate(float x, const SatArgs &s) {
    float t = tanhf(__fmul_rn(x, s.drive));
    return __fadd_rn(__fmul_rn(s.keep, x), __fmul_rn(s.mix, t));
}

// audioop.mul of one int16 sample (pydub compressor output, AME:207-209).
__device__ __forceinline__ int16_t audioop_mul(int16_t x, double g) {
    double v = (double)x * g;
    if (v > 32767.0) v = 32767.0;
    else if (v < -32767.0) v = -32768.0;
    return (int16_t)(int32_t)floor(v);
}

__device__ __forceinline__ int16_t sat16(int32_t v) {
    return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v));
}

// ---------------------------------------------------------------- biquads
// DF2T section (scipy sosfilt / lfilter form): y = b0 x + z0;
// z0 = b1 x - a1 y + z1; z1 = b2 x - a2 y.  State s = (z0, z1).
// Written so that the y-independent halves (b1 x + z1, b2 x) sit off the
// recurrence's critical path.
__device__ __forceinline__ double df2t(double x, double &z0, double &z1, const double *c) {
    double y = fma(c[0], x, z0);
    double t0 = fma(c[1], x, z1);
    double t1 = c[2] * x;
    z0 = fma(-c[3], y, t0);
    z1 = fma(-c[4], y, t1);
    return y;
}

template <int NS>
__device__ __forceinline__ double cascade(double x, double (&z)[NS][2], const double (*sos)[5]) {
#pragma unroll
    for (int s = 0; s < NS; ++s) x = df2t(x, z[s][0], z[s][1], sos[s]);
    return x;
}

// ------------------------------------------------------- stage A: pre-chain
// Input: natural interleaved f32 (PCM16/32768), frames >= N_in read as 0
// (pydub pads a short final slice with silence).  Saturation f32, EQ cascade
// f64 (each active AME stage is one sosfilt section; zero-gain stages are
// dropped on the host), width f64, quantise -> q1 (tile-major short2).
// branch-free: the address is clamped into the buffer, padding frames read as 0
template <int CH>
__device__ __forceinline__ float2 load_in(const float *in, int64_t f, int64_t N_in) {
    const int64_t fc = min(f, N_in - 1);
    float2 v;
    if constexpr (CH == 2) v = *reinterpret_cast<const float2 *>(in + 2 * fc);
    else v = make_float2(in[fc], 0.f);
    return f < N_in ? v : make_float2(0.f, 0.f);
}

template <int NS, bool PASS2, int CH>
__global__ void __launch_bounds__(256) eq_kernel(StageArgs a) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.G) return;
    const int64_t f0 = g * a.T;
    const int len = (int)min((int64_t)a.T, a.N_proc - f0);
    constexpr int ch = CH;
    constexpr int D = 8;  // state stride per channel (MM_MAX_DIM), unused entries 0
    double zl[NS][2], zr[NS][2];
    if (PASS2) {
        const double *s = a.s_in + (g * ch) * D;
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            zl[k][0] = s[2 * k];
            zl[k][1] = s[2 * k + 1];
            if (ch == 2) {
                zr[k][0] = s[D + 2 * k];
                zr[k][1] = s[D + 2 * k + 1];
            } else {
                zr[k][0] = zr[k][1] = 0.0;
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < NS; ++k) zl[k][0] = zl[k][1] = zr[k][0] = zr[k][1] = 0.0;
    }
    const double(*sos)[5] = a.sos;
    int pn = 0;
    stream<8, 3, float2>(
        len, [&](int i) { return load_in<CH>(a.in, f0 + min(i, len - 1), a.N_in); },
        [&](float2 v) {
            float l = v.x, r = v.y;
            if (a.sat.on) {
                l = saturate(l, a.sat);
                r = saturate(r, a.sat);
            }
            double yl = cascade<NS>((double)l, zl, sos);
            double yr = ch == 2 ? cascade<NS>((double)r, zr, sos) : 0.0;
            if (PASS2) {
                if (a.width_on) {  // apply_stereo_width (AME:136-144) in f64
                    double mid = (yl + yr) / 2;
                    double side = (yl - yr) / 2 * a.width;
                    yl = mid + side;
                    yr = mid - side;
                }
                a.q_out[(int64_t)pn * a.G + g] = make_short2(quantize(yl), quantize(yr));
            }
            ++pn;
        });
    if (!PASS2) {
        double *z = a.z_out + (g * ch) * D;
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            z[2 * k] = zl[k][0];
            z[2 * k + 1] = zl[k][1];
            if (ch == 2) {
                z[D + 2 * k] = zr[k][0];
                z[D + 2 * k + 1] = zr[k][1];
            }
        }
        for (int k = 2 * NS; k < D; ++k) {
            z[k] = 0.0;
            if (ch == 2) z[D + k] = 0.0;
        }
    }
}

// No active EQ stage: the chain stays f32 (AME:152-162 returns the f32 input;
// width then runs in f32).
template <int CH>
__global__ void __launch_bounds__(256) pre_pointwise_kernel(StageArgs a) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.G) return;
    const int64_t f0 = g * a.T;
    const int len = (int)min((int64_t)a.T, a.N_proc - f0);
    int pn = 0;
    stream<8, 2, float2>(
        len, [&](int i) { return load_in<CH>(a.in, f0 + min(i, len - 1), a.N_in); },
        [&](float2 v) {
            float l = v.x, r = v.y;
            if (a.sat.on) {
                l = saturate(l, a.sat);
                r = saturate(r, a.sat);
            }
            if (a.width_on) {
                float w = (float)a.width;
                float mid = __fdiv_rn(__fadd_rn(l, r), 2.0f);
                float side = __fmul_rn(__fdiv_rn(__fsub_rn(l, r), 2.0f), w);
                l = __fadd_rn(mid, side);
                r = __fsub_rn(mid, side);
            }
            a.q_out[(int64_t)pn * a.G + g] =
                make_short2(quantize((double)l), a.ch == 2 ? quantize((double)r) : (int16_t)0);
            ++pn;
        });
}

// ------------------------------------------------------ stage B: crossover
// apply_multiband_compressor (AME:196-206): x = int16/32768 (f32), LP = butter(4)
// 250 Hz (2 SOS), HP = butter(4) 4 kHz (2 SOS), f64; mid = (x - lo) - hi;
// each band quantised.  Two branches of 2 sections share the input.
template <bool PASS2>
__global__ void __launch_bounds__(256) xover_kernel(StageArgs a) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.G) return;
    const int64_t f0 = g * a.T;
    const int len = (int)min((int64_t)a.T, a.N_proc - f0);
    const int ch = a.ch;
    constexpr int D = 8;
    double lo[2][2][2], hi[2][2][2];  // [channel][section][z]
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (PASS2 && c < ch) {
                const double *s = a.s_in + (g * ch + c) * D;
                lo[c][k][0] = s[2 * k];
                lo[c][k][1] = s[2 * k + 1];
                hi[c][k][0] = s[4 + 2 * k];
                hi[c][k][1] = s[4 + 2 * k + 1];
            } else {
                lo[c][k][0] = lo[c][k][1] = hi[c][k][0] = hi[c][k][1] = 0.0;
            }
        }
    const double(*sos)[5] = a.sos;
    int pn = 0;
    stream<8, 3, short2>(
        len, [&](int i) { return a.q_in[(int64_t)min(i, len - 1) * a.G + g]; },
        [&](short2 q) {
            const double x[2] = {(double)((float)q.x / 32768.0f), (double)((float)q.y / 32768.0f)};
            int32_t ob0[2] = {0, 0}, ob1[2] = {0, 0}, ob2[2] = {0, 0};
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (c >= ch) break;
                double yl = df2t(x[c], lo[c][0][0], lo[c][0][1], sos[0]);
                yl = df2t(yl, lo[c][1][0], lo[c][1][1], sos[1]);
                double yh = df2t(x[c], hi[c][0][0], hi[c][0][1], sos[2]);
                yh = df2t(yh, hi[c][1][0], hi[c][1][1], sos[3]);
                if (PASS2) {
                    double ym = (x[c] - yl) - yh;
                    ob0[c] = quantize(yl);
                    ob1[c] = quantize(ym);
                    ob2[c] = quantize(yh);
                }
            }
            if (PASS2) {
                const int64_t idx = (int64_t)pn * a.G + g;
                a.band_out[0][idx] = make_short2((int16_t)ob0[0], (int16_t)ob0[1]);
                a.band_out[1][idx] = make_short2((int16_t)ob1[0], (int16_t)ob1[1]);
                a.band_out[2][idx] = make_short2((int16_t)ob2[0], (int16_t)ob2[1]);
            }
            ++pn;
        });
    if (!PASS2) {
        for (int c = 0; c < ch; ++c) {
            double *z = a.z_out + (g * ch + c) * D;
            for (int k = 0; k < 2; ++k) {
                z[2 * k] = lo[c][k][0];
                z[2 * k + 1] = lo[c][k][1];
                z[4 + 2 * k] = hi[c][k][0];
                z[4 + 2 * k + 1] = hi[c][k][1];
            }
        }
    }
}

// ------------------------------------------------- stage D: K-weighting
// pyloudnorm Meter (AME:213-218): mono = f32 mean(L,R) (= (L+R)/65536 exactly),
// high_shelf lfilter in f64 stored back to f32, high_pass lfilter in f64
// stored to f32, then squared sums per 0.4 s/0.1 s block.  The whole track is
// one line (state carries across chunks).  Pass 2 accumulates per-tile partial
// energies of the (at most two) loudness segments the tile touches.
template <bool PASS2>
__global__ void __launch_bounds__(256) kweight_kernel(KwArgs a) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.G) return;
    const int64_t f0 = g * a.T;
    const int len = (int)min((int64_t)a.T, a.N_proc - f0);
    double z[2][2];
    if (PASS2) {
        const double *s = a.s_in + g * 4;
        z[0][0] = s[0];
        z[0][1] = s[1];
        z[1][0] = s[2];
        z[1][1] = s[3];
    } else {
        z[0][0] = z[0][1] = z[1][0] = z[1][1] = 0.0;
    }
    // segment bookkeeping
    int64_t seg = 0, seg_end = 0;
    if (PASS2) {
        int64_t lo = 0, hi = a.n_segs;  // largest s with bounds[s] <= f0
        while (hi - lo > 1) {
            int64_t mid = (lo + hi) >> 1;
            if (a.seg_bounds[mid] <= f0) lo = mid;
            else hi = mid;
        }
        seg = lo;
        seg_end = a.seg_bounds[seg + 1];
    }
    double e0 = 0.0, e1 = 0.0;
    int64_t pf = f0;
    stream<8, 3, short2>(
        len, [&](int i) { return a.mix[(int64_t)min(i, len - 1) * a.G + g]; },
        [&](short2 q) {
            float m = a.ch == 2 ? ((float)q.x + (float)q.y) * (1.0f / 65536.0f) : (float)q.x * (1.0f / 32768.0f);
            double y1 = df2t((double)m, z[0][0], z[0][1], a.sos[0]);
            float y1f = (float)y1;
            double y2 = df2t((double)y1f, z[1][0], z[1][1], a.sos[1]);
            if (PASS2) {
                float y2f = (float)y2;
                double e = (double)y2f * (double)y2f;
                if (pf < seg_end) e0 += e;
                else e1 += e;
            }
            ++pf;
        });
    if (PASS2) {
        a.part[2 * g] = e0;
        a.part[2 * g + 1] = e1;
        a.part_seg[g] = seg;
    } else {
        double *zo = a.z_out + g * 4;
        zo[0] = z[0][0];
        zo[1] = z[0][1];
        zo[2] = z[1][0];
        zo[3] = z[1][1];
    }
}

// Sum the per-tile partials into loudness segments (deterministic order).
__global__ void seg_reduce_kernel(KwArgs a, double *seg_energy) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= a.n_segs) return;
    int64_t b0 = a.seg_bounds[s], b1 = a.seg_bounds[s + 1];
    if (b1 > a.N_proc) b1 = a.N_proc;
    double acc = 0.0;
    if (b0 < b1) {
        int64_t g0 = b0 / a.T, g1 = (b1 - 1) / a.T;
        for (int64_t g = g0; g <= g1; ++g) {
            if (a.part_seg[g] == s) acc += a.part[2 * g];
            else if (a.part_seg[g] == s - 1) acc += a.part[2 * g + 1];
        }
    }
    seg_energy[s] = acc;
}

// ------------------------------------------------ stage E: gain + limiter
// AME:84-89: y = int16/32768 (f32); with a loudness target the gain is an
// np.float64 so y*gain, the soft limiter and the clip run in f64; without
// one they run in f32.  Output natural interleaved layout.  A block handles
// FIN_TILES tiles: the tile-major mix is read coalesced into LDS, then written
// out frame-major coalesced.
constexpr int FIN_TILES = 32;

__device__ __forceinline__ double limiter64(double y) {
    double ay = fabs(y);
    if (ay > 0.98) {
        double d = ay - 0.98;
        double t = d / 0.02;
        double den = sqrt(1.0 + t * t);
        double v = 0.98 + d / den;
        double sg = y > 0 ? 1.0 : (y < 0 ? -1.0 : y);
        y = v * sg;
    }
    return y;
}

__device__ __forceinline__ float limiter32(float y) {
    float ay = fabsf(y);
    if (ay > 0.98f) {
        float d = __fsub_rn(ay, 0.98f);
        float t = __fdiv_rn(d, 0.02f);
        float den = __fsqrt_rn(__fadd_rn(1.0f, __fmul_rn(t, t)));
        float v = __fadd_rn(0.98f, __fdiv_rn(d, den));
        float sg = y > 0 ? 1.0f : (y < 0 ? -1.0f : y);
        y = __fmul_rn(v, sg);
    }
    return y;
}

__global__ void __launch_bounds__(256) finalize_kernel(FinArgs a) {
    extern __shared__ short2 lds[];  // [FIN_TILES][T+1]
    const int T = a.T;
    const int stride = T + 1;
    const int64_t g0 = (int64_t)blockIdx.x * FIN_TILES;
    const int ntile = (int)min((int64_t)FIN_TILES, a.G - g0);
    for (int i = threadIdx.x; i < T * FIN_TILES; i += blockDim.x) {
        int n = i / FIN_TILES, t = i - n * FIN_TILES;
        if (t < ntile) lds[t * stride + n] = a.mix[(int64_t)n * a.G + g0 + t];
    }
    __syncthreads();
    const int64_t f_base = g0 * T;
    const int64_t nf = min((int64_t)ntile * T, a.N_proc - f_base);
    for (int64_t i = threadIdx.x; i < nf; i += blockDim.x) {
        int t = (int)(i / T), n = (int)(i - (int64_t)t * T);
        short2 q = lds[t * stride + n];
        int16_t o[2];
        const int16_t qq[2] = {q.x, q.y};
        for (int c = 0; c < a.ch; ++c) {
            float y = (float)qq[c] / 32768.0f;
            if (a.use_gain) {
                double v = (double)y * a.gain;
                o[c] = quantize(limiter64(v));
            } else {
                o[c] = quantize((double)limiter32(y));
            }
        }
        const int64_t f = f_base + i;
        if (a.out_kind == 0) {
            int16_t *out = reinterpret_cast<int16_t *>(a.out);
            if (a.ch == 2) *reinterpret_cast<short2 *>(out + 2 * f) = make_short2(o[0], o[1]);
            else out[f] = o[0];
        } else {
            float *out = reinterpret_cast<float *>(a.out);
            if (a.ch == 2) *reinterpret_cast<float2 *>(out + 2 * f) = make_float2(o[0] / 32768.0f, o[1] / 32768.0f);
            else out[f] = o[0] / 32768.0f;
        }
    }
}

// copy the tile-major mix to natural interleaved int16 (parity probe)
__global__ void mix_to_natural_kernel(const short2 *mix, int16_t *out, int64_t G, int T, int64_t N, int ch) {
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= N) return;
    int64_t g = f / T, n = f - g * T;
    short2 q = mix[n * G + g];
    if (ch == 2) {
        out[2 * f] = q.x;
        out[2 * f + 1] = q.y;
    } else {
        out[f] = q.x;
    }
}

// explicit instantiations used by the host
template __global__ void xover_kernel<false>(StageArgs);
template __global__ void xover_kernel<true>(StageArgs);
template __global__ void kweight_kernel<false>(KwArgs);
template __global__ void kweight_kernel<true>(KwArgs);

}  // namespace mm
