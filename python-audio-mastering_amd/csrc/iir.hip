// iir.hip — the three linear-recurrence stages of the chain, one launch each.
//
// A lane owns one tile (T frames) of ONE channel: stereo tiles use lane pairs
// (even lane = left, odd lane = right), which doubles the lanes in flight over a
// lane-per-tile layout and keeps the per-frame f64 chain short.  Each kernel
// runs its recurrence twice over the tile: pass 1 from the zero state (end state
// z), lookback.h's in-kernel carry, pass 2 from the exact carry producing the
// stage outputs.  Intermediates are tile-major int16 pairs: element (tile g,
// frame n, channel c) at (n*G + g)*2 + c, so a wave's 64 lanes touch 128
// consecutive bytes at every step.
//
//   eq_kernel      AME:55-63   f32 input -> exciter (f32) -> EQ (<=4 DF2T, f64)
//                              -> width (f64, lane-pair exchange) -> int16 q1
//   xover_kernel   AME:196-206 q1/32768 -> LP4 250 Hz + HP4 4 kHz (f64),
//                              mid = x - lo - hi -> three int16 band planes
//   kweight_kernel AME:213-218 mix -> mono f32 -> pyloudnorm high shelf + high
//                              pass (f64, f32 between) -> per-tile energies of
//                              the 0.1 s loudness segments
#include "lookback.h"

namespace mm {

// float_array_to_audio_segment (AME:123-126): clip to [-1,1] (NaN propagates),
// * 32768, astype(int16) == trunc to int32 then wrap to 16 bits; NaN -> 0.
// Three instructions: v * 2^15 is exact, v_cvt_i32_f64 truncates, saturates out
// of range values (infinities included) and maps NaN to 0, and v_med3_i32 clamps
// to [-32768, 32768] — the same integer as trunc(clip(v) * 32768) for every v.
// The caller keeps the low 16 bits (32768 wraps to -32768, as astype(int16)).
__device__ __forceinline__ int32_t quantize_i32(double v) {
    int32_t i;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(i) : "v"(v * 32768.0));
    return min(max(i, -32768), 32768);
}
__device__ __forceinline__ int16_t quantize(double v) { return (int16_t)quantize_i32(v); }

// tanhf without a branch: OCML's __ocml_tanh_f32 (ROCm 7.2 ocml.bc) operation for
// operation — |x| < 0.625: the odd polynomial |x| + x^2 |x| P(x^2) (FMAs), else
// 1 - 2 / (exp(2|x|) + 1) with OCML's expf and v_rcp_f32 — both evaluated and one
// selected, then copysign.  Bit-identical to tanhf (whose divergent if/else runs
// both paths in most waves anyway, behind exec-mask branches that keep the
// scheduler from overlapping a frame's tanh with the previous frame's f64 chain).
__device__ __forceinline__ float tanh_sel(float x) {
    const float ax = fabsf(x);
    const float x2 = __fmul_rn(x, x);
    float p = fmaf(x2, -0x1.758e7ap-8f, 0x1.521192p-6f);
    p = fmaf(x2, p, -0x1.b8389cp-5f);
    p = fmaf(x2, p, 0x1.110704p-3f);
    p = fmaf(x2, p, -0x1.555532p-2f);
    const float small = fmaf(x2, __fmul_rn(ax, p), ax);
    const float e = expf(__fmul_rn(ax, 2.0f));
    const float big = fmaf(-2.0f, __builtin_amdgcn_rcpf(__fadd_rn(e, 1.0f)), 1.0f);
    return copysignf(ax < 0.625f ? small : big, x);
}

// apply_saturation (AME:128-134), f32 throughout; no FMA contraction so the
// rounding sequence matches numpy: keep*x + mix*tanh(x*drive).  Inputs on the
// int16 grid (every decoded PCM16 sample, AME:121) read the host's table of the
// reference's own numpy evaluation (bit-identical); only off-grid inputs (f32
// WAV) evaluate tanhf here (within 2 ulp of numpy's float32 tanh).
// The device's own evaluation (tanhf: within 2 ulp of numpy's float32 tanh).
__device__ __forceinline__ float saturate_dev(float x, const SatArgs &s) {
#ifdef MM_ABLATE_TANH  // timing-only builds (tools/ablate.sh): the exciter without its tanh
    float t = __fmul_rn(x, s.drive);
#elif defined(MM_TANH_SEL)
    float t = tanh_sel(__fmul_rn(x, s.drive));
#else
    float t = tanhf(__fmul_rn(x, s.drive));
#endif
    return __fadd_rn(__fmul_rn(s.keep, x), __fmul_rn(s.mix, t));
}
// With the correction codes: the device value, then the signed 2-bit code of its
// grid entry (numpy minus device as float bit patterns: 0, +1, -1) moves it onto
// numpy's bits.  One code per grid index i = k + 32768 (16 per word, 16 KB, in the
// EQ kernel's LDS): one unsigned range check, one LDS word, one signed bit-field
// extract (round 6's first version folded |k| into an 8 KB table: 5 more VALU per
// sample).  The codes are only used when every entry is within one step
// (sat_corr_kernel's exception count, checked on the host once per table): then the
// exciter issues no global load in the EQ's per-frame loop (a conditional one there
// made the compiler drain the staging prefetch at every frame).  Without them
// (pointwise operators): the full table's entry, a gather per sample.
__device__ __forceinline__ float saturate_corr(float x, const SatArgs &s, const uint32_t *corr) {
    float y = saturate_dev(x, s);
    const float sc = x * 32768.0f;  // exact
    const int k = (int)sc;
    const unsigned i = (unsigned)(k + 32768);
    if ((float)k == sc && i < 65536u) {
        const int d = __builtin_amdgcn_sbfe((int)corr[i >> 4], (i & 15u) * 2u, 2u);
        y = __int_as_float(__float_as_int(y) + d);
    }
    return y;
}
__device__ __forceinline__ float saturate(float x, const SatArgs &s) {
    float y;
    if (s.corr) return saturate_corr(x, s, s.corr);
    if (s.tab && sat_lookup(x, s.tab, &y)) return y;
    return saturate_dev(x, s);
}

constexpr int SAT_CORR_WORDS = 4096;  // i = k + 32768 = 0 .. 65535, 16 codes per word (16 KB)
// Builds SatArgs::corr from SatArgs::tab: thread w packs i = 16w .. 16w + 15 as signed
// 2-bit fields; exceptions[0] counts entries more than one step apart (their field
// is 0 and the codes are not used).
__global__ void __launch_bounds__(256) sat_corr_kernel(SatArgs s, uint32_t *corr, unsigned *exceptions) {
    const int w = blockIdx.x * 256 + threadIdx.x;
    if (w >= SAT_CORR_WORDS) return;
    uint32_t word = 0;
    for (int e = 0; e < 16; ++e) {
        const int i = w * 16 + e, k = i - 32768;
        const float x = (float)k * (1.0f / 32768.0f);
        const int d = __float_as_int(s.tab[i]) - __float_as_int(saturate_dev(x, s));
        if (d < -1 || d > 1) atomicAdd(exceptions, 1u);
        else word |= ((uint32_t)d & 3u) << (2 * e);
    }
    corr[w] = word;
}

// The exciter as a pointwise pre-pass (decoded input -> f32), for the EQ kernel when
// the correction codes are incomplete: the full table per grid sample, tanhf off it.
__global__ void __launch_bounds__(256) sat_pre_kernel(const float *in, const int16_t *in16, int64_t n, SatArgs s,
                                                      float *out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = in16 ? (float)in16[i] * (1.0f / 32768.0f) : in[i];
    out[i] = saturate(x, s);
}

// apply_stereo_width (AME:136-144) on a lane pair, one formula for both lanes:
// with y this lane's sample and o its partner's, the left lane's mid + side and
// the right lane's mid - side are both RN(RN(y + o)/2 + RN(RN(y - o) * (w/2)))
// (RN(o - y) = -RN(y - o); halving and w/2 are exact), and RN(s/2 + side) is
// fma(s, 0.5, side).  No lane-dependent selects.  hw = width / 2.
__device__ __forceinline__ double widen_pair(double y, double hw) {
    const double o = pair_swap(y);
    const double side = (y - o) * hw;
    return fma(y + o, 0.5, side);
}

// DF2T section (scipy sosfilt / lfilter form): y = b0 x + z0;
// z0 = b1 x - a1 y + z1; z1 = b2 x - a2 y.  State s = (z0, z1).
// SCIPY: scipy's _sosfilt operation order, every product and sum rounded
// (y = b0*x + z0; z0 = (b1*x - a1*y) + z1; z1 = b2*x - a2*y; matched bit for bit
// against scipy.signal.sosfilt on random data): the passes whose outputs are
// quantised (AME:63, 204-206) use it, so with the same state they produce
// scipy's bits.  Otherwise fused (the zero-state passes that only feed the
// tiles' carry maps).
// scipy.signal.lfilter's order (_sigtools lfilter.c, one section, a0 == 1): y = Z0 +
// b0 x; Z0 = (Z1 + x b1) - y a1; Z1 = x b2 - y a2, every product and sum rounded
// (no contraction: built with -ffp-contract=off).  pyloudnorm's K-weighting
// filters are lfilter calls (AME:217).
__device__ __forceinline__ double df2t_lfilter(double x, double &z0, double &z1, const double *c) {
    const double y = z0 + c[0] * x;
    z0 = (z1 + x * c[1]) - y * c[3];
    z1 = x * c[2] - y * c[4];
    return y;
}

template <bool SCIPY = false>
__device__ __forceinline__ double df2t(double x, double &z0, double &z1, const double *c) {
    if constexpr (SCIPY) {
        const double y = c[0] * x + z0;
        z0 = (c[1] * x - c[3] * y) + z1;
        z1 = c[2] * x - c[4] * y;
        return y;
    } else {
        double y = fma(c[0], x, z0);
        double t0 = fma(c[1], x, z1);
        double t1 = c[2] * x;
        z0 = fma(-c[3], y, t0);
        z1 = fma(-c[4], y, t1);
        return y;
    }
}

// ------------------------------------------------------------------ EQ stage
#ifndef MM_EQ_STAGE
#define MM_EQ_STAGE 16
#endif
#ifndef MM_XO_NB
#define MM_XO_NB 3
#endif
#ifndef MM_EQ_NB
#define MM_EQ_NB 3
#endif
#ifndef MM_KW_NB
#define MM_KW_NB 3
#endif
constexpr int EQ_STAGE = MM_EQ_STAGE;  // frames per tile staged through LDS per step

struct EqArgs {
    const float *in;   // natural interleaved f32 input (or null when in16 is set)
    const int16_t *in16;  // natural interleaved int16 PCM input, decoded as x / 32768
    int64_t N_in;      // valid input frames (later frames read as 0: pydub pads)
    int64_t N_proc;    // processed frames
    int64_t G;         // tiles
    int T;             // frames per tile
    SatArgs sat;
    double width;
    int width_on;
    double sos[4][5];  // {b0,b1,b2,a1,a2}
    int16_t *q_out;    // tile-major int16 pairs
    float *xs;         // tile-major f32 scratch: pass 1 leaves the exciter's output here for pass 2
};

// Staging buffer: two steps of EQ_STAGE frames for the block's TPB tiles (rows
// padded by one frame against bank conflicts); the look-back scratch aliases it
// between the passes.  The exciter's codes are a static 16 KB beside it (51 KB per
// block: three blocks per CU, as with round 6's first 8 KB table; an unpadded
// XOR-swizzled stage with the codes in its place, four blocks per CU, measured
// slower: eq 0.234 against 0.173 ms).
template <int CH>
constexpr int eq_stage_bytes() {
    return 2 * (LB_THREADS / CH) * (EQ_STAGE + 1) * CH * (int)sizeof(float);
}
template <int NS, int CH>
constexpr int eq_lds_bytes() {
    return eq_stage_bytes<CH>() > lb_lds_bytes<2 * NS, CH>() ? eq_stage_bytes<CH>() : lb_lds_bytes<2 * NS, CH>();
}

// One pass over the block's tiles with the input staged through LDS: the block
// cooperatively loads EQ_STAGE frames of each of its tiles (16 consecutive
// threads read one tile's 128 contiguous bytes), double-buffered so the next
// stage's loads are in flight while lanes run the recurrence.
template <int NS, int CH, bool P2, bool I16>
__device__ void eq_pass(const EqArgs &a, int64_t g0, int t, int c, int len, double (&z)[NS][2], float *stage,
                        const uint32_t *codes) {
    constexpr int TPB = LB_THREADS / CH;
    constexpr int ROW = (EQ_STAGE + 1) * CH;       // floats per staged tile row (padded)
    constexpr int ITEMS = TPB * EQ_STAGE / LB_THREADS;  // frames each thread loads per step
    const int T = a.T;
    const int nsteps = (T + EQ_STAGE - 1) / EQ_STAGE;
    const int tid = threadIdx.x;
    const double(*sos)[5] = a.sos;
    float regs[ITEMS][CH];
    auto load = [&](int step) {
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const int idx = tid + r * LB_THREADS;
            const int tt = idx / EQ_STAGE, j = idx % EQ_STAGE;
            const int n = step * EQ_STAGE + j;
            const int64_t f = (g0 + tt) * T + n;
            const bool ok = n < T && f < a.N_in;  // also excludes tiles past the track end
            const int64_t fc = ok ? f : 0;
            if constexpr (I16) {  // int16 -> f32 / 32768 is exact (AME:117-121)
                if constexpr (CH == 2) {
                    const short2 v = *reinterpret_cast<const short2 *>(a.in16 + 2 * fc);
                    regs[r][0] = ok ? (float)v.x * (1.0f / 32768.0f) : 0.f;
                    regs[r][1] = ok ? (float)v.y * (1.0f / 32768.0f) : 0.f;
                } else {
                    regs[r][0] = ok ? (float)a.in16[fc] * (1.0f / 32768.0f) : 0.f;
                }
            } else if constexpr (CH == 2) {
                const float2 v = *reinterpret_cast<const float2 *>(a.in + 2 * fc);
                regs[r][0] = ok ? v.x : 0.f;
                regs[r][1] = ok ? v.y : 0.f;
            } else {
                const float v = a.in[fc];
                regs[r][0] = ok ? v : 0.f;
            }
        }
    };
    // The exciter runs here, on the staged values, once per sample (its codes are LDS
    // reads: no vector-memory wait in the per-frame loop below)
    // The exciter runs in the per-frame loop below: tanhf fills the issue slots the
    // f64 chain leaves, and its correction codes are LDS reads, so no vector-memory
    // wait sits in that loop (one would drain the staging prefetch at every frame).
    // An incomplete code table (no known input) is applied by sat_pre_kernel before
    // this kernel instead (the EQ then runs with the exciter off).
    auto store = [&](int buf) {
#pragma unroll
        for (int r = 0; r < ITEMS; ++r) {
            const int idx = tid + r * LB_THREADS;
            const int tt = idx / EQ_STAGE, j = idx % EQ_STAGE;
            float *dst = stage + buf * TPB * ROW + tt * ROW + j * CH;
#pragma unroll
            for (int q = 0; q < CH; ++q) dst[q] = regs[r][q];
        }
    };
    load(0);
    store(0);
    lds_barrier();
    const int64_t g = g0 + t;
    for (int step = 0; step < nsteps; ++step) {
        const int cur = step & 1;
        if (step + 1 < nsteps) load(step + 1);
        const float *row = stage + cur * TPB * ROW + t * ROW;
#pragma unroll 4
        for (int j = 0; j < EQ_STAGE; ++j) {
            const int n = step * EQ_STAGE + j;
            if (n >= len) break;
            float x = row[j * CH + c];
            // (no global load may sit in this loop, even unexecuted: the compiler's waits
            // would drain the staging prefetch; the full-table case runs as a pre-pass)
            if (a.sat.on) x = codes ? saturate_corr(x, a.sat, codes) : saturate_dev(x, a.sat);
            if (!P2) a.xs[((int64_t)n * a.G + g0 + t) * CH + c] = x;  // pass 2 reads it back coalesced
            double y = (double)x;
#pragma unroll
            for (int s = 0; s < NS; ++s) y = df2t<P2>(y, z[s][0], z[s][1], sos[s]);
            if (P2) {
                if (CH == 2 && a.width_on) y = widen_pair(y, a.width * 0.5);  // AME:136-144, f64
                const int64_t o = ((int64_t)n * a.G + g) * 2;
                if (CH == 2) a.q_out[o + c] = quantize(y);
                else *reinterpret_cast<short2 *>(a.q_out + o) = make_short2(quantize(y), 0);  // mono: R = 0
            }
        }
        if (step + 1 < nsteps) store(cur ^ 1);
        lds_barrier();
    }
}

// Pass 2 from the tile-major exciter output pass 1 left in a.xs: the lane's own
// frames, 64 lanes reading 256 contiguous bytes per step, no LDS staging, barrier
// or second tanh.  EQ -> width (lane-pair exchange) -> int16.
template <int NS, int CH>
__device__ void eq_pass2(const EqArgs &a, int64_t g, int c, int len, double (&z)[NS][2]) {
    const double(*sos)[5] = a.sos;
    const int64_t G = a.G;
    const float *xs = a.xs;
    int n = 0;
    stream<8, MM_EQ_NB, float>(
        len, [&](int i) { return xs[((int64_t)min(i, len - 1) * G + g) * CH + c]; },
        [&](float x) {
            double y = (double)x;
#pragma unroll
            for (int s = 0; s < NS; ++s) y = df2t<true>(y, z[s][0], z[s][1], sos[s]);
            if (CH == 2 && a.width_on) y = widen_pair(y, a.width * 0.5);  // AME:136-144, f64
            const int64_t o = ((int64_t)n * G + g) * 2;
            if (CH == 2) a.q_out[o + c] = quantize(y);
            else *reinterpret_cast<short2 *>(a.q_out + o) = make_short2(quantize(y), 0);  // mono: R = 0
            ++n;
        });
}

// ---- full-tile fast paths ----------------------------------------------------
// Every block but the track's last holds TPB whole tiles, so its lanes run the
// same T frames: the frame index is wave-uniform, every row address is a scalar
// row base plus the lane's constant offset (no per-frame 64-bit index math), the
// loops carry no per-lane exit, and the exciter / width switches are template
// arguments instead of per-frame tests.

// pass 2 from the scratch: EQ (scipy order) -> width -> int16, all rows uniform
template <int NS, int CH, bool WIDTH>
__device__ void eq_pass2_full(const EqArgs &a, int64_t g0, double (&z)[NS][2]) {
    const double(*sos)[5] = a.sos;
    const int T = a.T;
    const uint32_t tid = threadIdx.x;  // (unsigned: scalar row base + 32-bit lane offset)
    const int64_t GC = a.G * CH;
    const float *xs0 = a.xs + g0 * CH;
    const double hw = a.width * 0.5;
    int16_t *q0 = a.q_out + g0 * 2;  // the block's first pair of row 0
    const int64_t G2 = a.G * 2;
    int n = 0;
    stream<8, MM_EQ_NB, float>(
        T, [&](int i) { return (xs0 + (int64_t)min(i, T - 1) * GC)[tid]; },
        [&](float x) {
            double y = (double)x;
#pragma unroll
            for (int s = 0; s < NS; ++s) y = df2t<true>(y, z[s][0], z[s][1], sos[s]);
            if constexpr (CH == 2 && WIDTH) y = widen_pair(y, hw);
            int16_t *qr = q0 + (int64_t)n * G2;
            if constexpr (CH == 2) qr[tid] = quantize(y);
            else reinterpret_cast<short2 *>(qr)[tid] = make_short2(quantize(y), 0);  // mono: R = 0
            ++n;
        });
}

// I16: the input is int16 PCM (a.in16), else f32 (a.in); a template parameter so
// the staging loads carry no runtime branch (it costs registers and spills).
template <int NS, int CH, bool I16>
__global__ void __launch_bounds__(LB_THREADS, 4) eq_kernel(EqArgs a, LbArgs lb, int64_t line_tiles) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int TPB = LB_THREADS / CH;
    constexpr int DIM = 2 * NS;
    __shared__ int ticket_slot;
    __shared__ uint32_t codes_lds[SAT_CORR_WORDS];  // the exciter's correction codes for pass 1
    const int blk = lb_ticket(lb, &ticket_slot);
    const int tid = threadIdx.x;
    const int c = CH == 2 ? (tid & 1) : 0;
    const int t = tid / CH;
    const int64_t g0 = (int64_t)blk * TPB;
    const int64_t g = g0 + t;
    const bool valid = g < a.G;
    const int len = valid ? (int)min((int64_t)a.T, a.N_proc - g * a.T) : 0;
    // the look-back scratch is live only between the passes: it aliases the
    // staging buffer, so four blocks fit a CU (eq_lds_bytes)
    float *stage = reinterpret_cast<float *>(smem);
    double *lds = smem;
    double zs[NS][2];
#pragma unroll
    for (int s = 0; s < NS; ++s) zs[s][0] = zs[s][1] = 0.0;
    // block-uniform: every tile of the block is whole (all blocks but the track's last).
    // Pass 1 stays the general LDS-staged loop at every block (a uniform-row variant
    // with the exciter switch as a template argument measured slower: eq 0.152 ->
    // 0.166 ms); pass 2 takes the uniform-row path on full blocks.
    const bool full = (g0 + TPB) * a.T <= a.N_proc;
#ifndef MM_ABL_EQ_NOP1  // (ablation builds: timing only)
    // the exciter's correction codes into LDS (ordered before their reads by eq_pass's
    // first barrier)
    const bool codes_on = a.sat.on && a.sat.corr;
    if (codes_on)
        for (int i = tid; i < SAT_CORR_WORDS; i += LB_THREADS) codes_lds[i] = a.sat.corr[i];
    eq_pass<NS, CH, false, I16>(a, g0, t, c, len, zs, stage, codes_on ? codes_lds : nullptr);
#endif
    double z[DIM], s[DIM], rst[DIM];
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) {
        z[2 * s_] = zs[s_][0];
        z[2 * s_ + 1] = zs[s_][1];
    }
#pragma unroll
    for (int d = 0; d < DIM; ++d) rst[d] = 0.0;
#ifndef MM_ABL_EQ_NOLB  // (ablation builds: timing only)
    lb_carry<DIM, CH>(lb, blk, t, c, valid, valid && (g % line_tiles) == 0, rst, z, s, lds);
#else
#pragma unroll
    for (int d = 0; d < DIM; ++d) s[d] = z[d] + rst[d];
#endif
    __syncthreads();  // every lane has read the look-back scratch before pass 2 stages into it
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) {
        zs[s_][0] = s[2 * s_];
        zs[s_][1] = s[2 * s_ + 1];
    }
#ifdef MM_ABL_EQ_NOP2  // (ablation builds: timing only)
    return;
#endif
#ifdef MM_EQ_P2_GENERIC  // (ablation builds)
    if (false) {
#else
    if (full) {
#endif
        if (CH == 2 && a.width_on) eq_pass2_full<NS, CH, true>(a, g0, zs);
        else eq_pass2_full<NS, CH, false>(a, g0, zs);
    } else if (valid) {
        eq_pass2<NS, CH>(a, g, c, len, zs);
    }
}

// No active EQ stage: the chain stays f32 (AME:152-162 returns the f32 input;
// width then runs in f32).  Pointwise; natural layout in, tile-major out.
template <int CH>
__global__ void __launch_bounds__(256) pre_pointwise_kernel(EqArgs a) {
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= a.N_proc) return;
    float v[2] = {0.f, 0.f};
    if (f < a.N_in && a.in16) {
        v[0] = (float)a.in16[CH * f] * (1.0f / 32768.0f);
        if constexpr (CH == 2) v[1] = (float)a.in16[2 * f + 1] * (1.0f / 32768.0f);
    } else if (f < a.N_in) {
        if constexpr (CH == 2) {
            const float2 x = *reinterpret_cast<const float2 *>(a.in + 2 * f);
            v[0] = x.x;
            v[1] = x.y;
        } else {
            v[0] = a.in[f];
        }
    }
    if (a.sat.on) {
        v[0] = saturate(v[0], a.sat);
        v[1] = saturate(v[1], a.sat);
    }
    if (CH == 2 && a.width_on) {
        const float w = (float)a.width;
        const float mid = __fdiv_rn(__fadd_rn(v[0], v[1]), 2.0f);
        const float side = __fmul_rn(__fdiv_rn(__fsub_rn(v[0], v[1]), 2.0f), w);
        v[0] = __fadd_rn(mid, side);
        v[1] = __fsub_rn(mid, side);
    }
    const int64_t g = f / a.T, n = f - g * a.T;
    const int64_t o = (n * a.G + g) * 2;
    a.q_out[o] = quantize((double)v[0]);
    a.q_out[o + 1] = CH == 2 ? quantize((double)v[1]) : (int16_t)0;
}

// ------------------------------------------------------------ crossover stage
struct XoArgs {
    int64_t N_proc, G;
    int T;
    double sos[4][5];     // LP s0, LP s1, HP s0, HP s1
    const int16_t *q_in;  // tile-major int16 pairs
    int16_t *band[3];     // low / mid / high planes, same layout
    // per tile and band, for the compressor's RMS windows (exact integer sums in
    // f64): E = sum of L^2 + R^2 over the tile, tail = the same over its last
    // frames n >= tail_from (the window's partial tile, look % T frames)
    double *E[3], *tail[3];
    int tail_from[3];
    const double *zw;     // [T][8] zero-state weights (zs_weights; null: pass 1 runs the recurrence)
};

// this lane's channel's q^2; the lane pair's sums are added once per tile (exact
// integers below 2^53 in any order), so no per-frame lane exchange
__device__ __forceinline__ double sample_energy(int16_t q) {
    const int32_t v = q;
    return (double)(uint32_t)(v * v);
}

template <int CH, bool P2>
__device__ __forceinline__ void xo_pass(const XoArgs &a, int64_t g, int c, int len, double (&z)[4][2]) {
    const double(*sos)[5] = a.sos;
    const int64_t G = a.G;
    int pn = 0;
    double E[3] = {0.0, 0.0, 0.0}, tl[3] = {0.0, 0.0, 0.0};
    stream<8, MM_XO_NB, int16_t>(
        len, [&](int i) { return a.q_in[((int64_t)min(i, len - 1) * G + g) * 2 + c]; },
        [&](int16_t q) {
            const double x = (double)((float)q / 32768.0f);  // AME:199 int16 -> f32
            double yl = df2t<P2>(x, z[0][0], z[0][1], sos[0]);
            yl = df2t<P2>(yl, z[1][0], z[1][1], sos[1]);
            double yh = df2t<P2>(x, z[2][0], z[2][1], sos[2]);
            yh = df2t<P2>(yh, z[3][0], z[3][1], sos[3]);
            if (P2) {
                const double ym = (x - yl) - yh;  // AME:202
                const int64_t o = ((int64_t)pn * G + g) * 2;
                const int16_t q[3] = {quantize(yl), quantize(ym), quantize(yh)};
                if (CH == 2) {
#pragma unroll
                    for (int b = 0; b < 3; ++b) a.band[b][o + c] = q[b];
                } else {  // mono: the second half of every pair stays 0
#pragma unroll
                    for (int b = 0; b < 3; ++b) *reinterpret_cast<short2 *>(a.band[b] + o) = make_short2(q[b], 0);
                }
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    const double e = sample_energy(q[b]);
                    E[b] += e;
                    tl[b] += pn >= a.tail_from[b] ? e : 0.0;
                }
            }
            ++pn;
        });
    if (P2 && CH == 2) {  // L^2 + R^2 sums of the lane pair
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            E[b] += pair_swap(E[b]);
            tl[b] += pair_swap(tl[b]);
        }
    }
    if (P2 && c == 0) {
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            a.E[b][g] = E[b];
            a.tail[b][g] = tl[b];
        }
    }
}

// Full-tile fast path (every block but the track's last): uniform rows, scalar
// row bases, int16 -> f64 in two instructions (q * 2^-15 is exact, and equals
// AME:199's f32 q / 32768 widened), and the band energies as exact 64-bit integer
// multiply-adds (v_mad_i64_i32) of the pre-wrap quantiser output (+-32768 square
// alike); the tail sums take the frames n >= tail_from through a select on the
// uniform frame index.
// ZW (pass 1 of a block of whole tiles): the tile's zero-state end state as the
// product of its T inputs with the stage's zero-state weights, z_d = sum_n W[n][d]
// x_n (mastering.hip zs_weights): 8 independent FMAs per frame for the two
// branches' 4 sections in place of the recurrence's chained sections, the weights
// read from LDS (wl: the block's copy, broadcast reads; as scalar loads the
// per-frame load latency was exposed: xover 0.150 against 0.126 ms).
template <int CH, bool P2, bool ZW = false>
__device__ __forceinline__ void xo_pass_full(const XoArgs &a, int64_t g0, int tid, double (&z)[4][2],
                                             const double *wl = nullptr) {
    const double(*sos)[5] = a.sos;
    const int T = a.T;
    const int64_t G2 = a.G * 2;
    const int16_t *qin0 = a.q_in + g0 * 2;  // the block's first element of row 0
    const uint32_t lo = CH == 2 ? (uint32_t)tid : 2u * tid;  // this lane's int16 within the row
    int16_t *b0 = a.band[0] + g0 * 2, *b1 = a.band[1] + g0 * 2, *b2 = a.band[2] + g0 * 2;
    int pn = 0;
    // exact integer sums in doubles (< 2^53); the tail weight is 0 or 1 (uniform)
    double Ed[3] = {0.0, 0.0, 0.0}, td[3] = {0.0, 0.0, 0.0};
    stream<8, MM_XO_NB, int16_t>(
        T, [&](int i) { return (qin0 + (int64_t)min(i, T - 1) * G2)[lo]; },
        [&](int16_t q) {
            const double x = (double)(int32_t)q * (1.0 / 32768.0);  // AME:199 int16 -> f32, exact
            if constexpr (ZW && !P2) {
                const double2 *w2 = reinterpret_cast<const double2 *>(wl + pn * 8);
                double w[8];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const double2 v = w2[k];
                    w[2 * k] = v.x;
                    w[2 * k + 1] = v.y;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    z[k][0] = fma(w[2 * k], x, z[k][0]);
                    z[k][1] = fma(w[2 * k + 1], x, z[k][1]);
                }
                ++pn;
                return;
            }
            double yl = df2t<P2>(x, z[0][0], z[0][1], sos[0]);
            yl = df2t<P2>(yl, z[1][0], z[1][1], sos[1]);
            double yh = df2t<P2>(x, z[2][0], z[2][1], sos[2]);
            yh = df2t<P2>(yh, z[3][0], z[3][1], sos[3]);
            if (P2) {
                const double ym = (x - yl) - yh;  // AME:202
                const int32_t qi[3] = {quantize_i32(yl), quantize_i32(ym), quantize_i32(yh)};
                const int64_t ro = (int64_t)pn * G2;
                int16_t *rows[3] = {b0 + ro, b1 + ro, b2 + ro};
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    if constexpr (CH == 2) rows[b][lo] = (int16_t)qi[b];
                    else reinterpret_cast<short2 *>(rows[b])[(uint32_t)tid] = make_short2((int16_t)qi[b], 0);
                    const double e = (double)(uint32_t)(qi[b] * qi[b]);  // <= 2^30 (v_mul_i32_i24)
                    Ed[b] += e;
                    td[b] = fma(pn >= a.tail_from[b] ? 1.0 : 0.0, e, td[b]);
                }
            }
            ++pn;
        });
    if (P2) {
        if (CH == 2) {  // L^2 + R^2 sums of the lane pair
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                Ed[b] += pair_swap(Ed[b]);
                td[b] += pair_swap(td[b]);
            }
        }
        const int c = CH == 2 ? (tid & 1) : 0;
        const int64_t g = g0 + tid / CH;
        if (c == 0) {
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                a.E[b][g] = Ed[b];
                a.tail[b][g] = td[b];
            }
        }
    }
}

template <int CH>
__global__ void __launch_bounds__(LB_THREADS, 4) xover_kernel(XoArgs a, LbArgs lb, int64_t line_tiles) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int TPB = LB_THREADS / CH;
    __shared__ int ticket_slot;
    const int blk = lb_ticket(lb, &ticket_slot);
    const int tid = threadIdx.x;
    const int c = CH == 2 ? (tid & 1) : 0;
    const int t = tid / CH;
    const int64_t g = (int64_t)blk * TPB + t;
    const bool valid = g < a.G;
    const int len = valid ? (int)min((int64_t)a.T, a.N_proc - g * a.T) : 0;
    double zs[4][2] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}};
    const int64_t g0 = (int64_t)blk * TPB;
    const bool full = (g0 + TPB) * a.T <= a.N_proc;  // block-uniform
    if (full && a.zw) {  // the weights into LDS (the look-back scratch is free until lb_carry)
        for (int i = tid; i < a.T * 8; i += LB_THREADS) smem[i] = a.zw[i];
        __syncthreads();
        xo_pass_full<CH, false, true>(a, g0, tid, zs, smem);
        __syncthreads();  // (every wave has read the weights before lb_carry writes its scratch)
    } else if (full) {
        xo_pass_full<CH, false>(a, g0, tid, zs);
    } else if (valid) {
        xo_pass<CH, false>(a, g, c, len, zs);
    }
    double z[8], s[8], rst[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        z[2 * k] = zs[k][0];
        z[2 * k + 1] = zs[k][1];
        rst[2 * k] = rst[2 * k + 1] = 0.0;
    }
    lb_carry<8, CH, 2>(lb, blk, t, c, valid, valid && (g % line_tiles) == 0, rst, z, s, smem);  // LP | HP branches
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        zs[k][0] = s[2 * k];
        zs[k][1] = s[2 * k + 1];
    }
    if (full) xo_pass_full<CH, true>(a, g0, tid, zs);
    else if (valid) xo_pass<CH, true>(a, g, c, len, zs);
}

// ----------------------------------------------------------- K-weighting stage
struct KwArgs {
    int64_t N_proc, G;     // G sub-tiles of T frames (T divides the mix's tile Tt)
    int T, ch;
    int64_t Gt;            // tiles of the tile-major mix (its row stride)
    int sub;               // sub-tiles per tile (Tt = sub * T)
    double sos[2][5];
    const int16_t *mix;     // tile-major int16 pairs (pre-gain chain output)
    int64_t n_segs;
    const int64_t *seg_bounds;
    double *part;           // [G][2] energies of the (at most two) segments a tile touches
    int64_t *part_seg;      // [G]   first segment of the tile
    double *line_end;       // optional [4]: state after the last frame
    // fused batch (several tracks on one timeline, each starting at a chunk
    // boundary): n_trk > 0 gives each track's first tile (its K-weighting line
    // restarts there) and the end of its real frames (later frames of its last
    // chunk are padding: zero energy).  n_trk == 0: one line from tile 0.
    int n_trk;
    const int64_t *trk_tile0;  // [n_trk] ascending
    const int64_t *trk_end;    // [n_trk] timeline frame
    // exact block energies (kw_blocks_kernel): pass 2 writes the f32 square of every
    // K-weighted frame here instead of segment partials, in frame order with every
    // mix tile padded to sq_tp = Tt rounded up to 4 frames (frame n of mix tile g at
    // g * sq_tp + n): a lane stores 16 bytes every 4 frames, and a loudness chunk's
    // frames are ~37 contiguous runs the block sums load 16 bytes at a time
    float *sq;
    int sq_tp;
};

// pyloudnorm Meter (AME:213-218): mono = f32 mean(L,R) (== (L+R)/65536 exactly),
// high_shelf lfilter in f64 stored back to f32, high_pass lfilter in f64 stored
// to f32, then squared sums per 0.4 s / 0.1 s block.  The whole track is one line.
// A lane runs one (sub-)tile of T = Tt / sub frames of a mix tile; the chain uses
// sub = 1 (5 sub-tiles per tile measured 2x slower: 5x the look-back blocks and
// 5-line mix loads), the operator path any tile its tables were made for.
// P2 && SQ: pass 2 in lfilter's own operation order, writing np.square's f32 value
// of every frame (pyloudnorm squares the f32 filter output, AME:218) for the exact
// block sums; P2 && !SQ: f64 energies of the (at most two) segments of the tile.
template <bool P2, bool SQ = false>
__device__ __forceinline__ void kw_pass(const KwArgs &a, int64_t g, int len, double (&z)[2][2], int64_t seg_end,
                                        int64_t e_end, double &e0, double &e1) {
    const int64_t gt = g / a.sub;  // the mix tile holding sub-tile g, and its first row
    const short2 *mix = reinterpret_cast<const short2 *>(a.mix) + (g - gt * a.sub) * a.T * a.Gt + gt;
    const int64_t Gt = a.Gt;
    int64_t pf = g * a.T;
    float *sq = SQ ? a.sq + gt * a.sq_tp + (g - gt * a.sub) * a.T : nullptr;  // (sub-tile starts: multiples of T)
    float4 sq4 = make_float4(0.f, 0.f, 0.f, 0.f);
    int nsq = 0;
    stream<8, MM_KW_NB, short2>(
        len, [&](int i) { return mix[(int64_t)min(i, len - 1) * Gt]; },
        [&](short2 q) {
            const float m = a.ch == 2 ? ((float)q.x + (float)q.y) * (1.0f / 65536.0f)
                                      : (float)q.x * (1.0f / 32768.0f);
            if constexpr (P2 && SQ) {
                const float y1f = (float)df2t_lfilter((double)m, z[0][0], z[0][1], a.sos[0]);
                const float y2f = (float)df2t_lfilter((double)y1f, z[1][0], z[1][1], a.sos[1]);
                // 16-byte stores when the tile starts 16-byte aligned (the chain: sub = 1,
                // sq_tp % 4 == 0), else one word per frame
                const float v = __fmul_rn(y2f, y2f);
                if (a.sub == 1) {  // (a shift register: no per-frame component select)
                    sq4.x = sq4.y;
                    sq4.y = sq4.z;
                    sq4.z = sq4.w;
                    sq4.w = v;
                    if (++nsq == 4) {
                        *reinterpret_cast<float4 *>(sq) = sq4;
                        sq += 4;
                        nsq = 0;
                    }
                } else {
                    *sq++ = v;
                }
            } else {
                const double y1 = df2t((double)m, z[0][0], z[0][1], a.sos[0]);
                const float y1f = (float)y1;
                const double y2 = df2t((double)y1f, z[1][0], z[1][1], a.sos[1]);
                if (P2) {
                    const float y2f = (float)y2;
                    const double e = pf < e_end ? (double)y2f * (double)y2f : 0.0;
                    if (pf < seg_end) e0 += e;
                    else e1 += e;
                }
            }
            ++pf;
        });
    if constexpr (P2 && SQ) {  // the tile's last T % 4 frames: the newest nsq entries of the register
        if (nsq == 1) sq[0] = sq4.w;
        if (nsq == 2) sq[0] = sq4.z, sq[1] = sq4.w;
        if (nsq == 3) sq[0] = sq4.y, sq[1] = sq4.z, sq[2] = sq4.w;
    }
}

template <bool SQ>
__global__ void __launch_bounds__(LB_THREADS, 2) kweight_kernel(KwArgs a, LbArgs lb) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    __shared__ int ticket_slot;
    const int blk = lb_ticket(lb, &ticket_slot);
    const int t = threadIdx.x;
    const int64_t g = (int64_t)blk * LB_THREADS + t;
    const bool valid = g < a.G;
    const int len = valid ? (int)min((int64_t)a.T, a.N_proc - g * a.T) : 0;
    double zs[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
    double e0 = 0.0, e1 = 0.0;
    // this tile's track (fused batch): its line start and real-frame end
    int64_t line0 = 0, e_end = INT64_MAX;
    if (a.n_trk > 0 && valid) {  // (trk_tile0 counts mix tiles: sub lanes each)
        int lo = 0, hi = a.n_trk;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (a.trk_tile0[mid] * a.sub <= g) lo = mid;
            else hi = mid;
        }
        line0 = a.trk_tile0[lo] * a.sub;
        e_end = a.trk_end[lo];
    }
    if (valid) kw_pass<false>(a, g, len, zs, 0, e_end, e0, e1);
    double z[4] = {zs[0][0], zs[0][1], zs[1][0], zs[1][1]}, s[4], rst[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) rst[d] = lb.init ? lb.init[d] : 0.0;
    lb_carry<4, 1>(lb, blk, t, 0, valid, valid && g == line0, rst, z, s, smem);
    if (!valid) return;
    if constexpr (SQ) {
        zs[0][0] = s[0];
        zs[0][1] = s[1];
        zs[1][0] = s[2];
        zs[1][1] = s[3];
        kw_pass<true, true>(a, g, len, zs, 0, e_end, e0, e1);
        if (a.line_end && g == a.G - 1) {
            a.line_end[0] = zs[0][0];
            a.line_end[1] = zs[0][1];
            a.line_end[2] = zs[1][0];
            a.line_end[3] = zs[1][1];
        }
        return;
    }
    // loudness segment of the tile's first frame (largest s with bounds[s] <= f0)
    const int64_t f0 = g * a.T;
    int64_t lo = 0, hi = a.n_segs;
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (a.seg_bounds[mid] <= f0) lo = mid;
        else hi = mid;
    }
    zs[0][0] = s[0];
    zs[0][1] = s[1];
    zs[1][0] = s[2];
    zs[1][1] = s[3];
    kw_pass<true>(a, g, len, zs, a.seg_bounds[lo + 1], e_end, e0, e1);
    a.part[2 * g] = e0;
    a.part[2 * g + 1] = e1;
    a.part_seg[g] = lo;
    if (a.line_end && g == a.G - 1) {
        a.line_end[0] = zs[0][0];
        a.line_end[1] = zs[0][1];
        a.line_end[2] = zs[1][0];
        a.line_end[3] = zs[1][1];
    }
}

// Sum the per-tile partials into loudness segments: one wave per segment, lane
// k takes tiles g0+k, g0+k+64, ...; fixed-order butterfly (deterministic).
__global__ void __launch_bounds__(256) seg_reduce_kernel(KwArgs a, double *seg_energy) {
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (s >= a.n_segs) return;  // wave-uniform
    int64_t b0 = a.seg_bounds[s], b1 = a.seg_bounds[s + 1];
    if (b1 > a.N_proc) b1 = a.N_proc;
    double acc = 0.0;
    if (b0 < b1) {
        const int64_t g0 = b0 / a.T, g1 = (b1 - 1) / a.T;
        for (int64_t g = g0 + lane; g <= g1; g += 64) {
            const int64_t ps = a.part_seg[g];
            acc += ps == s ? a.part[2 * g] : (ps == s - 1 ? a.part[2 * g + 1] : 0.0);
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) seg_energy[s] = acc;
}

}  // namespace mm
