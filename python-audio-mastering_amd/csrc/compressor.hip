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
//                  the compacted super-tile-major array (per chunk: [U][SPC]);
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
#include "lookback.h"  // sc1 loads/stores and the global address-space types

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

#ifndef MM_RMS_NB
#define MM_RMS_NB 3
#endif
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
    stream<8, MM_RMS_NB, Pair>(
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

// Column of super-tile s (chunk c, index k in it) in Mc / ck.  Every chunk has a
// block of its own (rows RS elements apart: a walk's rows stay within a few MB,
// where one track-wide array put them a whole band-width apart and its walks and
// scatters missed the TLB on big batches).  Pass-0 lane j of a chunk owns its
// super-tiles j*own .. j*own + own-1, so super-tile j*own + t lives in column
// t*ocols + j and the 64 lanes of a wave touch 64 consecutive columns (512
// contiguous bytes) at every step of every walk, whatever `own` is.
__device__ __forceinline__ int64_t cm_col(const CompArgs &a, int64_t s) {
    const int64_t c = s / a.SPC, k = s - c * a.SPC;
    return c * a.CB + (k % a.own) * a.ocols + k / a.own;
}
__device__ __forceinline__ int64_t ck_col(const CompArgs &a, int64_t s) {
    const int64_t c = s / a.SPC, k = s - c * a.SPC;
    return c * a.CKB + (k % a.own) * a.ocols + k / a.own;
}

#ifndef MM_COMPACT_B
#define MM_COMPACT_B 32
#endif
#ifndef MM_COMPACT_NB
#define MM_COMPACT_NB 2
#endif
// frames per gather block (the table gathers run one block ahead; C2: 0.18 ms at 8,
// 0.16 at 16, 0.15 at 32 (208 VGPRs: fewer waves, more gathers in flight)) and rms
// blocks in flight
constexpr int COMPACT_B = MM_COMPACT_B, COMPACT_NB = MM_COMPACT_NB;

// 3. scatter M of active frames into the compacted array.  grid (ceil(G/256), 3)
// Inactive frames store into this lane's own padding slot (row U of the array),
// so every store is unconditional; the element index is 32-bit and advanced
// with selects (no per-frame branch), keeping the load pipeline counted.
// ONE_CROSS (U >= T, checked on the host): a tile's active frames cross at most
// one super-tile boundary, so the element of its j-th active frame is
// j*RS + (j < jb ? a0 : a1) — the only per-frame chain is j*RS += act*RS; the
// general form below carries row, column and owner through a select chain.
template <bool ONE_CROSS>
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
    const uint32_t cb = (uint32_t)(g / a.K) * (uint32_t)a.CB;  // the chunk's block
    uint32_t t = k % own, col = cb + t * ocols + k / own;  // column of its super-tile
    uint32_t idx = o * RS + col;  // its element
    const uint32_t dummy = cb + U * RS + g32 % RS;
    double *Mc = a.Mc[b];
    if constexpr (ONE_CROSS) {
        const uint32_t jbRS = (U - o) * RS;  // j*RS at the boundary (row 0 of super-tile sg + 1)
        const uint32_t k1 = k + 1, col1 = cb + (k1 % own) * ocols + k1 / own;  // (unused past the chunk's last)
        const uint32_t a0 = idx, a1 = col1 - jbRS;  // mod 2^32: a1 + jbRS == col1
        uint32_t jRS = 0;
        stream2<COMPACT_B, COMPACT_NB, uint16_t, double>(
            len, [&](int i) { return R[(uint32_t)min(i, len - 1) * G32]; },
            [&](uint16_t r) { return lut[r]; },
            [&](uint16_t r, double m) {
                const bool act = (uint32_t)r >= r0;
                const uint32_t e = jRS + (jRS < jbRS ? a0 : a1);
                Mc[act ? e : dummy] = m;
                jRS += act ? RS : 0u;
            });
        return;
    }
    stream2<COMPACT_B, COMPACT_NB, uint16_t, double>(
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

// IEEE binade of a positive normal double: x in [2^e, 2^(e+1))
__device__ __forceinline__ int binade(double x) { return (int)((uint64_t)__double_as_longlong(x) >> 52) - 1023; }

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
#ifndef MM_WALK_WB
#define MM_WALK_WB 40
#endif
constexpr int WALK_WB = MM_WALK_WB;  // M values in flight per walker (a multiple of CK_Q)
#ifndef MM_P0_WB
#define MM_P0_WB 40
#endif
constexpr int P0_WB = MM_P0_WB;     // the same for pass 0's walkers (latency of a lockstep wave's loads)
constexpr int WALK_PAD = WALK_WB > P0_WB ? WALK_WB : P0_WB;  // padding rows after the compacted array (prefetch past a super-tile's end)
constexpr int CK_Q = 10;     // checkpoint stride (compacted frames); divides WALK_WB and SEG
// Release jumps: a super-tile is cut into segments of SEG compacted
// frames; for each, pass 0 records the exact effect of SEG release steps on any
// state of binade e0 + k (k < JB, per mantissa parity), so a fix-up walker whose
// exact state releases through the whole segment moves past it in O(1).
constexpr int SEG = 100;     // divides U (host), multiple of CK_Q and DESC_B
constexpr int JB = 4;        // binades per segment descriptor: e0 .. e0 + JB - 1

// A column of Mc / ck walked row by row.  BUF: buffer loads/stores with the
// column's byte offset in a VGPR (constant over the walk) and the row's in an
// SGPR (the rows of a walk are wave-uniform), so stepping costs no VALU address
// arithmetic; needs the array under 2 GB (CompArgs::buf_ok).  Else flat pointers.
template <bool BUF>
struct ColWalk;
template <>
struct ColWalk<false> {
    double *p;
    size_t step;
    // rows rs elements apart from row row0 (or from element offset `skip` when given)
    __device__ __forceinline__ ColWalk(const double *base, int64_t col, int64_t rs, uint32_t, int row0 = 0,
                                       int64_t skip = -1)
        : p(const_cast<double *>(base) + col + (skip >= 0 ? skip : (int64_t)row0 * rs)), step((size_t)rs) {}
    __device__ __forceinline__ double ld() {
        const double v = *p;
        p += step;
        return v;
    }
    __device__ __forceinline__ void st(double v) {
        *p = v;
        p += step;
    }
};
template <>
struct ColWalk<true> {
    // the row offset advances in the per-lane (VGPR) offset: lanes walk different
    // rows and trip counts (an SGPR offset that diverges becomes a waterfall loop
    // around every load); the SGPR offset stays 0
    __amdgpu_buffer_rsrc_t r;
    int vo, step;
    __device__ __forceinline__ ColWalk(const double *base, int64_t col, int64_t rs, uint32_t bytes, int row0 = 0,
                                       int64_t skip = -1)
        : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(base), (short)0, (int)bytes, 0x00020000)),
          vo((int)((col + (skip >= 0 ? skip : (int64_t)row0 * rs)) * 8)), step((int)(rs * 8)) {}
    __device__ __forceinline__ double ld() {
        const double v = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vo, 0, 0));
        vo += step;
        return v;
    }
    __device__ __forceinline__ void st(double v) {
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, vo, 0, 0);
        vo += step;
    }
};

template <bool CK, bool BUF = false, int WB = WALK_WB>
__device__ __forceinline__ double comp_walk(double att, const CompArgs &a, int b, int64_t s, int len,
                                            const BandStep &bs, int row0 = 0) {
    constexpr int WP = 4;
    if (len <= 0) return att;
    // column s from row row0 (a multiple of CK_Q), rows RS apart; loads run up to WB
    // rows past the end (padding rows)
    ColWalk<BUF> pl(a.Mc[b], cm_col(a, s), a.RS, a.mc_bytes, row0);
    ColWalk<BUF> pc(CK ? a.ck[b] : a.Mc[b], CK ? ck_col(a, s) : 0, a.RS, a.ck_bytes, CK ? row0 / CK_Q : 0);  // checkpoint rows
    double buf[WB], inc[WP], dec[WP];
#pragma unroll
    for (int k = 0; k < WB; ++k) buf[k] = pl.ld();
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
            if (CK && k % CK_Q == 0) pc.st(att);
            att = lean_step(att, m, ik, dk);
            buf[k] = pl.ld();
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
            if (CK && k % CK_Q == 0) pc.st(att);
            att = lean_step(att, m, ik, dk);
        }
    }
    return att;
}

// Re-walk of segment [i0, i0 + sl) of a super-tile by a fix sweep: comp_walk<true>
// from the corrected state, which also compares the state at every WB-frame
// block start with the checkpoint stored there by the previous walk (loaded one
// block ahead, before this walk overwrites it).  Equal states mean the stored
// trajectory from there on (and the stored end) came from the same state: the
// walk stops (coalesced).  Returns the state after the segment (meaningless when
// coalesced); *nw = frames walked.
template <bool BUF>
__device__ __forceinline__ double comp_rewalk_seg(double att, const CompArgs &a, int b, int64_t s, int i0, int sl,
                                                  const BandStep &bs, bool *coalesced, int *nw, bool check = true) {
    constexpr int WB = WALK_WB, WP = 4, CKB = WB / CK_Q;  // checkpoint rows per block
    *coalesced = false;
    *nw = sl;
    if (sl <= 0) return att;
    const int64_t cs = ck_col(a, s);
    ColWalk<BUF> pl(a.Mc[b], cm_col(a, s), a.RS, a.mc_bytes, i0);
    ColWalk<BUF> pc(a.ck[b], cs, a.RS, a.ck_bytes, i0 / CK_Q);
    ColWalk<BUF> po(a.ck[b], cs, CKB * a.RS, a.ck_bytes, 0, (int64_t)(i0 / CK_Q) * a.RS);  // old checkpoint of the next block start (padding rows)
    double buf[WB], inc[WP], dec[WP];
#pragma unroll
    for (int k = 0; k < WB; ++k) buf[k] = pl.ld();
#pragma unroll
    for (int k = 0; k < WP; ++k) {
        inc[k] = div_cr(buf[k], bs.A, bs.rA);
        dec[k] = div_cr(buf[k], bs.R, bs.rR);
    }
    // (with !check the stored checkpoints inside the segment are not this
    // trajectory's: never compared; NaN never equals a state)
    const double nan = __longlong_as_double(0x7ff8000000000000ll);
    double old = check ? po.ld() : nan;
    int i = 0;
    for (; i + WB <= sl; i += WB) {
        if (__double_as_longlong(old) == __double_as_longlong(att)) {
            *coalesced = true;
            *nw = i;
            return att;
        }
        old = check ? po.ld() : nan;
#pragma unroll
        for (int k = 0; k < WB; ++k) {
            const double m = buf[k], ik = inc[k % WP], dk = dec[k % WP];
            const double mn = buf[(k + WP) % WB];
            inc[k % WP] = div_cr(mn, bs.A, bs.rA);
            dec[k % WP] = div_cr(mn, bs.R, bs.rR);
            if (k % CK_Q == 0) pc.st(att);
            att = lean_step(att, m, ik, dk);
            buf[k] = pl.ld();
        }
    }
    const int rem = sl - i;
    if (rem > 0 && __double_as_longlong(old) == __double_as_longlong(att)) {
        *coalesced = true;
        *nw = i;
        return att;
    }
#pragma unroll
    for (int k = 0; k < WB; ++k) {
        if (k < rem) {
            const double m = buf[k], ik = inc[k % WP], dk = dec[k % WP];
            const double mn = buf[(k + WP) % WB];
            inc[k % WP] = div_cr(mn, bs.A, bs.rA);
            dec[k % WP] = div_cr(mn, bs.R, bs.rR);
            if (k % CK_Q == 0) pc.st(att);
            att = lean_step(att, m, ik, dk);
        }
    }
    return att;
}

// ---- release jumps -----------------------------------------------------------
// Exactness ("release jumps").  Let a be a double in binade e
// (2^e <= a < 2^(e+1)), so a = A u with u = 2^(e-52) and integer A.  A release step
// a' = RN(a - d) whose exact result a - d stays >= 2^e rounds on the grid u:
// a' = a - rho u with rho the nearest integer to d/u, a tie going to the even
// result.  rho therefore depends only on d, e and the parity of A.  A reference
// walk r that starts in binade e with the same parity and stays in it rounds
// every step exactly like a, so after SEG release steps a ends at a - (r0 - rL).
// Pass 0 walks 2 * JB such references per segment (binades e0 .. e0+JB-1, both
// parities; e0 = binade of the segment's first M) and stores q = r0 - rL (exact,
// NaN if the reference left its binade) and the segment's max M.  A fix-up walker
// in state a (binade e, parity p) may jump iff x = a - q[e - e0][p] satisfies
//   x > max M  (every entry state of the segment, all >= x, is > its M: release)
//   x >= 2^e + u (every exact difference a_k - d_k >= a_{k+1} - u/2 > 2^e: grid u)
// and then lands EXACTLY on the state the step-by-step walk reaches.
struct SegDesc {
    double mx;
    int e0;
    double q[2 * JB];
};
constexpr int DREC = 2 + 2 * JB;  // doubles per descriptor record: max M, e0, q[2 JB]

// Record of segment t of super-tile s: [s][SPT][DREC] (a lane's records contiguous)
__device__ __forceinline__ const double2 *desc_rec(const CompArgs &a, int b, int64_t s, int t) {
    return reinterpret_cast<const double2 *>(a.desc[b] + ((s * a.SPT + t) * DREC));
}
__device__ __forceinline__ SegDesc load_desc(const double2 *r) {
    SegDesc d;
    double2 v[DREC / 2];
#pragma unroll
    for (int k = 0; k < DREC / 2; ++k) v[k] = r[k];
    d.mx = v[0].x;
    d.e0 = (int)v[0].y;
#pragma unroll
    for (int k = 0; k < JB; ++k) {
        d.q[2 * k] = v[k + 1].x;
        d.q[2 * k + 1] = v[k + 1].y;
    }
    return d;
}

__device__ __forceinline__ bool release_jump(const SegDesc &d, double att, double *out) {
    constexpr uint64_t MANT = (1ull << 52) - 1;
    const uint64_t ab = (uint64_t)__double_as_longlong(att);
    const int k = (int)(ab >> 52) - 1023 - d.e0;
    if (!(att > 0.0) || k < 0 || k >= JB) return false;
    const int idx = 2 * k + (int)(ab & 1);
    double q = d.q[0];
#pragma unroll
    for (int j = 1; j < 2 * JB; ++j) q = idx == j ? d.q[j] : q;
    const double x = att - q;  // exact: both multiples of u, result checked to stay in binade e
    const uint64_t xb = (uint64_t)__double_as_longlong(x);
    if (!(x > d.mx) || (xb >> 52) != (ab >> 52) || (xb & MANT) == 0) return false;
    *out = x;
    return true;
}

// Descriptors of the full segments of super-tile s (pass 0's second wave): one
// pass over the column, the 2 * JB reference walks per frame off any dependency
// chain but their own.
constexpr int DESC_B = 20;  // M values in flight per describing lane (divides SEG)

__device__ __forceinline__ void comp_describe(const CompArgs &a, int b, int64_t s, int len, const BandStep &bs) {
    constexpr int WB = DESC_B;
    constexpr uint64_t MANT = (1ull << 52) - 1;
    const int nseg = min(len / SEG, a.SPT);
    if (nseg <= 0) return;
    ColWalk<false> pl(a.Mc[b], cm_col(a, s), a.RS, 0);
    double buf[WB];
#pragma unroll
    for (int k = 0; k < WB; ++k) buf[k] = pl.ld();
    for (int t = 0; t < nseg; ++t) {
        const int e0 = binade(buf[0]);  // buf[0] = the segment's first M (> 0)
        double r0[2 * JB], r[2 * JB];
#pragma unroll
        for (int k = 0; k < 2 * JB; ++k) {  // top of binade e0 + k/2, parity k % 2
            const uint64_t bits = ((uint64_t)(e0 + k / 2 + 1023) << 52) | (MANT - 63 + (uint64_t)(k % 2));
            r0[k] = r[k] = __longlong_as_double((long long)bits);
        }
        double mx = 0.0;
        for (int blk = 0; blk < SEG / WB; ++blk) {
#pragma unroll
            for (int k = 0; k < WB; ++k) {
                const double m = buf[k];
                const double dec = div_cr(m, bs.R, bs.rR);
                mx = fmax(mx, m);
#pragma unroll
                for (int j = 0; j < 2 * JB; ++j) r[j] = r[j] - dec;
                buf[k] = pl.ld();
            }
        }
        double q[2 * JB];
#pragma unroll
        for (int k = 0; k < 2 * JB; ++k) {
            // the reference stayed in its binade with a nonzero mantissa (>= 2^e + u) at the end
            const uint64_t rb = (uint64_t)__double_as_longlong(r[k]);
            const bool ok = (rb >> 52) == (uint64_t)(e0 + k / 2 + 1023) && (rb & MANT) != 0;
            q[k] = ok ? r0[k] - r[k] : __longlong_as_double(0x7ff8000000000000ll);
        }
        double2 *rec = const_cast<double2 *>(desc_rec(a, b, s, t));
        rec[0] = make_double2(mx, (double)e0);
#pragma unroll
        for (int k = 0; k < JB; ++k) rec[k + 1] = make_double2(q[2 * k], q[2 * k + 1]);
    }
}

// Re-walk of a whole super-tile from its corrected start: segment by segment,
// each one checked for coalescence with the stored trajectory at its start,
// then jumped (exact release jump, its checkpoints left to comp_refill) or
// walked.  A jump stores the segment's entry state as its first checkpoint and
// marks it (jmark = tag, jstart); its inner checkpoints stay stale until
// comp_refill, so a later walk of a marked segment does not compare with them.
// The descriptor record, mark and first stored checkpoint of the next two
// segments are loaded ahead (a chain of jumps costs no load latency per jump).
// *nw = frames walked, *nj = frames jumped.
template <bool BUF>
__device__ __forceinline__ double comp_rewalk(double att, const CompArgs &a, int b, int64_t s, int len,
                                              const BandStep &bs, bool *coalesced, int *nw, int *nj) {
    *coalesced = false;
    *nw = 0;
    *nj = 0;
    if (len <= 0) return att;
    const int64_t cs = ck_col(a, s);
    const int nseg = (len + SEG - 1) / SEG;
    const double *ck = a.ck[b];
    const uint32_t *jm = a.jmark[b];
    auto seg_old = [&](int t) { return ck[(int64_t)(min(t, nseg - 1) * (SEG / CK_Q)) * a.RS + cs]; };
    auto seg_mark = [&](int t) { return jm[(int64_t)min(t, nseg - 1) * a.GS + s]; };
    SegDesc d0 = load_desc(desc_rec(a, b, s, 0)), d1 = load_desc(desc_rec(a, b, s, min(1, nseg - 1)));
    double o0 = seg_old(0), o1 = seg_old(1);
    uint32_t m0 = seg_mark(0), m1 = seg_mark(1);
    for (int t = 0; t < nseg; ++t) {
        const int i0 = t * SEG, sl = min(SEG, len - i0);
        const int64_t sg = (int64_t)t * a.GS + s;
        const SegDesc d2 = load_desc(desc_rec(a, b, s, min(t + 2, nseg - 1)));
        const double o2 = seg_old(t + 2);
        const uint32_t m2 = seg_mark(t + 2);
        if (__double_as_longlong(o0) == __double_as_longlong(att)) {
            *coalesced = true;
            return att;
        }
        double x;
        if (sl == SEG && a.jumps && release_jump(d0, att, &x)) {
            a.ck[b][(int64_t)(i0 / CK_Q) * a.RS + cs] = att;  // the entry state (refill writes the rest)
            a.jstart[b][sg] = att;
            a.jmark[b][sg] = a.tag;
            if (m0 != a.tag) {  // newly marked this chain: queue it for comp_refill
                const uint32_t k = atomicAdd(a.jlist_n + b, 1u);
                if (k < a.jlist_cap) a.jlist[b][k] = (uint32_t)sg;
            }
            att = x;
            *nj += SEG;
        } else {
            const bool stale_inside = m0 == a.tag;  // jumped earlier this chain: inner checkpoints stale
            if (stale_inside) a.jmark[b][sg] = 0u;  // walked now: every checkpoint rewritten below
            bool co;
            int w;
            att = comp_rewalk_seg<BUF>(att, a, b, s, i0, sl, bs, &co, &w, !stale_inside);
            *nw += w;
            if (co) {
                *coalesced = true;
                return att;
            }
        }
        d0 = d1;
        d1 = d2;
        o0 = o1;
        o1 = o2;
        m0 = m1;
        m1 = m2;
    }
    return att;
}

// 4. speculative pass.  grid: (ceil(GS/(own*BLOCK)), 3), two waves per block:
// wave 0 walks, wave 1 describes the same super-tiles' segments for the release
// jumps (comp_describe; it reads the same lines of Mc, mostly from L1/L2).  Each
// walking lane walks `own` consecutive super-tiles.  The start of the first is
// guessed: the M of its first frame (the state tracks M closely; tools/study), or
// with `warmup` > 0 by walking that many previous super-tiles of its chunk from
// the M of the first warm-up frame; the later ones start from the end of the one
// before.  Exactness never depends on the guess (the fix-up sweeps); the jumps
// make stale stretches cheap to repair, so the default warm-up is 0.
#ifndef MM_PASS0_BLOCK
#define MM_PASS0_BLOCK 64
#endif
constexpr int PASS0_BLOCK = MM_PASS0_BLOCK;

// (flat column walks: the buffer-load form measured slower here, 0.27 -> 0.30 ms on
// C2, though it helps the sweeps' lone walkers)
__global__ void __launch_bounds__(2 * PASS0_BLOCK) comp_pass0_kernel(CompArgs a) {
    const bool describer = threadIdx.x >= PASS0_BLOCK;
    const int64_t L = (int64_t)blockIdx.x * PASS0_BLOCK + (threadIdx.x % PASS0_BLOCK);  // lane j of chunk c
    const int b = blockIdx.y;
    const int64_t c = L / a.ocols, j = L - c * a.ocols;
    if (c * a.SPC >= a.GS) return;
    const int64_t s0 = c * a.SPC + j * a.own, s1 = c * a.SPC + min(j * a.own + a.own, a.SPC);
    const BandStep bs = band_step(a, b);
    if (describer) {
        if (a.jumps)
            for (int64_t s = s0; s < s1; ++s) comp_describe(a, b, s, super_of(a, b, s).len, bs);
        return;
    }
    double att = 0.0;
    bool warm = false;
    for (int64_t s = s0; s < s1; ++s) {
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
            for (int64_t w = w0; w < s; ++w) att = comp_walk<false, false, P0_WB>(att, a, b, w, a.U, bs);
        } else if (!warm) {
            att = a.Mc[b][cm_col(a, s)];  // the M of its first frame
        }
        a.start[b][s] = att;
        att = comp_walk<true, false, P0_WB>(att, a, b, s, st.len, bs);
        a.end[b][s] = att;
        warm = true;
    }
}

// 5. one fix-up sweep (exits at once if the previous sweep left nothing stale).
// grid: (ceil(GS/64), 3), lane = super-tile.  A lane whose start differs from
// its predecessor's end CLAIMS its super-tile (atomic max of the sweep stamp:
// one writer per super-tile per sweep) and re-walks it from that end
// (comp_rewalk: storing checkpoints, stopping once it meets the stored
// trajectory, after which the stored trajectory and end are right).  A re-walk
// that reaches the end without meeting it publishes the new end and CONTINUES
// into the successor in the same chunk (whose stored trajectory started from
// the old end) if it can claim it; if the successor's own lane claimed it
// first, that lane may have read the old end, so the sweep flags `changed` and
// the next sweep re-checks.  Every stale start is caught that way (a lane that
// read an old end either lost the successor's claim to the continuing walker,
// or the continuing walker lost it and flagged), so a sweep that flags nothing
// leaves every start equal to its predecessor's end: exact by induction from
// the chunk start.  Non-coalescing stretches (heavily compressed material) are
// walked through in one sweep instead of one super-tile per sweep.
constexpr int FIX_MAX_U = 8192; // cap on frames per super-tile (lengths are int)

__device__ __forceinline__ bool comp_claim(const CompArgs &a, int b, int64_t s) {
    return __hip_atomic_fetch_max((gu32 *)(a.claim[b] + s), a.stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
           a.stamp;
}

// Sweep 1 (a.heads == 0) is a Jacobi step: every stale super-tile re-walks from
// its predecessor's current end.  Later sweeps start a walker only at the HEAD of
// each run of consecutive stale super-tiles (its predecessor is not stale): the
// head's walker carries its value through the run by continuation, where Jacobi
// walkers inside the run would claim the run's super-tiles first and stop the
// correction after one super-tile per sweep.  Every lane that sees its super-tile
// stale flags the sweep, so a sweep that flags nothing saw every start equal to
// its predecessor's end and changed nothing (the fixed point: exact).
template <bool BUF>
__global__ void __launch_bounds__(64) comp_fix_kernel(CompArgs a, const unsigned int *prev_changed) {
    if (prev_changed && *prev_changed == 0u) return;
    const int64_t s = (int64_t)blockIdx.x * 64 + threadIdx.x;
    const int b = blockIdx.y;
    if (s >= a.GS) return;
    Super st = super_of(a, b, s);
    if (st.len <= 0 || st.p0 == 0) return;  // chunk starts are exact
    double *end = a.end[b];
    double att = ld_sc1(end + s - 1);
    if (__double_as_longlong(att) == __double_as_longlong(a.start[b][s])) return;
    *a.changed = 1u;  // stale: the next sweep re-checks (benign race: every writer stores 1)
    if (a.heads && st.p0 > 0 && (st.p0 / a.U) > 1) {  // the predecessor is not a chunk start
        const double pe = ld_sc1(end + s - 2);
        if (__double_as_longlong(pe) != __double_as_longlong(a.start[b][s - 1])) return;  // inside a run
    }
    if (!comp_claim(a, b, s)) return;  // a walker continuing from s - 1 owns it
    const BandStep bs = band_step(a, b);
    unsigned long long walked = 0, jumped = 0;
    int64_t cur = s;
    for (;;) {
        a.start[b][cur] = att;
        bool coalesced;
        int nw, nj;
        const double t = comp_rewalk<BUF>(att, a, b, cur, st.len, bs, &coalesced, &nw, &nj);
        walked += nw;
        jumped += nj;
        if (coalesced) break;
        st_sc1(end + cur, t);
        if (st.last) break;  // the chunk's last super-tile: no successor
        const int64_t nxt = cur + 1;
        if (!comp_claim(a, b, nxt)) break;  // its owner read an older end of cur: it is stale (flagged) next sweep
        att = t;
        cur = nxt;
        st = super_of(a, b, cur);
    }
    atomicAdd(a.walked, walked);
    if (jumped) atomicAdd(a.walked + 1, jumped);
}

// 6. checkpoints of the segments the sweeps jumped over.  grid (n, 3): the lanes
// of band blockIdx.y stride over its list of segments newly marked this chain
// (or, if the list overflowed, over all its segments) and re-walk each one still
// marked with this chain's tag (a segment walked again after its jump was
// unmarked by that walk) from its recorded exact entry state.  The band is
// uniform per block: the walks' buffer descriptors stay scalar.
template <bool BUF>
__global__ void __launch_bounds__(64) comp_refill_kernel(CompArgs a) {
    const int b = blockIdx.y;
    const uint32_t n = a.jlist_n[b];
    const int64_t NG = (int64_t)a.SPT * a.GS;
    const bool all = n > a.jlist_cap;
    const int64_t total = all ? NG : (int64_t)n;
    const BandStep bs = band_step(a, b);
    for (int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 64) {
        const int64_t sg = all ? i : (int64_t)a.jlist[b][i];
        if (a.jmark[b][sg] != a.tag) continue;
        const int64_t t = sg / a.GS, s = sg - t * a.GS;
        comp_walk<true, BUF>(a.jstart[b][sg], a, b, s, SEG, bs, (int)t * SEG);
    }
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
    // the <= CK_Q frames' M are independent loads: issue them with the checkpoint's,
    // then step (frames past p read as M = 0, the identity step)
    const int32_t n = p - q;
    double m[CK_Q];
#pragma unroll
    for (int j = 0; j < CK_Q; ++j) m[j] = a.Mc[b][cm_index(a, c, q + min(j, max(n - 1, 0)))];
    double att = a.ck[b][(int64_t)(o / CK_Q) * a.RS + ck_col(a, c * a.SPC + k)];
#pragma unroll
    for (int j = 0; j < CK_Q; ++j) att = comp_step(att, j < n ? m[j] : 0.0, bs);
    return att;
}

// 7. gains + overlay.  A block = 64 tiles x 3 bands: wave w runs band w's exact
// trajectory for its 64 tiles from the checkpoints (audioop.mul floor on both
// channels), APPLY_STEP frames at a time into LDS; then all 192 threads overlay
// sat16(sat16(lo + mid) + hi) (AME:210) and store q2 coalesced.
// Branch-free per frame so a group's steps, gains and multiplies interleave:
//  * M == 0 (rms <= threshold) needs no test: the step is then the identity;
//  * att == 0 gives gain 10^-0 = 1.0 exactly, for which audioop.mul is the
//    identity (pydub skips the multiply there);
//  * the group's 10^(-att/20) are skipped (wave-uniformly) when no lane's att
//    changed since the last gain (the sparse band's wave, almost always).
// Loads run two groups ahead (R, samples) and the table gathers one group ahead.
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

#ifndef MM_APPLY_MINB
#define MM_APPLY_MINB 1
#endif
__global__ void __launch_bounds__(192, MM_APPLY_MINB) comp_apply_kernel(CompArgs a) {
    constexpr int S = APPLY_STEP;
    __shared__ short2 lds[3][S][APPLY_TILES];
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
    double gain = 1.0, gain_att = -1.0;  // gain of gain_att; att >= 0 never equals -1
    // a wave whose 64 tiles hold no active frame (the sparse band, almost
    // everywhere) keeps each tile's entry state: one constant gain per lane, no
    // rms loads, table gathers or steps
    const bool quiet = __all(!valid || a.cnt[b][g] == 0);
    if (quiet) {
        gain = exp10(neg_div20(att));
        gain_att = att;
    }
    const uint32_t G32 = (uint32_t)G, gl = valid ? (uint32_t)g : 0u;
    const int last = max(len - 1, 0);
    uint16_t r1[S], r2[S];
    short2 v1[S], v2[S];
    double m1[S];
    auto load = [&](int n0, uint16_t (&r)[S], short2 (&v)[S]) {
#pragma unroll
        for (int j = 0; j < S; ++j) {
            const uint32_t idx = (uint32_t)min(n0 + j, last) * G32 + gl;
            r[j] = R[idx];
            v[j] = X[idx];
        }
    };
    // frames past the tile's end read lut[0] = 0 (rms 0 is below every threshold:
    // the identity step; their output is unused).  The index select keeps the
    // gather unconditional (a conditional load would be an exec-mask branch).
    auto gather = [&](int n0, const uint16_t (&r)[S], double (&m)[S]) {
#pragma unroll
        for (int j = 0; j < S; ++j) m[j] = lut[n0 + j < len ? r[j] : 0];
    };
    load(0, r1, v1);
    load(S, r2, v2);
    gather(0, r1, m1);
    for (int n0 = 0; n0 < T; n0 += S) {
        // this group: v1, m1; next: r2, v2
        short2 v[S];
        double m[S];
#pragma unroll
        for (int j = 0; j < S; ++j) {
            v[j] = v1[j];
            m[j] = m1[j];
            v1[j] = v2[j];
        }
        double gj[S];
        if (quiet) {  // wave-uniform: only the samples stream
#pragma unroll
            for (int j = 0; j < S; ++j) {
                const uint32_t idx = (uint32_t)min(n0 + 2 * S + j, last) * G32 + gl;
                v2[j] = X[idx];
                gj[j] = gain;
            }
        } else {
            gather(n0 + S, r2, m1);
            load(n0 + 2 * S, r2, v2);
            double at[S];
            bool same = true;
#pragma unroll
            for (int j = 0; j < S; ++j) {
                att = lean_step(att, m[j], div_cr(m[j], bs.A, bs.rA), div_cr(m[j], bs.R, bs.rR));
                at[j] = att;
                same = same && att == gain_att;
            }
            if (__all(same)) {  // wave-uniform: no lane's attenuation moved
#pragma unroll
                for (int j = 0; j < S; ++j) gj[j] = gain;
            } else {
#pragma unroll
                for (int j = 0; j < S; ++j) gj[j] = exp10(neg_div20(at[j]));  // db_to_float(-att); exp10(-0) == 1 exactly
                gain = gj[S - 1];
                gain_att = at[S - 1];
            }
        }
#pragma unroll
        for (int j = 0; j < S; ++j) {
            short2 s = v[j];
            s.x = audioop_mul(s.x, gj[j]);
            s.y = audioop_mul(s.y, gj[j]);
            lds[b][j][lane] = s;
        }
        lds_barrier();
        for (int p = threadIdx.x; p < S * APPLY_TILES; p += 3 * APPLY_TILES) {
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
