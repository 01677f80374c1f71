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
// is held: the step is the identity).
//
// The recurrence is solved EXACTLY per (chunk, band) over the chunk's ACTIVE
// tiles (T = 225 frames at 44.1 kHz, design.choose_tile; a tile without an active
// frame holds the state), in super-tiles of TPS = 4 consecutive active tiles (900
// frames).  Data flow:
//  1. comp_rms_t per (column block of 256 tiles, band): exact integer rms per frame
//                (window sums in doubles, one-sided f32 estimate + one exact check),
//                M = lut[r] gathered ONCE and stored as f64 into the super-tile-major
//                M plane (column blocks of 64, so 64 walkers read 512 contiguous
//                bytes per step), plus per tile its active count, largest M and
//                (max,+) release summary `ce`, per column block its active-tile count.
//                Consumers gate every read of M on the tile's count: rows of tiles
//                with no active frame are never stored (comp_rms's quiet-tile skip).
//  2. comp_describe per column block: ranks and lists the chunk's active tiles in
//                compact order and records per active tile the exact effect of its T
//                release steps on any state of the EIGHT binades above its largest M
//                (release jumps, JB = 8, both mantissa parities).
//  3. comp_pass0 walker lanes (one per super-tile, a wave in lockstep) walk from a
//                guess (the (max,+) release envelope folded over the preceding 32
//                active tiles; exactly 0 at the chunk's first active tile), storing
//                every tile's entry state and the end, and compose each full
//                super-tile's super-jump record.
//  4. comp_fix   sweeps: a super-tile whose start differs from its predecessor's
//                end is claimed and re-walked from it — super jumps, release jumps
//                over pure-release tiles, steps otherwise — and stops as soon as its
//                state equals a tile's stored entry state (the stored trajectory from
//                there on came from the same state).  At the fixed point every start
//                is its predecessor's end: exact by induction from the chunk start.
//  5. comp_apply per (64 tiles, 3 bands): from the tile's entry state, the exact
//                trajectory, gains (table exp10), audioop.mul and the overlay
//                through LDS.
// Pass 0 needs no warm-up: the true trajectory is in release ~90 % of the time
// and every stretch between its clamps is crossed by jumps in the sweeps
// (tools/study/envelope_model.c).
#include "common.h"
#include "lookback.h"  // sc1 loads/stores and the global address-space types

namespace mm {

// x^2 + y^2 of one frame: at most 2 * 32768^2 = 2^31, exact in uint32
template <bool V>
struct BoolTag {
    static constexpr bool value = V;
};

__device__ __forceinline__ uint32_t frame_energy(short2 v) {
    return (uint32_t)((int32_t)v.x * v.x) + (uint32_t)((int32_t)v.y * v.y);
}

// correctly rounded m / d given rd = RN(1/d) (Markstein; tests/test_oracle.py)
__device__ __forceinline__ double div_cr(double m, double d, double rd) {
    const double q = m * rd;
    const double rem = fma(-q, d, m);
    return fma(rem, rd, q);
}

#ifndef MM_RMS_NB
#define MM_RMS_NB 3
#endif
constexpr int RMS_B = 8;  // frames per load block of comp_rms
constexpr int RMS_TPS = 4;  // tiles per super-tile comp_rms_t is written for (its four waves)

// Super-tile-major M plane of a band: frame n of tile g — the k-th tile of
// super-tile s — is row k*TP + n of column s (TP = T rounded up to whole walk load
// blocks; rows past a tile's frames hold M = 0, identity steps).  Columns come in
// blocks of 64 (one pass-0 wave): element (s, row) at ((s / 64) * RP + row) * 64 +
// s % 64, RP = TPS*TP + WALK_PAD rows (prefetch padding), so the 64 walkers of a
// wave read 512 contiguous bytes at every step and a column's rows lie 512 B apart
// (a tile's rows and a block's walks stay within a few pages).  Each chunk's
// columns (SPC, whole column blocks) form a plane of their own, chunk_elems
// elements from the chunk's base: offsets within it fit 32 bits at any track
// length (every kernel that walks it does so within one chunk per wave).
__device__ __forceinline__ void tile_col(const CompArgs &a, int64_t g, int64_t *s, int *k) {
    const int64_t c = g / a.K, j = g - c * a.K;
    *s = c * a.SPC + j / a.TPS;
    *k = (int)(j - (j / a.TPS) * a.TPS);
}
// element index of row 0 of column s within its chunk's plane
__device__ __forceinline__ uint32_t col_elem(const CompArgs &a, int64_t s) {
    const int64_t sl = s % a.SPC;
    return (uint32_t)((sl >> 6) * (int64_t)a.RP * 64 + (sl & 63));
}
// chunk c's plane of band b
__device__ __forceinline__ double *chunk_plane(const CompArgs &a, int b, int64_t c) {
    return a.Ms[b] + c * a.chunk_elems;
}

// 1. rms and M per frame.  grid: (GS * TPS / 256, 3 bands) of 256-thread blocks,
// one wave per (column block, position k): wave v handles tile k = v % TPS of the 64
// super-tiles (columns) of column block v / TPS, lane l the one of column 64 (v /
// TPS) + l.  SPC is a multiple of 64, so a column block lies in one chunk and the
// wave's 64 lanes store row k*T + n of 64 consecutive columns: every M store is
// one 512-byte run (round 3 mapped lanes to consecutive tiles: 8 runs of 64 B per
// store).  The band loads are TPS tiles apart across the lanes (the block's TPS
// waves share those lines).  The window [max(chunk0, f-look), f) slides one frame
// per step: + frame f-1 (this lane's own previous frame), - frame f-1-look (up to
// ~4 tiles back: another tile's data).  The window sum is an exact integer held in
// a double.  M = lut[r] is gathered ONCE here (a block of RMS_B frames' gathers is
// stored one block later) and written to the super-tile-major plane that the
// walkers and comp_apply read; rows past the end of a partial last tile get M = 0
// (identity steps).  Also the tile's active count and largest M (the table is
// nondecreasing in r), its (max,+) release summary for the pass-0 guesses, and the
// per-chunk active count.
#ifndef MM_RMS_MINB
#define MM_RMS_MINB 1
#endif
// rms_exact with one correction: the f32 estimate of sqrt(S * (1/n)) taken with
// the reciprocal scaled by (1 - 2^-18) (inv_b) lies in sqrt(S/n) * [1 - 2^-19 -
// 2^-22, 1 - 2^-19 + 2^-22] (rcp, product and sqrt each within a few ulp), so
// below sqrt(S/n) and above it minus 0.07 at r <= 32768: its truncation is r or
// r - 1, and one exact check n (r+1)^2 <= S (integers below 2^53 in f64) fixes it.
__device__ __forceinline__ uint32_t rms_exact1(double S, double n, float inv_b) {
    int32_t r = (int32_t)__builtin_amdgcn_sqrtf((float)S * inv_b);
    const double rd = (double)(r + 1);
    r += (n * rd * rd <= S) ? 1 : 0;
    return (uint32_t)r;
}
__device__ __forceinline__ float rcp_biased(double n) {
    return __fmul_rn(__builtin_amdgcn_rcpf((float)n), 1.0f - 0x1p-18f);
}
// x^2 + y^2 of one frame in one v_dot2_i32_i16 (the 2^31 of two -32768s wraps to the
// same uint32)
__device__ __forceinline__ uint32_t frame_energy2(short2 v) {
    uint32_t r;  // (VOP3P with an inline 0 accumulator: no v_mov to clear a v_dot2c destination)
    asm("v_dot2_i32_i16 %0, %1, %1, 0" : "=v"(r) : "v"(v));
    return r;
}
// max of two non-NaN doubles without fmax's operand canonicalisation
__device__ __forceinline__ double vmax(double x, double y) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}

// ---- comp_rms with the table gathers and M stores transposed through LDS -------
// (TPS == 4: a workgroup = one column block = 256 consecutive tiles of a chunk.)
// The per-frame rms runs as in comp_rms (lane = tile, coalesced band rows); per
// block of RMS_B frames three phases exchange through LDS:
//   A  lane = tile: the exact rms r of RMS_B frames -> R[j][tile];
//   B  each wave gathers M = lut[r] for its own 64 tiles x RMS_B frames with lanes
//      over (8 tiles x 8 CONSECUTIVE frames): a lane group of one tile reads
//      nearly the same r, so a gather touches ~8 table lines instead of 64 (the
//      round-5 profile had comp_rms TA-bound: L1 address stalls 55 % of its time);
//   C  lane = column, wave = tile position: M rows of 64 consecutive columns are
//      stored as one 512-byte run, and the lane keeps its tile's (max,+) release
//      summary (frames in order).
// Gathers of block q are in flight while block q+1's rms runs; one workgroup
// barrier per block (double-buffered R and M stages).
constexpr int RT_SLOTS = 4 * 68;                      // M stage slots: position-major, 68 per position
constexpr int RT_RPAD = 264, RT_MPAD = 296;           // row strides (words / doubles), bank spread
__device__ __forceinline__ int rt_slot(int tl) { return (tl & 3) * 68 + (tl >> 2); }

__global__ void __launch_bounds__(256, MM_RMS_MINB) comp_rms_t_kernel(CompArgs a) {
    __shared__ uint16_t Rs[2][RMS_B][RT_RPAD];
    __shared__ double Mst[2][RMS_B][RT_MPAD];
    const int b = blockIdx.y;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t cbk = blockIdx.x;                   // global column block
    const int64_t cc = (cbk * 64) / a.SPC;
    const int64_t jt0 = (cbk * 64 - cc * a.SPC) * 4;  // its first tile in the chunk
    const short2 *x = a.band[b];
    const int look = a.look[b], T = a.T, ch = a.ch;
    const uint32_t G = (uint32_t)a.G;
    const uint32_t r0 = a.r0[b];
    const double *lut = a.lut[b];
    const double Rf = a.release_frames[b], rR = a.rcp_release[b];
    const int64_t chunk0 = cc * a.K * T;
    // ---- phase A role: tile tlA = 64 w + lane of the block
    const int tlA = w * 64 + lane;
    const int64_t jtA = jt0 + tlA, gA = cc * a.K + jtA;
    const bool vA = jtA < a.K && gA < a.G;
    // invalid lanes (past the chunk's tiles or the track: a wave's LAST lanes, so lane 0
    // is valid whenever any lane is) load as lane 0 does: in bounds, never used
    const uint32_t g32 = vA ? (uint32_t)gA : (uint32_t)__builtin_amdgcn_readfirstlane((int)gA);
    const int64_t f0 = (int64_t)g32 * T;
    const int lenA = vA ? (int)min((int64_t)T, a.N_proc - f0) : 0;
    const int64_t lo0 = max(chunk0, f0 - look);
    double S = 0.0;
    if (vA) {
        const int kf = look / T;
        for (int t = 1; t <= kf; ++t)
            if (((int64_t)g32 - t) * T >= chunk0) S += a.E[b][g32 - t];
        if (look % T != 0 && ((int64_t)g32 - kf - 1) * T >= chunk0) S += a.tail[b][g32 - kf - 1];
    }
    const int64_t d_first = max(f0 - look, chunk0);
    const int skip = vA ? (int)(d_first - (f0 - look)) : 0;
    const uint32_t gd = (uint32_t)(d_first / T);
    const int nd = (int)(d_first - (int64_t)gd * T);
    double n = (double)((f0 - lo0) * ch);
    float inv = n > 0.0 ? rcp_biased(n) : 0.f;
    int i_proc = 0, active = 0;
    uint32_t rmx = 0;
    struct Pair {
        short2 in, drop;
    };
    const bool steady = __all(!vA || (skip == 0 && lenA == T)) && look > 0;
    const int64_t dgo = (int64_t)__builtin_amdgcn_readfirstlane((int)((int64_t)gd - (int64_t)g32));
    const int nd_u = __builtin_amdgcn_readfirstlane(nd);
    auto ld_steady = [&](int i) __attribute__((always_inline)) {
        i = min(i, T - 1);
        Pair p;
        p.in = (x + (int64_t)i * G)[g32];
        int k = nd_u + i;
        const int wrap = k >= T ? 1 : 0;
        k -= wrap * T;
        p.drop = (x + (int64_t)k * G + dgo + wrap)[g32];
        return p;
    };
    auto ld = [&](int i) __attribute__((always_inline)) {
        i = max(min(i, lenA - 1), 0);
        Pair p;
        p.in = x[(uint32_t)i * G + g32];
        int k = nd + max(i - skip, 0);
        const int wrap = k >= T ? 1 : 0;
        k -= wrap * T;
        p.drop = x[(uint32_t)k * G + gd + (uint32_t)wrap];
        return p;
    };
    auto rms_step = [&](Pair p, auto st) __attribute__((always_inline)) {
        uint32_t r;
        if constexpr (decltype(st)::value) {
            r = rms_exact1(S, n, inv);
            S += (double)frame_energy2(p.in) - (double)frame_energy2(p.drop);
        } else {
            r = n > 0.0 ? rms_exact1(S, n, inv) : 0u;
            const bool drops = i_proc >= skip;
            S += (double)frame_energy2(p.in) - (drops ? (double)frame_energy2(p.drop) : 0.0);
            if (!drops) {
                n += ch;
                inv = rcp_biased(n);
            }
            ++i_proc;
        }
        active += r >= r0 ? 1 : 0;
        rmx = max(rmx, r);
        return r;
    };
    // ---- phase B role: lanes over (8 tiles x 8 frames) of the wave's own tiles
    const int jB = lane & 7;                          // frame in the block
    // ---- phase C role: column lane of the block, tile position w
    const int tlC = lane * 4 + w;
    const int64_t jtC = jt0 + tlC, gC = cc * a.K + jtC;
    const bool vC = jtC < a.K && gC < a.G;
    const int lenC = vC ? (int)min((int64_t)T, a.N_proc - gC * T) : 0;
    double *Mo = chunk_plane(a, b, cc);
    uint32_t eC = col_elem(a, cc * a.SPC + jtC / 4) + (uint32_t)(w * a.TP) * 64u;  // row w*TP of its column
    double ce = 0.0, De = 0.0;
    const int slotC = w * 68 + lane;                  // == rt_slot(tlC)

    constexpr int B = RMS_B, NB = MM_RMS_NB;
    const int NBK = (T + B - 1) / B;
    const int NBKP = (NBK + NB - 1) / NB * NB;        // blocks run (a multiple of NB; past NBK: empty)
    Pair buf[NB][B];
    double gm[B];                                     // phase B gathers in flight
#pragma unroll
    for (int j = 0; j < B; ++j) gm[j] = 0.0;
    auto issue_gathers = [&](int q) __attribute__((always_inline)) {
        asm volatile("" ::: "memory");                // (R written by this wave above: keep the reads after)
#pragma unroll
        for (int r8 = 0; r8 < B; ++r8) {
            const int tl = w * 64 + r8 * 8 + (lane >> 3);
#ifdef MM_RMS_NOGATHER  // (ablation builds: timing only)
            gm[r8] = (double)Rs[q & 1][jB][tl];
#else
            gm[r8] = lut[Rs[q & 1][jB][tl]];
#endif
        }
    };
    auto finish_gathers = [&](int q) __attribute__((always_inline)) {
#pragma unroll
        for (int r8 = 0; r8 < B; ++r8) {
            const int tl = w * 64 + r8 * 8 + (lane >> 3);
            Mst[q & 1][jB][rt_slot(tl)] = gm[r8];
        }
    };
    // Phase C's stores are unconditional buffer stores (an invalid lane or a row past
    // the tile gets an offset past the plane: the store is dropped), so the compiler
    // counts them exactly: with exec-masked stores its gather waits also waited for
    // the previous block's stores (vmcnt is in order).  Measured neutral (0.203 ms
    // either way: the kernel is bound by its L1 -> L2 request rate).
    const __amdgpu_buffer_rsrc_t Mr =
        __builtin_amdgcn_make_buffer_rsrc(Mo, (short)0, (int)(a.chunk_elems * 8), 0x00020000);
    constexpr uint32_t DROP = 0xFFFFFFF0u;            // >= the plane's bytes (offsets fit 32 bits)
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    auto phase_c = [&](int q) __attribute__((always_inline)) {
        const int nv = q >= 0 ? max(min(B, T - q * B), 0) : 0;  // uniform (q = -1, past the tile: none)
        double m[B];
#pragma unroll
        for (int j = 0; j < B; ++j) m[j] = Mst[q & 1][j][slotC];
#pragma unroll
        for (int j = 0; j < B; ++j) {
#ifndef MM_RMS_NOSTORE  // (ablation builds: timing only)
            const uint32_t off = (vC && j < nv) ? (eC + (uint32_t)j * 64u) * 8u : DROP;
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, m[j]), Mr, off, 0, 0);
#endif
        }
        eC += (uint32_t)nv * 64u;
#pragma unroll
        for (int j = 0; j < B; ++j) {  // (rows past the tile: M = 0 is the identity here)
            const double mj = j < nv ? m[j] : 0.0;
            const double d = div_cr(mj, Rf, rR);
            ce = vmax(mj, ce - d);
            De += d;
        }
    };
    auto run = [&](auto st, auto &&load) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < NB; ++k) {
#pragma unroll
            for (int j = 0; j < B; ++j) buf[k][j] = load(k * B + j);
            __builtin_amdgcn_sched_barrier(0);
        }
        auto body = [&](int k, int q) __attribute__((always_inline)) {
            // A: rms of block q (frames past the lane's tile: r = 0, M = 0)
            uint32_t r[B];
            const int nvA = lenA - q * B;             // (uniform when steady)
#pragma unroll
            for (int j = 0; j < B; ++j) r[j] = j < nvA ? rms_step(buf[k][j], st) : 0u;
#pragma unroll
            for (int j = 0; j < B; ++j) buf[k][j] = load((q + NB) * B + j);
#pragma unroll
            for (int j = 0; j < B; ++j) Rs[q & 1][j][tlA] = (uint16_t)r[j];
            finish_gathers(q - 1);                    // (q = 0: zeros into the idle stage)
            issue_gathers(q);
            __syncthreads();
            phase_c(q - 1);
        };
        // every body issues the same vector memory operations (no conditional loads,
        // gathers or stores; blocks past the tile are empty), so the compiler's vmcnt
        // waits count exactly and never wait on the stores
        for (int q0 = 0; q0 < NBKP; q0 += NB) {
#pragma unroll
            for (int k = 0; k < NB; ++k) body(k, q0 + k);
        }
    };
    // (a wave's invalid tiles are its last lanes: lane 0 is valid iff any lane is, so
    // the readfirstlane values above are a valid lane's; a wave past the chunk's tiles
    // loads nothing)
    if (!__any(vA)) run(BoolTag<true>{}, [](int) { return Pair{make_short2(0, 0), make_short2(0, 0)}; });
    else if (steady) run(BoolTag<true>{}, ld_steady);
    else run(BoolTag<false>{}, ld);
    finish_gathers(NBKP - 1);
    __syncthreads();
    phase_c(NBKP - 1);
    // rows past the tile's frames (the padding to TP) hold M = 0 (identity steps)
    if (vC)
        for (int i = T; i < a.TP; ++i, eC += 64u) Mo[eC] = 0.0;
    if (vC) reinterpret_cast<double2 *>(a.ced[b])[gC] = make_double2(ce, De);
    (void)lenC;
    if (vA) {
        a.cnt[b][gA] = active;
        a.mmax[b][gA] = lut[rmx];
    }
    {  // active tiles of the column block
        const int na = (int)__popcll(__ballot(vA && active != 0));
        if (lane == 0 && na) atomicAdd(a.cbtot[b] + cbk, na);
    }
    int v = vA ? active : 0;  // per-chunk active count (statistics)
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0 && v) atomicAdd(a.total[b] + cc, v);
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

// v_min_f64 without the operand canonicalisation fmin adds
// (operands here are never NaN; equal operands and signed zeros give the same
// observable att)
__device__ __forceinline__ double vmin(double x, double y) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}

// the step given M and its (precomputed) increments.  The release branch needs no
// max(., 0): it is taken for att > m, and dec = RN(m/R) <= m (R >= 1, checked on
// the host), so att - dec > 0 and its rounding is >= 0 (pydub's max is the identity)
__device__ __forceinline__ double lean_step(double att, double m, double inc, double dec) {
    const double up = vmin(att + inc, m);
    const double dn = att - dec;
    return att <= m ? up : dn;
}

// ---- envelope walks over the M plane ------------------------------------------
// The solve runs over each chunk's ACTIVE tiles (an inactive tile holds the
// state): comp_describe ranks them (rank[g] = active tiles before tile g in its
// chunk, compact index ci = chunk * K + rank), and super-tile j of chunk c is
// the active tiles of ranks [j*TPS, min((j+1)*TPS, nact[c])) — empty past the
// chunk's active tiles.  Its state on entry, the tiles' entry states (tstc) and
// jump records (descc) live at compact indices.
struct Super {
    int64_t ci0;  // compact index of its first tile
    int ntiles;   // 0: empty
    bool first;   // the chunk's first (starts exactly at 0)
    bool last;    // the chunk's last non-empty one
};

// (na: the chunk's active tiles, a.nact)
__device__ __forceinline__ Super super_of_na(const CompArgs &a, int64_t s, int na) {
    Super r;
    const int64_t c = s / a.SPC, j = s - c * a.SPC;
    r.ci0 = c * a.K + j * a.TPS;
    r.ntiles = (int)max((int64_t)0, min((int64_t)a.TPS, (int64_t)na - j * a.TPS));
    r.first = j == 0;
    r.last = (j + 1) * a.TPS >= na;
    return r;
}
__device__ __forceinline__ Super super_of(const CompArgs &a, int b, int64_t s) {
    return super_of_na(a, s, a.nact[b][s / a.SPC]);
}

#ifndef MM_WALK_B
#define MM_WALK_B 25
#endif
#ifndef MM_WALK_NB
#define MM_WALK_NB 2
#endif
constexpr int WB = MM_WALK_B;   // rows per load block (divides TP)
constexpr int WNB = MM_WALK_NB; // blocks in flight (sweep walkers)
#ifndef MM_FIX_WNB
#define MM_FIX_WNB MM_WALK_NB
#endif
constexpr int FIX_WNB = MM_FIX_WNB;  // blocks in flight of a fix-up walker's tile walk
#ifndef MM_P0_NB
#define MM_P0_NB 2
#endif
constexpr int P0_NB = MM_P0_NB;  // blocks in flight (pass 0)
constexpr int WP = 5;           // divisions run WP frames ahead of their step (divides WB)
static_assert(WB % WP == 0, "WP must divide WB");
constexpr int WALK_PAD = WB * (WNB > P0_NB ? WNB : P0_NB);  // padding rows after a column's TPS*T (prefetch)

// Buffer view of one band's M plane (byte offset of row 0 of column s: col_elem * 8)
struct Plane {
    __amdgpu_buffer_rsrc_t r;
    int RP;
};
constexpr uint32_t ROWB = 64u * 8u;  // bytes per row of a column block
// (c: the wave's chunk, made uniform here: the descriptor lives in SGPRs)
__device__ __forceinline__ Plane plane(const CompArgs &a, int b, int64_t c) {
    Plane p;
    const int64_t cu = ((int64_t)__builtin_amdgcn_readfirstlane((int)(c >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((int)(c & 0xffffffff));
    p.r = __builtin_amdgcn_make_buffer_rsrc(chunk_plane(a, b, cu), (short)0, (int)(a.chunk_elems * 8), 0x00020000);
    p.RP = a.RP;
    return p;
}
// byte offset of row 0 of tile g (its column and row k*TP) in its chunk's plane
__device__ __forceinline__ uint32_t tile_off(const CompArgs &a, int64_t g) {
    int64_t s;
    int k;
    tile_col(a, g, &s, &k);
    return (col_elem(a, s) + (uint32_t)(k * a.TP) * 64u) * 8u;
}
__device__ __forceinline__ double ld_plane(const Plane &p, uint32_t vo, uint32_t so) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(p.r, vo, so, 0));
}

// Stream ntiles tiles of T rows to f, in order: f.tile(i) before tile i's first
// row (and f.tile(ntiles) after the last), f.frame(j, m, m_ahead) per row (j: row
// in the block, m_ahead: the M WP rows later).  offs(i) = byte offset of tile i's
// row 0 (called once per tile, when the loads reach it).  NBK blocks in flight;
// no conditional loads in the loop (counted waits).  LOCK: the wave's lanes step
// the same rows (pass 0), so the row offset is an SGPR.
template <bool LOCK, int NBK, typename OFF, typename F>
__device__ __forceinline__ void stream_col(const Plane &p, OFF &&offs, int ntiles, int T, F &f) {
    constexpr int WNB = NBK;
    const int bpt = T / WB, nblk = ntiles * bpt;
    if (nblk <= 0) return;
    double mb[WNB][WB];
    int lt = 0, lb = 0;  // load cursor: tile, block in tile
    uint32_t vo = offs(0);
    auto load = [&](double (&d)[WB]) __attribute__((always_inline)) {
        // LOCK: every lane is at the same row, so the row offset is one SGPR (a
        // per-lane soffset would become a waterfall loop around every load)
        const uint32_t rb = LOCK ? (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)(lb * WB) * ROWB))
                                 : (uint32_t)(lb * WB) * ROWB;
#pragma unroll
        for (int j = 0; j < WB; ++j)
            d[j] = LOCK ? ld_plane(p, vo, rb + (uint32_t)j * ROWB) : ld_plane(p, vo + rb + (uint32_t)j * ROWB, 0);
        if (++lb == bpt) {  // next tile (past the last: reload it, never consumed)
            lb = 0;
            if (++lt < ntiles) vo = offs(lt);
            else lb = bpt - 1;
        }
    };
#pragma unroll
    for (int k = 0; k < WNB; ++k) {
        load(mb[k]);
        __builtin_amdgcn_sched_barrier(0);
    }
    f.init(mb[0]);
    int ct = 0, cb = 0;  // tile, block in tile
    auto consume = [&](int k, bool reload) __attribute__((always_inline)) {
        if (cb == 0) f.tile(ct);
#pragma unroll
        for (int j = 0; j < WB; ++j) f.frame(j, mb[k][j], j + WP < WB ? mb[k][j + WP] : mb[(k + 1) % WNB][j + WP - WB]);
        __builtin_amdgcn_sched_barrier(0);
        if (reload) load(mb[k]);
        __builtin_amdgcn_sched_barrier(0);
        if (++cb == bpt) {
            cb = 0;
            ++ct;
        }
    };
    const int nfull = nblk / WNB;
    for (int r = 0; r < nfull; ++r) {
#pragma unroll
        for (int k = 0; k < WNB; ++k) consume(k, true);
    }
    const int rem = nblk - nfull * WNB;
#pragma unroll
    for (int k = 0; k < WNB; ++k)
        if (k < rem) consume(k, false);
    f.tile(ct);  // (the boundary after the last row)
}

// The envelope walk as a stream consumer: with ST, the state on entry to stream
// tiles [i0, i0 + nst) into tst[i - i0]; `out` = the state on entry to tile
// i0 + nst (the end of a lane's own tiles in a lockstep walk of the longest).
template <bool ST>
struct Walker {
    double att, out, sv;  // sv: the state on entry to tile i0
    double inc[WP], dec[WP];
    BandStep bs;
    double *tst;
    int i0, nst;
    __device__ __forceinline__ void init(const double (&m)[WB]) {
#pragma unroll
        for (int k = 0; k < WP; ++k) {
            inc[k] = div_cr(m[k], bs.A, bs.rA);
            dec[k] = div_cr(m[k], bs.R, bs.rR);
        }
    }
    __device__ __forceinline__ void tile(int i) {
        if (ST && i >= i0 && i < i0 + nst) tst[i - i0] = att;
        if (i == i0) sv = att;
        if (i == i0 + nst) out = att;
    }
    __device__ __forceinline__ void frame(int j, double m, double ma) {
        const double ik = inc[j % WP], dk = dec[j % WP];
        inc[j % WP] = div_cr(ma, bs.A, bs.rA);
        dec[j % WP] = div_cr(ma, bs.R, bs.rR);
        att = lean_step(att, m, ik, dk);
    }
};

// ---- release jumps -----------------------------------------------------------
// Exactness ("release jumps").  Let a be a double in binade e
// (2^e <= a < 2^(e+1)), so a = A u with u = 2^(e-52) and integer A.  A release step
// a' = RN(a - d) whose exact result a - d stays >= 2^e rounds on the grid u:
// a' = a - rho u with rho the nearest integer to d/u, a tie going to the even
// result.  rho therefore depends only on d, e and the parity of A.  A reference
// walk r that starts in binade e with the same parity and stays in it rounds
// every step exactly like a, so after the tile's T release steps a ends at
// a - (r0 - rT).  The describer walks 2 * JB such references per active tile
// (binades e0 .. e0+JB-1 from their tops, both parities; e0 = binade of the
// tile's largest M, below which no releasing state lies) and stores q = r0 - rT
// (exact; NaN if the reference left its binade) and the largest M.  A fix-up
// walker in state a (binade e, parity p) may jump iff x = a - q[e - e0][p] has
//   x > max M  (every entry state of the tile, all >= x, is > its M: release)
//   x >= 2^e + u (every exact difference a_k - d_k >= a_{k+1} - u/2 > 2^e: grid u)
// and then lands EXACTLY on the state the step-by-step walk reaches.  Inactive
// frames (M = 0) are d = 0 steps for both.
#ifndef MM_JB
#define MM_JB 8
#endif
constexpr int JB = MM_JB;  // binades per descriptor: e0 .. e0 + JB - 1
constexpr int JF = JB < 4 ? JB : 4;  // binades of the records the pass-0 guess folds use (e_fold_tile)
struct SegDesc {
    double mx;
    int e0;
    double q[2 * JB];
};
constexpr int DREC = 2 * JB;  // doubles per descriptor record: q[2 JB] (max M: mmax, e0 = its binade)

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

// The describer of one active tile as a stream consumer: the 2 * JB reference
// walks over its T rows, each off every dependency chain but its own.
struct Describer {
    static constexpr uint64_t MANT = (1ull << 52) - 1;
    double r0[2 * JB], r[2 * JB];
    int e0;
    BandStep bs;
    __device__ __forceinline__ void init(const double (&)[WB]) {}
    __device__ __forceinline__ void tile(int i) {
        if (i != 0) return;
#pragma unroll
        for (int k = 0; k < 2 * JB; ++k) {  // top of binade e0 + k/2, parity k % 2
            const uint64_t bits = ((uint64_t)(e0 + k / 2 + 1023) << 52) | (MANT - 63 + (uint64_t)(k % 2));
            r0[k] = r[k] = __longlong_as_double((long long)bits);
        }
    }
    __device__ __forceinline__ void frame(int, double m, double) {
        const double dec = div_cr(m, bs.R, bs.rR);
#pragma unroll
        for (int k = 0; k < 2 * JB; ++k) r[k] = r[k] - dec;
    }
    __device__ __forceinline__ void store(double *rec_) const {
        double2 *rec = reinterpret_cast<double2 *>(rec_);
        double q[2 * JB];
#pragma unroll
        for (int k = 0; k < 2 * JB; ++k) {
            // the reference stayed in its binade with a nonzero mantissa (>= 2^e + u) at the end
            const uint64_t rb = (uint64_t)__double_as_longlong(r[k]);
            const bool ok = (rb >> 52) == (uint64_t)(e0 + k / 2 + 1023) && (rb & MANT) != 0;
            q[k] = ok ? r0[k] - r[k] : __longlong_as_double(0x7ff8000000000000ll);
        }
#pragma unroll
        for (int k = 0; k < JB; ++k) rec[k] = make_double2(q[2 * k], q[2 * k + 1]);
    }
};

// 2. links + describers, ONE launch.  grid: (column blocks, 3), a block of
// 64 * TPS threads = one column block (64 super-tiles x TPS tiles = 64 TPS
// consecutive tiles of one chunk), lanes mapped to tiles as in comp_rms (wave k:
// tile position k of the 64 columns), so the describers' M loads are 512-byte runs.
//  * links: ranks the chunk's active tiles (rank[g] = active tiles before g in its
//    chunk: the counts comp_rms left per column block for the blocks before this
//    one, plus a scan over the block's tiles in tile order), lists them at compact
//    index ci = chunk * K + rank (tl = the tile, mmaxc = its largest M, cedc = its
//    (max,+) summary) and counts them (nact[c], by the chunk's last block);
//  * describers: an active tile's release-jump record (Describer).
// (Round 3 ran the links as one 1024-thread block per chunk and band: 30 blocks
// for a 5-min track, 26 us of latency before the describers' own launch.)
#ifndef MM_DESC_NB
#define MM_DESC_NB 1
#endif
constexpr int DESC_MAX_TPS = 8;  // block = 64 * TPS <= 512 threads (tile rounding: TPS = round(500 / T) <= 8)

__global__ void __launch_bounds__(64 * DESC_MAX_TPS) comp_describe_kernel(CompArgs a) {
    __shared__ int32_t wsum[DESC_MAX_TPS], base_s;
    __shared__ uint8_t flag[64 * DESC_MAX_TPS];
    __shared__ int32_t pre[64 * DESC_MAX_TPS];
    const int b = blockIdx.y;
    const int TPS = a.TPS, NT = 64 * TPS;
    const int kc = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int64_t cb = blockIdx.x;  // column block
    const int64_t sc = cb * 64 + l;
    const int64_t cc = sc / a.SPC;
    const int64_t cbl = (sc - cc * a.SPC) >> 6;  // column block within the chunk
    const int64_t jt = (sc - cc * a.SPC) * TPS + kc;
    const int64_t g = cc * a.K + jt;
    const bool valid = jt < a.K && g < a.G;
    const bool live = valid && a.cnt[b][g] != 0;
    // tile order within the block: tile jt = (column block base) + l * TPS + kc
    flag[l * TPS + kc] = live ? 1 : 0;
    if (threadIdx.x < 64) {  // active tiles of the chunk's earlier column blocks (comp_rms counts), wave 0
        int32_t acc = 0;
        const int32_t *ct = a.cbtot[b] + cc * (a.SPC >> 6);
        for (int64_t q = threadIdx.x; q < cbl; q += 64) acc += ct[q];
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (threadIdx.x == 0) base_s = acc;
    }
    __syncthreads();
    // exclusive scan of the flags in tile order: thread t takes entry t
    const int t = threadIdx.x;
    const bool f = flag[t] != 0;
    const uint64_t bal = __ballot(f);
    const int wp = (int)__popcll(bal & ((1ull << (t & 63)) - 1ull));
    if ((t & 63) == 0) wsum[t >> 6] = (int32_t)__popcll(bal);
    __syncthreads();
    int32_t woff = base_s;
    for (int w = 0; w < (t >> 6); ++w) woff += wsum[w];
    pre[t] = woff + wp;
    if (t == NT - 1 && cbl == (a.SPC >> 6) - 1) a.nact[b][cc] = woff + wp + (f ? 1 : 0);  // the chunk's last block
    __syncthreads();
    const int32_t r = pre[l * TPS + kc];
    const int64_t ci = cc * a.K + r;
    if (valid) a.rank[b][g] = r;
    if (live) {
        a.tl[b][ci] = (int32_t)g;
        a.mmaxc[b][ci] = a.mmax[b][g];
        reinterpret_cast<double2 *>(a.cedc[b])[ci] = reinterpret_cast<const double2 *>(a.ced[b])[g];
    }
    if (!a.jumps || __all(!live)) return;
    const int64_t gc = live ? g : cc * a.K;  // (dead lanes: the chunk's first tile)
    Describer d;
    d.bs = band_step(a, b);
    const double mx = a.mmax[b][gc];
    d.e0 = mx > 0.0 ? binade(mx) : 0;
    const uint32_t off = tile_off(a, gc);
    stream_col<true, MM_DESC_NB>(plane(a, b, cc), [&](int) { return off; }, 1, a.TP, d);
    if (live) d.store(a.descc[b] + ci * DREC);
}

// ---- super-tile release jumps --------------------------------------------------
// A full super-tile (SJ_TPS active tiles) gets a record composed from its tiles'
// release-jump records (pass 0 writes it): for a state a of binade e = e0s + kb
// (e0s: binade of the super-tile's largest M, kb < JB) and mantissa parity p, the
// SJ_TPS tile jumps are taken one after another iff a > L[kb][p] and a - Q[SJ_TPS]
// stays in binade e with a nonzero mantissa; Q[t] is the exact offset after t tiles
// (so the tiles' entry states are a - Q[t]).  Exactness: tile t's jump from
// a_t = a - Q[t] needs a_t - q_t > mx_t (L >= mx_t + Q[t+1], rounded up), x_t in
// binade e with a nonzero mantissa (x_t >= the final state >= 2^e + u, x_t < a <
// 2^(e+1)), and tile t's record to cover binade e with the parity of a_t (tracked:
// a_t - q_t flips it iff q_t / u is odd).  L = NaN: some tile's record does not
// cover (e, p), or the offsets leave the binade.  The fix-up walkers cross a
// release stretch a super-tile per jump (the long sweep chains are jump chains:
// tools/study/envelope_model.c), with the next record prefetched.
constexpr int SJ_TPS = 4;               // tiles per super-tile with records
constexpr int SJ_ENT = SJ_TPS + 1;      // doubles per (kb, p) entry: L, Q[1..SJ_TPS]
#ifndef MM_SJB
#define MM_SJB 4
#endif
constexpr int SJB = MM_SJB < JB ? MM_SJB : JB;  // binades per super-tile record: e0s .. e0s + SJB - 1
constexpr int SREC = 2 * SJB * SJ_ENT;  // doubles per super-tile record
constexpr int SJ_NONE = -100000;        // se0 of a super-tile without a record

__device__ __forceinline__ double next_up(double x) {
    return x > 0.0 ? __longlong_as_double(__double_as_longlong(x) + 1) : x;
}

// pass 0, lane = a full super-tile s with its first tile at compact index ci0 (the
// tiles' records are loaded before any store: the stores could alias them)
__device__ void compose_super(const CompArgs &a, int b, int64_t s, int64_t ci0) {
    double mxt[SJ_TPS], q[SJ_TPS][2 * JB];
#pragma unroll
    for (int t = 0; t < SJ_TPS; ++t) {
        mxt[t] = a.mmaxc[b][ci0 + t];
        const double2 *r = reinterpret_cast<const double2 *>(a.descc[b] + (ci0 + t) * DREC);
#pragma unroll
        for (int k = 0; k < JB; ++k) {
            const double2 v = r[k];
            q[t][2 * k] = v.x;
            q[t][2 * k + 1] = v.y;
        }
    }
    double mxs = 0.0;
#pragma unroll
    for (int t = 0; t < SJ_TPS; ++t) mxs = fmax(mxs, mxt[t]);
    const int e0s = binade(mxs);
    double *out = a.sdesc[b] + s * SREC;
#pragma unroll
    for (int k = 0; k < 2 * SJB; ++k) {
        double rec[SJ_ENT];
        double Q = 0.0, L = 0.0;
        int par = k & 1;
        bool ok = true;
        const int e = e0s + k / 2;
#pragma unroll
        for (int t = 0; t < SJ_TPS; ++t) {
            const int kt = e - binade(mxt[t]);
            const int idx = 2 * min(max(kt, 0), JB - 1) + par;
            double qv = q[t][0];
#pragma unroll
            for (int j = 1; j < 2 * JB; ++j) qv = idx == j ? q[t][j] : qv;
            ok = ok && kt >= 0 && kt < JB && qv == qv;
            Q += ok ? qv : 0.0;
            ok = ok && Q < ldexp(1.0, e);
            if (ok) par ^= (int)((int64_t)ldexp(qv, 52 - e) & 1);  // qv / u, an exact integer
            L = fmax(L, next_up(mxt[t] + Q));
            rec[1 + t] = Q;
        }
        rec[0] = ok ? L : __longlong_as_double(0x7ff8000000000000ll);
#pragma unroll
        for (int j = 0; j < SJ_ENT; ++j) out[k * SJ_ENT + j] = rec[j];  // (entry k: its own stores)
    }
    a.se0[b][s] = e0s;
}

// The pass-0 guess across one tile: the exit of the per-frame (max,+) walk E <-
// max(M, E - M/R) from entry E, bit for bit (tests/test_envelope_jumps.py) when the
// tile's release-jump record covers E: E = 0 or below the tile's largest M clamps
// in the tile and ends on ct (the walk from 0, comp_rms); above it the pure release
// E - q (exact while it stays in E's binade: the offsets do not depend on M), max'ed
// with ct (a walk that clamps ends on ct's values: the steps are monotone).  An
// uncovered E takes E - Dt (a guess; exactness never depends on it).
template <typename QF>
__device__ __forceinline__ double e_fold_tile(double E, double ct, double Dt, double mx, QF &&qat) {
    constexpr uint64_t MANT = (1ull << 52) - 1;
    if (!(E > 0.0)) return ct;
    const uint64_t ab = (uint64_t)__double_as_longlong(E);
    const int k = (int)(ab >> 52) - 1023 - binade(mx);
    if (k < 0) return ct;
    double x = E - Dt;
    if (k < JF) {
        const double y = E - qat(2 * k + (int)(ab & 1));  // (qat: the record entry, loaded by index)
        const uint64_t yb = (uint64_t)__double_as_longlong(y);
        if (y == y && (yb >> 52) == (ab >> 52) && (yb & MANT) != 0) x = y;
    }
    return fmax(ct, x);
}

// 3b. speculative pass.  grid: (ceil(GS/64), 3) of 64-lane blocks, lane =
// super-tile; the wave's 64 lanes step their tiles' rows in lockstep (their
// M-plane offsets staged in LDS).  A walker's start is exactly 0 for the chunk's
// first super-tile, else guessed: the (max,+) release envelope of the E_TILES
// active tiles before it (with `warmup` = 1, before a walk of the previous
// super-tile).  Exactness never depends on the guess (the fix-up sweeps).
constexpr int PASS0_BLOCK = 64, P0_MAXL = 64;  // lanes; tiles per walker (warm-up included)
constexpr int E_TILES = 32;  // active tiles folded into a pass-0 guess by default (~4000 frames of release history)

constexpr int EW_MAX = 64 * SJ_TPS + 64;  // tiles a pass-0 block stages for its guesses (TPS <= 4, window <= 64)
constexpr int P0_SMEM = (EW_MAX * (3 + 2 * JF) * 8 > P0_MAXL * PASS0_BLOCK * 4) ? EW_MAX * (3 + 2 * JF) * 8
                                                                                 : P0_MAXL * PASS0_BLOCK * 4;

__global__ void __launch_bounds__(PASS0_BLOCK) comp_pass0_kernel(CompArgs a) {
    // LDS: first the staged tile summaries of the guesses, then the walk's tile offsets
    __shared__ __attribute__((aligned(16))) char smem[P0_SMEM];
    uint32_t(*offs_lds)[PASS0_BLOCK] = reinterpret_cast<uint32_t(*)[PASS0_BLOCK]>(smem);
    const int b = blockIdx.y;
    const BandStep bs = band_step(a, b);
    const Plane p = plane(a, b, (int64_t)blockIdx.x * PASS0_BLOCK / a.SPC);  // (a block's 64 columns: one chunk)
    const int lane = threadIdx.x;
    const int64_t s = (int64_t)blockIdx.x * PASS0_BLOCK + lane;
    const int64_t sc = min(s, a.GS - 1);
    const Super st = super_of(a, b, sc);
    const bool live = s < a.GS && st.ntiles > 0;
    if (__all(!live)) return;
    const int64_t cK = (sc / a.SPC) * a.K;
    const int W = min(a.warmup, 1);
    const int64_t cw0 = max(cK, st.ci0 - (int64_t)W * a.TPS);  // first compact index walked
    const int nwarm = live ? (int)(st.ci0 - cw0) : 0, ntot = live ? nwarm + st.ntiles : 0;
    // the guess: the (max,+) walk of the e_tiles active tiles before the walk, from 0
    // (every attack an instant clamp, release at M/R per frame): bit-exact across
    // covered tiles, so after a loud stretch it carries the very release values a
    // speculative walk that clamped at the same peak computes (the M of the first
    // frame left ~all super-tiles stale).  The block's 64 windows
    // overlap: their tiles are staged in LDS once (coalesced), then each lane folds
    // its own window from LDS.
    double att = 0.0;
    {
        const int64_t nact_c = a.nact[b][sc / a.SPC];
        const int64_t lo = max(cK, (int64_t)__shfl(cw0, 0) - a.e_tiles);
        const int64_t hi = min(cK + nact_c, (int64_t)__shfl(cw0, 63));
        const int64_t n = hi - lo;
        const bool staged = n <= EW_MAX;
        double *sc_c = reinterpret_cast<double *>(smem);
        double *sc_d = sc_c + EW_MAX, *sc_m = sc_d + EW_MAX, *sc_q = sc_m + EW_MAX;  // q: [2 JF][EW_MAX]
        if (staged && n > 0) {
            const double2 *cd = reinterpret_cast<const double2 *>(a.cedc[b]);
            const double2 *qd = reinterpret_cast<const double2 *>(a.descc[b]);
            for (int i = lane; i < n; i += PASS0_BLOCK) {
                const double2 v = cd[lo + i];
                sc_c[i] = v.x;
                sc_d[i] = v.y;
                sc_m[i] = a.mmaxc[b][lo + i];
#pragma unroll
                for (int k = 0; k < JF; ++k) {
                    const double2 q = qd[(lo + i) * (DREC / 2) + k];
                    sc_q[(2 * k) * EW_MAX + i] = q.x;
                    sc_q[(2 * k + 1) * EW_MAX + i] = q.y;
                }
            }
        }
        __syncthreads();
        if (live && cw0 != cK && staged) {  // (a larger window or super-tile than the stage holds: guess 0)
            for (int64_t i = max(cK, cw0 - a.e_tiles) - lo; i < cw0 - lo; ++i)
                att = e_fold_tile(att, sc_c[i], sc_d[i], sc_m[i], [&](int idx) { return sc_q[idx * EW_MAX + i]; });
        }
        __syncthreads();  // (the stage is reused for the walk's offsets)
    }
    int nmax = ntot;
    for (int o = 32; o > 0; o >>= 1) nmax = max(nmax, __shfl_xor(nmax, o));
    nmax = __builtin_amdgcn_readfirstlane(nmax);
    const int32_t *tl = a.tl[b];
    for (int i = 0; i < nmax; ++i)  // the walk's tile offsets (lanes past their own repeat their last)
        offs_lds[i][lane] = tile_off(a, ntot ? tl[cw0 + min(i, ntot - 1)] : 0);
    __syncthreads();
    if (a.sjump) {  // the super-tile's release-jump record (the sweeps' super jumps)
        if (live && st.ntiles == SJ_TPS && a.TPS == SJ_TPS) compose_super(a, b, s, st.ci0);
        else if (s < a.GS) a.se0[b][s] = SJ_NONE;
    }
    Walker<true> w;
    w.att = att;
    w.out = att;
    w.sv = att;
    w.bs = bs;
    w.tst = a.tstc[b] + st.ci0;
    w.i0 = nwarm;
    w.nst = live ? st.ntiles : 0;
    stream_col<true, P0_NB>(p, [&](int i) { return offs_lds[i][lane]; }, nmax, a.TP, w);
    if (live) {
        a.start[b][s] = w.sv;
        a.end[b][s] = w.out;
    }
}

// 4. one fix-up sweep (exits at once if the previous sweep left nothing stale).
// grid: (ceil(GS/64), 3), lane = super-tile.  A lane whose start differs from its
// predecessor's end CLAIMS its super-tile (atomic max of the sweep stamp: one
// writer per super-tile per sweep) and re-walks it from that end, tile by tile:
// coalesced (stop) when the state equals the tile's stored entry state (the
// stored trajectory from there on, and the stored end, came from the same
// state), else it stores the state and jumps (exact release jump) or steps
// through the tile.  A re-walk that reaches the end without meeting the stored
// trajectory publishes the new end and CONTINUES into the successor (whose stored
// trajectory started from the old end) if it can claim it; if the successor's own
// lane claimed it first, that lane may have read the old end, so the sweep flags
// `changed` and the next sweep re-checks.  Every stale start is caught that way,
// so a sweep that flags nothing leaves every start equal to its predecessor's
// end: exact by induction from the chunk start.
//
// A chunk's active tiles are contiguous in compact index, so the walker's
// sequence runs on across super-tile boundaries: the stored state, largest M,
// jump record and plane offset of the tiles FIX_AHEAD ahead are loaded while it
// works on the current one, and a chain of jumps waits on no load.  In run-head
// sweeps the successor is claimed on entry (a Jacobi sweep's successors belong to
// their own lanes, so it claims at the end).
__device__ __forceinline__ bool comp_claim(const CompArgs &a, int b, int64_t s) {
    return __hip_atomic_fetch_max((gu32 *)(a.claim[b] + s), a.stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
           a.stamp;
}

struct TileMeta {
    double old, mx;
    double q[2 * JB];
    int32_t g;
};

#ifndef MM_FIX_AHEAD
#define MM_FIX_AHEAD 3
#endif
constexpr int FIX_AHEAD = MM_FIX_AHEAD;

// Sweep 1 (a.heads == 0) is a Jacobi step: every stale super-tile re-walks from
// its predecessor's current end.  Later sweeps start a walker only at the HEAD of
// each run of consecutive stale super-tiles (its predecessor is not stale): the
// head's walker carries its value through the run by continuation, where Jacobi
// walkers inside the run would claim the run's super-tiles first and stop the
// correction after one super-tile per sweep.  Every lane that sees its super-tile
// stale flags the sweep, so a sweep that flags nothing saw every start equal to
// its predecessor's end and changed nothing (the fixed point: exact).
__global__ void __launch_bounds__(64) comp_fix_kernel(CompArgs a, const unsigned int *prev_changed) {
    if (prev_changed && *prev_changed == 0u) return;
    const int64_t s = (int64_t)blockIdx.x * 64 + threadIdx.x;
    const int b = blockIdx.y;
    if (s >= a.GS) return;
    const int na_c = a.nact[b][s / a.SPC];  // (a walk stays in its chunk)
    Super st = super_of_na(a, s, na_c);
    if (st.ntiles == 0 || st.first) return;  // chunk starts are exact
    double *end = a.end[b];
    double att = ld_sc1(end + s - 1);
    if (__double_as_longlong(att) == __double_as_longlong(a.start[b][s])) return;
    *a.changed = 1u;  // stale: the next sweep re-checks (benign race: every writer stores 1)
    if (a.heads && (s - 1) % a.SPC != 0 &&
        __double_as_longlong(ld_sc1(end + s - 2)) != __double_as_longlong(a.start[b][s - 1]))
        return;  // inside a run
    if (!comp_claim(a, b, s)) return;  // a walker continuing from the predecessor owns it
    const uint64_t t_start = a.trace ? wall_clock64() : 0;
    int n_vis = 1;
    const BandStep bs = band_step(a, b);
    const Plane p = plane(a, b, s / a.SPC);  // (the wave's 64 columns and their walks: one chunk)
    double *tst = a.tstc[b];
    const int T = a.T;
    int64_t walked = 0, jumped = 0;
    const int64_t cend = st.ci0 + (int64_t)na_c - (s % a.SPC) * a.TPS;  // past the chunk's last
    auto ld = [&](int64_t ci) __attribute__((always_inline)) {
        TileMeta m;
        ci = min(ci, cend - 1);
        m.old = tst[ci];
        m.mx = a.mmaxc[b][ci];
        m.g = a.tl[b][ci];
        const double2 *r = reinterpret_cast<const double2 *>(a.descc[b] + ci * DREC);
#pragma unroll
        for (int k = 0; k < JB; ++k) {
            const double2 v = r[k];
            m.q[2 * k] = v.x;
            m.q[2 * k + 1] = v.y;
        }
        return m;
    };
    int64_t cur = s;
    bool nx_claimed = a.heads && !st.last ? comp_claim(a, b, cur + 1) : false;
    // super jumps (full super-tiles of SJ_TPS tiles): the record entries (both
    // parities) of the next super-tile are loaded one super-tile ahead for the
    // binade the state has now (a release stretch stays in its binade for many
    // super-tiles), its se0 two ahead, so a stretch is crossed without waiting on
    // memory; a binade change costs one dependent load.
    const bool sj = a.sjump && a.jumps && a.TPS == SJ_TPS;
    const double *srec = a.sdesc[b];
    const int32_t *se0 = a.se0[b];
    const int64_t slast = (s / a.SPC) * a.SPC + a.SPC - 1;  // (clamp for the prefetches: the chunk's columns)
    int e0_c = SJ_NONE, e0_n = SJ_NONE, e0_nn = SJ_NONE;  // se0 of cur, cur + 1, cur + 2
    int kb_c = -1, kb_n = -1;             // binade offsets the prefetched entries are for
    double old_c = 0.0, old_n = 0.0;      // stored entry states of cur's, cur + 1's first tile
    double ec[2][SJ_ENT], en[2][SJ_ENT];  // entries (parity 0, 1) of cur, cur + 1
    auto ld_ent = [&](int64_t sx, int kb, double (&e)[2][SJ_ENT]) __attribute__((always_inline)) {
        const double *r = srec + min(sx, slast) * SREC + 2 * min(max(kb, 0), SJB - 1) * SJ_ENT;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int j = 0; j < SJ_ENT; ++j) e[q][j] = r[q * SJ_ENT + j];
    };
    if (sj) {
        e0_c = se0[cur];
        e0_n = se0[min(cur + 1, slast)];
        e0_nn = se0[min(cur + 2, slast)];
        old_c = tst[st.ci0];
        kb_c = binade(att) - e0_c;
        ld_ent(cur, kb_c, ec);
    }
    // advance the prefetch pipeline to super-tile cur (its predecessor's data shifts in)
    auto sj_advance = [&]() __attribute__((always_inline)) {
        e0_c = e0_n;
        kb_c = kb_n;
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int j = 0; j < SJ_ENT; ++j) ec[q][j] = en[q][j];
        e0_n = e0_nn;
        e0_nn = se0[min(cur + 2, slast)];  // (used one super-tile later: its latency hides)
        old_c = old_n;
    };
    auto sj_prefetch = [&]() __attribute__((always_inline)) {  // cur + 1: first stored state, entries
        old_n = tst[min(st.ci0 + st.ntiles, cend - 1)];
        kb_n = binade(att) - e0_n;
        ld_ent(cur + 1, kb_n, en);
    };
    if (sj) sj_prefetch();
    TileMeta ring[FIX_AHEAD];
    bool ring_ok = !sj;  // the ring holds tiles ci .. ci + FIX_AHEAD - 1
    if (ring_ok) {
#pragma unroll
        for (int k = 0; k < FIX_AHEAD; ++k) ring[k] = ld(st.ci0 + k);
    }
    a.start[b][cur] = att;
    int64_t ci = st.ci0, ce = st.ci0 + st.ntiles;  // position, end of cur
    bool sj_try = sj && st.ntiles == SJ_TPS;       // at the start of a full super-tile
    // after tile ci: the end of cur publishes its end and continues into the
    // successor if it is (or can be) claimed; false: the walk ends
    auto next = [&]() __attribute__((always_inline)) -> bool {
        if (++ci < ce) return true;
        st_sc1(end + cur, att);
        if (st.last) return false;  // the chunk's last super-tile
        // continue into the successor if it could be claimed (else its owner read an
        // older end of cur: it is stale next sweep, which this walk's own `changed`
        // flag queues); with jacobi_stop the Jacobi sweep's walkers stop here instead
        // (C2: 5 sweeps, fix 0.295 ms against 3 and 0.269 continuing)
        if (!a.heads && a.jacobi_stop) return false;
        if (!a.heads) nx_claimed = comp_claim(a, b, cur + 1);
        if (!nx_claimed) return false;
        ++cur;
        st = super_of_na(a, cur, na_c);
        a.start[b][cur] = att;
        ce = st.ci0 + st.ntiles;
        nx_claimed = a.heads && !st.last ? comp_claim(a, b, cur + 1) : false;
        ++n_vis;
        if (sj) {
            sj_advance();
            sj_prefetch();
            sj_try = st.ntiles == SJ_TPS;
        }
        return true;
    };
    // Lanes run through coalescence checks and jumps on their own until each needs
    // to step through a tile (or is done); then every lane that needs to walks its
    // tile at once, in lockstep: divergent lanes never serialise their walks.
    TileMeta m;
    bool run = true, walk = false;
    for (;;) {
        while (run && !walk) {
            if (sj_try) {  // a whole super-tile in one jump?
                sj_try = false;
                const double old0 = ring_ok ? ring[0].old : old_c;
                if (__double_as_longlong(old0) == __double_as_longlong(att)) {  // coalesced
                    run = false;
                    break;
                }
                constexpr uint64_t MANT = (1ull << 52) - 1;
                const uint64_t ab = (uint64_t)__double_as_longlong(att);
                const int kb = (int)(ab >> 52) - 1023 - e0_c;
                if (att > 0.0 && kb >= 0 && kb < SJB) {
                    if (kb != kb_c) {  // the state left the prefetched binade
                        kb_c = kb;
                        ld_ent(cur, kb, ec);
                    }
                    const int par = (int)(ab & 1);
                    const double L = par ? ec[1][0] : ec[0][0];
                    const double Qt = par ? ec[1][SJ_TPS] : ec[0][SJ_TPS];
                    const double x = att - Qt;
                    const uint64_t xb = (uint64_t)__double_as_longlong(x);
                    if (att > L && (xb >> 52) == (ab >> 52) && (xb & MANT) != 0) {
                        tst[ci] = att;
#pragma unroll
                        for (int t = 1; t < SJ_TPS; ++t) tst[ci + t] = att - (par ? ec[1][t] : ec[0][t]);
                        att = x;
                        jumped += (int64_t)SJ_TPS * T;
                        ci += SJ_TPS - 1;
                        ring_ok = false;
                        run = next();
                        continue;
                    }
                }
            }
            if (!ring_ok) {  // tile by tile from ci
#pragma unroll
                for (int k = 0; k < FIX_AHEAD; ++k) ring[k] = ld(ci + k);
                ring_ok = true;
            }
            m = ring[0];
#pragma unroll
            for (int k = 0; k + 1 < FIX_AHEAD; ++k) ring[k] = ring[k + 1];
            ring[FIX_AHEAD - 1] = ld(ci + FIX_AHEAD);
            if (__double_as_longlong(m.old) == __double_as_longlong(att)) {  // coalesced
                run = false;
                break;
            }
            tst[ci] = att;
            double x;
            SegDesc d;
            d.mx = m.mx;
            d.e0 = binade(m.mx);
#pragma unroll
            for (int k = 0; k < 2 * JB; ++k) d.q[k] = m.q[k];
            if (a.jumps && release_jump(d, att, &x)) {
                att = x;
                jumped += T;
                run = next();
            } else {
                walk = true;
            }
        }
        if (!__any(walk)) break;
        if (walk) {
            Walker<false> w;
            w.att = att;
            w.bs = bs;
            w.i0 = 0;
            w.nst = 1;
            const uint32_t off = tile_off(a, m.g);
            stream_col<true, FIX_WNB>(p, [&](int) { return off; }, 1, a.TP, w);  // (the walking lanes step the same rows)
            att = w.att;
            walked += T;
            walk = false;
            run = next();
        }
    }
    if (a.trace && a.sweep_idx < 16) {
        uint32_t *r = a.trace + (((int64_t)a.sweep_idx * 3 + b) * a.GS + s) * 4;
        r[0] = (uint32_t)(wall_clock64() - t_start);  // 100 MHz ticks
        r[1] = (uint32_t)(walked / a.T);
        r[2] = (uint32_t)(jumped / a.T);
        r[3] = (uint32_t)n_vis;
    }
    if (walked) atomicAdd(a.walked, (unsigned long long)walked);
    if (jumped) atomicAdd(a.walked + 1, (unsigned long long)jumped);
}

// 5. gains + overlay.  A block = 64 tiles x 3 bands: wave w runs band w's exact
// trajectory for its 64 tiles from their entry states (audioop.mul floor
// on both channels), APPLY_STEP frames at a time into LDS; then all 192 threads
// overlay sat16(sat16(lo + mid) + hi) (AME:210) and store q2 coalesced.
// Branch-free per frame so a group's steps, gains and multiplies interleave:
//  * M == 0 (rms <= threshold) needs no test: the step is then the identity;
//  * att == 0 gives gain 10^-0 = 1.0 exactly, for which audioop.mul is the
//    identity (pydub skips the multiply there);
//  * the group's 10^(-att/20) are skipped (wave-uniformly) when no lane's att
//    changed since the last gain (the sparse band's wave, almost always).
// M and sample loads run two groups ahead.
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

// 2^(j/64), j < 64, as double-double {hi, lo} (hi = RN(2^(j/64)), lo = RN(2^(j/64) - hi);
// generated with Python's decimal module at 60 digits)
__constant__ double2 EXP2_TAB64[64] = {
    {0x1.0000000000000p+0, 0x0.0p+0}, {0x1.02c9a3e778061p+0, -0x1.19083535b085dp-56},
    {0x1.059b0d3158574p+0, 0x1.d73e2a475b465p-55}, {0x1.0874518759bc8p+0, 0x1.186be4bb284ffp-57},
    {0x1.0b5586cf9890fp+0, 0x1.8a62e4adc610bp-54}, {0x1.0e3ec32d3d1a2p+0, 0x1.03a1727c57b53p-59},
    {0x1.11301d0125b51p+0, -0x1.6c51039449b3ap-54}, {0x1.1429aaea92de0p+0, -0x1.32fbf9af1369ep-54},
    {0x1.172b83c7d517bp+0, -0x1.19041b9d78a76p-55}, {0x1.1a35beb6fcb75p+0, 0x1.e5b4c7b4968e4p-55},
    {0x1.1d4873168b9aap+0, 0x1.e016e00a2643cp-54}, {0x1.2063b88628cd6p+0, 0x1.dc775814a8495p-55},
    {0x1.2387a6e756238p+0, 0x1.9b07eb6c70573p-54}, {0x1.26b4565e27cddp+0, 0x1.2bd339940e9d9p-55},
    {0x1.29e9df51fdee1p+0, 0x1.612e8afad1255p-55}, {0x1.2d285a6e4030bp+0, 0x1.0024754db41d5p-54},
    {0x1.306fe0a31b715p+0, 0x1.6f46ad23182e4p-55}, {0x1.33c08b26416ffp+0, 0x1.32721843659a6p-54},
    {0x1.371a7373aa9cbp+0, -0x1.63aeabf42eae2p-54}, {0x1.3a7db34e59ff7p+0, -0x1.5e436d661f5e3p-56},
    {0x1.3dea64c123422p+0, 0x1.ada0911f09ebcp-55}, {0x1.4160a21f72e2ap+0, -0x1.ef3691c309278p-58},
    {0x1.44e086061892dp+0, 0x1.89b7a04ef80d0p-59}, {0x1.486a2b5c13cd0p+0, 0x1.3c1a3b69062f0p-56},
    {0x1.4bfdad5362a27p+0, 0x1.d4397afec42e2p-56}, {0x1.4f9b2769d2ca7p+0, -0x1.4b309d25957e3p-54},
    {0x1.5342b569d4f82p+0, -0x1.07abe1db13cadp-55}, {0x1.56f4736b527dap+0, 0x1.9bb2c011d93adp-54},
    {0x1.5ab07dd485429p+0, 0x1.6324c054647adp-54}, {0x1.5e76f15ad2148p+0, 0x1.ba6f93080e65ep-54},
    {0x1.6247eb03a5585p+0, -0x1.383c17e40b497p-54}, {0x1.6623882552225p+0, -0x1.bb60987591c34p-54},
    {0x1.6a09e667f3bcdp+0, -0x1.bdd3413b26456p-54}, {0x1.6dfb23c651a2fp+0, -0x1.bbe3a683c88abp-57},
    {0x1.71f75e8ec5f74p+0, -0x1.16e4786887a99p-55}, {0x1.75feb564267c9p+0, -0x1.0245957316dd3p-54},
    {0x1.7a11473eb0187p+0, -0x1.41577ee04992fp-55}, {0x1.7e2f336cf4e62p+0, 0x1.05d02ba15797ep-56},
    {0x1.82589994cce13p+0, -0x1.d4c1dd41532d8p-54}, {0x1.868d99b4492edp+0, -0x1.fc6f89bd4f6bap-54},
    {0x1.8ace5422aa0dbp+0, 0x1.6e9f156864b27p-54}, {0x1.8f1ae99157736p+0, 0x1.5cc13a2e3976cp-55},
    {0x1.93737b0cdc5e5p+0, -0x1.75fc781b57ebcp-57}, {0x1.97d829fde4e50p+0, -0x1.d185b7c1b85d1p-54},
    {0x1.9c49182a3f090p+0, 0x1.c7c46b071f2bep-56}, {0x1.a0c667b5de565p+0, -0x1.359495d1cd533p-54},
    {0x1.a5503b23e255dp+0, -0x1.d2f6edb8d41e1p-54}, {0x1.a9e6b5579fdbfp+0, 0x1.0fac90ef7fd31p-54},
    {0x1.ae89f995ad3adp+0, 0x1.7a1cd345dcc81p-54}, {0x1.b33a2b84f15fbp+0, -0x1.2805e3084d708p-57},
    {0x1.b7f76f2fb5e47p+0, -0x1.5584f7e54ac3bp-56}, {0x1.bcc1e904bc1d2p+0, 0x1.23dd07a2d9e84p-55},
    {0x1.c199bdd85529cp+0, 0x1.11065895048ddp-55}, {0x1.c67f12e57d14bp+0, 0x1.2884dff483cadp-54},
    {0x1.cb720dcef9069p+0, 0x1.503cbd1e949dbp-56}, {0x1.d072d4a07897cp+0, -0x1.cbc3743797a9cp-54},
    {0x1.d5818dcfba487p+0, 0x1.2ed02d75b3707p-55}, {0x1.da9e603db3285p+0, 0x1.c2300696db532p-54},
    {0x1.dfc97337b9b5fp+0, -0x1.1a5cd4f184b5cp-54}, {0x1.e502ee78b3ff6p+0, 0x1.39e8980a9cc8fp-55},
    {0x1.ea4afa2a490dap+0, -0x1.e9c23179c2893p-54}, {0x1.efa1bee615a27p+0, 0x1.dc7f486a4b6b0p-54},
    {0x1.f50765b6e4540p+0, 0x1.9d3e12dd8a18bp-54}, {0x1.fa7c1819e90d8p+0, 0x1.74853f3a5931ep-55}};

// 10^y for the compressor's gains (y = RN(-att/20) <= 0): 2^(y log2 10) with the
// exponent split t = k/64 + r (|r| <= 1/128; y log2 10 carried to ~106 bits by two
// FMAs), 2^r by its degree-6 Taylor polynomial (truncation 3e-20) and 2^(k/64) from
// the double-double table in LDS.  Within 1.5 ulp of 10^y on [-3, 0] (pydub's libm
// pow within 0.5): a gain one or two ulp off moves floor(x * gain) (audioop.mul) only
// when x * gain lies within ~1e-11 of an integer, as with OCML's exp10.
// y = 0 gives exactly 1.0 (the identity gain of an unattenuated frame).  18 VALU + one
// LDS read against OCML exp10's ~70.
__device__ __forceinline__ double exp10_tab(double y, const double2 *tab) {
    constexpr double L_HI = 0x1.a934f0979a371p+1, L_LO = 0x1.7f2495fb7fa6dp-53;
    const double th = y * L_HI;
    const double tl = fma(y, L_LO, fma(y, L_HI, -th));
    const double kd = rint(th * 64.0);
    const int k = (int)kd;
    const double r = fma(-kd, 0.015625, th) + tl;
    double p = 0x1.430912f86c787p-13;
    p = fma(p, r, 0x1.5d87fe78a6731p-10);
    p = fma(p, r, 0x1.3b2ab6fba4e77p-7);
    p = fma(p, r, 0x1.c6b08d704a0c0p-5);
    p = fma(p, r, 0x1.ebfbdff82c58fp-3);
    p = fma(p, r, 0x1.62e42fefa39efp-1);
    p = fma(p, r, 1.0);
    const double2 t = tab[k & 63];
    return ldexp(fma(t.x, p, t.y * p), k >> 6);
}

// Verification of the compressor's two hand-made elementary functions on the
// device (mm_check_compressor_math, tests/test_compressor_math.py): what 0: out =
// exp10_tab(a) (10^a); what 1: out = rms_exact1(a, b) with comp_rms's biased
// reciprocal (isqrt(floor(a / b)) for integers a < 2^53, b >= 1).
__global__ void __launch_bounds__(256) comp_math_kernel(int what, const double *xa, const double *xb, int64_t n,
                                                       double *out) {
    __shared__ double2 etab[64];
    if (threadIdx.x < 64) etab[threadIdx.x] = EXP2_TAB64[threadIdx.x];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (what == 0) out[i] = exp10_tab(xa[i], etab);
    else out[i] = (double)rms_exact1(xa[i], xb[i], rcp_biased(xb[i]));
}

#ifndef MM_APPLY_MINB
#define MM_APPLY_MINB 1
#endif
#ifdef MM_APPLY_OCML  // (A/B builds: OCML's exp10)
#define MM_GAIN(att) exp10(neg_div20(att))
#else
#define MM_GAIN(att) exp10_tab(neg_div20(att), etab)
#endif
__global__ void __launch_bounds__(192, MM_APPLY_MINB) comp_apply_kernel(CompArgs a) {
    constexpr int S = APPLY_STEP;
    __shared__ short2 lds[3][S][APPLY_TILES];
    __shared__ double2 etab[64];
    if (threadIdx.x < 64) etab[threadIdx.x] = EXP2_TAB64[threadIdx.x];
    __syncthreads();
    const int b = threadIdx.x / APPLY_TILES;
    const int lane = threadIdx.x % APPLY_TILES;
    const int64_t G = a.G;
    // chunk-aligned blocks (the M rows of a block's 64 tiles are whole cache lines)
    const int64_t WPC = ((int64_t)a.K + APPLY_TILES - 1) / APPLY_TILES;
    const int64_t cb = blockIdx.x / WPC;
    const int64_t j0 = (blockIdx.x - cb * WPC) * APPLY_TILES;  // first tile of the block in its chunk
    const int64_t g0 = cb * a.K + j0;
    const int64_t g = g0 + lane;
    const int jn = (int)min((int64_t)APPLY_TILES, a.K - j0);  // the block's tiles (the chunk's last block: fewer)
    const bool valid = lane < jn && g < G;
    const int T = a.T;
    const int len = valid ? (int)min((int64_t)T, a.N_proc - g * T) : 0;
    const BandStep bs = band_step(a, b);
    const short2 *X = a.band[b];
    // this tile's column and rows in the M plane
    int64_t sg;
    int kg;
    tile_col(a, valid ? g : 0, &sg, &kg);
    constexpr uint32_t GS32 = 64;  // elements per row of a column block
    const uint32_t e0 = col_elem(a, sg) + (uint32_t)(kg * a.TP) * GS32;
    const double *Mp = chunk_plane(a, b, valid ? g / a.K : 0);
    double att = 0.0;
    if (valid) {  // the entry state of the tile, or of the next active one (held), or the chunk's end
        const int64_t c = g / a.K;
        const int32_t r = a.rank[b][g], na = a.nact[b][c];
        att = r < na ? a.tstc[b][c * a.K + r] : na > 0 ? a.end[b][c * a.SPC + (na - 1) / a.TPS] : 0.0;
    }
    double gain = 1.0, gain_att = -1.0;  // gain of gain_att; att >= 0 never equals -1
    // a wave whose 64 tiles hold no active frame (the sparse band, almost
    // everywhere) keeps each tile's entry state: one constant gain per lane, no
    // M loads or steps
    const bool quiet = __all(!valid || a.cnt[b][g] == 0);
    if (quiet) {
        gain = MM_GAIN(att);
        gain_att = att;
    }
    const uint32_t G32 = (uint32_t)G, gl = valid ? (uint32_t)g : 0u;
    const uint32_t last = (uint32_t)max(len - 1, 0);
    const short2 *Xl = X + gl;       // this lane's tile, row 0
    const double *Ml = Mp + e0;      // this lane's column, its tile's row 0
    // rows past the tile's frames hold M = 0 (comp_rms): identity steps whose
    // output is unused; samples are clamped to the tile
    // a tile without active frames has M = 0 throughout: comp_rms may not have
    // stored its rows (quiet tiles), so it takes 0 instead of loading them
    const bool act = valid && a.cnt[b][g] != 0;
    // the overlay's fast path: the block's 64 tiles all whole (every block but a
    // chunk's last and the track's last), so its rows need no per-element bounds
    const bool full = jn == APPLY_TILES && (g0 + APPLY_TILES) * T <= a.N_proc;
    const bool stereo = a.ch == 2;
    short2 *const qrow0 = a.q_out + g0;  // row 0 of the block's first tile
    auto load = [&](int n0, double (&m)[S], short2 (&v)[S], bool with_m) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < S; ++j) {
            if (with_m) m[j] = act ? Ml[(size_t)min(n0 + j, T - 1) * GS32] : 0.0;  // (uniform row)
            v[j] = Xl[(size_t)min((uint32_t)(n0 + j), last) * G32];
        }
    };
    // one group of S frames from its buffers (m, v), then the buffers refilled with
    // the group two ahead: two groups unrolled per iteration, so the buffers never
    // rotate through register copies
    auto group = [&](int n0, double (&m)[S], short2 (&v)[S]) __attribute__((always_inline)) {
        double gj[S];
        if (quiet) {  // wave-uniform: only the samples stream
#pragma unroll
            for (int j = 0; j < S; ++j) gj[j] = gain;
        } else {
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
                for (int j = 0; j < S; ++j)
#ifdef MM_APPLY_NOEXP  // timing experiment only (wrong gains)
                    gj[j] = 1.0 + neg_div20(at[j]);
#else
                    gj[j] = MM_GAIN(at[j]);  // db_to_float(-att); exactly 1 at att == 0
#endif
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
        load(n0 + 2 * S, m, v, !quiet);
        lds_barrier();
        if (full) {  // every tile of the block whole: wave w takes rows w, w + 3, ... (uniform)
            const int nv = min(S, T - n0);
            for (int j = b; j < nv; j += 3) {
                const short2 lo = lds[0][j][lane], mi = lds[1][j][lane], hi = lds[2][j][lane];
                const int16_t l = sat16(sat16((int32_t)lo.x + mi.x) + hi.x);
                const int16_t rr = sat16(sat16((int32_t)lo.y + mi.y) + hi.y);
                (qrow0 + (int64_t)(n0 + j) * G)[lane] = make_short2(l, stereo ? rr : (int16_t)0);
            }
        } else for (int p = threadIdx.x; p < S * APPLY_TILES; p += 3 * APPLY_TILES) {
            const int j = p / APPLY_TILES, tl = p % APPLY_TILES;
            const int64_t gt = g0 + tl;
            const int n = n0 + j;
            if (tl < jn && gt < G && n < (int)min((int64_t)T, a.N_proc - gt * T)) {
                const short2 lo = lds[0][j][tl], mi = lds[1][j][tl], hi = lds[2][j][tl];
                const int16_t l = sat16(sat16((int32_t)lo.x + mi.x) + hi.x);
                const int16_t rr = sat16(sat16((int32_t)lo.y + mi.y) + hi.y);
                a.q_out[(int64_t)n * G + gt] = make_short2(l, a.ch == 2 ? rr : (int16_t)0);
            }
        }
        lds_barrier();
    };
    double mA[S], mB[S];
    short2 vA[S], vB[S];
    load(0, mA, vA, !quiet);
    load(S, mB, vB, !quiet);
    for (int n0 = 0; n0 < T; n0 += 2 * S) {
        group(n0, mA, vA);
        if (n0 + S < T) group(n0 + S, mB, vB);
    }
}

}  // namespace mm
