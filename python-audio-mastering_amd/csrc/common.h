// common.h — shared device-side argument blocks of the mastering kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Python float / numpy semantics: no implicit FMA contraction anywhere.  The
// linear-recurrence kernels call fma() explicitly where it is wanted.  The pragma
// covers code in these files; the Makefile also passes -ffp-contract=off, because
// HIP's __fmul_rn/__fadd_rn bodies are compiled before it and were fused into
// v_fma_f32 when inlined next to each other (seen in the f32 soft limiter).
#pragma clang fp contract(off)

namespace mm {

// Workgroup barrier that orders LDS only.  __syncthreads()' fence also waits for
// every outstanding global access (vmcnt(0)), i.e. it stalls on the block's own
// in-flight stores and drains register prefetch pipelines at every barrier.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The value held by the partner lane (lane ^ 1) of a stereo lane pair: a DPP
// quad_perm [1,0,3,2] move (VALU), not __shfl_xor's ds_bpermute LDS round trip.
// (every lane reads a lane of its own quad, so no "old" value is ever kept:
// mov_dpp with bound_ctrl needs no zero-initialised destination)
__device__ __forceinline__ int32_t pair_swap(int32_t v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true); }
__device__ __forceinline__ double pair_swap(double v) {
    const int64_t b = __double_as_longlong(v);
    const int32_t lo = pair_swap((int32_t)(b & 0xffffffff)), hi = pair_swap((int32_t)(b >> 32));
    return __longlong_as_double(((int64_t)hi << 32) | (uint32_t)lo);
}

// Correctly rounded f32 square root (numpy's np.sqrt / x ** 0.5 on float32).
// __fsqrt_rn lowers to v_sqrt_f32 (1 ulp) on gfx950; the f64 square root is
// correctly rounded and rounding it to f32 is exact-safe (53 >= 2*24 + 2 bits).
__device__ __forceinline__ float sqrt_f32_cr(float x) { return (float)__dsqrt_rn((double)x); }

// Software-pipelined sequential stream over elements 0..len-1: ld(i) returns
// element i and MUST be safe (clamped) for any i < len + NB*B; proc(v) consumes
// elements in order.  NB*B elements stay in flight in registers, hiding
// HBM/Infinity-Cache latency behind a lane's dependent chain.  The main loop is
// branch-free (no conditional loads or stores), which lets the compiler use
// counted s_waitcnt vmcnt(N) instead of draining every load; the ragged tail
// is consumed once after it.
template <int B, int NB, typename V, typename LD, typename PROC>
__device__ __forceinline__ void stream(int len, LD &&ld, PROC &&proc) {
    constexpr int R = B * NB;
    if (len <= 0) return;
    // sched_barrier pins the issue order of the load blocks to be the same in
    // the prologue and in the loop body; without it the scheduler permutes the
    // prologue loads, the two paths into the loop header disagree on which
    // register is oldest, and the waitcnt pass falls back to vmcnt(0).
    V buf[NB][B];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
#pragma unroll
        for (int j = 0; j < B; ++j) buf[k][j] = ld(k * B + j);
        __builtin_amdgcn_sched_barrier(0);
    }
    const int nfull = len / R;
    int base = 0;
    for (int r = 0; r < nfull; ++r, base += R) {
#pragma unroll
        for (int k = 0; k < NB; ++k) {
#pragma unroll
            for (int j = 0; j < B; ++j) proc(buf[k][j]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < B; ++j) buf[k][j] = ld(base + R + k * B + j);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    const int rem = len - base;
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
        for (int j = 0; j < B; ++j)
            if (k * B + j < rem) proc(buf[k][j]);
}

// Two-stage variant for dependent gathers: ld1(i) is streamed NB blocks ahead,
// ld2(v1) (e.g. a table lookup indexed by the loaded value) is issued one block
// ahead of its use, so both latencies hide behind the consumer proc(v1, v2).
// ld2 must be safe for any v1 that ld1 can return.
template <int B, int NB, typename V1, typename V2, typename LD1, typename LD2, typename PROC>
__device__ __forceinline__ void stream2(int len, LD1 &&ld1, LD2 &&ld2, PROC &&proc) {
    constexpr int R = B * NB;
    if (len <= 0) return;
    V1 a[NB][B];
    V2 m[B];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
#pragma unroll
        for (int j = 0; j < B; ++j) a[k][j] = ld1(k * B + j);
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 0; j < B; ++j) m[j] = ld2(a[0][j]);
    __builtin_amdgcn_sched_barrier(0);
    const int nfull = len / R;
    int base = 0;
    for (int r = 0; r < nfull; ++r, base += R) {
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            V2 mn[B];
#pragma unroll
            for (int j = 0; j < B; ++j) mn[j] = ld2(a[(k + 1) % NB][j]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < B; ++j) proc(a[k][j], m[j]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < B; ++j) a[k][j] = ld1(base + R + k * B + j);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < B; ++j) m[j] = mn[j];
        }
    }
    const int rem = len - base;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        V2 mn[B];
#pragma unroll
        for (int j = 0; j < B; ++j) mn[j] = ld2(a[(k + 1) % NB][j]);
#pragma unroll
        for (int j = 0; j < B; ++j)
            if (k * B + j < rem) proc(a[k][j], m[j]);
#pragma unroll
        for (int j = 0; j < B; ++j) m[j] = mn[j];
    }
}

struct SatArgs {
    float keep, mix, drive;
    int on;
    const float *tab;  // [65536] the reference's apply_saturation on the int16 grid (mm_job.sat_table), or null
    // [4096] signed 2-bit codes per grid index k + 32768 (16 per word): numpy's value
    // minus the device's tanhf evaluation, as float bit patterns (0, +1, -1); built on
    // the device from tab (sat_corr_kernel) and used only when complete (no entry off
    // by more than one step), else null (tab alone: a gather per sample)
    const uint32_t *corr;
};

// apply_saturation's value for x = k / 32768 from the host table (numpy's float32
// tanh, bit for bit); false when x is not on the int16 grid (the caller evaluates
// the expression itself).  x * 32768 is exact; v_cvt_i32_f32 truncates.
__device__ __forceinline__ bool sat_lookup(float x, const float *tab, float *y) {
    const float t = x * 32768.0f;
    const int k = (int)t;
    if ((float)k != t || k < -32768 || k > 32767) return false;
    *y = tab[k + 32768];
    return true;
}

struct CompArgs {
    int64_t N_proc, G;
    int T, K, ch, warmup;
    int TPS;                   // tiles per super-tile (envelope solve unit)
    int64_t SPC;               // super-tiles (columns) per chunk: ceil(K / TPS) rounded up to a multiple of 64
    int64_t GS;                // super-tiles = chunks * SPC
    const short2 *band[3];
    const double *lut[3];      // device tables [32769]: M per integer rms
    uint32_t r0[3];            // smallest rms with M != 0 ("above threshold")
    int look[3];
    double attack_frames[3], release_frames[3];
    double rcp_attack[3], rcp_release[3];
    double *Ms[3];             // super-tile-major M plane, column blocks of 64 x RP rows (compressor.hip tile_col)
    int TP;                    // plane rows per tile: T rounded up to whole walk load blocks
    int RP;                    // rows per column of the M plane (TPS*TP + prefetch padding)
    int64_t chunk_elems;       // elements of one chunk's part of a band's plane (buffer descriptors: < 4 GB)
    const double *E[3], *tail[3];  // per tile: sum of L^2+R^2, and over its last look % T frames
    int32_t *cnt[3];           // per tile: active frames
    double *mmax[3];           // per tile: largest M
    double *ced[3];            // per tile: (max,+) release summary {c, D} (double2; comp_rms)
    int32_t *total[3];         // per chunk: active frames (statistics)
    int32_t *cbtot[3];         // per column block: active tiles (comp_rms; zeroed per chain)
    int32_t *rank[3];          // per tile: active tiles before it in its chunk (comp_describe)
    int32_t *nact[3];          // per chunk: active tiles
    // per active tile at compact index ci = chunk * K + rank:
    int32_t *tl[3];            // the tile
    double *mmaxc[3];          // its largest M
    double *cedc[3];           // its (max,+) release summary (double2; pass-0 guesses)
    double *tstc[3];           // envelope state on entry (written by the owning walks)
    double *descc[3];          // release-jump record [2 JB] (compressor.hip Describer)
    double *start[3];          // per-super-tile start state
    double *end[3];            // per-super-tile end state (one buffer; sweeps hand ends over with sc1 accesses)
    uint32_t *claim[3];        // per super-tile: the last sweep stamp that claimed it (zeroed per chain)
    int jumps;                 // release jumps enabled (MM_COMP_NOJUMP=1 disables them: diagnostics)
    int sjump;                 // super-tile jumps enabled (MM_COMP_NOSJUMP=1 disables them: diagnostics)
    double *sdesc[3];          // per super-tile: composed release-jump record (compressor.hip compose_super)
    int32_t *se0[3];           // per super-tile: binade of its largest M (SJ_NONE: no record)
    uint32_t stamp;            // this sweep's stamp (> every earlier one of the chain)
    int heads;                 // 0: Jacobi sweep (every stale super-tile walks); 1: run heads only
    int jacobi_stop;           // a Jacobi walker stops at its super-tile's end (MM_JACOBI_STOP=1: experiments)
    int e_tiles;               // active tiles of a pass-0 guess's (max,+) fold (MM_E_TILES; E_TILES)
    unsigned int *changed;
    unsigned long long *walked;  // [0] frames re-walked, [1] frames jumped by the fix-up sweeps (statistics)
    uint32_t *trace;           // diagnostics (MM_FIX_TRACE): per sweep, band, super-tile {10 ns ticks, walked, jumped, visited}
    int sweep_idx;
    short2 *q_out;
};

struct FinArgs {
    int64_t N_proc, G;       // frames and tiles of this track
    int64_t Gs, g_off;       // row stride of the tile-major mix, this track's first tile in it
    int T, ch, out_kind, use_gain;
    double gain;
    const double *gain_dev;  // device gain (loudness gated on the device) or null
    const short2 *mix;
    void *out;
    // The chain's tail (its last finalize launch; ctl null otherwise): every block
    // zeroes its slice of the control block past the readback area, and the last
    // block to finish copies the readback area into the mapped host block, then
    // zeroes it, so the next chain starts on a zeroed block with no fill or copy.
    char *ctl;
    int64_t ctl_bytes, rb_area;  // the control block, its readback area (both multiples of 4)
    int rb_bytes;                // readback bytes copied out (a multiple of 4)
    char *rb_host;               // device address of the mapped host block
    unsigned *done;              // finished-block counters: FIN_DONE_LINES + 1, 128 B apart
};
// Blocks count themselves on FIN_DONE_LINES counters (block b on b % FIN_DONE_LINES),
// the block completing a counter on one more: ONE device-scope atomic per block on
// a shared address serialises (3.7 K blocks on C2: finalize 0.067 against 0.040 ms).
constexpr int FIN_DONE_LINES = 64;

}  // namespace mm
