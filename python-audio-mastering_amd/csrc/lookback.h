// lookback.h — single-pass carry of a linear recurrence across tiles (CDNA4).
//
// Every lane owns one tile of T frames of one channel line.  A tile maps its
// start state s to Phi_T s + z (z = its zero-state end state from pass 1).  The
// carry-in of every tile is the exclusive scan of these affine maps along the
// line, reset to a known state at line starts (chunk starts for the per-chunk
// filters, the track start for K-weighting).  This header computes it inside the
// pass kernel, so a filter stage is ONE launch:
//
//   1. block-local Kogge-Stone scan in LDS over the block's TPB tiles
//      (Phi_T^(2^k) from a host table);
//   2. the block publishes its aggregate (state at its end from a zero carry-in;
//      already exact when the block contains a line start) with write-through
//      (sc1) stores, then a status word (1 = aggregate, 2 = inclusive);
//   3. decoupled look-back by one wave: lane i reads predecessor block b-1-i,
//      terms Phi_B^i x_i are summed across the wave until the first predecessor
//      with an inclusive prefix (or a line start); windows of 64 blocks;
//   4. the block publishes its own inclusive prefix; every lane adds
//      Phi_T^t C_b to its local prefix when no line start lies before it.
//
// Logical block order comes from an atomic ticket, so a block only ever waits
// on blocks that started before it (no dispatch-order assumption).  Handed-off
// words are stored with agent-scope relaxed atomics (sc1, write-through), every
// storing wave drains them (vmcnt(0)) before the workgroup barrier behind which
// one lane stores the status word; the consumer wave polls relaxed, then takes
// ONE agent-scope acquire before loading the payload (cdna_hip_programming.md
// Guideline 16: producer R1, consumer poll -> acquire -> loads).  Status words
// are zeroed by a hipMemsetAsync before every launch.  Spins are bounded: on
// timeout the kernel records an error word and proceeds (the host reports it).
#pragma once
#include "common.h"

namespace mm {

constexpr int LB_THREADS = 256;
constexpr int LB_WIN = 64;      // predecessors per look-back window (one wave)
constexpr int LB_TILE_POW = 8;  // Phi_T^(2^k), k < 8  (TPB <= 256)
constexpr int LB_SPIN_LIMIT = 1 << 22;

struct LbArgs {
    const double *pw_tile;  // [LB_TILE_POW][64]  Phi_T^(2^k), row-major 8x8
    const double *pw_blk;   // [LB_WIN + 1][64]   Phi_B^e, e = 0..64 (Phi_B = Phi_T^TPB)
    double *agg;            // [nblk][CH][8]
    double *incl;           // [nblk][CH][8]
    unsigned *status;       // [nblk]   zeroed before every launch
    unsigned *ticket;       // [1]      zeroed before every launch
    unsigned *error;        // [1]      set to 1 on a spin timeout
    const double *init;     // [CH][8]  state at the track start (or null = 0)
    int64_t line_tiles;     // line starts at tiles g % line_tiles == 0
};

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ void st_sc1(double *p, double v) {
    __hip_atomic_store((gu64 *)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p) {
    return __longlong_as_double(
        (long long)__hip_atomic_load((gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_flag(unsigned *p, unsigned v) {
    __hip_atomic_store((gu32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ld_flag(const unsigned *p) {
    return __hip_atomic_load((gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sparsity of the state maps.  State component d belongs to DF2T section d/2;
// sections [0, NB0) form one cascade (branch 0), the rest a second cascade fed
// by the same input (branch 1).  A section's zero-input update reads only the
// states of its own branch up to itself, so the one-frame matrix A is block
// lower-triangular within a block-diagonal, and so is every power and product
// of powers: M[r][k] is exactly 0 unless lb_nz(r, k).  The matrix-vector
// products below skip those entries at compile time (EQ: 40 of 64 FMAs,
// crossover: 24 of 64).
template <int NB0>
__device__ __forceinline__ constexpr bool lb_nz(int r, int k) {
    return ((r / 2 < NB0) == (k / 2 < NB0)) && (k / 2 <= r / 2);
}

// o = M v  (M row-major with stride 8)
template <int DIM, int NB0 = DIM / 2>
__device__ __forceinline__ void mv(const double *M, const double (&v)[DIM], double (&o)[DIM]) {
#pragma unroll
    for (int r = 0; r < DIM; ++r) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < DIM; ++k)
            if (lb_nz<NB0>(r, k)) acc = fma(M[r * 8 + k], v[k], acc);
        o[r] = acc;
    }
}

// Logical block index in start order.
__device__ __forceinline__ int lb_ticket(const LbArgs &a, int *lds_slot) {
    if (threadIdx.x == 0) *lds_slot = (int)atomicAdd(a.ticket, 1u);
    __syncthreads();
    return *lds_slot;
}

// LDS scratch the carry needs (bytes), for CH lines of TPB tiles.
template <int DIM, int CH>
constexpr int lb_lds_bytes() {
    return (LB_THREADS * 8 + LB_TILE_POW * 64 + 2 * CH * 8 + 64) * (int)sizeof(double) + LB_THREADS * 4 + 16;
}

// Carry-in state s of this lane's tile.  z: the tile's zero-state end state;
// `reset`: the tile starts a line; `rst` : state at a line start (zero, or the
// track-start init for g == 0).  Must be called by every thread of the block.
// NB0: sections in the first cascade (lb_nz); DIM / 2 = one cascade.
template <int DIM, int CH, int NB0 = DIM / 2>
__device__ void lb_carry(const LbArgs &a, int blk, int t, int c, bool valid, bool reset, const double (&rst)[DIM],
                         const double (&z)[DIM], double (&s)[DIM], double *lds) {
    constexpr int TPB = LB_THREADS / CH;
    double *buf = lds;                            // [CH][TPB][8]
    double *pw = buf + LB_THREADS * 8;            // [LB_TILE_POW][64]
    double *cb = pw + LB_TILE_POW * 64;           // [CH][8] block carry
    double *aux = cb + 2 * CH * 8;                // [64] matrix scratch
    int *flg = reinterpret_cast<int *>(aux + 64); // [CH][TPB]
    const int tid = threadIdx.x;
    for (int i = tid; i < LB_TILE_POW * 64; i += LB_THREADS) pw[i] = a.pw_tile[i];

    // element of this tile: (reset, state at its end)
    double v[DIM], tmp[DIM];
    int f = reset ? 1 : 0;
    if (reset) {
        mv<DIM, NB0>(a.pw_tile, rst, tmp);  // Phi_T rst  (pw_tile[0] = Phi_T)
#pragma unroll
        for (int d = 0; d < DIM; ++d) v[d] = tmp[d] + z[d];
    } else {
#pragma unroll
        for (int d = 0; d < DIM; ++d) v[d] = z[d];
    }
    if (!valid) {
        f = 0;
#pragma unroll
        for (int d = 0; d < DIM; ++d) v[d] = 0.0;
    }
    double *mine = buf + (c * TPB + t) * 8;
#pragma unroll
    for (int d = 0; d < DIM; ++d) mine[d] = v[d];
    flg[c * TPB + t] = f;
    __syncthreads();
    // 1. block-local inclusive scan
#pragma unroll
    for (int k = 0; (1 << k) < TPB; ++k) {
        const int dist = 1 << k;
        double o[DIM];
        int of = 1;
        const bool has = t >= dist;
        if (has) {
            const double *src = buf + (c * TPB + t - dist) * 8;
#pragma unroll
            for (int d = 0; d < DIM; ++d) o[d] = src[d];
            of = flg[c * TPB + t - dist];
        }
        __syncthreads();
        if (has && !f) {
            mv<DIM, NB0>(pw + k * 64, o, tmp);
#pragma unroll
            for (int d = 0; d < DIM; ++d) v[d] += tmp[d];
            f = of;
        }
#pragma unroll
        for (int d = 0; d < DIM; ++d) mine[d] = v[d];
        flg[c * TPB + t] = f;
        __syncthreads();
    }
    // local exclusive prefix of this tile
    double sp[DIM];
    int fp = 0;
    if (t > 0) {
        const double *src = buf + (c * TPB + t - 1) * 8;
#pragma unroll
        for (int d = 0; d < DIM; ++d) sp[d] = src[d];
        fp = flg[c * TPB + t - 1];
    } else {
#pragma unroll
        for (int d = 0; d < DIM; ++d) sp[d] = 0.0;
    }
    const bool blk_reset = flg[0 * TPB + TPB - 1] != 0;  // same line structure for every channel
#ifndef MM_ABL_NOLOOK  // (ablation builds: timing only)
    const bool need_carry = !flg[0 * TPB + 0];           // tile 0 of the block is not a line start
#else
    const bool need_carry = false;
#endif
    // 2. publish the aggregate
    if (t == TPB - 1) {
        double *ag = a.agg + ((int64_t)blk * CH + c) * 8;
#pragma unroll
        for (int d = 0; d < DIM; ++d) {
            st_sc1(ag + d, v[d]);
            if (blk_reset) st_sc1(a.incl + ((int64_t)blk * CH + c) * 8 + d, v[d]);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) st_flag(a.status + blk, blk_reset ? 2u : 1u);
    // 3. look-back (wave 0); the block carry accumulates in LDS (cb)
    if (need_carry && tid < 64) {
        const int lane = tid;
        if (lane < CH * 8) cb[lane] = 0.0;
        // Pw = Phi_B^(64 w), kept in LDS (aux) as 8x8; identity for w = 0
        aux[lane] = (lane / 8 == lane % 8) ? 1.0 : 0.0;
        __builtin_amdgcn_wave_barrier();
        bool done = false;
        for (int w = 0; !done; ++w) {
            const int64_t j = (int64_t)blk - 1 - lane - (int64_t)w * LB_WIN;
            unsigned st = j >= 0 ? ld_flag(a.status + j) : 2u;
            // Wait only for the predecessors up to the nearest one with an inclusive
            // prefix (lanes 0 .. first): the ones past it do not contribute.  (Round 5
            // waited for all 64 flags of the window, so a block also waited for the
            // slowest of up to 64 predecessors, the previous chunk's included: eq's
            // look-back cost 26 us of its 158 on C2)
            for (int spins = 0;; ++spins) {
                const unsigned long long inc = __ballot(st == 2u), zero = __ballot(st == 0u);
                const int first = inc ? __builtin_ctzll(inc) : LB_WIN - 1;
                const unsigned long long need = first >= 63 ? ~0ull : (2ull << first) - 1ull;
                if (!(zero & need)) break;
                if (spins > LB_SPIN_LIMIT) {
                    if (st == 0u) {
                        st_flag(a.error, 1u);
                        st = 2u;
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
                if (st == 0u) st = ld_flag(a.status + j);
            }
            // agent-scope acquire after the polls (cdna_hip_programming.md Guideline 16:
            // ONE relaxed poll, ONE agent acquire, then the loads): this CU's L1 holds
            // no stale copy of a predecessor's aggregate or prefix, whatever the
            // placement.  The payload loads below stay sc1 (L2-served) as well.
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned long long m = __ballot(st == 2u);
            const int first = m ? __builtin_ctzll(m) : LB_WIN;  // lanes <= first contribute
#pragma unroll 1
            for (int q = 0; q < CH; ++q) {
                double x[DIM], term[DIM];
                if (lane <= first && j >= 0) {
                    const double *src = (lane == first ? a.incl : a.agg) + (j * CH + q) * 8;
#pragma unroll
                    for (int d = 0; d < DIM; ++d) x[d] = ld_sc1(src + d);
                } else {  // past the first inclusive predecessor, or the track start
#pragma unroll
                    for (int d = 0; d < DIM; ++d)
                        x[d] = (lane == first && a.init) ? a.init[q * 8 + d] : 0.0;
                }
                mv<DIM, NB0>(a.pw_blk + lane * 64, x, term);
#pragma unroll
                for (int d = 0; d < DIM; ++d) {  // wave sum
                    double r = term[d];
#pragma unroll
                    for (int off = 32; off >= 1; off >>= 1) r += __shfl_xor(r, off);
                    term[d] = r;
                }
                if (lane < DIM) {  // cb[q] += Pw * window sum, one row per lane
                    double acc = 0.0;
#pragma unroll
                    for (int k = 0; k < DIM; ++k) acc = fma(aux[lane * 8 + k], term[k], acc);
                    cb[q * 8 + lane] += acc;
                }
                __builtin_amdgcn_wave_barrier();
            }
            done = first < LB_WIN;
            if (!done) {  // Pw <- Pw * Phi_B^64, one element per lane
                const double *P64 = a.pw_blk + LB_WIN * 64;
                const int r = lane / 8, col = lane % 8;
                double acc = 0.0;
                for (int k = 0; k < 8; ++k) acc = fma(aux[r * 8 + k], P64[k * 8 + col], acc);
                __builtin_amdgcn_wave_barrier();
                aux[lane] = acc;
                __builtin_amdgcn_wave_barrier();
            }
        }
        // inclusive prefix of this block = Phi_B C_b + aggregate
        if (!blk_reset && lane < CH * DIM) {
            const int q = lane / DIM, r = lane % DIM;
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < DIM; ++k) acc = fma(a.pw_blk[64 + r * 8 + k], cb[q * 8 + k], acc);
            acc += buf[(q * TPB + TPB - 1) * 8 + r];
            st_sc1(a.incl + ((int64_t)blk * CH + q) * 8 + r, acc);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (!blk_reset && lane == 0) st_flag(a.status + blk, 2u);
    }
    __syncthreads();
    // 4. carry-in of this tile
    if (reset) {
#pragma unroll
        for (int d = 0; d < DIM; ++d) s[d] = rst[d];
    } else if (fp || !need_carry) {
#pragma unroll
        for (int d = 0; d < DIM; ++d) s[d] = sp[d];
    } else {
        double cv[DIM];
#pragma unroll
        for (int d = 0; d < DIM; ++d) cv[d] = cb[c * 8 + d];
#pragma unroll
        for (int k = 0; k < LB_TILE_POW; ++k) {
            if ((t >> k) & 1) {
                mv<DIM, NB0>(pw + k * 64, cv, tmp);
#pragma unroll
                for (int d = 0; d < DIM; ++d) cv[d] = tmp[d];
            }
        }
#pragma unroll
        for (int d = 0; d < DIM; ++d) s[d] = sp[d] + cv[d];
    }
}

}  // namespace mm
