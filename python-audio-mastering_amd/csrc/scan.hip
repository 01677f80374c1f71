// scan.hip — chip-wide exclusive scan of affine IIR state maps across tiles.
//
// Tile g's zero-input map over its T frames is  s -> Phi s + z_g  (Phi = A^T,
// z_g = zero-state end state from pass 1).  At a line start (chunk boundary for
// the per-chunk filters; the track start for K-weighting) the incoming state is
// reset to 0, so the element becomes the constant z_g.  Elements compose as
//   (f_a, v_a) then (f_b, v_b)  ->  (f_a|f_b,  f_b ? v_b : Phi^{n_b} v_a + v_b)
// which is associative, so the carry-in state of every tile is a segmented
// exclusive scan.  Three launches spread it over the whole chip:
//   A scan_local   one 256-thread block per 256 tiles: Kogge-Stone in LDS with
//                  Phi^(2^k); writes the block-local prefix and the block aggregate
//   B scan_blocks  one 1024-thread block per channel over the block aggregates
//                  (serial folds of c blocks + Kogge-Stone with Phi^(256 c 2^k))
//   C scan_apply   per tile: s = s_local + Phi^t C_block when no reset lies
//                  between the block start and the tile (binary powers of Phi)
#include "common.h"

namespace mm {

constexpr int SCAN_BLOCK = 256;   // tiles per block (kernel A)
constexpr int SCAN_THREADS = 1024;  // kernel B
// matrix table layout in ScanArgs.mats (each 8x8 row-major)
constexpr int MAT_PHI = 0, MAT_POW2 = 1, MAT_BLK = 13, MAT_BLKPOW = 14, MAT_LAST = 26, MAT_COUNT = 27;

template <int DIM>
__device__ __forceinline__ void matvec(const double *Mx, const double (&v)[DIM], double (&o)[DIM]) {
#pragma unroll
    for (int r = 0; r < DIM; ++r) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < DIM; ++k) acc = fma(Mx[r * 8 + k], v[k], acc);
        o[r] = acc;
    }
}

// A. grid (nblk, ch), block 256
template <int DIM>
__global__ void __launch_bounds__(SCAN_BLOCK) scan_local_kernel(ScanArgs a) {
    __shared__ double buf[SCAN_BLOCK * DIM];
    __shared__ int flg[SCAN_BLOCK];
    __shared__ double pw[8 * 64];
    const int blk = blockIdx.x, chn = blockIdx.y, t = threadIdx.x;
    for (int i = t; i < 8 * 64; i += SCAN_BLOCK) pw[i] = a.mats[MAT_POW2 * 64 + i];
    const int64_t g = (int64_t)blk * SCAN_BLOCK + t;
    const bool valid = g < a.G;
    double v[DIM], tmp[DIM];
    int f = 1;
    if (valid) {
        const double *z = a.z + (g * a.ch + chn) * a.dim;
#pragma unroll
        for (int d = 0; d < DIM; ++d) v[d] = z[d];
        // line starts reset the state; the track start (g == 0) is kernel B's
        // leading (reset, init) element instead, so it takes the block carry
        f = g > 0 && (g % a.line_tiles) == 0;
    } else {
#pragma unroll
        for (int d = 0; d < DIM; ++d) v[d] = 0.0;
    }
    const int my_reset = f;
#pragma unroll
    for (int d = 0; d < DIM; ++d) buf[t * DIM + d] = v[d];
    flg[t] = f;
    __syncthreads();
    for (int k = 0, dist = 1; dist < SCAN_BLOCK; ++k, dist <<= 1) {
        double o[DIM];
        int of = 1;
        const bool has = t >= dist;
        if (has) {
#pragma unroll
            for (int d = 0; d < DIM; ++d) o[d] = buf[(t - dist) * DIM + d];
            of = flg[t - dist];
        }
        __syncthreads();
        if (has && !f) {
            matvec<DIM>(pw + k * 64, o, tmp);
#pragma unroll
            for (int d = 0; d < DIM; ++d) v[d] += tmp[d];
            f = of;
        }
#pragma unroll
        for (int d = 0; d < DIM; ++d) buf[t * DIM + d] = v[d];
        flg[t] = f;
        __syncthreads();
    }
    if (valid) {
        double *s = a.s + (g * a.ch + chn) * a.dim;
        const bool prev_reset = t > 0 ? flg[t - 1] != 0 : false;
#pragma unroll
        for (int d = 0; d < DIM; ++d) s[d] = (my_reset || t == 0) ? 0.0 : buf[(t - 1) * DIM + d];
        a.need[g * a.ch + chn] = (uint8_t)!(my_reset || prev_reset);
    }
    if (t == SCAN_BLOCK - 1) {
        double *ag = a.agg + ((int64_t)blk * a.ch + chn) * a.dim;
#pragma unroll
        for (int d = 0; d < DIM; ++d) ag[d] = v[d];
        a.agg_f[blk * a.ch + chn] = f;
    }
}

// B. grid (ch), block 1024: carry-in state of every block
template <int DIM>
__global__ void __launch_bounds__(SCAN_THREADS) scan_blocks_kernel(ScanArgs a) {
    __shared__ double buf[SCAN_THREADS * DIM];
    __shared__ int flg[SCAN_THREADS];
    __shared__ double mats[13 * 64];  // blk, blk_pow[12]
    const int chn = blockIdx.x, t = threadIdx.x;
    for (int i = t; i < 13 * 64; i += SCAN_THREADS) mats[i] = a.mats[MAT_BLK * 64 + i];
    __syncthreads();
    const double *blkm = mats;
    const double *bpow = mats + 64;
    const int64_t b0 = (int64_t)t * a.c, b1 = min(b0 + a.c, a.nblk);
    auto agg = [&](int64_t b) { return a.agg + (b * a.ch + chn) * a.dim; };
    double v[DIM], tmp[DIM];
    int f = 0;
#pragma unroll
    for (int d = 0; d < DIM; ++d) v[d] = 0.0;
    if (t == 0) {  // the track start: an element (reset, init)
        f = 1;
        if (a.init) {
#pragma unroll
            for (int d = 0; d < DIM; ++d) v[d] = a.init[(int64_t)chn * a.dim + d];
        }
    }
    for (int64_t b = b0; b < b1; ++b) {
        const double *x = agg(b);
        if (a.agg_f[b * a.ch + chn]) {
#pragma unroll
            for (int d = 0; d < DIM; ++d) v[d] = x[d];
            f = 1;
        } else {
            matvec<DIM>(blkm, v, tmp);
#pragma unroll
            for (int d = 0; d < DIM; ++d) v[d] = tmp[d] + x[d];
        }
    }
#pragma unroll
    for (int d = 0; d < DIM; ++d) buf[t * DIM + d] = v[d];
    flg[t] = f;
    __syncthreads();
    for (int k = 0, dist = 1; dist < SCAN_THREADS; ++k, dist <<= 1) {
        double o[DIM];
        int of = 1;
        const bool has = t >= dist;
        if (has) {
#pragma unroll
            for (int d = 0; d < DIM; ++d) o[d] = buf[(t - dist) * DIM + d];
            of = flg[t - dist];
        }
        __syncthreads();
        if (has && !f) {
            matvec<DIM>(bpow + k * 64, o, tmp);
#pragma unroll
            for (int d = 0; d < DIM; ++d) v[d] += tmp[d];
            f = of;
        }
#pragma unroll
        for (int d = 0; d < DIM; ++d) buf[t * DIM + d] = v[d];
        flg[t] = f;
        __syncthreads();
    }
    // exclusive: state at each block start (the t == 0 fold began with a reset,
    // so every prefix is a constant)
    double e[DIM];
    if (t > 0) {
#pragma unroll
        for (int d = 0; d < DIM; ++d) e[d] = buf[(t - 1) * DIM + d];
    } else {
#pragma unroll
        for (int d = 0; d < DIM; ++d) e[d] = a.init ? a.init[(int64_t)chn * a.dim + d] : 0.0;
    }
    for (int64_t b = b0; b < b1; ++b) {
        double *C = a.carry + (b * a.ch + chn) * a.dim;
#pragma unroll
        for (int d = 0; d < DIM; ++d) C[d] = e[d];
        const double *x = agg(b);
        if (a.agg_f[b * a.ch + chn]) {
#pragma unroll
            for (int d = 0; d < DIM; ++d) e[d] = x[d];
        } else {
            matvec<DIM>(blkm, e, tmp);
#pragma unroll
            for (int d = 0; d < DIM; ++d) e[d] = tmp[d] + x[d];
        }
    }
}

// C. grid (nblk, ch), block 256: add Phi^t C_block where no reset intervenes
template <int DIM>
__global__ void __launch_bounds__(SCAN_BLOCK) scan_apply_kernel(ScanArgs a) {
    __shared__ double pw[8 * 64];
    const int blk = blockIdx.x, chn = blockIdx.y, t = threadIdx.x;
    for (int i = t; i < 8 * 64; i += SCAN_BLOCK) pw[i] = a.mats[MAT_POW2 * 64 + i];
    __syncthreads();
    const int64_t g = (int64_t)blk * SCAN_BLOCK + t;
    if (g >= a.G) return;
    double *s = a.s + (g * a.ch + chn) * a.dim;
    double st[DIM], tmp[DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) st[d] = s[d];
    if (a.need[g * a.ch + chn]) {
        double v[DIM];
        const double *C = a.carry + ((int64_t)blk * a.ch + chn) * a.dim;
#pragma unroll
        for (int d = 0; d < DIM; ++d) v[d] = C[d];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if ((t >> k) & 1) {
                matvec<DIM>(pw + k * 64, v, tmp);
#pragma unroll
                for (int d = 0; d < DIM; ++d) v[d] = tmp[d];
            }
        }
#pragma unroll
        for (int d = 0; d < DIM; ++d) st[d] += v[d];
#pragma unroll
        for (int d = 0; d < DIM; ++d) s[d] = st[d];
    }
    if (a.line_end && g == a.G - 1) {
        const double *z = a.z + (g * a.ch + chn) * a.dim;
        matvec<DIM>(a.mats + MAT_LAST * 64, st, tmp);
#pragma unroll
        for (int d = 0; d < DIM; ++d) a.line_end[(int64_t)chn * a.dim + d] = tmp[d] + z[d];
    }
}

template __global__ void scan_local_kernel<4>(ScanArgs);
template __global__ void scan_local_kernel<8>(ScanArgs);
template __global__ void scan_blocks_kernel<4>(ScanArgs);
template __global__ void scan_blocks_kernel<8>(ScanArgs);
template __global__ void scan_apply_kernel<4>(ScanArgs);
template __global__ void scan_apply_kernel<8>(ScanArgs);

}  // namespace mm
