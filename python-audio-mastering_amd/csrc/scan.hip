// scan.hip — exclusive scan of affine IIR state maps across tiles.
//
// For a line of tiles (one chunk x channel for the per-chunk filters, or the whole
// track for K-weighting) with per-tile zero-state end states z_m, the state at
// the start of tile m is  s_m = sum_{i<m} Phi^(m-1-i) z_i  (+ Phi^m init),
// Phi = A^T the zero-input transition over one tile.  One 1024-thread workgroup
// per line: each thread folds c consecutive tiles serially (z streamed with the
// register pipeline), a Kogge-Stone scan over the 1024 block aggregates uses the
// precomputed powers Phi^(c*2^k) held in LDS, and a final serial pass writes
// every tile's carry-in state.
#include "common.h"

namespace mm {

constexpr int SCAN_THREADS = 1024;
constexpr int SCAN_MATS = 2 + 12;  // phi, phi_pow[12], phi_last  (MM_SCAN_POWERS == 12)

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

template <int DIM>
struct Vec {
    double v[DIM];
};

template <int DIM>
__global__ void __launch_bounds__(SCAN_THREADS) scan_kernel(ScanArgs a) {
    __shared__ double buf[SCAN_THREADS * DIM];
    __shared__ double mats[SCAN_MATS * 64];
    const int line = blockIdx.x;
    const int chunk = line / a.ch, chn = line - chunk * a.ch;
    const int64_t t0 = (int64_t)chunk * a.line_tiles;
    const int64_t n = min(a.line_tiles, a.G - t0);
    const int tid = threadIdx.x;
    for (int i = tid; i < SCAN_MATS * 64; i += SCAN_THREADS) {
        mats[i] = i < 64 ? a.phi[i] : (i < 13 * 64 ? a.phi_pow[i - 64] : a.phi_last[i - 13 * 64]);
    }
    __syncthreads();
    const double *phi = mats;
    const double *phi_pow = mats + 64;
    const double *phi_last = mats + 13 * 64;
    const int64_t b0 = (int64_t)tid * a.c;
    const int64_t b1 = min(b0 + a.c, n);
    const int cnt = (int)max((int64_t)0, b1 - b0);
    auto zp = [&](int64_t m) { return a.z + ((t0 + m) * a.ch + chn) * a.dim; };

    double acc[DIM], tmp[DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) acc[d] = 0.0;
    {
        int64_t lm = b0;
        stream<2, 2, Vec<DIM>>(
            cnt,
            [&]() {
                Vec<DIM> z;
                const double *p = zp(lm++);
#pragma unroll
                for (int d = 0; d < DIM; ++d) z.v[d] = p[d];
                return z;
            },
            [&](const Vec<DIM> &z) {
                matvec<DIM>(phi, acc, tmp);
#pragma unroll
                for (int d = 0; d < DIM; ++d) acc[d] = tmp[d] + z.v[d];
            });
    }
#pragma unroll
    for (int d = 0; d < DIM; ++d) buf[tid * DIM + d] = acc[d];
    __syncthreads();
    // inclusive Kogge-Stone over block aggregates
    for (int k = 0, dist = 1; dist < SCAN_THREADS; ++k, dist <<= 1) {
        double other[DIM];
        const bool has = tid >= dist;
        if (has) {
#pragma unroll
            for (int d = 0; d < DIM; ++d) other[d] = buf[(tid - dist) * DIM + d];
        }
        __syncthreads();
        if (has) {
            matvec<DIM>(phi_pow + k * 64, other, tmp);
#pragma unroll
            for (int d = 0; d < DIM; ++d) acc[d] += tmp[d];
#pragma unroll
            for (int d = 0; d < DIM; ++d) buf[tid * DIM + d] = acc[d];
        }
        __syncthreads();
    }
    // exclusive prefix of this thread's block
    double s[DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) s[d] = tid > 0 ? buf[(tid - 1) * DIM + d] : 0.0;
    if (a.init) {
        // + Phi^(c*tid) init, via the binary powers of Phi^c
        double v[DIM];
        const double *ini = a.init + ((int64_t)line) * a.dim;
#pragma unroll
        for (int d = 0; d < DIM; ++d) v[d] = ini[d];
        for (int k = 0; (tid >> k) != 0; ++k) {
            if ((tid >> k) & 1) {
                matvec<DIM>(phi_pow + k * 64, v, tmp);
#pragma unroll
                for (int d = 0; d < DIM; ++d) v[d] = tmp[d];
            }
        }
#pragma unroll
        for (int d = 0; d < DIM; ++d) s[d] += v[d];
    }
    {
        int64_t lm = b0, pm = b0;
        stream<2, 2, Vec<DIM>>(
            cnt,
            [&]() {
                Vec<DIM> z;
                const double *p = zp(lm++);
#pragma unroll
                for (int d = 0; d < DIM; ++d) z.v[d] = p[d];
                return z;
            },
            [&](const Vec<DIM> &z) {
                double *out = a.s + ((t0 + pm) * a.ch + chn) * a.dim;
#pragma unroll
                for (int d = 0; d < DIM; ++d) out[d] = s[d];
                if (pm == n - 1) {
                    if (a.line_end) {
                        matvec<DIM>(phi_last, s, tmp);
                        double *e = a.line_end + (int64_t)line * a.dim;
#pragma unroll
                        for (int d = 0; d < DIM; ++d) e[d] = tmp[d] + z.v[d];
                    }
                } else {
                    matvec<DIM>(phi, s, tmp);
#pragma unroll
                    for (int d = 0; d < DIM; ++d) s[d] = tmp[d] + z.v[d];
                }
                ++pm;
            });
    }
}

template __global__ void scan_kernel<4>(ScanArgs);
template __global__ void scan_kernel<8>(ScanArgs);

}  // namespace mm
