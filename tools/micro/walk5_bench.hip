// Microbenchmark: the envelope walk split over two waves of one workgroup.  Wave 1
// (producer) loads a block of WB frames of M for the 64 walkers and computes the two
// correctly rounded divisions per frame into LDS; wave 0 (consumer) walks the block
// from LDS (M, inc, dec) with only the step's own VALU.  Double-buffered blocks, one
// workgroup barrier per block.  Against the one-wave walk (divisions inline).  All
// 64 lanes walk (pass 0's geometry), M coalesced across lanes.  ns per frame.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#pragma clang fp contract(off)

constexpr int WB = 25, WP = 5;
__device__ __forceinline__ double div_cr(double m, double d, double rd) {
    double q = m * rd; double rem = fma(-q, d, m); return fma(rem, rd, q);
}
__device__ __forceinline__ double vmin(double x, double y) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
__device__ __forceinline__ double lean(double att, double m, double inc, double dec) {
    const double up = vmin(att + inc, m);
    const double dn = att - dec;
    return att <= m ? up : dn;
}
struct K { double A, rA, R, rR; };

// one wave: divisions WP frames ahead (the product's Walker)
__global__ void __launch_bounds__(64) walk1(const double *M, int nblk, int S, double *out, long long *t, K k) {
    const int lane = threadIdx.x;
    const double *p = M + (size_t)blockIdx.x * 64 + lane;
    double att = 0.0, mb[2][WB], inc[WP], dec[WP];
    long long w0 = wall_clock64();
#pragma unroll
    for (int j = 0; j < WB; ++j) mb[0][j] = p[(size_t)j * S];
#pragma unroll
    for (int j = 0; j < WB; ++j) mb[1][j] = p[(size_t)(WB + j) * S];
#pragma unroll
    for (int q = 0; q < WP; ++q) {
        inc[q] = div_cr(mb[0][q], k.A, k.rA);
        dec[q] = div_cr(mb[0][q], k.R, k.rR);
    }
    for (int b = 0; b < nblk; b += 2) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
            for (int j = 0; j < WB; ++j) {
                const double m = mb[kk][j];
                const double ma = j + WP < WB ? mb[kk][j + WP] : mb[kk ^ 1][j + WP - WB];
                const double ik = inc[j % WP], dk = dec[j % WP];
                inc[j % WP] = div_cr(ma, k.A, k.rA);
                dec[j % WP] = div_cr(ma, k.R, k.rR);
                att = lean(att, m, ik, dk);
            }
            __builtin_amdgcn_sched_barrier(0);
            const int nb = min(b + kk + 2, nblk - 1);
#pragma unroll
            for (int j = 0; j < WB; ++j) mb[kk][j] = p[(size_t)(nb * WB + j) * S];
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    long long w1 = wall_clock64();
    out[blockIdx.x * 64 + lane] = att;
    if (lane == 0) t[blockIdx.x] = w1 - w0;
}

// two waves: wave 1 produces {M, inc, dec} blocks into LDS, wave 0 walks them
__global__ void __launch_bounds__(128) walk2(const double *M, int nblk, int S, double *out, long long *t, K k) {
    __shared__ double L[2][3][WB][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double *p = M + (size_t)blockIdx.x * 64 + lane;
    long long w0 = wall_clock64();
    if (w == 1) {
        double mb[WB];
        auto produce = [&](int b, int s) __attribute__((always_inline)) {
#pragma unroll
            for (int j = 0; j < WB; ++j) {
                L[s][0][j][lane] = mb[j];
                L[s][1][j][lane] = div_cr(mb[j], k.A, k.rA);
                L[s][2][j][lane] = div_cr(mb[j], k.R, k.rR);
            }
            const int nb = min(b + 1, nblk - 1);
#pragma unroll
            for (int j = 0; j < WB; ++j) mb[j] = p[(size_t)(nb * WB + j) * S];
        };
#pragma unroll
        for (int j = 0; j < WB; ++j) mb[j] = p[(size_t)j * S];
        produce(0, 0);
        __syncthreads();
        for (int b = 1; b <= nblk; ++b) {  // block b while the consumer walks block b-1
            if (b < nblk) produce(b, b & 1);
            __syncthreads();
        }
    } else {
        double att = 0.0;
        __syncthreads();
        for (int b = 0; b < nblk; ++b) {
            const int s = b & 1;
#pragma unroll
            for (int j = 0; j < WB; ++j) att = lean(att, L[s][0][j][lane], L[s][1][j][lane], L[s][2][j][lane]);
            __syncthreads();
        }
        out[blockIdx.x * 64 + lane] = att;
    }
    long long w1 = wall_clock64();
    if (threadIdx.x == 0) t[blockIdx.x] = w1 - w0;
}

int main() {
    const int nwg = 256, S = nwg * 64, nblk = 36;  // 900 frames per walker
    const size_t n = (size_t)S * (nblk + 2) * WB;
    std::vector<double> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (i % 7 == 0) ? 0.0 : 5.0 + (i % 97) * 0.05;
    double *M, *o1, *o2;
    long long *t;
    hipMalloc(&M, n * 8);
    hipMalloc(&o1, S * 8);
    hipMalloc(&o2, S * 8);
    hipMalloc(&t, nwg * 8);
    hipMemcpy(M, h.data(), n * 8, hipMemcpyHostToDevice);
    K k{441.0, 1.0 / 441.0, 8820.0, 1.0 / 8820.0};
    std::vector<long long> ht(nwg);
    for (int wg : {1, 256}) {
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(walk1, wg, 64, 0, 0, (const double *)M, nblk, S, o1, t, k);
            hipDeviceSynchronize();
            hipMemcpy(ht.data(), t, wg * 8, hipMemcpyDeviceToHost);
            long long mx = 0;
            for (int i = 0; i < wg; ++i) mx = ht[i] > mx ? ht[i] : mx;
            printf("one wave    wgs %3d rep %d: %.1f ns per frame\n", wg, rep, mx * 10.0 / (nblk * WB));
            hipLaunchKernelGGL(walk2, wg, 128, 0, 0, (const double *)M, nblk, S, o2, t, k);
            hipDeviceSynchronize();
            hipMemcpy(ht.data(), t, wg * 8, hipMemcpyDeviceToHost);
            mx = 0;
            for (int i = 0; i < wg; ++i) mx = ht[i] > mx ? ht[i] : mx;
            printf("two waves   wgs %3d rep %d: %.1f ns per frame\n", wg, rep, mx * 10.0 / (nblk * WB));
        }
        std::vector<double> a(S), b(S);
        hipMemcpy(a.data(), o1, wg * 64 * 8, hipMemcpyDeviceToHost);
        hipMemcpy(b.data(), o2, wg * 64 * 8, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < wg * 64; ++i) bad += a[i] != b[i];
        printf("wgs %d: results differ in %d lanes\n", wg, bad);
    }
    return 0;
}
