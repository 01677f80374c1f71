// Microbenchmark: cycles per envelope step for one lane, by formulation.
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang fp contract(off)
__device__ __forceinline__ double div_cr(double m, double d, double rd) {
    double q = m * rd; double rem = fma(-q, d, m); return fma(rem, rd, q);
}
template <int V>
__device__ __forceinline__ double step(double att, double M, double inc, double dec) {
    if (V == 0) {  // min/max
        double up = fmin(att + inc, M), dn = fmax(att - dec, 0.0);
        return att <= M ? up : dn;
    } else if (V == 1) {  // selects, no clamp at 0 (provably inactive)
        double t = att + inc, d = att - dec;
        double up = (M < t) ? M : t;
        return att <= M ? up : d;
    } else if (V == 2) {  // min without canonicalize via integer compare of non-negative doubles
        double t = att + inc, d = att - dec;
        double up = fmin(t, M);
        return att <= M ? up : d;
    } else {  // the product's lean_step: v_min_f64 without canonicalisation + select
        double t = att + inc, d = att - dec, up;
        asm("v_min_f64 %0, %1, %2" : "=v"(up) : "v"(t), "v"(M));
        return att <= M ? up : d;
    }
}
template <int V, int CHAINS>
__global__ void bench(const double* in, int n, double* out, long long* cyc, int act) {
    if ((int)threadIdx.x >= act) return;
    double att[CHAINS];
    for (int c = 0; c < CHAINS; ++c) att[c] = 0.1 * c;
    double M[4], inc[4], dec[4];
    for (int k = 0; k < 4; ++k) { M[k] = in[k] + 1e-3 * threadIdx.x; inc[k] = div_cr(M[k], 441.0, 1.0/441.0); dec[k] = div_cr(M[k], 8820.0, 1.0/8820.0); }
    long long t0 = clock64(), w0 = wall_clock64();
    for (int i = 0; i < n; i += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) att[c] = step<V>(att[c], M[k], inc[k], dec[k]);
    }
    long long t1 = clock64(), w1 = wall_clock64();
    double s = 0; for (int c = 0; c < CHAINS; ++c) s += att[c];
    out[threadIdx.x] = s; if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = w1 - w0; }
}
template <int CHAINS>
__global__ void bench_div(const double* in, int n, double* out, long long* cyc, int act) {
    if ((int)threadIdx.x >= act) return;
    double att[CHAINS];
    for (int c = 0; c < CHAINS; ++c) att[c] = 0.1 * c;
    double M[4]; for (int k = 0; k < 4; ++k) M[k] = in[k] + 1e-3 * threadIdx.x;
    long long t0 = clock64();
    for (int i = 0; i < n; i += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            double inc = div_cr(M[k], 441.0, 1.0/441.0), dec = div_cr(M[k], 8820.0, 1.0/8820.0);
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) att[c] = step<0>(att[c], M[k], inc, dec);
        }
    }
    long long t1 = clock64();
    double s = 0; for (int c = 0; c < CHAINS; ++c) s += att[c];
    out[threadIdx.x] = s; if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
template <class K>
void run(const char* name, K k, const double* d, double* o, long long* c, int n, int chains) {
    for (int act : {1, 64}) {
        long long cy[2] = {0, 0};
        hipMemset(c, 0, 16);
        hipLaunchKernelGGL(k, 1, 64, 0, 0, d, n, o, c, act); hipDeviceSynchronize();
        hipLaunchKernelGGL(k, 1, 64, 0, 0, d, n, o, c, act); hipDeviceSynchronize();
        hipMemcpy(cy, c, 16, hipMemcpyDeviceToHost);
        printf("%-28s lanes=%2d chains=%d  %.1f cycles/step/chain  %.2f ns/step/chain (wall)\n", name, act, chains,
               (double)cy[0] / n / chains, cy[1] > 0 ? (double)cy[1] * 10.0 / n / chains : -1.0);
    }
}
int main() {
    double h[4] = {9.5, 9.6, 9.4, 9.55};
    double *d, *o; long long *c;
    hipMalloc(&d, 32); hipMalloc(&o, 64 * 8); hipMalloc(&c, 16);
    hipMemcpy(d, h, 32, hipMemcpyHostToDevice);
    const int n = 200000;
    run("div_cr inline + minmax", bench_div<1>, d, o, c, n, 1);
    run("div_cr inline + minmax", bench_div<2>, d, o, c, n, 2);
    run("precomp minmax", bench<0, 1>, d, o, c, n, 1);
    run("precomp selects", bench<1, 1>, d, o, c, n, 1);
    run("precomp fmin, no clamp0", bench<2, 1>, d, o, c, n, 1);
    run("precomp lean_step (asm)", bench<3, 1>, d, o, c, n, 1);
    run("precomp lean_step (asm)", bench<3, 2>, d, o, c, n, 2);
    run("precomp selects", bench<1, 2>, d, o, c, n, 2);
    run("precomp selects", bench<1, 4>, d, o, c, n, 4);
    return 0;
}
