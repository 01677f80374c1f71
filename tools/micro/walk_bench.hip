// Microbenchmark: per-step latency of the compressor envelope walk for ONE lane
// (the Jacobi fix-up critical path), with M read (a) from LDS, (b) from global
// memory at a large stride (super-tile-major layout), (c) contiguous.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#pragma clang fp contract(off)

__device__ __forceinline__ double div_cr(double m, double d, double rd) {
    double q = m * rd; double rem = fma(-q, d, m); return fma(rem, rd, q);
}
__device__ __forceinline__ double step(double att, double M, double A, double rA, double R, double rR) {
    double inc = div_cr(M, A, rA), dec = div_cr(M, R, rR);
    double up = fmin(att + inc, M), dn = fmax(att - dec, 0.0);
    return att <= M ? up : dn;
}
__global__ void walk_strided(const double* Mc, long stride, int n, double* out, long long* cyc) {
    if (threadIdx.x != 0) return;
    double att = 0.0; const double A = 441.0, rA = 1.0/441.0, R = 8820.0, rR = 1.0/8820.0;
    long long t0 = clock64();
    double buf[32];
    for (int k = 0; k < 32; ++k) buf[k] = Mc[(long)k * stride];
    for (int i = 0; i < n; i += 32) {
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            att = step(att, buf[k], A, rA, R, rR);
            int nx = i + 32 + k; nx = nx < n ? nx : n - 1;
            buf[k] = Mc[(long)nx * stride];
        }
    }
    long long t1 = clock64();
    out[0] = att; cyc[0] = t1 - t0;
}
__global__ void walk_regs(const double* Mc, int n, double* out, long long* cyc) {
    if (threadIdx.x != 0) return;
    double att = 0.0; const double A = 441.0, rA = 1.0/441.0, R = 8820.0, rR = 1.0/8820.0;
    double m0 = Mc[0], m1 = Mc[1];
    long long t0 = clock64();
    for (int i = 0; i < n; ++i) { att = step(att, (i & 1) ? m1 : m0, A, rA, R, rR); }
    long long t1 = clock64();
    out[0] = att; cyc[0] = t1 - t0;
}
int main() {
    const int n = 100000; const long stride_big = 13230;
    std::vector<double> h((size_t)n * stride_big / 64 + n * 2);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 5.0 + (i % 97) * 0.05;
    double *d; hipMalloc(&d, h.size() * 8); hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    double *o; long long *c; hipMalloc(&o, 8); hipMalloc(&c, 8);
    long long cy; hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1); float ms;
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0); hipLaunchKernelGGL(walk_regs, 1, 64, 0, 0, d, n, o, c); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1); hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
        printf("regs:       %.1f cycles/step  %.1f ns/step\n", (double)cy / n, ms * 1e6 / n);
        long strides[3] = {1, 1000 / 8 * 0 + 16, stride_big / 64};
        const char* names[3] = {"contiguous", "stride 128B", "stride ~1.6KB"};
        for (int s = 0; s < 3; ++s) {
            int nn = (int)std::min<long>(n, (long)(h.size() - 64) / strides[s]);
            hipEventRecord(e0); hipLaunchKernelGGL(walk_strided, 1, 64, 0, 0, d, strides[s], nn, o, c); hipEventRecord(e1); hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1); hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
            printf("%-12s %.1f cycles/step  %.1f ns/step (n=%d)\n", names[s], (double)cy / nn, ms * 1e6 / nn, nn);
        }
    }
    return 0;
}
