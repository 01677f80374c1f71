// Microbenchmark: throughput of the per-lane f64 DF2T cascade (the EQ/crossover
// recurrence) as a function of waves in flight.  Input synthesized in registers,
// output reduced to one store per lane, so only the recurrence is timed.
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ double df2t(double x, double &z0, double &z1, const double *c) {
    double y = fma(c[0], x, z0);
    double t0 = fma(c[1], x, z1);
    double t1 = c[2] * x;
    z0 = fma(-c[3], y, t0);
    z1 = fma(-c[4], y, t1);
    return y;
}
struct Sos { double c[4][5]; };
template <int NS, int SAT, int CHAINS>
__global__ void __launch_bounds__(256) casc(Sos s, int F, double *out) {
    const int lane = blockIdx.x * blockDim.x + threadIdx.x;
    double z[CHAINS][NS][2] = {};
    double acc = 0;
    float x0 = (float)(lane & 255) * 1e-3f;
    for (int i = 0; i < F; ++i) {
#pragma unroll
        for (int ch = 0; ch < CHAINS; ++ch) {
            float xf = x0 + (float)(i + ch) * 1e-4f;
            if (SAT) xf = 0.7f * xf + 0.3f * tanhf(xf * 2.2f);
            double y = (double)xf;
#pragma unroll
            for (int k = 0; k < NS; ++k) y = df2t(y, z[ch][k][0], z[ch][k][1], s.c[k]);
            acc += y > 0.5 ? 1.0 : 0.0;
        }
    }
    out[lane] = acc;
}
// the cascade skewed by one frame per section: section k runs frame i-k, so the
// NS section updates of an iteration are independent (ILP) instead of a chain
template <int NS, int SAT, int CHAINS>
__global__ void __launch_bounds__(256) casc_skew(Sos s, int F, double *out) {
    const int lane = blockIdx.x * blockDim.x + threadIdx.x;
    double z[NS][2] = {};
    double p[NS] = {};
    double acc = 0;
    float x0 = (float)(lane & 255) * 1e-3f;
    for (int i = 0; i < F; ++i) {
        float xf = x0 + (float)i * 1e-4f;
        if (SAT) xf = 0.7f * xf + 0.3f * tanhf(xf * 2.2f);
        p[0] = (double)xf;
        double q[NS];
#pragma unroll
        for (int k = 0; k < NS; ++k) q[k] = df2t(p[k], z[k][0], z[k][1], s.c[k]);
        acc += q[NS - 1] > 0.5 ? 1.0 : 0.0;
#pragma unroll
        for (int k = 1; k < NS; ++k) p[k] = q[k - 1];
    }
    out[lane] = acc;
}
template <int NS, int SAT, int CHAINS, bool SKEW = false>
void run(const char *name, Sos s, double *d) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int F = 1000;
    for (int wps : {1, 2, 4, 8}) {  // waves per SIMD (256 CUs x 4 SIMDs)
        const int lanes = 256 * 4 * 64 * wps / CHAINS;
        auto k = SKEW ? casc_skew<NS, SAT, CHAINS> : casc<NS, SAT, CHAINS>;
        k<<<lanes / 256, 256>>>(s, F, d);
        hipEventRecord(a);
        k<<<lanes / 256, 256>>>(s, F, d);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        const double lane_frames = (double)lanes * CHAINS * F;
        printf("%-22s waves/SIMD %d: %.3f ms, %.2f G lane-frames/s, %.1f SIMD-cycles per wave-frame @2.4GHz\n",
               name, wps, ms, lane_frames / ms / 1e6, ms * 1e-3 * 2.4e9 / (F * (double)wps * CHAINS));
    }
}
int main() {
    Sos s;
    for (int k = 0; k < 4; ++k) { s.c[k][0] = 0.2; s.c[k][1] = 0.3; s.c[k][2] = 0.1; s.c[k][3] = -0.9; s.c[k][4] = 0.3; }
    double *d; hipMalloc(&d, 256 * 4 * 64 * 8 * 8);
    run<4, 0, 1>("4 sections", s, d);
    run<4, 1, 1>("4 sections + tanhf", s, d);
    run<4, 0, 2>("4 sections x2 chains", s, d);
    run<2, 0, 1>("2 sections", s, d);
    run<4, 0, 1, true>("4 sections skewed", s, d);
    run<4, 1, 1, true>("4 sections skewed+tanhf", s, d);
    return 0;
}
