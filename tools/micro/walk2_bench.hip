// Microbenchmark: cycles per envelope step for a FULL wave of walkers (pass0's
// geometry: one wave per SIMD, every lane walks its own sequence), by step
// formulation.  M streamed from global memory, coalesced across lanes.
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang fp contract(off)
__device__ __forceinline__ double div_cr(double m, double d, double rd) {
    double q = m * rd; double rem = fma(-q, d, m); return fma(rem, rd, q);
}
__device__ __forceinline__ double vmin(double a, double b) {  // v_min_f64 without operand canonicalization
    double r; asm volatile("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r;
}
__device__ __forceinline__ double vmax0(double a) {
    double r; asm volatile("v_max_f64 %0, %1, 0" : "=v"(r) : "v"(a)); return r;
}
struct C { double A, rA, R, rR; };
template <int V, int P>
__global__ void __launch_bounds__(64) walk(const double *M, int n, C c, double *out, long long *cyc) {
    const int lane = threadIdx.x + blockIdx.x * 64;
    const double *p = M + lane;
    const int S = gridDim.x * 64;
    double att = 0.0;
    constexpr int B = 32;
    double buf[B];
#pragma unroll
    for (int k = 0; k < B; ++k) buf[k] = p[(long)k * S];
    double inc[P], dec[P];
#pragma unroll
    for (int k = 0; k < P; ++k) { inc[k] = div_cr(buf[k], c.A, c.rA); dec[k] = div_cr(buf[k], c.R, c.rR); }
    long long t0 = clock64();
    for (int i = 0; i < n; i += B) {
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const double m = buf[k];
            if (V == 0) {  // current: divisions inline, fmin/fmax
                const double a = div_cr(m, c.A, c.rA), d = div_cr(m, c.R, c.rR);
                const double up = fmin(att + a, m), dn = fmax(att - d, 0.0);
                att = att <= m ? up : dn;
            } else if (V == 1) {  // divisions P frames ahead (rotating registers)
                const double a = inc[k % P], d = dec[k % P];
                const double mn = buf[(k + P) % B];
                inc[k % P] = div_cr(mn, c.A, c.rA);
                dec[k % P] = div_cr(mn, c.R, c.rR);
                const double up = fmin(att + a, m), dn = fmax(att - d, 0.0);
                att = att <= m ? up : dn;
            } else if (V == 2) {  // as 1, min/max without canonicalize
                const double a = inc[k % P], d = dec[k % P];
                const double mn = buf[(k + P) % B];
                inc[k % P] = div_cr(mn, c.A, c.rA);
                dec[k % P] = div_cr(mn, c.R, c.rR);
                const double up = vmin(att + a, m), dn = vmax0(att - d);
                att = att <= m ? up : dn;
            } else {  // lean bound: increments "free" (m/A approximated by a multiply)
                const double up = fmin(att + m * c.rA, m), dn = fmax(att - m * c.rR, 0.0);
                att = att <= m ? up : dn;
            }
            buf[k] = p[(long)(i + B + k < n ? i + B + k : n - 1) * S];
        }
    }
    long long t1 = clock64();
    out[lane] = att;
    if (lane == 0) cyc[0] = t1 - t0;
}
// rms code r (uint16, 2 B/step from HBM) + L2-resident table gathers: G == 1
// gathers M and divides inline; G == 2 gathers {M, M/A, M/R, 0} (32 B rows)
template <int G, int L = 8>
__global__ void __launch_bounds__(64) walk_r(const uint16_t *Rc, const double *lut, const double4 *lut4, int n, C c,
                                             double *out, long long *cyc) {
    const int lane = threadIdx.x + blockIdx.x * 64;
    const uint16_t *p = Rc + lane;
    const int S = gridDim.x * 64;
    double att = 0.0;
    constexpr int B = 32;  // r prefetched B ahead, table rows L ahead
    uint16_t rb[B];
#pragma unroll
    for (int k = 0; k < B; ++k) rb[k] = p[(long)k * S];
    double m[L];
    double4 q[L];
#pragma unroll
    for (int k = 0; k < L; ++k) {
        if (G == 1) m[k] = lut[rb[k]];
        else q[k] = lut4[rb[k]];
    }
    long long t0 = clock64();
    for (int i = 0; i < n; i += B) {
#pragma unroll
        for (int k = 0; k < B; ++k) {
            double mm, a, d;
            if (G == 1) {
                mm = m[k % L];
                a = div_cr(mm, c.A, c.rA);
                d = div_cr(mm, c.R, c.rR);
                m[k % L] = lut[rb[(k + L) % B]];
            } else {
                const double4 v = q[k % L];
                mm = v.x; a = v.y; d = v.z;
                q[k % L] = lut4[rb[(k + L) % B]];
            }
            const double up = vmin(att + a, mm), dn = vmax0(att - d);
            att = att <= mm ? up : dn;
            rb[k] = p[(long)(i + B + k < n ? i + B + k : n - 1) * S];
        }
    }
    long long t1 = clock64();
    out[lane] = att;
    if (lane == 0) cyc[0] = t1 - t0;
}
template <int G, int L = 8>
void run_r(const char *name, const uint16_t *R, const double *lut, const double4 *lut4, int n, double *o, long long *cy, int blocks) {
    C c{441.0, 1.0 / 441.0, 8820.0, 1.0 / 8820.0};
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    walk_r<G, L><<<blocks, 64>>>(R, lut, lut4, n, c, o, cy);
    (void)hipEventRecord(e0);
    walk_r<G, L><<<blocks, 64>>>(R, lut, lut4, n, c, o, cy);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    long long h; (void)hipMemcpy(&h, cy, 8, hipMemcpyDeviceToHost);
    printf("%-34s blocks %4d: %6.1f cycles/step (clock64), %6.2f ns/step (events)\n", name, blocks, (double)h / n, ms * 1e6 / n);
}
template <int V, int P>
void run(const char *name, const double *M, int n, double *o, long long *cy, int blocks) {
    C c{441.0, 1.0 / 441.0, 8820.0, 1.0 / 8820.0};
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    walk<V, P><<<blocks, 64>>>(M, n, c, o, cy);
    (void)hipEventRecord(e0);
    walk<V, P><<<blocks, 64>>>(M, n, c, o, cy);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    long long h; (void)hipMemcpy(&h, cy, 8, hipMemcpyDeviceToHost);
    printf("%-34s blocks %4d: %6.1f cycles/step (clock64), %6.2f ns/step (events)\n", name, blocks, (double)h / n, ms * 1e6 / n);
}
int main() {
    const int n = 4096, maxb = 1024;
    size_t cnt = (size_t)n * maxb * 64 + 64;
    double *M; (void)hipMalloc(&M, cnt * 8);
    double *hM = new double[1 << 20];
    for (int i = 0; i < (1 << 20); ++i) hM[i] = (i % 7) ? 3.0 + (i % 97) * 0.1 : 0.0;
    for (size_t o = 0; o < cnt; o += (1 << 20)) (void)hipMemcpy(M + o, hM, 8 * std::min<size_t>(1 << 20, cnt - o), hipMemcpyHostToDevice);
    double *o; long long *cy; (void)hipMalloc(&o, maxb * 64 * 8); (void)hipMalloc(&cy, 8);
    // rms codes: slowly varying per lane (as a real rms track), spread over the table
    uint16_t *R; (void)hipMalloc(&R, cnt * 2);
    {
        uint16_t *hR = new uint16_t[1 << 20];
        for (int i = 0; i < (1 << 20); ++i) { const int lane = i % 65536 / 64 * 0 + (i & 63), t = i >> 6; hR[i] = (uint16_t)(3000 + (lane * 397 + (t / 50) * 13) % 29000); }
        for (size_t o2 = 0; o2 < cnt; o2 += (1 << 20)) (void)hipMemcpy(R + o2, hR, 2 * std::min<size_t>(1 << 20, cnt - o2), hipMemcpyHostToDevice);
    }
    double *lut; double4 *lut4; (void)hipMalloc(&lut, 32769 * 8); (void)hipMalloc(&lut4, 32769 * 32);
    {
        double *h = new double[32769 * 4];
        for (int r = 0; r < 32769; ++r) { h[r] = r * 1e-3; }
        (void)hipMemcpy(lut, h, 32769 * 8, hipMemcpyHostToDevice);
        for (int r = 0; r < 32769; ++r) { h[4*r] = r * 1e-3; h[4*r+1] = h[4*r] / 441.0; h[4*r+2] = h[4*r] / 8820.0; h[4*r+3] = 0; }
        (void)hipMemcpy(lut4, h, 32769 * 32, hipMemcpyHostToDevice);
    }
    for (int blocks : {312, 1024}) {  // <= maxb (the buffers hold maxb blocks)
        run_r<1>("r16 + gather M, divide", R, lut, lut4, n, o, cy, blocks);
        run_r<2>("r16 + gather {M,M/A,M/R}", R, lut, lut4, n, o, cy, blocks);
        run_r<2, 16>("r16 + gather rows, 16 ahead", R, lut, lut4, n, o, cy, blocks);
        run_r<2, 24>("r16 + gather rows, 24 ahead", R, lut, lut4, n, o, cy, blocks);
        run<0, 1>("inline divisions (current)", M, n, o, cy, blocks);
        run<1, 2>("divisions 2 frames ahead", M, n, o, cy, blocks);
        run<1, 4>("divisions 4 frames ahead", M, n, o, cy, blocks);
        run<2, 4>("4 ahead, no canonicalize", M, n, o, cy, blocks);
        run<3, 1>("lean (no divisions)", M, n, o, cy, blocks);
    }
    return 0;
}
