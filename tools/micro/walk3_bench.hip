// Microbenchmark: one walker lane stepping whole tiles of the super-tile-major M
// plane (rows 512 B apart, 225 rows per tile, tiles at random columns of a 320 MB
// plane), with WNB blocks of WB rows in flight -- the comp_fix walk's memory
// pattern -- against the same steps from registers.  ns per frame (wall clock).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#pragma clang fp contract(off)

constexpr int WB = 25, T = 225, ROW = 64;  // doubles per row of a column block
__device__ __forceinline__ double div_cr(double m, double d, double rd) {
    double q = m * rd; double rem = fma(-q, d, m); return fma(rem, rd, q);
}
__device__ __forceinline__ double lean(double att, double m, double inc, double dec) {
    double t = att + inc, d = att - dec, up;
    asm("v_min_f64 %0, %1, %2" : "=v"(up) : "v"(t), "v"(m));
    return att <= m ? up : d;
}
// XA: the next tile's first blocks are loaded during the current tile's last ones
template <int WNB, bool XA>
__global__ void __launch_bounds__(64) walk(const double *P, const unsigned *tiles, int ntiles, double *out,
                                           long long *t) {
    if (threadIdx.x != 0) return;
    const double A = 441.0, rA = 1.0 / 441.0, R = 8820.0, rR = 1.0 / 8820.0;
    double att = 0.0;
    double mb[WNB][WB];
    const int bpt = T / WB;
    long long w0 = wall_clock64();
    int lt = 0, lb = 0;
    const double *base = P + (size_t)tiles[0];
    auto load = [&](double (&d)[WB]) {
#pragma unroll
        for (int j = 0; j < WB; ++j) d[j] = base[(size_t)(lb * WB + j) * ROW];
        if (++lb == bpt) {
            lb = 0;
            if (XA) base = P + (size_t)tiles[min(++lt, ntiles - 1)];
        }
    };
    for (int tile = 0; tile < ntiles; ++tile) {
        if (!XA) {
            base = P + (size_t)tiles[tile];
            lb = 0;
        }
        if (!XA || tile == 0) {
#pragma unroll
            for (int k = 0; k < WNB; ++k) load(mb[k]);
        }
        for (int b = 0; b < bpt; b += WNB) {
#pragma unroll
            for (int k = 0; k < WNB; ++k) {
                if (b + k < bpt) {
#pragma unroll
                    for (int j = 0; j < WB; ++j) {
                        const double m = mb[k][j];
                        att = lean(att, m, div_cr(m, A, rA), div_cr(m, R, rR));
                    }
                    if (XA || b + k + WNB < bpt) load(mb[k]);
                }
            }
        }
    }
    long long w1 = wall_clock64();
    out[0] = att;
    t[0] = w1 - w0;
}
template <int WNB>
__global__ void __launch_bounds__(64) walk_regs(const double *P, const unsigned *, int ntiles, double *out, long long *t) {
    if (threadIdx.x != 0) return;
    const double A = 441.0, rA = 1.0 / 441.0, R = 8820.0, rR = 1.0 / 8820.0;
    double att = 0.0, m0 = P[0], m1 = P[1];
    long long w0 = wall_clock64();
    for (int i = 0; i < ntiles * T; ++i) {
        const double m = (i & 1) ? m1 : m0;
        att = lean(att, m, div_cr(m, A, rA), div_cr(m, R, rR));
    }
    long long w1 = wall_clock64();
    out[0] = att;
    t[0] = w1 - w0;
}

int main() {
    const size_t plane = 40u << 20;  // doubles: 320 MB
    double *P, *F, *o;
    long long *t;
    unsigned *tl;
    hipMalloc(&P, plane * 8);
    hipMalloc(&F, plane * 8);
    hipMalloc(&o, 64);
    hipMalloc(&t, 64);
    std::vector<double> h(plane);
    for (size_t i = 0; i < plane; ++i) h[i] = 5.0 + (i % 97) * 0.05;
    hipMemcpy(P, h.data(), plane * 8, hipMemcpyHostToDevice);
    const int ntiles = 64;
    std::vector<unsigned> ht(ntiles);
    srand(1);
    const size_t cols = plane / ROW / (T + 4);  // column blocks x 64 columns... (rough: any row-0 offset)
    for (int i = 0; i < ntiles; ++i) {
        const size_t cb = (size_t)rand() % cols;
        ht[i] = (unsigned)(cb * (size_t)(T + 4) * ROW + (size_t)(rand() % 64));
    }
    hipMalloc(&tl, ntiles * 4);
    hipMemcpy(tl, ht.data(), ntiles * 4, hipMemcpyHostToDevice);
    auto run = [&](const char *name, auto k, bool) {
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(F, rep, plane * 8);  // evict L2 / MALL
            hipDeviceSynchronize();
            hipLaunchKernelGGL(k, 1, 64, 0, 0, (const double *)P, (const unsigned *)tl, ntiles, o, t);
            hipDeviceSynchronize();
            long long w;
            hipMemcpy(&w, t, 8, hipMemcpyDeviceToHost);
            printf("%-26s rep %d: %.2f us per tile, %.1f ns per frame\n", name, rep, w * 0.01 / ntiles,
                   w * 10.0 / ntiles / T);
        }
    };
    run("registers", walk_regs<2>, true);
    run("plane WNB 2", walk<2, false>, false);
    run("plane WNB 3", walk<3, false>, false);
    run("plane WNB 4", walk<4, false>, false);
    run("plane WNB 2 cross-tile", walk<2, true>, false);
    run("plane WNB 4 cross-tile", walk<4, true>, false);
    return 0;
}
