// Microbenchmark: the envelope walk's instruction schedule.  One walker lane steps
// tiles of a super-tile-major M plane (rows 512 B apart, 225 rows, 2 blocks of 25
// rows in flight, as comp_fix's walk).  Variants of how the two correctly rounded
// divisions per frame (inc = M/A, dec = M/R: 3 dependent f64 ops each) are placed
// against the att chain (add -> min -> select per frame):
//   0: the product's Walker (divisions WP = 5 frames ahead, compiler-scheduled)
//   1: divisions software-pipelined by stage: each frame issues stage 3 of frame
//      j+1, stage 2 of j+2 and stage 1 of j+3 (no dependent pair inside a frame)
//   2: no divisions (inc, dec precomputed in the plane: the chain's own floor)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#pragma clang fp contract(off)

constexpr int WB = 25, T = 225, ROW = 64, WP = 5;
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

template <int V>
__global__ void __launch_bounds__(64) walk(const double *P, const unsigned *tiles, int ntiles, double *out,
                                           long long *t, K k) {
    if (threadIdx.x != 0) return;
    double att = 0.0;
    double mb[2][WB];
    const int bpt = T / WB;
    long long w0 = wall_clock64();
    for (int tile = 0; tile < ntiles; ++tile) {
        const double *base = P + (size_t)tiles[tile];
        int lb = 0;
        auto load = [&](double (&d)[WB]) {
#pragma unroll
            for (int j = 0; j < WB; ++j) d[j] = base[(size_t)(min(lb, bpt - 1) * WB + j) * ROW];
            ++lb;
        };
        load(mb[0]);
        load(mb[1]);
        if (V == 0) {
            double inc[WP], dec[WP];
#pragma unroll
            for (int q = 0; q < WP; ++q) {
                inc[q] = div_cr(mb[0][q], k.A, k.rA);
                dec[q] = div_cr(mb[0][q], k.R, k.rR);
            }
            for (int b = 0; b < bpt; b += 2) {
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    if (b + kk < bpt) {
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
                        load(mb[kk]);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
        } else if (V == 1) {
            // pipeline registers: frame j+1's stage-2 results (rem) -> stage 3 this frame,
            // frame j+2's stage-1 results (q) -> stage 2 this frame, frame j+3 -> stage 1
            double iq1, ir1, dq1, dr1;  // frame j+1: q and rem (stage 2 done)
            double iq2, dq2;            // frame j+2: q (stage 1 done)
            double m1, m2;              // M of frames j+1, j+2
            double inc0, dec0;          // frame j: finished
            auto M_at = [&](int kk, int j) __attribute__((always_inline)) {
                return j < WB ? mb[kk][j] : mb[kk ^ 1][j - WB];
            };
            {  // prologue: frame 0 finished, frame 1 through stage 2, frame 2 through stage 1
                const double m0 = mb[0][0];
                inc0 = div_cr(m0, k.A, k.rA);
                dec0 = div_cr(m0, k.R, k.rR);
                m1 = mb[0][1];
                iq1 = m1 * k.rA;
                ir1 = fma(-iq1, k.A, m1);
                dq1 = m1 * k.rR;
                dr1 = fma(-dq1, k.R, m1);
                m2 = mb[0][2];
                iq2 = m2 * k.rA;
                dq2 = m2 * k.rR;
            }
            for (int b = 0; b < bpt; b += 2) {
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    if (b + kk < bpt) {
#pragma unroll
                        for (int j = 0; j < WB; ++j) {
                            const double m = M_at(kk, j);
                            const double m3 = M_at(kk, j + 3);
                            // independent stages (none depends on another in this frame)
                            const double inc1 = fma(ir1, k.rA, iq1), dec1 = fma(dr1, k.rR, dq1);
                            const double ir2 = fma(-iq2, k.A, m2), dr2 = fma(-dq2, k.R, m2);
                            const double iq3 = m3 * k.rA, dq3 = m3 * k.rR;
                            att = lean(att, m, inc0, dec0);
                            inc0 = inc1; dec0 = dec1;
                            iq1 = iq2; ir1 = ir2; dq1 = dq2; dr1 = dr2; m1 = m2;
                            iq2 = iq3; dq2 = dq3; m2 = m3;
                        }
                        __builtin_amdgcn_sched_barrier(0);
                        load(mb[kk]);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
            (void)m1;
        } else {
            for (int b = 0; b < bpt; b += 2) {
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    if (b + kk < bpt) {
#pragma unroll
                        for (int j = 0; j < WB; ++j) {
                            const double m = mb[kk][j];
                            att = lean(att, m, m * 0.001, m * 0.0001);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                        load(mb[kk]);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
        }
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
    const size_t cols = plane / ROW / (T + 4);
    for (int i = 0; i < ntiles; ++i)
        ht[i] = (unsigned)(((size_t)rand() % cols) * (size_t)(T + 4) * ROW + (size_t)(rand() % 64));
    hipMalloc(&tl, ntiles * 4);
    hipMemcpy(tl, ht.data(), ntiles * 4, hipMemcpyHostToDevice);
    K k{441.0, 1.0 / 441.0, 8820.0, 1.0 / 8820.0};
    double res[3];
    auto run = [&](const char *name, auto kern, int v) {
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(F, rep, plane * 8);  // evict L2 / MALL
            hipDeviceSynchronize();
            hipLaunchKernelGGL(kern, 1, 64, 0, 0, (const double *)P, (const unsigned *)tl, ntiles, o, t, k);
            hipDeviceSynchronize();
            long long w;
            double r;
            hipMemcpy(&w, t, 8, hipMemcpyDeviceToHost);
            hipMemcpy(&r, o, 8, hipMemcpyDeviceToHost);
            res[v] = r;
            printf("%-34s rep %d: %.2f us per tile, %.1f ns per frame  (att %.17g)\n", name, rep, w * 0.01 / ntiles,
                   w * 10.0 / ntiles / T, r);
        }
    };
    run("0 product Walker (WP 5)", walk<0>, 0);
    run("1 divisions pipelined by stage", walk<1>, 1);
    run("2 no divisions (floor)", walk<2>, 2);
    printf("variants 0 and 1 agree: %s\n", res[0] == res[1] ? "yes" : "NO");
    return 0;
}
