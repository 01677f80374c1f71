// Study: an approximate (f32) warm-up in place of pass 0's exact f64 warm-up.
// For every super-tile start S = k*U: walk f32 from the guess M[S-W] over
// [S-W, S) (inc = m * RN(1/A), no correct rounding), optionally snap the state to
// the exact M[S-1] (or 0) when the f32 walk ended clamped there, then walk the
// exact f64 step from S and report how far past S it merges with the true
// trajectory (0 = exact at S).  Compare with the exact f64 warm-up (mode "f64").
// Build: gcc -O2 -o /tmp/coalesce_f32 tools/study/coalesce_f32.c -lm
// Usage: /tmp/coalesce_f32 U A R file.f64 ...
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

static double step(double a, double m, double A, double R) {
    const double inc = m / A, dec = m / R;
    if (a <= m) { a = a + inc; return a < m ? a : m; }
    a = a - dec;
    return a > 0.0 ? a : 0.0;
}
static int cmp(const void *x, const void *y) { long a = *(const long *)x, b = *(const long *)y; return a < b ? -1 : a > b; }

int main(int argc, char **argv) {
    const int U = atoi(argv[1]);
    const double A = atof(argv[2]), R = atof(argv[3]);
    const float rA = (float)(1.0 / A), rR = (float)(1.0 / R);
    const int Ws[] = {1000, 2000, 3000, 4000, 6000};
    const int NW = 5, NM = 3;  // modes: f64 exact warm-up, f32, f32 + snap
    const char *mname[] = {"f64 warm-up", "f32 warm-up", "f32 warm-up + clamp snap"};
    long *d[5][3];
    long cnt = 0, cap = 1 << 20;
    for (int w = 0; w < NW; ++w) for (int g = 0; g < NM; ++g) d[w][g] = malloc(cap * sizeof(long));
    for (int f = 4; f < argc; ++f) {
        FILE *fp = fopen(argv[f], "rb");
        fseek(fp, 0, SEEK_END);
        long n = ftell(fp) / 8;
        fseek(fp, 0, SEEK_SET);
        double *M = malloc(n * 8), *tr = malloc((n + 1) * 8);
        if (fread(M, 8, n, fp) != (size_t)n) return 1;
        fclose(fp);
        tr[0] = 0.0;
        for (long i = 0; i < n; ++i) tr[i + 1] = step(tr[i], M[i], A, R);
        for (long S = U; S < n; S += U) {
            for (int w = 0; w < NW; ++w) {
                const long s0 = S - Ws[w] < 0 ? 0 : S - Ws[w];
                for (int g = 0; g < NM; ++g) {
                    double a;
                    if (g == 0) {
                        a = s0 == 0 ? 0.0 : M[s0];
                        for (long i = s0; i < S; ++i) a = step(a, M[i], A, R);
                    } else {
                        float x = s0 == 0 ? 0.f : (float)M[s0];
                        int clamp = 0;  // 1: ended at m, 2: ended at 0
                        for (long i = s0; i < S; ++i) {
                            const float m = (float)M[i];
                            if (x <= m) { x = fminf(x + m * rA, m); clamp = x == m ? 1 : 0; }
                            else { x = fmaxf(x - m * rR, 0.f); clamp = x == 0.f ? 2 : 0; }
                        }
                        a = (double)x;
                        if (g == 2 && clamp == 1) a = M[S - 1];
                        if (g == 2 && clamp == 2) a = 0.0;
                    }
                    long i = S, dist = -1;
                    for (; i < n; ++i) {
                        if (a == tr[i]) { dist = i - S; break; }
                        a = step(a, M[i], A, R);
                    }
                    if (dist < 0) dist = n - S;
                    d[w][g][cnt] = dist;
                }
            }
            if (++cnt >= cap) break;
        }
        free(M);
        free(tr);
    }
    printf("super-tiles %ld (U=%d, A=%.1f, R=%.1f)\n", cnt, U, A, R);
    for (int g = 0; g < NM; ++g) {
        printf("%s\n", mname[g]);
        for (int w = 0; w < NW; ++w) {
            long *v = d[w][g];
            qsort(v, cnt, sizeof(long), cmp);
            long nz = 0, sum = 0;
            for (long k = 0; k < cnt; ++k) { nz += v[k] > 0; sum += v[k]; }
            printf("  W=%5d  miss %6.3f%%  mean %7.1f  p50 %6ld  p90 %6ld  p99 %6ld  p99.9 %6ld  max %7ld\n", Ws[w],
                   100.0 * nz / cnt, (double)sum / cnt, v[cnt / 2], v[cnt * 9 / 10], v[cnt * 99 / 100],
                   v[cnt * 999 / 1000], v[cnt - 1]);
        }
    }
    return 0;
}
