// Coalescence study for the envelope solve's speculative warm-up (CPU only).
// Reads raw M sequences (one chunk-band each) and, for every super-tile start
// S = k*U, walks a guessed trajectory from S - W and reports how far past S it
// merges with the true one (0 = merged before S).
// Build: gcc -O2 -o /tmp/coalesce tools/study/coalesce.c -lm
// Usage: /tmp/coalesce U A R file.f64 ...   (file: raw little-endian doubles)
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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
    const int Ws[] = {0, 500, 1000, 2000, 3000, 4000, 6000};
    const int NW = 7, NG = 4;
    const char *gname[] = {"M[S-W]", "zero", "maxM(2000 before)", "true+1ulp-ish(high)"};
    long *d[7][4];
    long cnt = 0, cap = 1 << 20;
    for (int w = 0; w < NW; ++w) for (int g = 0; g < NG; ++g) d[w][g] = malloc(cap * sizeof(long));
    for (int f = 4; f < argc; ++f) {
        FILE *fp = fopen(argv[f], "rb");
        fseek(fp, 0, SEEK_END);
        long n = ftell(fp) / 8;
        fseek(fp, 0, SEEK_SET);
        double *M = malloc(n * 8), *tr = malloc((n + 1) * 8);
        if (fread(M, 8, n, fp) != (size_t)n) return 1;
        fclose(fp);
        tr[0] = 0.0;
        for (long i = 0; i < n; ++i) tr[i + 1] = step(tr[i], M[i], A, R);  // tr[i] = state on entry to frame i
        for (long S = U; S < n; S += U) {
            for (int w = 0; w < NW; ++w) {
                const long s0 = S - Ws[w] < 0 ? 0 : S - Ws[w];
                for (int g = 0; g < NG; ++g) {
                    double a;
                    if (g == 0) a = M[s0];
                    else if (g == 1) a = 0.0;
                    else if (g == 2) { a = 0; for (long j = s0 - 2000 < 0 ? 0 : s0 - 2000; j <= s0; ++j) if (M[j] > a) a = M[j]; }
                    else a = tr[s0] * 1.5 + 1.0;
                    long i = s0, dist = -1;
                    if (s0 == 0) { a = 0.0; }
                    for (; i < n; ++i) {
                        if (a == tr[i]) { dist = i <= S ? 0 : i - S; break; }
                        a = step(a, M[i], A, R);
                    }
                    if (dist < 0) dist = n - S;  // never merged before the chunk end
                    d[w][g][cnt] = dist;
                }
            }
            if (++cnt >= cap) break;
        }
        free(M);
        free(tr);
    }
    printf("super-tiles %ld (U=%d, A=%.1f, R=%.1f)\n", cnt, U, A, R);
    for (int g = 0; g < NG; ++g) {
        printf("guess %s\n", gname[g]);
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
