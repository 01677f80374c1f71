// CPU study for VERDICT r03 item 2 (the associative-scan envelope): compose pydub's
// per-frame envelope maps  a -> (a <= M) ? min(a + M/A, M) : max(a - M/R, 0)  over a
// tile of TL active frames as a piecewise map of the entry state (pieces of slope 1,
// a + c, or constant), as a scan over tiles would, and report
//   * the pieces a tile's composed map needs (the "bounded-breakpoint" overflow rate
//     for a budget of K pieces), and
//   * how often the composed map, evaluated at the TRUE entry state, lands bit for bit
//     on the sequential pydub value (pieces of slope 1 add the tile's offsets in a
//     different order than the walk rounds them).
// Data: tools/study/coalesce_data.py + envelope_data.py (the compacted M streams of
// the bench track; M = 0 frames are identities, so tiles are TL active frames).
// gcc -O2 -o /tmp/ms tools/study/map_scan.c && /tmp/ms /tmp/study/full.idx 225
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
typedef struct { double lo, hi, c; int s; } Piece;  // a in (lo, hi]: s ? a + c : c
static double step(double a, double m, double A, double R) {
  double inc = m / A, dec = m / R;
  if (a <= m) { double u = a + inc; return u < m ? u : m; }
  double d = a - dec; return d > 0 ? d : 0;
}
static int cmpint(const void *x, const void *y) { return *(const int *)x - *(const int *)y; }
int main(int argc, char **argv) {
  FILE *f = fopen(argv[1], "r"); int TL = argc > 2 ? atoi(argv[2]) : 225;
  char path[256]; int b; long n; double A, R;
  long ntile[3] = {0}, exact[3] = {0}, over[3][4] = {{0}}; int *npc[3]; long cap[3] = {0};
  const int K[4] = {4, 8, 16, 32};
  for (int q = 0; q < 3; ++q) { cap[q] = 1 << 20; npc[q] = malloc(cap[q] * sizeof(int)); }
  Piece *p = malloc(sizeof(Piece) * 8 * (TL + 4)), *t = malloc(sizeof(Piece) * 8 * (TL + 4));
  while (fscanf(f, "%s %d %ld %lf %lf", path, &b, &n, &A, &R) == 5) {
    double *M = malloc(n * 8); FILE *g = fopen(path, "rb");
    if (fread(M, 8, n, g) != (size_t)n) return 1; fclose(g);
    double att = 0.0;  // the true (sequential) state
    for (long t0 = 0; t0 + TL <= n; t0 += TL) {
      int np = 1; p[0] = (Piece){-1.0, 1e300, 0.0, 1};  // identity over the state domain
      for (int i = 0; i < TL; ++i) {
        double m = M[t0 + i], inc = m / A, dec = m / R; int nt = 0;
        for (int k = 0; k < np; ++k) {
          Piece x = p[k];
          if (!x.s) { t[nt++] = (Piece){x.lo, x.hi, step(x.c, m, A, R), 0}; continue; }
          double sa = m - x.c, sm = m - inc - x.c;  // a <= sa: attack; a <= sm: a + c + inc <= M
          if (x.lo < sm) t[nt++] = (Piece){x.lo, x.hi < sm ? x.hi : sm, x.c + inc, 1};
          double l2 = x.lo > sm ? x.lo : sm, h2 = x.hi < sa ? x.hi : sa;
          if (l2 < h2) t[nt++] = (Piece){l2, h2, m, 0};
          if (x.hi > sa) t[nt++] = (Piece){x.lo > sa ? x.lo : sa, x.hi, x.c - dec, 1};
        }
        np = 0;  // merge neighbours with the same form
        for (int k = 0; k < nt; ++k) {
          if (np && p[np - 1].s == t[k].s && p[np - 1].c == t[k].c) p[np - 1].hi = t[k].hi;
          else p[np++] = t[k];
        }
      }
      double a0 = att;
      for (int i = 0; i < TL; ++i) att = step(att, M[t0 + i], A, R);
      double v = 0.0;
      for (int k = 0; k < np; ++k) if (a0 > p[k].lo && a0 <= p[k].hi) { v = p[k].s ? a0 + p[k].c : p[k].c; break; }
      if (ntile[b] == cap[b]) { cap[b] *= 2; npc[b] = realloc(npc[b], cap[b] * sizeof(int)); }
      npc[b][ntile[b]++] = np;
      exact[b] += v == att;
      for (int q = 0; q < 4; ++q) over[b][q] += np > K[q];
    }
    free(M);
  }
  for (int q = 0; q < 3; ++q) {
    if (!ntile[q]) continue;
    qsort(npc[q], ntile[q], sizeof(int), cmpint);
    long N = ntile[q];
    printf("band %d: %ld tiles of %d active frames; pieces p50 %d p90 %d p99 %d max %d; overflow >4 %.3f >8 %.3f "
           ">16 %.3f >32 %.3f; composed map bit-exact at the true entry state %.3f\n", q, N, TL, npc[q][N / 2],
           npc[q][N * 9 / 10], npc[q][N * 99 / 100], npc[q][N - 1], (double)over[q][0] / N, (double)over[q][1] / N,
           (double)over[q][2] / N, (double)over[q][3] / N, (double)exact[q] / N);
  }
  return 0;
}
