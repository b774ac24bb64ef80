/* Convergence of traceback paths (DESIGN.md segmented traceback): for one
 * pair, the true path (from (m, n)) and, per 2048-row band, a path started on
 * the band's last row at a guessed column; prints how many rows up the guess
 * path meets the true path (a shared cell: the paths coincide from there), or
 * "none" within the band.  Linear gaps, the reference's recurrence and
 * traceback order (oracle/nw_oracle.c nwo_pair: DIAG, UP, LEFT).
 * usage: segconv <seqfile: two lines> pxy pgap */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int *D;
static int W;
#define AT(i, j) D[(size_t)(i) * W + (size_t)(j)]

int main(int argc, char **argv) {
  if (argc < 4) return 1;
  FILE *f = fopen(argv[1], "r");
  static char bx[1 << 21], by[1 << 21];
  if (!f || !fgets(bx, sizeof bx, f) || !fgets(by, sizeof by, f)) return 1;
  fclose(f);
  int m = (int)strcspn(bx, "\r\n"), n = (int)strcspn(by, "\r\n");
  const int pxy = atoi(argv[2]), pgap = atoi(argv[3]);
  W = n + 1;
  D = (int *)malloc(sizeof(int) * (size_t)(m + 1) * W);
  if (!D) return 2;
  for (int i = 0; i <= m; ++i) AT(i, 0) = i * pgap;
  for (int j = 0; j <= n; ++j) AT(0, j) = j * pgap;
  for (int i = 1; i <= m; ++i)
    for (int j = 1; j <= n; ++j) {
      int d = AT(i - 1, j - 1) + (bx[i - 1] == by[j - 1] ? 0 : pxy);
      int u = AT(i - 1, j) + pgap, l = AT(i, j - 1) + pgap;
      if (bx[i - 1] == by[j - 1]) { AT(i, j) = AT(i - 1, j - 1); continue; }
      int v = d < u ? d : u;
      AT(i, j) = v < l ? v : l;
    }
  /* true path: the column range per row (cells (i, j), 1-based) */
  int *lo = (int *)malloc(sizeof(int) * (m + 1)), *hi = (int *)malloc(sizeof(int) * (m + 1));
  for (int i = 0; i <= m; ++i) lo[i] = 1 << 30, hi[i] = -1;
  int i = m, j = n;
  while (i > 0 && j > 0) {
    if (j < lo[i]) lo[i] = j;
    if (j > hi[i]) hi[i] = j;
    if (bx[i - 1] == by[j - 1] || AT(i - 1, j - 1) + pxy == AT(i, j)) { i--; j--; }
    else if (AT(i - 1, j) + pgap == AT(i, j)) i--;
    else j--;
  }
  const int nb = (m + 2047) / 2048;
  for (int b = 0; b + 1 < nb; ++b) {
    const int R = 2048 * (b + 1); /* 1-based row of the band's last row */
    const int top = 2048 * b + 1;
    const int cdiag = (int)((long long)R * n / m);
    printf("band %2d: true entry %6d..%6d  diag %6d (off %+6d):", b, lo[R], hi[R], cdiag, cdiag - hi[R]);
    /* argmin over the band's last row of H[R][c] + pgap |(n - c) - (m - R)| (the gaps the suffix cannot avoid) */
    int cam = 1;
    long long best = 1LL << 60;
    for (int c = 1; c <= n; ++c) {
      const long long v = AT(R, c) + (long long)pgap * llabs((long long)(n - c) - (m - R));
      if (v < best) best = v, cam = c;
    }
    printf(" argmin %6d (off %+6d)", cam, cam - hi[R]);
    const int offs[] = {0, 16, 64, 256, 1024, -16, -64, -256, -1024, 99999, 77777};
    for (int g = 0; g < 11; ++g) {
      int c0 = offs[g] == 99999 ? n : offs[g] == 77777 ? cam : cdiag + offs[g];
      if (c0 < 1) c0 = 1;
      if (c0 > n) c0 = n;
      int ii = R, jj = c0, met = -1;
      while (ii >= 1 && jj > 0) {  /* (past the band's top too: the depth of the merge) */
        if (jj >= lo[ii] && jj <= hi[ii]) { met = R - ii; break; }
        if (bx[ii - 1] == by[jj - 1] || AT(ii - 1, jj - 1) + pxy == AT(ii, jj)) { ii--; jj--; }
        else if (AT(ii - 1, jj) + pgap == AT(ii, jj)) ii--;
        else jj--;
      }
      (void)top;
      if (offs[g] == 99999) printf("  n:%s", met < 0 ? "none" : "");
      else if (offs[g] == 77777) printf("  AM:%s", met < 0 ? "none" : "");
      else printf("  %+d:%s", offs[g], met < 0 ? "none" : "");
      if (met >= 0) printf("%d", met);
    }
    printf("\n");
  }
  return 0;
}
