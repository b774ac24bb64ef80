/*
 * oracle/msa_oracle.c -- CPU restatement of the k-way sum-of-pairs
 * progressive MSA.  TEST INFRASTRUCTURE ONLY (same rules
 * as nw_oracle.c: only tests/ and the bench's cpu_baseline leg load it).
 *
 * The reference has no multiple alignment (its metric name says "k-way SoP
 * MSA" but the code stops at the pairwise penalties and the hash chain,
 * seqalign-mpi-skeleton.cpp:117-175), so the build defines it:
 *
 *   guide tree   UPGMA on the pairwise penalty matrix of getMinimumPenalties
 *                (canonical order, skel:122-123); cluster distance = mean
 *                pairwise penalty, compared exactly as integer ratios; ties
 *                -> the pair with the smallest (older id, younger id), new
 *                clusters get ids k, k+1, ...
 *   merge        profile-profile Needleman-Wunsch of the younger cluster (rows
 *                X, like genes[i], i > j, in skel:122-123) against the older
 *                (columns Y) under sum-of-pairs costs
 *                from the reference's scoring: c(a,a) = 0, c(a,b) = pxy,
 *                c(a,'_') = c('_',a) = pgap, c('_','_') = 0, linear gaps:
 *                  sub(i,j) = sum over rows r of X, s of Y of c(X[r][i], Y[s][j])
 *                  gx(i)    = nongap(X col i) * |Y| * pgap   (X column vs a gap column)
 *                  gy(j)    = nongap(Y col j) * |X| * pgap
 *                  H = min(H[i-1][j-1] + sub, H[i-1][j] + gx(i), H[i][j-1] + gy(j))
 *                traceback priority DIAG > UP > LEFT (skel:236-262), prefix
 *                as skel:263-272; merged rows = X's rows then Y's rows.
 *                The merge order of a UPGMA step is (younger, older) so that
 *                for k = 2 the DP is exactly skel's pair (1, 0).
 *   output       rows in input order, SoP score = sum over row pairs and
 *                columns of c() = the sum of the merge costs.
 *
 * Pins: for k = 2 the MSA is exactly the reference's pairwise alignment
 * (profile costs reduce to the pairwise ones; the match shortcut equals the
 * minimum for non-negative penalties), so every k = 2 golden
 * vector pins it; for any k the SoP of the rows must equal the summed merge
 * costs.  Beyond that, parity with a reference is unpinned.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int cost(unsigned char a, unsigned char b, int pxy, int pgap) {
  if (a == '_' || b == '_') return (a == '_' && b == '_') ? 0 : pgap;
  return a == b ? 0 : pxy;
}

/*
 * Profile X (nx rows of length lx, row-major) against Y (ny x ly).  Writes the
 * alignment columns in forward order to ops ('D' X col with Y col, 'U' X col
 * with a gap column, 'L' a gap column with Y col; capacity lx + ly) and
 * returns the cost H[lx][ly] (-1 on allocation failure).
 */
long long nwo_profile_align(const unsigned char *X, int nx, int lx, const unsigned char *Y, int ny, int ly,
                            int pxy, int pgap, unsigned char *ops, int *nops) {
  const size_t W = (size_t)ly + 1;
  long long *H = (long long *)malloc(sizeof(long long) * (size_t)(lx + 1) * W);
  long long *gx = (long long *)malloc(sizeof(long long) * (size_t)(lx + 1));
  long long *gy = (long long *)malloc(sizeof(long long) * (size_t)(ly + 1));
  if (!H || !gx || !gy) { free(H); free(gx); free(gy); return -1; }
  for (int i = 1; i <= lx; ++i) {
    long long ng = 0;
    for (int r = 0; r < nx; ++r) ng += X[(size_t)r * lx + i - 1] != '_';
    gx[i] = ng * ny * pgap;
  }
  for (int j = 1; j <= ly; ++j) {
    long long ng = 0;
    for (int s = 0; s < ny; ++s) ng += Y[(size_t)s * ly + j - 1] != '_';
    gy[j] = ng * nx * pgap;
  }
  H[0] = 0;
  for (int j = 1; j <= ly; ++j) H[j] = H[j - 1] + gy[j];
  for (int i = 1; i <= lx; ++i) {
    long long *row = H + (size_t)i * W, *up = row - W;
    row[0] = up[0] + gx[i];
    for (int j = 1; j <= ly; ++j) {
      long long s = 0;
      for (int r = 0; r < nx; ++r)
        for (int q = 0; q < ny; ++q) s += cost(X[(size_t)r * lx + i - 1], Y[(size_t)q * ly + j - 1], pxy, pgap);
      long long v = up[j - 1] + s;
      if (up[j] + gx[i] < v) v = up[j] + gx[i];
      if (row[j - 1] + gy[j] < v) v = row[j - 1] + gy[j];
      row[j] = v;
    }
  }
  const long long total = H[(size_t)lx * W + ly];
  /* traceback from (lx, ly), moves collected reversed */
  int i = lx, j = ly, n = 0;
  while (i > 0 && j > 0) {
    const long long h = H[(size_t)i * W + j];
    long long s = 0;
    for (int r = 0; r < nx; ++r)
      for (int q = 0; q < ny; ++q) s += cost(X[(size_t)r * lx + i - 1], Y[(size_t)q * ly + j - 1], pxy, pgap);
    if (H[(size_t)(i - 1) * W + j - 1] + s == h) { ops[n++] = 'D'; --i; --j; }
    else if (H[(size_t)(i - 1) * W + j] + gx[i] == h) { ops[n++] = 'U'; --i; }
    else { ops[n++] = 'L'; --j; }
  }
  while (i > 0) { ops[n++] = 'U'; --i; }
  while (j > 0) { ops[n++] = 'L'; --j; }
  for (int a = 0, b = n - 1; a < b; ++a, --b) { unsigned char t = ops[a]; ops[a] = ops[b]; ops[b] = t; }
  *nops = n;
  free(H); free(gx); free(gy);
  return total;
}

/* SoP score of k rows of length len. */
long long nwo_sop(const unsigned char *rows, int k, int len, int pxy, int pgap) {
  long long s = 0;
  for (int a = 0; a < k; ++a)
    for (int b = a + 1; b < k; ++b)
      for (int c = 0; c < len; ++c) s += cost(rows[(size_t)a * len + c], rows[(size_t)b * len + c], pxy, pgap);
  return s;
}

/*
 * Progressive MSA of k sequences.  penalties: the P = k(k-1)/2 pairwise
 * penalties in canonical order.  rows: k x cap bytes (cap >= sum of lengths);
 * *len = MSA length, *sop = SoP score (= summed merge costs).  Returns 0, or
 * -1 on allocation failure / cap too small.
 */
int nwo_msa(const unsigned char *seqs, const int64_t *offsets, int k, int pxy, int pgap, const int *penalties,
            unsigned char *rows, int cap, int *len, long long *sop) {
  *len = 0;
  *sop = 0;
  if (k <= 0) return 0;
  const int nc = 2 * k - 1;
  unsigned char **prof = (unsigned char **)calloc((size_t)nc, sizeof(unsigned char *));
  int *plen = (int *)calloc((size_t)nc, sizeof(int)), *psz = (int *)calloc((size_t)nc, sizeof(int));
  int **mem = (int **)calloc((size_t)nc, sizeof(int *));
  char *alive = (char *)calloc((size_t)nc, 1);
  long long *S = (long long *)calloc((size_t)nc * nc, sizeof(long long));  /* summed pairwise penalties */
  if (!prof || !plen || !psz || !mem || !alive || !S) return -1;
  for (int c = 0; c < k; ++c) {
    const int L = (int)(offsets[c + 1] - offsets[c]);
    prof[c] = (unsigned char *)malloc((size_t)L + 1);
    memcpy(prof[c], seqs + offsets[c], (size_t)L);
    plen[c] = L;
    psz[c] = 1;
    mem[c] = (int *)malloc(sizeof(int));
    mem[c][0] = c;
    alive[c] = 1;
  }
  for (int i = 1; i < k; ++i)
    for (int j = 0; j < i; ++j) S[(size_t)i * nc + j] = S[(size_t)j * nc + i] = penalties[(size_t)i * (i - 1) / 2 + j];
  for (int nid = k; nid < nc; ++nid) {
    int ba = -1, bb = -1;
    for (int a = 0; a < nid; ++a) {
      if (!alive[a]) continue;
      for (int b = a + 1; b < nid; ++b) {
        if (!alive[b]) continue;
        if (ba < 0) { ba = a; bb = b; continue; }
        /* S(a,b)/(|a||b|) < S(ba,bb)/(|ba||bb|), exactly */
        const __int128 lhs = (__int128)S[(size_t)a * nc + b] * psz[ba] * psz[bb];
        const __int128 rhs = (__int128)S[(size_t)ba * nc + bb] * psz[a] * psz[b];
        if (lhs < rhs) { ba = a; bb = b; }
      }
    }
    const int xa = bb, ya = ba;  /* rows: the younger cluster (skel's x = genes[i], i > j) */
    const int lx = plen[xa], ly = plen[ya], nx = psz[xa], ny = psz[ya];
    unsigned char *ops = (unsigned char *)malloc((size_t)lx + ly + 1);
    int nops = 0;
    const long long c = nwo_profile_align(prof[xa], nx, lx, prof[ya], ny, ly, pxy, pgap, ops, &nops);
    if (c < 0) return -1;
    *sop += c;
    unsigned char *np = (unsigned char *)malloc((size_t)(nx + ny) * nops + 1);
    for (int r = 0; r < nx + ny; ++r) {
      const unsigned char *src = r < nx ? prof[xa] + (size_t)r * lx : prof[ya] + (size_t)(r - nx) * ly;
      const int isx = r < nx;
      int p = 0;
      for (int t = 0; t < nops; ++t) {
        const unsigned char o = ops[t];
        const int take = isx ? (o != 'L') : (o != 'U');
        np[(size_t)r * nops + t] = take ? src[p++] : (unsigned char)'_';
      }
    }
    prof[nid] = np;
    plen[nid] = nops;
    psz[nid] = nx + ny;
    mem[nid] = (int *)malloc(sizeof(int) * (size_t)(nx + ny));
    memcpy(mem[nid], mem[xa], sizeof(int) * (size_t)nx);
    memcpy(mem[nid] + nx, mem[ya], sizeof(int) * (size_t)ny);
    alive[ba] = alive[bb] = 0;
    alive[nid] = 1;
    for (int o = 0; o < nid; ++o) {
      if (!alive[o]) continue;
      const long long v = S[(size_t)ba * nc + o] + S[(size_t)bb * nc + o];
      S[(size_t)nid * nc + o] = S[(size_t)o * nc + nid] = v;
    }
    free(ops);
  }
  const int root = nc - 1;
  if (plen[root] > cap) return -1;
  *len = plen[root];
  for (int r = 0; r < k; ++r) memcpy(rows + (size_t)mem[root][r] * cap, prof[root] + (size_t)r * plen[root], (size_t)plen[root]);
  for (int c = 0; c < nc; ++c) { free(prof[c]); free(mem[c]); }
  free(prof); free(plen); free(psz); free(mem); free(alive); free(S);
  return 0;
}
