"""Traceback coalescence on CPU (numpy DP, skel tie rules): from a cell d columns off
the true path on row r0, how many moves/rows until the two paths share a cell.
usage: python tools/coalesce.py [L=8000]  (two C4-style synthetic sequences)"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multiple-sequence-alignment-openmp-openmpi_amd"))
import workloads
L = int(sys.argv[1]) if len(sys.argv) > 1 else 8000
g = workloads.synth(2, L)
x = np.frombuffer(g[0], np.uint8); y = np.frombuffer(g[1], np.uint8)
m, n = len(x), len(y); pxy, pgap = 3, 2
H = np.zeros((m + 1, n + 1), np.int32)
H[0] = np.arange(n + 1) * pgap
jj = np.arange(n + 1, dtype=np.int64) * pgap
for i in range(1, m + 1):
    cost = np.where(x[i - 1] == y, 0, pxy).astype(np.int32)
    T = np.empty(n + 1, np.int64); T[0] = i * pgap
    T[1:] = np.minimum(H[i - 1, :-1] + cost, H[i - 1, 1:] + pgap)
    H[i] = (np.minimum.accumulate(T - jj) + jj).astype(np.int32)
def step(i, j):
    if x[i - 1] == y[j - 1] or H[i - 1, j - 1] + pxy == H[i, j]: return i - 1, j - 1
    if H[i - 1, j] + pgap == H[i, j]: return i - 1, j
    return i, j - 1
def path(i, j):
    P = {}
    while i > 0 and j > 0:
        P[(i, j)] = None; i, j = step(i, j)
    return P
true = path(m, n)
rowcols = {}
for (i, j) in true: rowcols.setdefault(i, []).append(j)
for r0 in (m // 2, 3 * m // 4):
    jt = max(rowcols[r0])
    for d in (-1024, -256, -64, -16, 16, 64, 256, 1024):
        i, j = r0, jt + d
        if not (0 < j <= n): continue
        k = 0
        while i > 0 and j > 0 and (i, j) not in true:
            i, j = step(i, j); k += 1
        print("L=%d r0=%d offset %+5d: merged after %d moves, %d rows (at row %d)" % (L, r0, d, k, r0 - i, i), flush=True)
