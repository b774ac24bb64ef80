import sys, os
sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd"); sys.path.insert(0, "oracle")
import numpy as np, seqalign, oracle
rng = np.random.RandomState(0)
for (m, n) in [(20, 20), (600, 600), (1500, 1300), (200, 3000), (3000, 200)]:
    x = bytes(rng.choice(list(b"ACGT"), m).tolist()); y = bytes(rng.choice(list(b"ACGT"), n).tolist())
    with seqalign.Engine(device=0) as e:
        g = e.get_minimum_penalty(x, y, 3, 2)
    o = oracle.pair(x, y, 3, 2)
    ok = g == o
    print(m, n, "OK" if ok else "MISMATCH", "pen", g[0], o[0], "len", len(g[1]), len(o[1]))
    if not ok:
        a, b = g[1][::-1], o[1][::-1]
        k = next((t for t in range(min(len(a), len(b))) if a[t] != b[t] or g[2][::-1][t] != o[2][::-1][t]), None)
        print("  first diff from end at", k)
