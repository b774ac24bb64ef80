"""Small affine pairs on the GPU vs the oracle, printing the first mismatch."""
import sys, random
sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd"); sys.path.insert(0, "oracle")
import seqalign, oracle
r = random.Random(0)
with seqalign.Engine(device=0) as e:
    for (m, n) in [(1, 1), (3, 2), (8, 8), (20, 17), (64, 70), (300, 200), (600, 900), (1100, 1030)]:
        x = bytes(r.choice(b"ACGT") for _ in range(m)); y = bytes(r.choice(b"ACGT") for _ in range(n))
        for (pxy, go, ge) in [(2, 0, 2), (3, 4, 1)]:
            try:
                g = e.get_minimum_penalty_affine(x, y, pxy, go, ge)
            except Exception as ex:
                print("ERR", m, n, pxy, go, ge, ex, flush=True); continue
            o = oracle.pair_affine(x, y, pxy, go, ge)
            ok = g == o
            print(m, n, pxy, go, ge, "ok" if ok else "MISMATCH", g[0], o[0], flush=True)
            if not ok and m <= 64:
                print(" gpu", g[1], g[2]); print(" orc", o[1], o[2])
