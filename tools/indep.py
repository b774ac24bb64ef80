"""Throughput of independent band chains: pairs (i, 0) of an m-row x against one n-column y.
usage: python tools/indep.py m n npairs [m n npairs ...]   -- kernel GCUPS per config"""
import os, sys, time
sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import numpy as np
import seqalign
if os.environ.get("LIB"):
    seqalign.load_library(os.path.join(os.environ["LIB"], "libnwk.so"))
args = [int(a) for a in sys.argv[1:]]
rng = np.random.default_rng(1)
for q in range(0, len(args), 3):
    m, n, P = args[q:q + 3]
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    genes = [acgt[rng.integers(0, 4, n)].tobytes()] + [acgt[rng.integers(0, 4, m)].tobytes() for _ in range(P)]
    ids = np.array([i * (i - 1) // 2 for i in range(1, P + 1)], dtype=np.int64)
    with seqalign.Engine(device=0, verbose=int(os.environ.get("V", "0"))) as e:
        e.set_sequences(genes)
        ks = []
        for r in range(4):
            e.align_pairs(ids, 3, 2)
            ks.append(e.stats()["fill_ms"])
    cells = float(m) * n * P
    print("indep m=%d n=%d pairs=%d bands=%d: kernel ms min %.2f -> %.0f GCUPS" % (
        m, n, P, P * ((m + 511) // 512), min(ks), cells / min(ks) / 1e6), flush=True)
