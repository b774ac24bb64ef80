"""nw_align_pka throughput probe: chain-free (one band pair per pair) vs chained
(long pairs), affine go=3 ge=1 pxy=3.  Kernel GCUPS per config.
usage: python tools/pka_probe.py m n npairs [m n npairs ...]
(NWK_AFF_NOTRACE=1: fill only; NWK_VERBOSE=1: batch lines on stderr)"""
import os, sys
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
    with seqalign.Engine(device=0) as e:
        e.set_sequences(genes)
        ks = []
        for r in range(3):
            e.align_pairs_affine(ids, 3, 3, 1)
            st = e.stats()
            ks.append(st["fill_ms"])
    cells = float(m) * n * P
    print("pka m=%d n=%d pairs=%d tasks=%d batches=%s: kernel ms min %.2f -> %.0f GCUPS" % (
        m, n, P, P * ((m + 1023) // 1024), st.get("batches"), min(ks), cells / min(ks) / 1e6), flush=True)
