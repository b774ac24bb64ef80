"""Round 6: test_affine_packed_windowed_storage_and_full_rerun[40]'s job (the
round-5 intermittent nw_align_pka miss, profiles/r05/pka_flake_rate.txt) with
the fill-vs-walk guard on: every mismatch is logged by the engine
(NWK_GUARD_LOG: walked path cost vs the fill's H(m, n)) and re-run, so the
answers must now always equal the oracle's.  argv: iterations."""
import os, random, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np
import seqalign, oracle
from test_gpu import _mutants, ACGT
r = random.Random(5151)
genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in (900, 2600, 4100, 5200)]
genes += _mutants(r, bytes(r.choice(ACGT) for _ in range(4500)), 2, ACGT)
P, Q = (bytes(r.choice(ACGT) for _ in range(3000)) for _ in range(2))
genes += [P + Q, Q + P]
k = len(genes)
ids = np.arange(k * (k - 1) // 2, dtype=np.int64)
ref = {s: oracle.all_pairs_affine(genes, *s)[1] for s in ((3, 3, 1), (4, 2, 2))}
nbad = nguard = 0
for it in range(int(sys.argv[1])):
    for s in ((3, 3, 1), (4, 2, 2)):
        with seqalign.Engine(device=0, workspace_bytes=40 << 20) as e:
            e.set_sequences(genes)
            try:
                pen, hs = e.align_pairs_affine(ids, *s)
            except seqalign.NwkError as x:
                print(it, s, "ERROR", x, flush=True)
                nbad += 1
                continue
            st = e.stats()
        bad = [(int(p), seqalign.pair_ij(int(p)), int(pen[p]), ref[s][p]) for p in range(len(ids)) if int(pen[p]) != ref[s][p]]
        nbad += len(bad) > 0
        nguard += st["guard_reruns"] > 0
        print(it, s, "mode", st["mode"], "batches", st["batches"], "retries", st["window_retries"],
              "guard checked", st["guard_checked"], "reruns", st["guard_reruns"], "bad", bad, flush=True)
print("runs with a wrong pair:", nbad, "runs with a guard re-run:", nguard)
