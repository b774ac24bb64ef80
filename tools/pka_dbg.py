#!/usr/bin/env python3
"""Debug: one small affine call per process stage, with markers on stderr.

    python tools/pka_dbg.py <case> [kernel]     case: mseq | rand | big13deg
"""
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import seqalign  # noqa: E402


def log(*a):
    print("[%.2f]" % (time.time() - T0), *a, file=sys.stderr, flush=True)


T0 = time.time()
case = sys.argv[1]
kernel = sys.argv[2] if len(sys.argv) > 2 else "auto"
if case == "mseq":
    pxy, pgap, genes = seqalign.parse_input(open(os.path.join(REPO, "tests/golden/data/mseq.dat"), "rb").read())
    go, ge = 0, pgap
elif case == "rand":
    r = random.Random(5)
    genes = [bytes(r.choice(b"ACGT") for _ in range(L)) for L in (1, 2, 63, 64, 65, 700, 1500)]
    pxy, go, ge = 3, 3, 1
elif case == "pairs":
    pass
else:
    raise SystemExit("case?")
if case == "pairs":
    r = random.Random(11)
    fails = 0
    with seqalign.Engine(device=0, kernel=kernel) as e:
        for (pxy, go, ge) in [(3, 3, 1), (3, 0, 2), (4, 2, 1)]:
            for m, n in [(1, 1), (3, 5), (8, 8), (9, 9), (16, 3), (64, 64), (65, 65), (100, 100), (300, 40),
                         (40, 300), (520, 530), (700, 30), (30, 700), (1100, 1000)]:
                x = bytes(r.choice(b"ACGT") for _ in range(m))
                y = bytes(r.choice(b"ACGT") for _ in range(n))
                pg, g1, g2 = e.get_minimum_penalty_affine(x, y, pxy, go, ge)
                mode = e.stats()["mode"]
                po, o1, o2 = oracle.pair_affine(x, y, pxy, go, ge)
                ok = pg == po and g1 == o1 and g2 == o2
                if not ok:
                    fails += 1
                    # first difference counted from the end of the rows (where the trace starts)
                    k = 0
                    while k < min(len(g1), len(o1)) and g1[-1 - k] == o1[-1 - k] and g2[-1 - k] == o2[-1 - k]:
                        k += 1
                    log("MISMATCH pxy/go/ge", (pxy, go, ge), "m,n", (m, n), "mode", mode, "gpu", pg, "oracle", po,
                        "lens", len(g1), len(o1), "same tail", k,
                        "gpu..", g1[max(0, len(g1) - k - 12):len(g1) - k + 3], g2[max(0, len(g2) - k - 12):len(g2) - k + 3],
                        "ora..", o1[max(0, len(o1) - k - 12):len(o1) - k + 3], o2[max(0, len(o2) - k - 12):len(o2) - k + 3])
                else:
                    log("ok", (pxy, go, ge), (m, n), "mode", mode, pg)
    sys.exit(1 if fails else 0)
log("genes", [len(g) for g in genes], "pxy", pxy, "go", go, "ge", ge, "kernel", kernel)
with seqalign.Engine(device=0, kernel=kernel, verbose=3) as e:
    log("engine up")
    e.set_sequences(genes)
    log("sequences set")
    k = len(genes)
    pen, hs = e.align_pairs_affine(np.arange(k * (k - 1) // 2, dtype=np.int64), pxy, go, ge)
    log("aligned, mode", e.stats()["mode"])
    h, opens, ohs = oracle.all_pairs_affine(genes, pxy, go, ge)
    ok = [int(v) for v in pen] == opens and [x.tobytes().hex() for x in hs] == ohs
    log("penalties", [int(v) for v in pen][:10], "oracle", opens[:10], "OK" if ok else "MISMATCH")
    if not ok:
        ids = [(i, j) for i in range(1, k) for j in range(i)]
        for q, (v, o) in enumerate(zip([int(v) for v in pen], opens)):
            if v != o or hs[q].tobytes().hex() != ohs[q]:
                i, j = ids[q]
                log("pair", q, (i, j), "m,n", len(genes[i]), len(genes[j]), "gpu", v, "oracle", o)
        sys.exit(1)
