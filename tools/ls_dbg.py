#!/usr/bin/env python3
"""Debug: big13 through the linear-space path at several HBM budgets.

    python tools/ls_dbg.py G ws_gb [ws_gb ...]     (ws_gb 0 = automatic budget)
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
import numpy as np  # noqa: E402

if os.environ.get("LS_TORCH"):  # load torch's bundled HIP runtime first (as the test session does)
    import torch  # noqa: F401
import seqalign  # noqa: E402

G = int(sys.argv[1])
gold = {c["name"]: c for c in json.load(open(os.path.join(REPO, "tests/golden/golden.json")))["cases"]}["big13"]
pxy, pgap, genes = seqalign.parse_input(open(os.path.join(REPO, "tests/golden/data", gold["file"]), "rb").read())
ids = [(i, j) for i in range(1, len(genes)) for j in range(i)]
bad_total = 0
for ws in sys.argv[2:]:
    t0 = time.time()
    with seqalign.Engine(device=0, linear_space=G, workspace_bytes=int(float(ws) * (1 << 30))) as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(np.arange(len(ids), dtype=np.int64), pxy, pgap)
        st = e.stats()
    bad = [q for q in range(len(ids)) if int(pen[q]) != gold["penalties"][q]]
    bad_total += len(bad)
    print("ws %s GB: %.1f s, batches %d, bad pairs %s" % (ws, time.time() - t0, st["batches"],
          [(q, ids[q], len(genes[ids[q][0]]), len(genes[ids[q][1]]), int(pen[q]), gold["penalties"][q]) for q in bad]),
          flush=True)
sys.exit(1 if bad_total else 0)
