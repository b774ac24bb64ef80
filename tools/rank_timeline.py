"""One rank's shard of a W-rank job on one GPU with the engine's per-pair
timeline (nwk_opts.verbose = 2: filled / traced per pair, band cycles and the
share spent waiting on the band above; nwk_runtime.cpp "nwk timeline").

usage: python tools/rank_timeline.py [workload=c3] [W=8] [rank=0] [kernel=auto]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
import numpy as np  # noqa: E402

import seqalign  # noqa: E402
import workloads  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rank = int(sys.argv[3]) if len(sys.argv) > 3 else 0
kernel = sys.argv[4] if len(sys.argv) > 4 else "auto"
_, k, L, pxy, pgap, _ = workloads.SYNTH[wl]
genes = workloads.synth(k, L)
ids = seqalign.shard_pairs([len(g) for g in genes], rank, W)
with seqalign.Engine(device=0, kernel=kernel) as e:
    e.set_sequences(genes)
    e.align_pairs(ids, pxy, pgap)  # warm
    t0 = time.perf_counter()
    e.align_pairs(ids, pxy, pgap)
    print("rank %d of %d: %d pairs, %.2f ms (stats %s)" % (rank, W, len(ids), (time.perf_counter() - t0) * 1e3, e.stats()),
          flush=True)
with seqalign.Engine(device=0, kernel=kernel, verbose=2) as e:
    e.set_sequences(genes)
    e.align_pairs(ids, pxy, pgap)
