"""Per-rank time of a job LPT-sharded over W ranks: each rank's shard runs alone on
one GPU (one after another), so the slowest rank bounds an N-GPU run without its
all-gather (72-byte records, microseconds).  Wall time of align_pairs per shard
(fill + traceback + finalize), best of 3; cells from the shard's pairs.
usage: python tools/shardtime.py [workload=big13] [W ...]     (workload: big13, c3, c4)"""
import os
import sys
import time

sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import numpy as np  # noqa: E402
import seqalign  # noqa: E402
import workloads  # noqa: E402

args = sys.argv[1:]
wl = args.pop(0) if args and not args[0].isdigit() else "big13"
if wl == "big13":
    t = open(os.path.join(workloads.GOLDEN_DATA, "mseq-big13-example.txt"), "rb").read()
    pxy, pgap, g = seqalign.parse_input(t)
else:
    _, k, L, pxy, pgap, _ = workloads.SYNTH[wl]
    g = workloads.synth(k, L)
lens = [len(s) for s in g]
P = len(g) * (len(g) - 1) // 2
e = seqalign.Engine(device=0)
e.set_sequences(g)
e.align_pairs(np.arange(P, dtype=np.int64), pxy, pgap)  # warm
full = None
for W in [int(a) for a in args] or [1, 2, 4, 8]:
    worst, wcells = 0.0, 0
    for r in range(W):
        ids = seqalign.shard_pairs(lens, r, W)
        best = 1e9
        for rep in range(3):
            t0 = time.perf_counter()
            e.align_pairs(ids, pxy, pgap)
            best = min(best, time.perf_counter() - t0)
        if best > worst:
            worst, wcells = best, workloads.cells(g, ids)
    if W == 1:
        full = worst
    print("%s W=%d: slowest rank %.2f ms (%d pairs' cells %.3g, %.0f GCUPS on that rank)%s" % (
        wl, W, worst * 1e3, len(ids), wcells, wcells / worst / 1e9,
        "  speedup vs W=1: %.2fx" % (full / worst) if full else ""), flush=True)
