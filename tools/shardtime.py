"""Per-rank time of the big13 job when LPT-sharded over W ranks (rank shards run one after another on one GPU).
usage: python tools/shardtime.py [W ...]"""
import os, sys, time
sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import numpy as np
import seqalign
t = open("tests/golden/data/mseq-big13-example.txt", "rb").read()
pxy, pgap, g = seqalign.parse_input(t)
e = seqalign.Engine(device=0)
e.set_sequences(g)
e.align_pairs(np.arange(78, dtype=np.int64), pxy, pgap)  # warm
for W in [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]:
    worst = 0.0
    for r in range(W):
        ids = seqalign.shard_pairs([len(s) for s in g], r, W) if hasattr(seqalign, "shard_pairs") else None
        best = 1e9
        for rep in range(3):
            t0 = time.perf_counter()
            e.align_pairs(ids, pxy, pgap)
            best = min(best, time.perf_counter() - t0)
        worst = max(worst, best)
    print("W=%d: slowest rank %.2f ms" % (W, worst * 1e3), flush=True)
