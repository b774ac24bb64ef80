"""Timeline of rank 0's C4 shard at W = 8 (4,080 pairs, the streamed path's
one launch with the fused finalize), verbose >= 2 stamps to stderr.
usage: python tools/c4shard_tl.py [kernel=auto] [W=8]"""
import sys

sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import numpy as np  # noqa: E402

import seqalign  # noqa: E402
import workloads  # noqa: E402

kernel = sys.argv[1] if len(sys.argv) > 1 else "auto"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 8
_, k, L, pxy, pgap, _ = workloads.SYNTH["c4"]
g = workloads.synth(k, L)
ids = seqalign.shard_pairs([len(x) for x in g], 0, W)
with seqalign.Engine(device=0, finalize="fused", kernel=kernel, verbose=2) as e:
    e.set_sequences(g)
    for _ in range(2):
        e.align_pairs(ids, pxy, pgap)
    st = e.stats()
print("rank-0 shard of %d: %d pairs, fill %.2f ms, mode %s" % (W, len(ids), st["fill_ms"], seqalign.MODES.get(st["mode"])))
