"""C5's first batch on nw_align_gotoh with the engine's per-pair timeline
(verbose = 2): when each pair's last band finished and its walk ended, and
the share of band time spent waiting on the band above.

usage: python tools/c5_timeline.py [pairs=124]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
import numpy as np  # noqa: E402

import seqalign  # noqa: E402
import workloads  # noqa: E402

npairs = int(sys.argv[1]) if len(sys.argv) > 1 else 124
_, k, L, pxy, pgap, (go, ge) = workloads.SYNTH["c5"]
genes = workloads.synth(k, L)
with seqalign.Engine(device=0, verbose=2) as e:
    e.set_sequences(genes)
    e.align_pairs_affine(np.arange(npairs, dtype=np.int64), pxy, go, ge)
