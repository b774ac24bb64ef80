"""Traceback time of lone pairs (DESIGN.md §3.2 "Traceback"): one pair per job,
so the walk runs with the GPU otherwise idle; NWK_VERBOSE=2-style timeline
lines give each pair's fill end and trace end.
usage: [NWK_LIB=<variant .so>] [NWK_TP_KERNEL=nw_align_col] python tools/trace_probe.py [L ...]"""
import os
import sys

sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import numpy as np  # noqa: E402

import seqalign  # noqa: E402
import workloads  # noqa: E402

seqalign.load_library(os.environ.get("NWK_LIB", seqalign.LIB_PATH))
for L in [int(a) for a in sys.argv[1:]] or [8192, 50000]:
    g = workloads.synth(2, L)
    e = seqalign.Engine(device=0, verbose=2, kernel=os.environ.get("NWK_TP_KERNEL", "auto"))
    e.set_sequences(g)
    for rep in range(3):
        pen, hs = e.align_pairs(np.arange(1, dtype=np.int64), 3, 2)
    print("L=%d penalty %d" % (L, int(pen[0])), flush=True)
    e.close()
