"""A/B one libnwk.so variant on a bench workload: kernel ms and wall ms per step.
usage: python tools/ab_wl.py <lib dir> [workload=c3] [reps=3]   (one variant per process)"""
import os
import sys
import time

sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import seqalign  # noqa: E402
import workloads  # noqa: E402

lib = sys.argv[1]
wl = sys.argv[2] if len(sys.argv) > 2 else "c3"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
seqalign.load_library(os.path.join(lib, "libnwk.so"))
desc, k, L, pxy, pgap, affine = workloads.SYNTH[wl]
genes = workloads.synth(k, L)
with seqalign.Engine(device=0) as e:
    e.set_sequences(genes)
    ks, ws, hs = [], [], set()
    for r in range(reps + 1):
        t0 = time.perf_counter()
        h, pen, _ = e.align_all(pxy, pgap, affine=affine)
        if r:
            ws.append(time.perf_counter() - t0)
            ks.append(e.stats()["fill_ms"])
        hs.add(h)
cells = workloads.cells(genes)
print("ab %-32s %s kernel ms min %.1f | wall ms min %.1f -> %.0f GCUPS | hash %s" % (
    lib, wl, min(ks), 1e3 * min(ws), cells / min(ws) / 1e9, "/".join(x[:12] for x in hs)), flush=True)
