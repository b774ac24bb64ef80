"""C4 at full size through align_all, answer hash against tests/golden/large/c4.json
(fused-finalize debugging: NWK_STRIP / NWK_DEVHASH select the path).
usage: python tools/c4_check.py [workload=c4]"""
import json
import os
import sys
import time

sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import seqalign  # noqa: E402
import workloads  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c4"
g = json.load(open("tests/golden/large/%s.json" % wl))
_, k, L, pxy, pgap, _ = workloads.SYNTH[wl]
genes = workloads.synth(k, L)
with seqalign.Engine(device=0) as e:
    e.set_sequences(genes)
    for rep in range(2):
        t0 = time.perf_counter()
        try:
            h, pen, _ = e.align_all(pxy, pgap)
        except seqalign.NwkError as ex:
            print("%s rep %d: ERROR %s" % (wl, rep, ex), flush=True)
            sys.exit(1)
        st = e.stats()
        print("%s rep %d: %.1f ms, mode %s, batches %d, devfin %d, hash ok %s, penalties ok %s" % (
            wl, rep, 1e3 * (time.perf_counter() - t0), seqalign.MODES.get(st["mode"]), st["batches"],
            st["device_finalized"], h == g["hash"], [int(v) for v in pen] == g["penalties"]), flush=True)
