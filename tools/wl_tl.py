"""Per-pair fill timeline of one whole-workload align_all (verbose >= 2 stamps
to stderr: each pair's fill-done and trace-done time, fill band-cycles and the
share spent waiting on the band above).
usage: python tools/wl_tl.py [workload=big13] [kernel=auto]   (workload: big13, c3, c4)"""
import os
import sys

sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import seqalign  # noqa: E402
import workloads  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "big13"
kernel = sys.argv[2] if len(sys.argv) > 2 else "auto"
if wl == "big13":
    pxy, pgap, g = seqalign.parse_input(open(os.path.join(workloads.GOLDEN_DATA, "mseq-big13-example.txt"), "rb").read())
else:
    _, k, L, pxy, pgap, _ = workloads.SYNTH[wl]
    g = workloads.synth(k, L)
with seqalign.Engine(device=0, kernel=kernel, verbose=2) as e:
    e.set_sequences(g)
    for _ in range(2):
        h, pen, _ = e.align_all(pxy, pgap)
    st = e.stats()
print("%s: fill %.2f ms, mode %s, window %d, retries %d, hash %s" % (
    wl, st["fill_ms"], seqalign.MODES.get(st["mode"]), st["window"], st["window_retries"], h[:16]))
