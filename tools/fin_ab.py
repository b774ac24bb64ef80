"""align_all with the separate device finalize (nw_rows + nw_hash after each
launch) against the fused one (finalize="fused": records stream out of the
fill launch and the chain runs during it).  usage: python tools/fin_ab.py [wl ...]"""
import json
import sys
import time

sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import seqalign  # noqa: E402
import workloads  # noqa: E402

for wl in sys.argv[1:] or ["c4", "c3"]:
    g = json.load(open("tests/golden/large/%s.json" % wl))
    _, k, L, pxy, pgap, _ = workloads.SYNTH[wl]
    genes = workloads.synth(k, L)
    for fin in ("device", "fused", "device", "fused"):
        with seqalign.Engine(device=0, finalize=fin) as e:
            e.set_sequences(genes)
            best = 1e9
            for rep in range(4):
                t0 = time.perf_counter()
                h, pen, _ = e.align_all(pxy, pgap)
                dt = time.perf_counter() - t0
                if rep:
                    best = min(best, dt)
                assert h == g["hash"], "answer differs"
            st = e.stats()
            print("%s finalize=%-6s align_all best %.1f ms (fill %.1f ms, %s, %d batches)" % (
                wl, fin, best * 1e3, st["fill_ms"], seqalign.MODES.get(st["mode"]), st["batches"]), flush=True)
