"""Times align_pairs on a workload several times in one process (min/median).
usage: python tools/fill_timeit.py [lib_dir ...]  (each lib dir holds a libnwk.so variant)"""
import sys, os, time, ctypes, importlib
sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import numpy as np
import seqalign, json
GOLD = {c["name"]: c for c in json.load(open("tests/golden/golden.json"))["cases"]}["big13"]["hash"]
wl = os.environ.get("WL", "big13")
reps = int(os.environ.get("REPS", "5"))
t = open("tests/golden/data/mseq-big13-example.txt", "rb").read()
pxy, pgap, g = seqalign.parse_input(t)
libs = sys.argv[1:] or [os.path.dirname(seqalign.LIB_PATH)]
for d in libs * int(os.environ.get("ROUNDS", "1")):
    seqalign._lib = None
    seqalign.load_library(os.path.join(d, "libnwk.so"))
    e = seqalign.Engine(device=0, verbose=int(os.environ.get("V", "0")))
    e.set_sequences(g)
    ids = np.arange(78, dtype=np.int64)
    ks, ws = [], []
    for r in range(reps):
        aff = os.environ.get("AFF")  # "go,ge": affine variant (no golden check unless go == 0, ge == pgap)
        t0 = time.perf_counter()
        if aff:
            go, ge = (int(v) for v in aff.split(","))
            pen, hs = e.align_pairs_affine(ids, pxy, go, ge)
        else:
            pen, hs = e.align_pairs(ids, pxy, pgap)
        ws.append(time.perf_counter() - t0)
        if (not aff or aff == "0,%d" % pgap) and not os.environ.get("NWK_NOTRACE"):
            assert seqalign.chain_hash(hs) == GOLD, "big13 hash mismatch"
        ks.append(e.stats()["fill_ms"])
    e.close()
    print("timeit %-40s kernel ms min %.2f med %.2f | wall ms min %.2f med %.2f" % (d, min(ks), sorted(ks)[len(ks)//2], 1e3*min(ws), 1e3*sorted(ws)[len(ws)//2]), flush=True)
