"""big13's span-critical pairs vs the rest, each set timed alone (feasibility
of running them as two concurrent launches on disjoint CUs).

Critical = the pairs whose column-kernel span (n + 100 x bands) is >= 0.7 x the
longest (the runtime's issue-priority rule).  Env knobs of the run apply
(NWK_BPC=1: one 4-wave block per CU, i.e. one fill wave per SIMD;
NWK_CU_RESERVE=r: the engine's stream on all but r CUs).  Every penalty is
checked against the published answer.

usage: python tools/big13_split.py crit|rest|all [reps=3]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
import numpy as np  # noqa: E402

import seqalign  # noqa: E402
import workloads  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "all"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
text = open(os.path.join(REPO, "tests", "golden", "data", "mseq-big13-example.txt"), "rb").read()
pxy, pgap, genes = seqalign.parse_input(text)
gold = {c["name"]: c for c in json.load(open(os.path.join(REPO, "tests", "golden", "golden.json")))["cases"]}["big13"]
k = len(genes)
ids, span = [], []
p = 0
for i in range(1, k):
    for j in range(i):
        m, n = len(genes[i]), len(genes[j])
        ids.append(p)
        span.append(n + 100 * ((m + 2047) // 2048))
        p += 1
ids, span = np.array(ids), np.array(span)
crit = span >= 0.7 * span.max()
sel = ids[crit] if which == "crit" else ids[~crit] if which == "rest" else ids
cells = sum(len(genes[seqalign.pair_ij(int(q))[0]]) * len(genes[seqalign.pair_ij(int(q))[1]]) for q in sel)
with seqalign.Engine(device=0) as e:
    e.set_sequences(genes)
    e.align_pairs(sel[:1], pxy, pgap)
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        pen, _ = e.align_pairs(sel, pxy, pgap)
        best = min(best, time.perf_counter() - t0)
        if [int(v) for v in pen] != [gold["penalties"][int(q)] for q in sel]:
            sys.exit("big13_split: penalties differ from the published answer")
    st = e.stats()
print("big13 %-4s %2d pairs (%.3g cells, spans %d-%d): %.2f ms (fill %.2f ms, mode %s) env BPC=%s CU_RESERVE=%s; "
      "penalties ok" % (which, len(sel), cells, span[np.isin(ids, sel)].min(), span[np.isin(ids, sel)].max(),
                        best * 1e3, st["fill_ms"], seqalign.MODES.get(st["mode"]), os.environ.get("NWK_BPC", "-"),
                        os.environ.get("NWK_CU_RESERVE", "-")), flush=True)
