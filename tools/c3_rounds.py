"""C3 at 8 ranks: where a rank's time goes.

Rank 0's LPT shard of C3 at W = 8 is 252 pairs x 25 bands = 6,300 band tasks
on the column kernel's 5,120 wave slots (5 waves/SIMD): a full round and a
partial one.  This times, on one MI355X with the shard's own engine path
(Engine.align_pairs, best of 3):
  * the whole shard (the rank's fill + walks),
  * its first 204 pairs (5,100 tasks: exactly one round),
  * the other 48 pairs alone (the partial round on an otherwise idle chip),
  * one pair alone (the span: 50k + 25 x ~96 steps, then its walk),
and checks every penalty against tests/golden/large/c3.json.

usage: python tools/c3_rounds.py [W=8]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
import numpy as np  # noqa: E402

import seqalign  # noqa: E402
import workloads  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
_, k, L, pxy, pgap, _ = workloads.SYNTH["c3"]
genes = workloads.synth(k, L)
gold = json.load(open(os.path.join(REPO, "tests", "golden", "large", "c3.json")))["penalties"]
lens = [len(g) for g in genes]
ids = np.sort(seqalign.shard_pairs(lens, 0, W))
with seqalign.Engine(device=0) as e:
    e.set_sequences(genes)
    e.align_pairs(ids[:4], pxy, pgap)  # warm

    def run(sub, what):
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            pen, _ = e.align_pairs(sub, pxy, pgap)
            best = min(best, time.perf_counter() - t0)
            if [int(v) for v in pen] != [gold[int(p)] for p in sub]:
                sys.exit("c3_rounds: %s: penalties differ from c3.json" % what)
        st = e.stats()
        print("%-34s %4d pairs %6d band tasks: %7.2f ms (fill launch %.2f ms); penalties ok" % (
            what, len(sub), 25 * len(sub), best * 1e3, st["fill_ms"]), flush=True)
        return best

    full = run(ids, "rank 0's shard at W=%d" % W)
    r1 = run(ids[:204], "first 204 pairs (one round)")
    r2 = run(ids[204:], "last %d pairs alone" % (len(ids) - 204))
    one = run(ids[:1], "one pair alone")
    print("one round %.2f ms + the partial round's extra %.2f ms = %.2f ms; a lone pair %.2f ms" % (
        r1 * 1e3, (full - r1) * 1e3, full * 1e3, one * 1e3))
