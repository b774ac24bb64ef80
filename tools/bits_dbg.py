#!/usr/bin/env python3
"""Debug / bring-up: nw_align_bits against the oracle and the published big13 answer.

    python tools/bits_dbg.py small|multi|big13|all
"""
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import seqalign  # noqa: E402

T0 = time.time()


def log(*a):
    print("[%.2f]" % (time.time() - T0), *a, flush=True)


def check_set(e, genes, pxy, pgap, tag):
    e.set_sequences(genes)
    k = len(genes)
    pen, hs = e.align_pairs(np.arange(k * (k - 1) // 2, dtype=np.int64), pxy, pgap)
    mode = e.stats()["mode"]
    h, opens, ohs = oracle.all_pairs(genes, pxy, pgap)
    bad = [q for q in range(len(opens)) if int(pen[q]) != opens[q] or hs[q].tobytes().hex() != ohs[q]]
    ids = [(i, j) for i in range(1, k) for j in range(i)]
    log(tag, "pxy", pxy, "pgap", pgap, "mode", mode, "pairs", len(opens), "bad", len(bad),
        [(q, ids[q], len(genes[ids[q][0]]), len(genes[ids[q][1]]), int(pen[q]), opens[q]) for q in bad[:6]])
    return len(bad)


def main(what):
    r = random.Random(3)
    fails = 0
    with seqalign.Engine(device=0, kernel="nw_align_bits") as e:
        if what in ("small", "all"):
            for pxy, pgap in [(3, 2), (1, 1), (0, 2), (5, 2), (4, 2), (2, 1), (3, 1), (0, 1), (7, 2)]:
                lens = [1, 2, 5, 31, 32, 33, 63, 64, 65, 100, 300, 700]
                genes = [bytes(r.choice(b"ACGT") for _ in range(L)) for L in lens]
                fails += check_set(e, genes, pxy, pgap, "small")
        if what in ("multi", "all"):
            for pxy, pgap in [(3, 2), (1, 1), (6, 2)]:
                lens = [2047, 2048, 2049, 4100, 5000, 130, 3000]
                base = bytes(r.choice(b"ACGT") for _ in range(5000))
                genes = [bytes(r.choice(b"ACGT") for _ in range(L)) for L in lens]
                genes += [bytes(c if r.random() > 0.05 else r.choice(b"ACGT") for c in base[:4500])]
                fails += check_set(e, genes, pxy, pgap, "multi")
        if what in ("big13", "all"):
            gold = {c["name"]: c for c in json.load(open(os.path.join(REPO, "tests/golden/golden.json")))["cases"]}["big13"]
            pxy, pgap, genes = seqalign.parse_input(open(os.path.join(REPO, "tests/golden/data", gold["file"]), "rb").read())
            e.set_sequences(genes)
            for rep in range(2):
                t0 = time.time()
                h, pen, hs = e.align_all(pxy, pgap)
                st = e.stats()
                bad = [q for q in range(len(pen)) if int(pen[q]) != gold["penalties"][q]]
                log("big13 rep", rep, "%.1f ms" % ((time.time() - t0) * 1e3), "mode", st["mode"], "fill_ms %.2f" % st["fill_ms"],
                    "hash ok", h == gold["hash"], "bad", len(bad), bad[:8])
                fails += len(bad) + (h != gold["hash"])
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "all")
