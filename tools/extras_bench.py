"""Timings of the rows beyond the hot path: progressive SoP MSA (f3) and the
linear-space traceback (f2) on big13.  Prints one line per measurement."""
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import seqalign  # noqa: E402
from conftest import case_input, load_golden  # noqa: E402


def mutants(r, base, k):
    out = []
    for _ in range(k):
        s = bytearray()
        for ch in base:
            u = r.random()
            if u < 0.02:
                continue
            if u < 0.04:
                s.append(r.choice(b"ACGT"))
            s.append(r.choice(b"ACGT") if r.random() < 0.1 else ch)
        out.append(bytes(s))
    return out


def main():
    r = random.Random(1)
    with seqalign.Engine(device=0) as e:
        for k, L in ((16, 10000), (64, 5000), (8, 50000)):
            genes = mutants(r, bytes(r.choice(b"ACGT") for _ in range(L)), k)
            e.set_sequences(genes)
            pen = e.align_all(3, 2)[1]
            e.msa(3, 2, pen)  # warm
            t0 = time.perf_counter()
            rows, sop = e.msa(3, 2, pen)
            dt = time.perf_counter() - t0
            print("msa k=%d L=%d: %.1f ms, MSA length %d, SoP %d" % (k, L, dt * 1e3, len(rows[0]), sop), flush=True)
    big = next(c for c in load_golden() if c["name"] == "big13")
    pxy, pgap, genes = case_input(big)
    ids = list(range(len(genes) * (len(genes) - 1) // 2))
    for g in (0, 16, 64):
        with seqalign.Engine(device=0, linear_space=g if g else -1) as e:
            e.set_sequences(genes)
            e.align_pairs(ids, pxy, pgap)
            t0 = time.perf_counter()
            pen, hs = e.align_pairs(ids, pxy, pgap)
            dt = time.perf_counter() - t0
            st = e.stats()
            ok = seqalign.chain_hash(hs) == big["hash"]
            print("big13 linear_space=%s: %.1f ms wall, fill %.1f ms, traceback %.1f ms, matrix %.2f GB, hash %s"
                  % (g if g else "off", dt * 1e3, st["fill_ms"], st["traceback_ms"], st["matrix_bytes"] / 1e9,
                     "ok" if ok else "WRONG"), flush=True)


if __name__ == "__main__":
    main()
