"""Throughput of the progressive SoP MSA (nwk_msa -> nw_profile).

One JSON line per workload.  A workload is k mutants of one random base of
length L (seeded; 2% deletions, 2% insertions, 10% substitutions per position),
pairwise penalties from align_all (untimed), then nwk_msa timed `--reps` times
(best kept).  Reported:

  cells          sum over the k - 1 merges of |X| x |Y| (profile columns)
  fill_ms        the nw_profile launches, one per guide-tree level (HIP events)
  fill_gcups     cells / fill_ms
  e2e_gcups      cells / the whole call (UPGMA, profile build, merges on the host)
  valu_alg       cells x 11 lane-ops / fill time / the 2.4 GHz VALU peak
                 (256 CU x 4 SIMD x 32 lanes): a cell is six v_mad_u32_u24,
                 three adds and two mins
  levels         the guide tree's depth (one launch each); --levels prints
                 each level's merges, band tasks and time (stderr)

usage: python tools/msa_bench.py [--reps R] [--sets k:L,k:L,...] [--levels]
"""
import argparse
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))

import seqalign  # noqa: E402

VALU_PEAK = 256 * 4 * 32 * 2.4e9  # lane-ops/s at the spec clock (MI355X_MICROARCH.md)
OPS_PER_CELL = 11


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sets", default="16:10000,64:5000,8:50000,256:2000")
    ap.add_argument("--pxy", type=int, default=3)
    ap.add_argument("--pgap", type=int, default=2)
    ap.add_argument("--levels", action="store_true")
    args = ap.parse_args()
    sets = [tuple(int(v) for v in s.split(":")) for s in args.sets.split(",")]
    for k, L in sets:
        r = random.Random(1000 * k + L)
        genes = mutants(r, bytes(r.choice(b"ACGT") for _ in range(L)), k)
        with seqalign.Engine(device=0) as e:
            e.set_sequences(genes)
            pen = e.align_all(args.pxy, args.pgap)[1]
            ref = e.msa(args.pxy, args.pgap, pen)  # warm
            best = None
            wall = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                rows, sop = e.msa(args.pxy, args.pgap, pen)
                wall.append(time.perf_counter() - t0)
                if (rows, sop) != ref:
                    raise SystemExit("msa k=%d L=%d: result changed between repeats" % (k, L))
                st = e.stats()
                if best is None or st["total_ms"] < best["total_ms"]:
                    best = st
        if args.levels:
            with seqalign.Engine(device=0, verbose=2) as e:
                e.set_sequences(genes)
                e.msa(args.pxy, args.pgap, pen)
        cells = best["cells"]
        line = {
            "workload": "msa k=%d L=%d" % (k, L),
            "k": k, "L": L, "pxy": args.pxy, "pgap": args.pgap,
            "msa_len": len(ref[0][0]), "sop": ref[1],
            "levels": best["fill_launches"],
            "cells": cells,
            "fill_ms": round(best["fill_ms"], 3),
            "total_ms": round(best["total_ms"], 3),
            "wall_ms_min": round(min(wall) * 1e3, 3),
            "fill_gcups": round(cells / best["fill_ms"] / 1e6, 2) if best["fill_ms"] > 0 else None,
            "e2e_gcups": round(cells / best["total_ms"] / 1e6, 2) if best["total_ms"] > 0 else None,
            "valu_alg": round(cells * OPS_PER_CELL / (best["fill_ms"] * 1e-3) / VALU_PEAK, 4)
            if best["fill_ms"] > 0 else None,
        }
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
