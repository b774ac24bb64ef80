#!/usr/bin/env python3
"""Full-size golden answers for BASELINE configs C3/C4/C5 and the int16-range
edge sets -- written to tests/golden/large/<name>.json, one file per job.

Run in the build container (after oracle/build_ref.sh); each job is
independent and can run concurrently:

    python tests/golden/make_golden_large.py c3        # sub, ~75 min on 8 cores
    python tests/golden/make_golden_large.py c3_pairs  # skel_debug, first 9 seqs (36 pairs)
    python tests/golden/make_golden_large.py c4 c4_pairs
    python tests/golden/make_golden_large.py c4_oracle # oracle, 8 processes, ~25 min (c4.json
                                                       # as committed: sub would take ~9 h)
    python tests/golden/make_golden_large.py edge16    # skel_debug, 4 penalty pairs
    python tests/golden/make_golden_large.py c5_scores # oracle score-only, O(n) memory

Sources of truth:
  * "sub"         oracle/_ref/sub = submit/xuliny-seqalkway.cpp compiled from
                  the reference sources, singleton MPI rank (16 OpenMP threads);
                  the answer hash and the penalties line (sub:57-69, 334-337).
  * "skel_debug"  oracle/_ref/skel_debug = root seqalign-mpi-skeleton.cpp; its
                  debug prints (skel:158-169) give each pair's penalty and
                  problemhash.  The first 9 sequences of a config give exactly
                  its first 36 canonical pairs (i < 9).
  * "oracle score" oracle.score_affine / oracle.score (nw_oracle.c, O(n) memory):
                  C5 has no reference, so its pin is the oracle's
                  restatement of the build-defined recurrence.

Inputs are NOT stored: the GPU tests regenerate them bit-for-bit from
multiple-sequence-alignment-openmp-openmpi_amd/workloads.py (synth) and
tests/golden/gen_inputs.py (edge16).
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, HERE)

import gen_inputs  # noqa: E402
import oracle  # noqa: E402
import workloads  # noqa: E402
from make_golden import run_skel  # noqa: E402

OUT = os.path.join(HERE, "large")


def save(name, entry):
    os.makedirs(OUT, exist_ok=True)
    entry["name"] = name
    with open(os.path.join(OUT, name + ".json"), "w") as f:
        json.dump(entry, f, indent=0)
    print(name, "written", file=sys.stderr)


def run_sub(genes, pxy, pgap):
    text = workloads.token_text(pxy, pgap, genes)
    us, h, pens = oracle.run_cli(os.path.join(oracle.REF_DIR, "sub"), text, timeout=6 * 3600)
    return us, h, pens


def job_full(cfg):
    desc, k, L, pxy, pgap, _ = workloads.SYNTH[cfg]
    genes = workloads.synth(k, L)
    us, h, pens = run_sub(genes, pxy, pgap)
    save(cfg, {"config": desc, "k": k, "L": L, "pxy": pxy, "pgap": pgap, "hash": h, "penalties": pens,
               "source": "oracle/_ref/sub (submit/xuliny-seqalkway.cpp, singleton rank, 16 threads, "
                         "8-core build container): %d us" % us})


def _oracle_pair(args):
    x, y, pxy, pgap = args
    p, a1, a2 = oracle.pair(x, y, pxy, pgap)
    return p, oracle.problem_hash(a1, a2)


def job_full_oracle(cfg, procs=8):
    """The same answer from the C restatement (nw_oracle.c), pair-parallel over
    `procs` processes: for C4, whose 32,640 pairs take sub's singleton rank
    ~1 s each here (120 pairs of the config: 124 s), ~9 h.  The oracle is
    pinned to the reference (golden.json, test_oracle.py), and on this config
    its first 36 per-pair problemhashes must equal skel_debug's (c4_pairs.json)."""
    from multiprocessing import Pool
    desc, k, L, pxy, pgap, _ = workloads.SYNTH[cfg]
    genes = workloads.synth(k, L)
    args = [(genes[i], genes[j], pxy, pgap) for i in range(1, k) for j in range(i)]
    t0 = time.time()
    with Pool(procs) as pool:
        res = pool.map(_oracle_pair, args, chunksize=32)
    pens, hs = [r[0] for r in res], [r[1] for r in res]
    ref = json.load(open(os.path.join(OUT, cfg + "_pairs.json")))
    n = len(ref["pairs"])
    assert [pp["problemhash"] for pp in ref["pairs"]] == hs[:n], "oracle disagrees with skel_debug"
    assert ref["penalties"] == pens[:n], "oracle disagrees with skel_debug"
    save(cfg, {"config": desc, "k": k, "L": L, "pxy": pxy, "pgap": pgap, "hash": oracle.chain(hs),
               "penalties": pens,
               "source": "oracle nw_oracle.c (skel:186-280 restatement), %d processes, %.0f s; first %d "
                         "pairs' problemhashes = skel_debug's (%s_pairs.json). sub's singleton rank needs "
                         "~1 s per 8k pair here (~9 h for the config)" % (procs, time.time() - t0, n, cfg)})


def _skel_pair(args):
    """Pair p = (i, j) of a config through the reference program itself:
    skel_debug on the two-sequence input [genes[j], genes[i]], whose only pair
    (1, 0) has x = genes[i] (rows), y = genes[j] (columns) -- the same DP as
    canonical pair p of the full input (skel:122-130)."""
    p, xi, yj, pxy, pgap = args
    _, pens, pairs = run_skel(workloads.token_text(pxy, pgap, [yj, xi]).decode("latin-1"), debug=True,
                              timeout=3600)
    assert len(pairs) == 1 and pens == [pairs[0]["penalty"]]
    return p, pairs[0]["penalty"], pairs[0]["problemhash"]


def job_full_skel(cfg, procs=6):
    """The full answer from the reference program itself, pair-parallel: every
    canonical pair through skel_debug as a two-sequence job (_skel_pair), then
    the chain of skel:159 over the per-pair problemhashes.  C4 (32,640 pairs of
    8k x 8k, ~0.4 s each for the serial skel) takes ~40 min on 6 processes --
    against ~9 h for sub's singleton rank.  Progress is checkpointed to
    /tmp/<cfg>_skel.jsonl so an interrupted run resumes."""
    from multiprocessing import Pool
    desc, k, L, pxy, pgap, _ = workloads.SYNTH[cfg]
    genes = workloads.synth(k, L)
    P = k * (k - 1) // 2
    ck = "/tmp/%s_skel.jsonl" % cfg
    done = {}
    if os.path.exists(ck):
        for line in open(ck):
            r = json.loads(line)
            done[r[0]] = (r[1], r[2])
    todo = []
    p = 0
    for i in range(1, k):
        for j in range(i):
            if p not in done:
                todo.append((p, genes[i], genes[j], pxy, pgap))
            p += 1
    t0 = time.time()
    with Pool(procs) as pool, open(ck, "a") as f:
        for n, (p, pen, ph) in enumerate(pool.imap_unordered(_skel_pair, todo, chunksize=4)):
            done[p] = (pen, ph)
            f.write(json.dumps([p, pen, ph]) + "\n")
            if n % 500 == 0:
                f.flush()
                print("%s skel: %d/%d pairs, %.0f s" % (cfg, len(done), P, time.time() - t0), file=sys.stderr)
    pens = [done[p][0] for p in range(P)]
    hs = [done[p][1] for p in range(P)]
    h = oracle.chain(hs)
    save(cfg, {"config": desc, "k": k, "L": L, "pxy": pxy, "pgap": pgap, "hash": h, "penalties": pens,
               "source": "oracle/_ref/skel_debug (root seqalign-mpi-skeleton.cpp, the reference's own "
                         "program): every pair as a two-sequence job, %d processes, %.0f s; answer = the "
                         "skel:159 chain over its per-pair problemhashes" % (procs, time.time() - t0)})


def job_pairs(cfg, nseq=9):
    desc, k, L, pxy, pgap, _ = workloads.SYNTH[cfg]
    genes = workloads.synth(nseq, L)
    h, pens, pairs = run_skel(workloads.token_text(pxy, pgap, genes).decode("latin-1"), debug=True,
                              timeout=6 * 3600)
    save(cfg + "_pairs", {"config": desc + " -- first %d sequences (canonical pairs 0..%d)" % (nseq, len(pens) - 1),
                          "k": nseq, "L": L, "pxy": pxy, "pgap": pgap, "hash": h, "penalties": pens, "pairs": pairs,
                          "source": "oracle/_ref/skel_debug (root seqalign-mpi-skeleton.cpp, skel:158-169)"})


def job_edge16():
    cases = []
    for pxy, pgap in gen_inputs.EDGE16_PENALTIES:
        genes = gen_inputs.edge16_genes(pxy, pgap)
        t0 = time.time()
        h, pens, pairs = run_skel(workloads.token_text(pxy, pgap, genes).decode("latin-1"), debug=True,
                                  timeout=6 * 3600)
        cases.append({"pxy": pxy, "pgap": pgap, "lengths": [len(g) for g in genes], "hash": h,
                      "penalties": pens, "pairs": pairs})
        print("edge16", pxy, pgap, "%.0fs" % (time.time() - t0), file=sys.stderr)
    save("edge16", {"cases": cases, "source": "oracle/_ref/skel_debug (root seqalign-mpi-skeleton.cpp)",
                    "generator": "tests/golden/gen_inputs.py edge16_genes"})


def job_c5_scores():
    desc, k, L, pxy, pgap, (go, ge) = workloads.SYNTH["c5"]
    genes = workloads.synth(k, L)
    out = []
    for p, (i, j) in enumerate([(1, 0), (2, 0)]):
        t0 = time.time()
        a = oracle.score_affine(genes[i], genes[j], pxy, go, ge)
        lin = oracle.score(genes[i], genes[j], pxy, pgap)
        out.append({"pair": p, "i": i, "j": j, "affine_penalty": a, "linear_penalty": lin})
        print("c5 pair", p, a, lin, "%.0fs" % (time.time() - t0), file=sys.stderr)
    save("c5_scores", {"config": desc, "pxy": pxy, "pgap": pgap, "go": go, "ge": ge, "scores": out,
                       "source": "oracle nwo_score_affine / nwo_score (O(n)-memory restatement; the "
                                 "affine variant has no reference, SURVEY §8 a9)"})


def _c5_affine_pair(args):
    p, x, y, pxy, go, ge = args
    return p, oracle.score_affine(x, y, pxy, go, ge)


def job_c5_pen(procs=6):
    """All 496 C5 affine penalties (go=3, ge=1) from the oracle's O(n)-memory
    Gotoh scorer (nwo_score_affine), pair-parallel, checkpointed to
    /tmp/c5_pen.jsonl so an interrupted run resumes.  ~2e13 cells: ~1.5-2 h on
    6 processes here.  bench.py --workload c5 checks every penalty of its last
    timed step against this file."""
    from multiprocessing import Pool
    desc, k, L, pxy, pgap, (go, ge) = workloads.SYNTH["c5"]
    genes = workloads.synth(k, L)
    P = k * (k - 1) // 2
    ck = "/tmp/c5_pen.jsonl"
    done = {}
    if os.path.exists(ck):
        for line in open(ck):
            r = json.loads(line)
            done[r[0]] = r[1]
    todo, p = [], 0
    for i in range(1, k):
        for j in range(i):
            if p not in done:
                todo.append((p, genes[i], genes[j], pxy, go, ge))
            p += 1
    t0 = time.time()
    with Pool(procs) as pool, open(ck, "a") as f:
        for p, pen in pool.imap_unordered(_c5_affine_pair, todo, chunksize=1):
            done[p] = pen
            f.write(json.dumps([p, pen]) + "\n")
            f.flush()
            print("c5_pen: %d/%d pairs, %.0f s" % (len(done), P, time.time() - t0), file=sys.stderr)
    pens = [done[p] for p in range(P)]
    ref = json.load(open(os.path.join(OUT, "c5_scores.json")))
    for s in ref["scores"]:
        p = s["i"] * (s["i"] - 1) // 2 + s["j"]
        assert pens[p] == s["affine_penalty"], "c5_pen disagrees with c5_scores.json"
    save("c5_pen", {"config": desc, "k": k, "L": L, "pxy": pxy, "go": go, "ge": ge, "penalties": pens,
                    "source": "oracle nwo_score_affine (O(n)-memory Gotoh restatement; the affine variant "
                              "has no reference, SURVEY §8 a9), %d processes, %.0f s" % (procs, time.time() - t0)})


def main(argv):
    for a in argv or ["c3", "c3_pairs", "c4", "c4_pairs", "edge16", "c5_scores"]:
        if a == "c5_pen":
            job_c5_pen()
            continue
        if a in ("c3", "c4"):
            job_full(a)
        elif a in ("c3_oracle", "c4_oracle"):
            job_full_oracle(a[:2])
        elif a == "c4_skel":
            job_full_skel("c4")
        elif a in ("c3_pairs", "c4_pairs"):
            job_pairs(a[:2])
        elif a == "edge16":
            job_edge16()
        elif a == "c5_scores":
            job_c5_scores()
        else:
            raise SystemExit("unknown job " + a)


if __name__ == "__main__":
    main(sys.argv[1:])
