"""Per-rank time of a job LPT-sharded over W ranks, emulated on one GPU, with the
rank-0 hash chain included (tools for DESIGN.md §6).

Each rank's shard runs alone on the GPU (one rank after another) through the
rank-side object the ranks use (dist.emulate_ranks): dist.PipelinedShard, or
with --stream dist.StreamedShard (one launch per rank, records polled as they
stream out of the fused finalize).  Per rank and piece we record when the
piece's results are ready (best of 3 by the rank's last piece).  Every run's
gathered answer -- the blocks of all ranks concatenated in rank order, as the
all-gather returns them, then chained -- must equal the reference's (c3/c4:
tests/golden/large/<wl>.json, big13: the published answer) before a time is
printed.  Rank 0's chain (skel:159) is then replayed from the measured
per-link cost tau of this host's chain (nwk_chain_hash over P records):
    chain_end = max(chain_end, ready of piece c on every rank) + links(c) * tau
The exchange: streamed pieces reach rank 0 through node shared memory as they
are ready (dist.NodeRecords), and one all-gather (AG_S) follows the last rank's
launch; the alternative of one RCCL all-gather per piece is replayed too, with
no piece exchanged before every rank's launch has drained (an RCCL kernel cannot
start while the persistent fill holds the GPU, profiles/r05/overlap).
W = 1 is the single-GPU getMinimumPenalties (align_all: batches with the chain
overlapped), the bench's N=1 step.

--records (with --stream): no pieces -- each rank's launch is polled in a tight
loop and every record's ready time is the moment its rank's ready prefix
(Engine.align_pairs_poll) covered it; the chain is replayed per record in
canonical order,  chain_end = max(chain_end, ready(p)) + tau  (the bound of a
chain that consumes each record as soon as it exists: dist.RecordStream).

usage: [NWK_ST_LIB=lib] python tools/shardtime.py [workload=big13] [--chunks C|auto] [--stream [--records]] [W ...]   (workload: big13, c3, c4)"""
import json
import os
import sys
import time

sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import numpy as np  # noqa: E402

import dist as nwdist  # noqa: E402
import seqalign  # noqa: E402
import workloads  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")

args = sys.argv[1:]
wl = args.pop(0) if args and not args[0].isdigit() and not args[0].startswith("--") else "big13"
chunks_arg = "auto"
stream = "--stream" in args
if stream:
    args.remove("--stream")
records = "--records" in args
if records:
    args.remove("--records")
    stream = True
if "--chunks" in args:
    i = args.index("--chunks")
    chunks_arg = args[i + 1]
    del args[i:i + 2]
if wl == "big13":
    t = open(os.path.join(workloads.GOLDEN_DATA, "mseq-big13-example.txt"), "rb").read()
    pxy, pgap, g = seqalign.parse_input(t)
    gold = {c["name"]: c for c in json.load(open(os.path.join(GOLDEN, "golden.json")))["cases"]}["big13"]
else:
    _, k, L, pxy, pgap, _ = workloads.SYNTH[wl]
    g = workloads.synth(k, L)
    gold = json.load(open(os.path.join(GOLDEN, "large", wl + ".json")))
if os.environ.get("NWK_ST_LIB"):  # A/B: a libnwk.so variant (tools/abv/<name>/libnwk.so)
    seqalign.load_library(os.environ["NWK_ST_LIB"])
lens = [len(s) for s in g]
P = len(g) * (len(g) - 1) // 2


def check(h, pen, what):
    if h != gold["hash"] or [int(v) for v in pen] != gold["penalties"]:
        sys.exit("shardtime: %s: the gathered answer differs from %s" % (what, gold.get("source", "the golden")))


KERNEL = os.environ.get("NWK_ST_KERNEL", "auto")  # e.g. nw_align_col
e = seqalign.Engine(device=0, kernel=KERNEL)
e.set_sequences(g)
e.align_pairs(np.arange(P, dtype=np.int64), pxy, pgap)  # warm

# host chain cost per link (the chain thread's work: schedule + 3 compressions)
rnd = np.random.RandomState(0).randint(0, 256, size=(P, 64)).astype(np.uint8)
tau = min((lambda: (lambda t0: (seqalign.chain_hash(rnd), time.perf_counter() - t0)[1])(time.perf_counter()))()
          for _ in range(3)) / max(P, 1)
print("%s: %d pairs; host chain %.1f ns per link (%.2f ms for all %d links)" % (wl, P, tau * 1e9, tau * P * 1e3, P),
      flush=True)

es = None
t1 = None
# one small all-gather (72-B records of a piece or shard, 8 ranks over xGMI):
# launch to completion of an RCCL-shaped kernel on an idle GPU was 0.08 ms
# (profiles/r05/overlap); the transfer is kilobytes
AG_S = float(os.environ.get("NWK_ST_AG_MS", "0.1")) * 1e-3
for W in [int(a) for a in args] or [1, 2, 4, 8]:
    if W == 1:
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            h, pen, _ = e.align_all(pxy, pgap)
            best = min(best, time.perf_counter() - t0)
            check(h, pen, "W=1")
        t1 = best
        st = e.stats()
        print("%s W=1: align_all %.2f ms (fill %.2f ms, %d batch(es), mode %s); answer ok" % (
            wl, best * 1e3, st["fill_ms"], st["batches"], seqalign.MODES.get(st["mode"])), flush=True)
        continue
    if stream and es is None:  # records fused into the fill launch (dist.StreamedShard)
        e.close()  # (its workspace holds most of the HBM)
        es = seqalign.Engine(device=0, finalize="fused", kernel=KERNEL,
                             task_order=int(os.environ.get("NWK_ST_ORDER", "0")))
        es.set_sequences(g)
        es.align_pairs(np.arange(min(P, 64), dtype=np.int64), pxy, pgap)
    eng = es if stream else e
    if records:
        best = None
        for _ in range(3):
            shards = [seqalign.shard_pairs(lens, r, W) for r in range(W)]
            ready_p = np.zeros(P)
            first = []
            chain = seqalign.ChainStream(P)
            try:
                for r in range(W):
                    ids = np.sort(shards[r])
                    n = len(ids)
                    t0 = time.perf_counter()
                    eng.align_pairs_begin(ids, pxy, pgap)
                    got = 0
                    while got < n:
                        u, p_, h_ = eng.align_pairs_poll(got)
                        if u > got:
                            t = time.perf_counter() - t0
                            if got == 0:
                                first.append(t)
                            ready_p[ids[got:u]] = t
                            chain.feed(ids[got:u], p_, h_)
                            got = u
                    eng.align_pairs_end()
                h, pen, _ = chain.finish()
            finally:
                chain.close()
            check(h, pen, "W=%d records" % W)
            end = 0.0
            for p in range(P):  # (the replay: each record chained as soon as it is ready)
                end = max(end, ready_p[p]) + tau
            if best is None or end < best[0]:
                best = (end, ready_p.copy(), list(first))
        end, ready_p, first = best
        q = [ready_p[:max(1, P * f // 16)].max() * 1e3 for f in (1, 2, 4, 8, 16)]
        crit = int(np.argmax(ready_p + (P - np.arange(P)) * tau))
        print("%s W=%d records streamed: first record per rank %s ms; canonical prefix 1/16, 1/8, 1/4, 1/2, all "
              "ready by %s ms; chain ends %.2f ms (critical record %d ready at %.2f ms + %d links)%s; answer ok" % (
                  wl, W, " ".join("%.2f" % (x * 1e3) for x in first), " ".join("%.2f" % x for x in q), end * 1e3,
                  crit, ready_p[crit] * 1e3, P - crit, "  speedup vs W=1: %.2fx" % (t1 / end) if t1 else ""),
              flush=True)
        continue
    C = (16 if stream else nwdist.auto_chunks(P, W)) if chunks_arg == "auto" else int(chunks_arg)

    def make(r):
        parts, per = nwdist.chunk_parts(lens, r, W, C)
        if stream:
            return nwdist.StreamedShard(eng, parts, per, pxy, pgap)
        return nwdist.PipelinedShard(eng, parts, per, pxy, pgap)

    ready = None
    for _ in range(3):
        h, pen, _, rd = nwdist.emulate_ranks(make, W, C, P)
        check(h, pen, "W=%d" % W)
        ready = rd if ready is None else np.where((rd[:, -1] < ready[:, -1])[:, None], rd, ready)
    links = np.zeros(C)
    for r in range(W):
        parts, _ = nwdist.chunk_parts(lens, r, W, C)
        for c in range(C):
            links[c] += len(parts[c])
    # pieces reach rank 0 as they are ready (node shared memory, dist.NodeRecords:
    # microseconds), then ONE all-gather once every rank's launch has drained
    end = 0.0
    for c in range(C):
        end = max(end, ready[:, c].max()) + links[c] * tau
    fill_done = ready[:, -1].max()
    end = max(end, fill_done + AG_S)
    # one RCCL all-gather per piece instead: an RCCL kernel cannot start while a
    # rank's persistent fill launch holds the GPU (profiles/r05/overlap), so no
    # piece is exchanged before that rank's launch has drained (its last piece)
    end_rccl = 0.0
    for c in range(C):
        end_rccl = max(end_rccl, max(ready[r, c] if not stream else ready[r, -1] for r in range(W)) + AG_S) + links[c] * tau
    slow = int(np.argmax(ready[:, -1]))
    print("%s W=%d, %d piece(s)%s: slowest rank %d ready at %.2f ms (pieces %s ms); chain ends %.2f ms (exposed %.2f ms)%s;"
          " with an RCCL all-gather per piece %.2f ms%s; answer ok" % (
              wl, W, C, " streamed" if stream else "", slow, fill_done * 1e3,
              " ".join("%.2f" % (x * 1e3) for x in ready[slow]), end * 1e3, (end - fill_done) * 1e3,
              "  speedup vs W=1: %.2fx" % (t1 / end) if t1 else "", end_rccl * 1e3,
              " (%.2fx)" % (t1 / end_rccl) if t1 else ""), flush=True)
