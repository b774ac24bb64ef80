"""Per-rank time of a job LPT-sharded over W ranks, emulated on one GPU, with the
rank-0 hash chain included (tools for DESIGN.md §6).

Each rank's shard runs alone on the GPU (one rank after another), as
dist.align_sharded_pipelined runs it on its own GPU: in C pieces of ascending
canonical ids, piece c+1 aligning (Engine.align_pairs_begin) while piece c's
records would go through their all-gather.  Per rank and piece we record when
the piece's results are ready (best of 3 by the rank's last piece).  Rank 0's
chain (skel:159, a worker thread fed per piece) is then replayed from the
measured per-link cost tau of this host's chain (nwk_chain_hash over P records):
    chain_end = max(chain_end, ready of piece c on every rank) + links(c) * tau
The all-gather of 72-byte records is not emulated (microseconds of transfer).
W = 1 is the single-GPU getMinimumPenalties (align_all: batches with the chain
overlapped), the bench's N=1 step.

usage: [NWK_ST_LIB=lib] python tools/shardtime.py [workload=big13] [--chunks C|auto] [--stream [--hybrid H]] [W ...]   (workload: big13, c3, c4)"""
import os
import sys
import time

sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import numpy as np  # noqa: E402

import dist as nwdist  # noqa: E402
import seqalign  # noqa: E402
import workloads  # noqa: E402

args = sys.argv[1:]
wl = args.pop(0) if args and not args[0].isdigit() and not args[0].startswith("--") else "big13"
chunks_arg = "auto"
stream = "--stream" in args  # one launch per rank, records polled as they stream (dist.align_sharded_streamed)
if stream:
    args.remove("--stream")
hybrid = 0  # --hybrid H: the first H pieces as band tasks (nw_align_bits, pair-major) in a launch of their own beside the strips
if "--hybrid" in args:
    i = args.index("--hybrid")
    hybrid = int(args[i + 1])
    del args[i:i + 2]
if "--chunks" in args:
    i = args.index("--chunks")
    chunks_arg = args[i + 1]
    del args[i:i + 2]
if wl == "big13":
    t = open(os.path.join(workloads.GOLDEN_DATA, "mseq-big13-example.txt"), "rb").read()
    pxy, pgap, g = seqalign.parse_input(t)
else:
    _, k, L, pxy, pgap, _ = workloads.SYNTH[wl]
    g = workloads.synth(k, L)
if os.environ.get("NWK_ST_LIB"):  # A/B: a libnwk.so variant (tools/abv/<name>/libnwk.so)
    seqalign.load_library(os.environ["NWK_ST_LIB"])
lens = [len(s) for s in g]
P = len(g) * (len(g) - 1) // 2
e = seqalign.Engine(device=0)
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
for W in [int(a) for a in args] or [1, 2, 4, 8]:
    if W == 1:
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            e.align_all(pxy, pgap)
            best = min(best, time.perf_counter() - t0)
        t1 = best
        st = e.stats()
        print("%s W=1: align_all %.2f ms (fill %.2f ms, %d batch(es), mode %s)" % (
            wl, best * 1e3, st["fill_ms"], st["batches"], seqalign.MODES.get(st["mode"])), flush=True)
        continue
    if stream and es is None:  # records fused into the fill launch, polled as they stream (dist.align_sharded_streamed)
        e.close()  # (its workspace holds most of the HBM)
        es = seqalign.Engine(device=0, finalize="fused", kernel=os.environ.get("NWK_ST_KERNEL", "auto"),
                             task_order=int(os.environ.get("NWK_ST_ORDER", "0")), workspace_bytes=(100 << 30) if hybrid else 0)
        es.set_sequences(g)
        es.align_pairs(np.arange(min(P, 64), dtype=np.int64), pxy, pgap)
        if hybrid:
            eh = seqalign.Engine(device=0, finalize="fused", kernel="nw_align_bits", task_order=1,
                                 workspace_bytes=60 << 30)
            eh.set_sequences(g)
            eh.align_pairs(np.arange(min(P, 64), dtype=np.int64), pxy, pgap)
    C = nwdist.auto_chunks(P, W) if chunks_arg == "auto" else int(chunks_arg)
    ready = np.zeros((W, C))
    links = np.zeros(C)
    for r in range(W):
        parts, _ = nwdist.chunk_parts(lens, r, W, C)
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            ts = []
            if stream and hybrid:
                ia, ib = np.concatenate(parts[:hybrid]), np.concatenate(parts[hybrid:])
                eh.align_pairs_begin(ia, pxy, pgap)
                es.align_pairs_begin(ib, pxy, pgap)
                bounds = np.cumsum([len(x) for x in parts])
                ga = gb = 0
                for c in range(C):
                    eng, tgt = (eh, bounds[c]) if c < hybrid else (es, bounds[c] - len(ia))
                    while (ga if c < hybrid else gb) < tgt:
                        if c < hybrid:
                            ga, _, _ = eng.align_pairs_poll(ga)
                        else:
                            gb, _, _ = eng.align_pairs_poll(gb)
                        if (ga if c < hybrid else gb) < tgt:
                            time.sleep(50e-6)
                    ts.append(time.perf_counter() - t0)
                eh.align_pairs_end()
                es.align_pairs_end()
            elif stream:
                ids = np.concatenate(parts)
                bounds = np.cumsum([len(x) for x in parts])
                es.align_pairs_begin(ids, pxy, pgap)
                got = 0
                for c in range(C):
                    while got < bounds[c]:
                        got, _, _ = es.align_pairs_poll(got)
                        if got < bounds[c]:
                            time.sleep(50e-6)
                    ts.append(time.perf_counter() - t0)
                es.align_pairs_end()
            else:
                e.align_pairs_begin(parts[0], pxy, pgap)
                for c in range(C):
                    e.align_pairs_end()
                    ts.append(time.perf_counter() - t0)
                    if c + 1 < C:
                        e.align_pairs_begin(parts[c + 1], pxy, pgap)
            if best is None or ts[-1] < best[-1]:
                best = ts
        ready[r] = best
        for c in range(C):
            links[c] += len(parts[c])
    end = 0.0
    for c in range(C):
        end = max(end, ready[:, c].max()) + links[c] * tau
    fill_done = ready[:, -1].max()
    slow = int(np.argmax(ready[:, -1]))
    print("%s W=%d, %d piece(s)%s: slowest rank %d ready at %.2f ms (pieces %s ms); chain ends %.2f ms (exposed %.2f ms)%s"
          % (wl, W, C, (" streamed" + (" (%d band-task)" % hybrid if hybrid else "")) if stream else "", slow, fill_done * 1e3, " ".join("%.2f" % (x * 1e3) for x in ready[slow]), end * 1e3,
             (end - fill_done) * 1e3, "  speedup vs W=1: %.2fx" % (t1 / end) if t1 else ""), flush=True)
