"""Can a collective run while a rank's persistent fill launch holds the GPU?


RCCL's collective kernel on gfx950 (ncclDevKernel_Generic_*) needs 248-256
VGPRs and 37.7 KB of LDS per 256-thread block (librccl's code-object notes).
nw_align_col's persistent launch runs 4 waves/SIMD at <= 128 VGPRs on every CU:
the whole 512-entry register file of every SIMD.  So a collective's block can
only start on a CU that two fill blocks have left.

The probe (tools/probe/rccl_shape.hip) launches a kernel of exactly RCCL's
shape from a side stream and records when its first block starts and its last
block ends.  Measured, per configuration:
  * alone (no fill running): the launch-to-start latency;
  * during C4's 8-rank shard 0 (streamed, 16 pieces, fused finalize -- the
    bench's --gpus 8 path): after each piece's records are in, the collective
    for that piece is launched; its start delay is what the piece's
    all-gather would wait;
  * the same with NWK_CU_RESERVE=r (the fill's stream masked off r CUs, its grid
    sized for the rest);
  * the cost of the reserve on one GPU: C4 align_all (W = 1) with and without it.

usage: python tools/overlap_probe.py [reserve ...]   (default 0 8)"""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
import numpy as np  # noqa: E402

import dist as nwdist  # noqa: E402
import seqalign  # noqa: E402
import workloads  # noqa: E402

rs = ctypes.CDLL(os.path.join(REPO, "tools", "probe", "librccl_shape.so"))
rs.rs_now.restype = ctypes.c_ulonglong
assert rs.rs_init() == 0
BLOCKS, SPIN = 16, 2000  # 16 channels' blocks, ~20 us of work each (LL all-gather of a few KB)


def collective():
    """Launches the RCCL-shaped kernel; returns (start delay, end) in ms after the launch call."""
    buf = (ctypes.c_ulonglong * 4)()
    t0 = time.perf_counter()
    assert rs.rs_launch(BLOCKS, SPIN) == 0
    ts = None
    while True:
        rs.rs_poll(buf)
        if ts is None and buf[2] > 0:
            ts = time.perf_counter()
        if buf[3] == BLOCKS:
            break
    te = time.perf_counter()
    rs.rs_sync()
    return (ts - t0) * 1e3, (te - t0) * 1e3


_, k, L, pxy, pgap, _ = workloads.SYNTH["c4"]
genes = workloads.synth(k, L)
lens = [len(s) for s in genes]
P = k * (k - 1) // 2
gold = json.load(open(os.path.join(REPO, "tests", "golden", "large", "c4.json")))
W, C = 8, 16
reserves = [int(a) for a in sys.argv[1:]] or [0, 8]

alone = [collective() for _ in range(5)]
print("collective alone: start %.3f ms, end %.3f ms (best of 5)" % (min(a[0] for a in alone), min(a[1] for a in alone)),
      flush=True)

out = {"alone_start_ms": min(a[0] for a in alone), "alone_end_ms": min(a[1] for a in alone), "configs": []}
for r in reserves:
    os.environ["NWK_CU_RESERVE"] = str(r)
    # cost on one GPU: C4 align_all (the bench's N = 1 step), answer checked
    e = seqalign.Engine(device=0)
    e.set_sequences(genes)
    e.align_all(pxy, pgap)
    t1 = []
    for _ in range(3):
        t0 = time.perf_counter()
        h, pen, _ = e.align_all(pxy, pgap)
        t1.append((time.perf_counter() - t0) * 1e3)
        assert h == gold["hash"], "C4 answer differs"
    e.close()
    # rank 0 of 8, streamed: collective per piece as its records arrive
    es = seqalign.Engine(device=0, finalize="fused")
    es.set_sequences(genes)
    es.align_pairs(np.arange(64, dtype=np.int64), pxy, pgap)
    best = None
    for _ in range(3):
        parts, per = nwdist.chunk_parts(lens, 0, W, C)
        sh = nwdist.StreamedShard(es, parts, per, pxy, pgap)
        t0 = time.perf_counter()
        sh.start()
        rows = []
        for c in range(C):
            sh.block(c)
            tr = (time.perf_counter() - t0) * 1e3
            s, d = collective()
            rows.append((tr, s, d))
        assert sh.finish() is None
        tend = (time.perf_counter() - t0) * 1e3
        if best is None or tend < best[1]:
            best = (rows, tend)
    es.close()
    rows, tend = best
    cfg = {"reserve": r, "c4_w1_ms": min(t1), "shard0_end_ms": tend,
           "pieces": [{"ready_ms": round(a, 3), "collective_start_ms": round(b, 3), "collective_end_ms": round(c, 3)}
                      for a, b, c in rows]}
    out["configs"].append(cfg)
    print("reserve %d CUs: C4 W=1 align_all %.2f ms; shard 0 of 8 ends %.2f ms" % (r, min(t1), tend), flush=True)
    for c, (a, b, d) in enumerate(rows):
        print("  piece %2d ready %7.3f ms  collective starts +%.3f ms, ends +%.3f ms" % (c, a, b, d), flush=True)
print(json.dumps(out))
