"""overlap_probe.py, one configuration per process: is a side-stream kernel
held back by the persistent fill's CU occupancy, and does NWK_CU_RESERVE (or
more hardware queues, GPU_MAX_HW_QUEUES) free it?  C4's rank 0 of 8
(streamed, fused finalize) starts; 2 ms later one kernel is launched from a
side stream: a one-wave tiny kernel, or RCCL's collective shape with 2 or 16
blocks (tools/probe/rccl_shape.hip).  Prints the launch-to-start and
launch-to-end delays (ms) and when the shard's launch ended.

usage: [NWK_CU_RESERVE=r] [GPU_MAX_HW_QUEUES=q] python tools/overlap_probe2.py"""
import ctypes
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
import numpy as np  # noqa: E402

import dist as nwdist  # noqa: E402
import seqalign  # noqa: E402
import workloads  # noqa: E402

_, k, L, pxy, pgap, _ = workloads.SYNTH["c4"]
genes = workloads.synth(k, L)
lens = [len(s) for s in genes]
es = seqalign.Engine(device=0, finalize="fused")  # (created first: its stream is the first queue)
rs = ctypes.CDLL(os.path.join(REPO, "tools", "probe", "librccl_shape.so"))
assert rs.rs_init() == 0
es.set_sequences(genes)
es.align_pairs(np.arange(64, dtype=np.int64), pxy, pgap)


def side(blocks, spin):
    buf = (ctypes.c_ulonglong * 4)()
    t0 = time.perf_counter()
    assert rs.rs_launch(blocks, spin) == 0
    ts = None
    while True:
        rs.rs_poll(buf)
        if ts is None and buf[2] > 0:
            ts = time.perf_counter()
        if buf[3] == blocks:
            break
    te = time.perf_counter()
    rs.rs_sync()
    return round((ts - t0) * 1e3, 3), round((te - t0) * 1e3, 3)


res = {"reserve": int(os.environ.get("NWK_CU_RESERVE", "0")), "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default"),
       "alone": {n: side(b, s) for n, (b, s) in {"tiny": (1, -1), "rccl2": (2, 2000), "rccl16": (16, 2000)}.items()}}
for name, (b, s) in {"tiny": (1, -1), "rccl2": (2, 2000), "rccl16": (16, 2000)}.items():
    rows = []
    for _ in range(3):
        parts, per = nwdist.chunk_parts(lens, 0, 8, 16)
        sh = nwdist.StreamedShard(es, parts, per, pxy, pgap)
        t0 = time.perf_counter()
        sh.start()
        time.sleep(0.002)
        ts = (time.perf_counter() - t0) * 1e3
        d = side(b, s)
        for c in range(16):
            sh.block(c)
        assert sh.finish() is None
        rows.append({"launched_ms": round(ts, 3), "start_delay_ms": d[0], "end_delay_ms": d[1],
                     "shard_end_ms": round((time.perf_counter() - t0) * 1e3, 3)})
    res[name] = rows
print(json.dumps(res))
