"""Runs a synthetic k x L all-pairs job (bench.synth) with an optional workspace cap."""
import sys, time
sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
sys.path.insert(0, ".")
import numpy as np
import bench, seqalign
k, L = int(sys.argv[1]), int(sys.argv[2])
ws = int(float(sys.argv[3]) * (1 << 30)) if len(sys.argv) > 3 else 0
genes = bench.synth(k, L)
with seqalign.Engine(device=0, workspace_bytes=ws, verbose=int(__import__("os").environ.get("V", "1"))) as e:
    e.set_sequences(genes)
    t = time.time()
    pen, hs = e.align_pairs(np.arange(k * (k - 1) // 2, dtype=np.int64), 3, 2)
    print("k=%d L=%d ws=%s: %.2f s hash %s pen0 %d" % (k, L, sys.argv[3:] or "auto", time.time() - t,
          seqalign.chain_hash(hs)[:16], pen[0]), e.stats(), flush=True)
