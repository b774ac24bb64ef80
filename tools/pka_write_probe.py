"""One affine job on nw_align_pka for a WRITE_SIZE pass (write
amplification of the packed affine fill).  Prints the job's stored-code bytes
(nwk_stats.matrix_bytes) so the counter can be compared with them.
usage: NWK_BITS_WIN=<w|0> python tools/pka_write_probe.py [k=4] [L=20000]"""
import os
import sys

sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import numpy as np  # noqa: E402

import seqalign  # noqa: E402
import workloads  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
L = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
g = workloads.synth(k, L)
seqalign.load_library(os.environ.get("NWK_LIB", seqalign.LIB_PATH))  # A/B: a tools/build_variant.sh library
e = seqalign.Engine(device=0)
e.set_sequences(g)
P = k * (k - 1) // 2
for rep in range(2):
    e.align_pairs_affine(np.arange(P, dtype=np.int64), 3, 3, 1)
    st = e.stats()
    print("rep %d: mode %d, %d launch(es), window %d, retries %d, stored matrix bytes %.4g, fill %.2f ms" % (
        rep, st["mode"], st["fill_launches"], st["window"], st["window_retries"], st["matrix_bytes"], st["fill_ms"]),
        flush=True)
