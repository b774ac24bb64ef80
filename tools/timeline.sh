cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python3 - <<'PY' 2>&1 | tail -90
import sys, os
sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import numpy as np, seqalign
t = open("tests/golden/data/mseq-big13-example.txt","rb").read()
pxy, pgap, g = seqalign.parse_input(t)
e = seqalign.Engine(device=0, verbose=2)
e.set_sequences(g)
ids = np.arange(78, dtype=np.int64)
e.align_pairs(ids, pxy, pgap)
e.align_pairs(ids, pxy, pgap)
PY
