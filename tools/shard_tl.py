"""Timeline (verbose 2) of one rank's shard: python tools/shard_tl.py W rank [workload=big13]"""
import sys
sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import seqalign, workloads  # noqa: E402
W, r = int(sys.argv[1]), int(sys.argv[2])
wl = sys.argv[3] if len(sys.argv) > 3 else "big13"
if wl == "big13":
    t = open("tests/golden/data/mseq-big13-example.txt", "rb").read()
    pxy, pgap, g = seqalign.parse_input(t)
else:
    _, k, L, pxy, pgap, _ = workloads.SYNTH[wl]
    g = workloads.synth(k, L)
e = seqalign.Engine(device=0, verbose=2)
e.set_sequences(g)
ids = seqalign.shard_pairs([len(s) for s in g], r, W)
for rep in range(2):
    e.align_pairs(ids, pxy, pgap)
