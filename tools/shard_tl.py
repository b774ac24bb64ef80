"""Timeline (verbose 2) of one rank's big13 shard: python tools/shard_tl.py W rank"""
import os, sys
sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import numpy as np
import seqalign
W, r = int(sys.argv[1]), int(sys.argv[2])
t = open("tests/golden/data/mseq-big13-example.txt", "rb").read()
pxy, pgap, g = seqalign.parse_input(t)
e = seqalign.Engine(device=0, verbose=2)
e.set_sequences(g)
ids = seqalign.shard_pairs([len(s) for s in g], r, W)
for rep in range(2):
    e.align_pairs(ids, pxy, pgap)
