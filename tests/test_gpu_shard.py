"""Full-size answer check of the sharded paths a `bench.py --gpus 8` run takes.

Each of the W ranks' LPT shards runs on the one GPU, one rank after another,
through the same rank-side objects the ranks use (dist.StreamedShard for
jobs of >= 8,192 pairs, dist.PipelinedShard otherwise); the all-gather of
each piece is stood in for by concatenating the ranks' padded record blocks in
rank order (what all_gather_into_tensor returns), and rank 0's chain
(nwk_chain_*) runs over the pieces in order.  The answer hash and every
penalty must equal the reference's (tests/golden/large/c3.json: oracle/_ref/sub;
c4.json: skel_debug), as in sub:305-337, which collects the workers' records
and chains them.
"""
import json
import os

import numpy as np
import pytest

import dist as nwdist
import seqalign
import workloads
from conftest import GOLDEN_DIR

pytestmark = pytest.mark.gpu


def _fixture(name):
    f = os.path.join(GOLDEN_DIR, "large", name + ".json")
    if not os.path.exists(f):
        pytest.fail("fixture %s missing (tests/golden/make_golden_large.py)" % f)
    return json.load(open(f))


def _bench_path(P):
    """What bench.py picks for a sharded linear job: streamed, 16 pieces, fused
    finalize for >= 8,192 pairs; else pipelined with dist.auto_chunks pieces."""
    return (True, 16) if P >= 8192 else (False, nwdist.auto_chunks(P, 8))


@pytest.mark.parametrize("cfg,world", [("c4", 8), ("c3", 8), ("c4", 3)])
def test_sharded_full_size_answer(cfg, world):
    g = _fixture(cfg)
    _, k, L, pxy, pgap, _ = workloads.SYNTH[cfg]
    genes = workloads.synth(k, L)
    lengths = [len(x) for x in genes]
    P = k * (k - 1) // 2
    streamed, chunks = _bench_path(P)
    with seqalign.Engine(device=0, finalize="fused" if streamed else "auto") as eng:
        eng.set_sequences(genes)

        def make(r):
            parts, per = nwdist.chunk_parts(lengths, r, world, chunks)
            if streamed:
                return nwdist.StreamedShard(eng, parts, per, pxy, pgap)
            return nwdist.PipelinedShard(eng, parts, per, pxy, pgap)

        h, pen, _, ready = nwdist.emulate_ranks(make, world, chunks, P)
    assert [int(v) for v in pen] == g["penalties"]
    assert h == g["hash"]
    assert ready.shape == (world, chunks) and np.all(ready > 0)
