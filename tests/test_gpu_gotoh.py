"""GPU parity of nw_align_gotoh (csrc/nwk_gotoh.hip): the affine variant
(build-defined; oracle/nw_oracle.c nwo_pair_affine is the
restatement it must equal) as bit-sliced thermometer planes with a fused
device walk.

Bar: bit-exact penalties, per-pair problemhashes and alignment strings against
the oracle, for every instantiated scoring; pairs crossing the 2048-row bands,
32-column chunks and 256-move output blocks; windowed storage with forced
window exits (the pair re-runs wider); several batches; the device finalize.
For go > 0 parity is unpinned by the reference (it has no affine path); the
degenerate go = 0, ge = pgap reproduces the reference's linear vectors
(test_gpu.py::test_affine_degenerate_golden, big13 included, runs here by
default).
"""
import json
import os
import random
import subprocess
import sys

import numpy as np
import pytest

import oracle
import seqalign

pytestmark = pytest.mark.gpu

ACGT = b"ACGT"
# (pxy, go, ge) instantiated in nwk_gotoh.hip (kGotohSet)
SCORINGS = [(3, 3, 1), (3, 0, 2), (5, 0, 1), (3, 0, 1), (3, 4, 1), (1, 2, 2), (2, 1, 1), (4, 2, 2), (4, 2, 1),
            (2, 4, 2), (3, 5, 2), (9, 3, 2)]


@pytest.fixture(scope="module")
def gengine():
    if seqalign.device_count() < 1:
        pytest.fail("no HIP device visible for a -m gpu run")
    e = seqalign.Engine(device=0, kernel="nw_align_gotoh")
    yield e
    e.close()


def _ids(k):
    return np.arange(k * (k - 1) // 2, dtype=np.int64)


def _mutants(r, base, k, alpha):
    out = []
    for _ in range(k):
        s = bytearray()
        for c in base:
            u = r.random()
            if u < 0.03:
                continue
            if u < 0.06:
                s.append(r.choice(alpha))
            s.append(r.choice(alpha) if r.random() < 0.1 else c)
        out.append(bytes(s))
    return out


def _genes(seed):
    r = random.Random(seed)
    lens = [1, 2, 31, 33, 255, 257, 2047, 2048, 2049, 4100, r.randint(300, 3000), r.randint(3000, 6000)]
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in lens]
    genes += _mutants(r, bytes(r.choice(ACGT) for _ in range(2500)), 2, ACGT)
    genes.append(bytes(r.choice(b"AC") for _ in range(1500)))  # two symbols: many ties between the states
    return genes


@pytest.mark.parametrize("pxy,go,ge", SCORINGS)
def test_gotoh_vs_oracle(gengine, pxy, go, ge):
    genes = _genes(9000 + 100 * pxy + 10 * go + ge)
    gengine.set_sequences(genes)
    pen, hs = gengine.align_pairs_affine(_ids(len(genes)), pxy, go, ge)
    assert gengine.stats()["mode"] == 11, "nw_align_gotoh expected"
    h, opens, ohs = oracle.all_pairs_affine(genes, pxy, go, ge)
    assert [int(v) for v in pen] == opens
    assert [x.tobytes().hex() for x in hs] == ohs
    assert seqalign.chain_hash(hs) == h


@pytest.mark.parametrize("m,n", [(1, 1), (1, 3000), (3000, 1), (2048, 2048), (2049, 700), (700, 4097), (4500, 4500)])
def test_gotoh_single_pair_strings(m, n):
    r = random.Random(m * 7 + n)
    x = bytes(r.choice(ACGT) for _ in range(m))
    y = bytes(r.choice(ACGT) for _ in range(n)) if m != n else _mutants(r, x, 1, ACGT)[0]
    with seqalign.Engine(device=0, kernel="nw_align_gotoh") as e:
        for pxy, go, ge in ((3, 3, 1), (2, 4, 2), (3, 0, 2)):
            assert e.get_minimum_penalty_affine(x, y, pxy, go, ge) == oracle.pair_affine(x, y, pxy, go, ge)
            assert e.stats()["mode"] == 11


def test_gotoh_auto_choice_and_fallback(gengine):
    """Under "auto" the instantiated scorings take nw_align_gotoh; others (or
    more than four symbols) fall back to nw_align_pka / nw_align_affine."""
    r = random.Random(77)
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in (300, 900, 1200)]
    with seqalign.Engine(device=0) as e:
        e.set_sequences(genes)
        for (pxy, go, ge), mode in (((3, 3, 1), 11), ((4, 10, 1), 3), ((5, 0, 0), 7), ((6, 1, 1), 7)):
            pen, _ = e.align_pairs_affine(_ids(3), pxy, go, ge)
            assert e.stats()["mode"] == mode, (pxy, go, ge)
            assert [int(v) for v in pen] == oracle.all_pairs_affine(genes, pxy, go, ge)[1]
        genes5 = genes + [b"ACGTN" * 50]
        e.set_sequences(genes5)
        pen, _ = e.align_pairs_affine(_ids(4), 3, 3, 1)
        assert e.stats()["mode"] != 11
        assert [int(v) for v in pen] == oracle.all_pairs_affine(genes5, 3, 3, 1)[1]


_WIN_SCRIPT = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import seqalign
genes = [bytes.fromhex(g) for g in json.loads(sys.stdin.read())]
k = len(genes)
out = []
for pxy, go, ge in ((3, 3, 1), (4, 2, 2)):
    for fin in ("host", "device"):
        with seqalign.Engine(device=0, workspace_bytes=int(sys.argv[2]), kernel="nw_align_gotoh", finalize=fin) as e:
            e.set_sequences(genes)
            pen, hs = e.align_pairs_affine(np.arange(k * (k - 1) // 2, dtype=np.int64), pxy, go, ge)
            st = e.stats()
        out.append({"mode": st["mode"], "batches": st["batches"], "retries": st["window_retries"],
                    "window": st["window"], "pen": [int(v) for v in pen], "hs": [x.tobytes().hex() for x in hs]})
print(json.dumps(out))
"""


@pytest.mark.parametrize("win", ["auto", "40", "600", "2000"])
def test_gotoh_windowed_storage_and_rerun(win):
    """Windowed storage: band b stores only the 4-step blocks gotoh_blk_lo(b) ..
    + nblk around the diagonal; a walk that leaves them flags the pair and it
    re-runs in full.  Ragged multi-band pairs, mutated copies and swapped halves
    (paths ~3000 columns off the diagonal), in a workspace too small for full
    storage (several batches); host and device finalize; bit-exact vs the oracle
    for any W."""
    r = random.Random(6161)
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in (900, 2600, 4100, 5200)]
    genes += _mutants(r, bytes(r.choice(ACGT) for _ in range(4500)), 2, ACGT)
    P, Q = (bytes(r.choice(ACGT) for _ in range(3000)) for _ in range(2))
    genes += [P + Q, Q + P]
    env = dict(os.environ, **({} if win == "auto" else {"NWK_BITS_WIN": win}))
    res = subprocess.run([sys.executable, "-c", _WIN_SCRIPT, os.path.dirname(seqalign.__file__), str(60 << 20)],
                         input=json.dumps([g.hex() for g in genes]).encode(), env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert res.returncode == 0, res.stderr.decode()[-2000:]
    out = json.loads(res.stdout.decode().strip().splitlines()[-1])
    for (pxy, go, ge), o in zip(((3, 3, 1), (3, 3, 1), (4, 2, 2), (4, 2, 2)), out):
        assert o["mode"] == 11, "nw_align_gotoh expected"
        _, opens, ohs = oracle.all_pairs_affine(genes, pxy, go, ge)
        assert o["pen"] == opens
        assert o["hs"] == ohs
        if win == "40":
            assert o["retries"] > 0, "a 40-column window must send some pairs to the re-run"
        if win == "auto":
            assert o["batches"] >= 2, "the 60 MiB workspace must take several batches"


def test_gotoh_align_all_chain(gengine):
    """nwk_align_all_affine (chain of skel:159 over the pairs) on the gotoh path."""
    genes = _genes(4242)[:9]
    gengine.set_sequences(genes)
    h, pen, hs = gengine.align_all(3, None, affine=(3, 1))
    oh, opens, _ = oracle.all_pairs_affine(genes, 3, 3, 1)
    assert h == oh and [int(v) for v in pen] == opens
