"""GPU parity: the HIP path through the C-ABI against golden vectors and the oracle.

Bar: bit-exact (penalties, per-pair problemhash, alignment strings, answer
hash) -- this is integer/byte work.  Full-size inputs (big13 and its
permutation, 2.785e11 cells each) are checked against the reference's
published answers.
"""
import os
import random
import subprocess

import numpy as np
import pytest

import oracle
import seqalign
from conftest import GOLDEN_DIR, PKG, case_input, load_golden

pytestmark = pytest.mark.gpu

GOLDEN = load_golden()


@pytest.fixture(scope="module")
def engine():
    if seqalign.device_count() < 1:
        pytest.fail("no HIP device visible for a -m gpu run")
    e = seqalign.Engine(device=0)
    yield e
    e.close()


def _all_ids(k):
    return np.arange(k * (k - 1) // 2, dtype=np.int64)


@pytest.mark.parametrize("case", GOLDEN, ids=[c["name"] for c in GOLDEN])
def test_golden_cases(engine, case):
    pxy, pgap, genes = case_input(case)
    engine.set_sequences(genes)
    k = len(genes)
    pen, hs = engine.align_pairs(_all_ids(k), pxy, pgap)
    assert [int(v) for v in pen] == case["penalties"]
    if "pairs" in case:
        assert [h.tobytes().hex() for h in hs] == [p["problemhash"] for p in case["pairs"]]
    assert seqalign.chain_hash(hs) == case["hash"]


def _rand_genes(r, k, lo, hi, alpha):
    return [bytes(r.choice(alpha) for _ in range(r.randint(lo, hi))) for _ in range(k)]


def _mutants(r, base, k, alpha):
    out = []
    for _ in range(k):
        s = bytearray()
        for c in base:
            u = r.random()
            if u < 0.02:
                continue
            if u < 0.04:
                s.append(r.choice(alpha))
            s.append(r.choice(alpha) if r.random() < 0.1 else c)
        out.append(bytes(s))
    return out


PENALTIES = [(3, 2), (5, 1), (0, 0), (1, 0), (0, 1), (2, 7), (11, 2), (100, 70), (-1, 2), (3, -1), (-2, -3),
             (40000, 30000)]
ACGT = b"ACGT"


@pytest.mark.parametrize("pxy,pgap", PENALTIES)
def test_random_vs_oracle_penalties(engine, pxy, pgap):
    r = random.Random(hash((pxy, pgap)) & 0xffff)
    genes = _rand_genes(r, 6, 1, 700, ACGT) + _mutants(r, bytes(r.choice(ACGT) for _ in range(650)), 3, ACGT)
    engine.set_sequences(genes)
    pen, hs = engine.align_pairs(_all_ids(len(genes)), pxy, pgap)
    h, opens, ohs = oracle.all_pairs(genes, pxy, pgap)
    assert [int(v) for v in pen] == opens
    assert [x.tobytes().hex() for x in hs] == ohs


@pytest.mark.parametrize("bits", [4, 8, 16, 32])
@pytest.mark.parametrize("alpha", [b"ACGT", b"AC", b"ACGTNacgtn_*"])
def test_forced_widths_and_alphabets(bits, alpha):
    r = random.Random(bits * 7 + len(alpha))
    # lengths straddle the 64-column chunk and 512-row band boundaries
    lens = [1, 2, 63, 64, 65, 511, 512, 513, 1100]
    genes = [bytes(r.choice(alpha) for _ in range(L)) for L in lens]
    with seqalign.Engine(device=0, bits=bits) as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(_all_ids(len(genes)), 3, 2)
        st = e.stats()
    assert st["bits"] == bits
    _, opens, ohs = oracle.all_pairs(genes, 3, 2)
    assert [int(v) for v in pen] == opens
    assert [x.tobytes().hex() for x in hs] == ohs


BITS_PENALTIES = [(p, 2) for p in range(0, 6)] + [(p, 1) for p in range(0, 4)] + [(9, 2), (7, 1)]


@pytest.mark.parametrize("pxy,pgap", BITS_PENALTIES)
def test_bits_kernel_every_mismatch_level(pxy, pgap):
    """nw_align_bits (csrc/nwk_bits.hip) at every thermometer level of the
    mismatch score SR = 2 pgap - pxy (clamped to [-1, 2 pgap]), on lengths that
    straddle its 32-row lane words, 2048-row bands and 64-column chunks, plus
    mutated copies (paths off the diagonal); bit-exact against the oracle."""
    r = random.Random(pxy * 31 + pgap)
    lens = [1, 31, 33, 2047, 2048, 2049, 4200]
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in lens]
    genes += _mutants(r, bytes(r.choice(ACGT) for _ in range(3000)), 2, ACGT)
    with seqalign.Engine(device=0, kernel="nw_align_bits") as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(_all_ids(len(genes)), pxy, pgap)
        assert e.stats()["mode"] == 8, "nw_align_bits expected"
    _, opens, ohs = oracle.all_pairs(genes, pxy, pgap)
    assert [int(v) for v in pen] == opens
    assert [x.tobytes().hex() for x in hs] == ohs


def _strip_pairs(ncols, k):
    """Canonical ids of the pairs whose column sequence is one of the first
    ncols genes (strips need n in range; rows can be anything)."""
    return np.array([seqalign.pair_index(i, j) for i in range(1, k) for j in range(min(i, ncols))],
                    dtype=np.int64)


@pytest.mark.parametrize("pxy,pgap", BITS_PENALTIES)
def test_strip_kernel_every_mismatch_level(pxy, pgap):
    """nw_align_strip (rolling strips: one wave sweeps every 2048-row pass of
    a pair, csrc/nwk_bits.hip) at every mismatch level SR, forced
    (kernel="nw_align_strip"): column lengths at the n' = n + 32 edge (4064 ->
    4096) and just past the smallest admissible n' (4001), rows of one row, a
    lane word, one pass exactly, one row past a pass, a ragged two-pass strip;
    bit-exact against the oracle."""
    r = random.Random(pxy * 37 + pgap)
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in (4001, 4064, 1, 33, 2048, 2049, 4100)]
    ids = _strip_pairs(2, len(genes))
    with seqalign.Engine(device=0, kernel="nw_align_strip") as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(ids, pxy, pgap)
        assert e.stats()["mode"] == 9, "nw_align_strip expected"
    _, opens, ohs = oracle.all_pairs(genes, pxy, pgap)
    assert [int(v) for v in pen] == [opens[i] for i in ids]
    assert [x.tobytes().hex() for x in hs] == [ohs[i] for i in ids]


@pytest.mark.parametrize("pxy,pgap", [(3, 2), (5, 1)])
def test_strip_kernel_multi_pass_and_mutants(pxy, pgap):
    """Strips over 1-5 row passes (rows up to 9000, a partial last pass),
    columns 6000/8000 (C4's length), mutated copies (long diagonal runs, paths
    off the diagonal) and swapped halves (a path ~2500 columns off it), under
    the default workspace and under one small enough to force windowed storage
    (with re-runs for paths that leave it); bit-exact against the oracle."""
    r = random.Random(991 + pxy)
    base = bytes(r.choice(ACGT) for _ in range(7000))
    P, Q = (bytes(r.choice(ACGT) for _ in range(2500)) for _ in range(2))
    cols = [bytes(r.choice(ACGT) for _ in range(L)) for L in (6000, 8000)] + _mutants(r, base, 1, ACGT) + [P + Q]
    rows = [bytes(r.choice(ACGT) for _ in range(L)) for L in (2047, 6145, 9000)] + _mutants(r, base, 1, ACGT) + [Q + P]
    genes = cols + rows
    ids = _strip_pairs(len(cols), len(genes))
    _, opens, ohs = oracle.all_pairs(genes, pxy, pgap)
    for ws in (0, 40 << 20):
        with seqalign.Engine(device=0, kernel="nw_align_strip", workspace_bytes=ws) as e:
            e.set_sequences(genes)
            pen, hs = e.align_pairs(ids, pxy, pgap)
            st = e.stats()
        assert st["mode"] == 9
        if ws:
            assert st["window"] > 0 or st["batches"] > 1, st
        assert [int(v) for v in pen] == [opens[i] for i in ids], ws
        assert [x.tobytes().hex() for x in hs] == [ohs[i] for i in ids], ws


_ORDER_SCRIPT = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import seqalign
genes = [bytes.fromhex(g) for g in json.loads(sys.stdin.read())]
ws = int(sys.argv[2]) if len(sys.argv) > 2 else 64 << 20
k = len(genes)
out = []
for pxy, pgap in ((3, 2), (5, 1)):
    with seqalign.Engine(device=0, workspace_bytes=ws, kernel="nw_align_bits") as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(np.arange(k * (k - 1) // 2, dtype=np.int64), pxy, pgap)
        st = e.stats()
    out.append({"mode": st["mode"], "batches": st["batches"], "retries": st["window_retries"],
                "pen": [int(v) for v in pen], "hs": [x.tobytes().hex() for x in hs]})
print(json.dumps(out))
"""


def _run_child(genes, env_extra, ws=64 << 20):
    import json
    import sys

    env = dict(os.environ, **env_extra)
    res = subprocess.run([sys.executable, "-c", _ORDER_SCRIPT, os.path.dirname(seqalign.__file__), str(ws)],
                         input=json.dumps([g.hex() for g in genes]).encode(), env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert res.returncode == 0, res.stderr.decode()[-2000:]
    return json.loads(res.stdout.decode().strip().splitlines()[-1])


@pytest.mark.parametrize("order", ["0", "1", "3"])
def test_bits_kernel_task_orders_multi_batch(order):
    """nw_align_bits under each task order of the runtime (NWK_ORDER: 0
    pair-major, 1 band-major -- the default when a batch holds more than two
    rounds of tasks per wave slot, as C3/C4 do --, g >= 2 groups of g pairs)
    with a small workspace, so several batches reuse the granule region.  The
    order is read once per process, hence the child process.  Bit-exact vs the
    oracle on 3/2 and 5/1 (the reference's two penalty sets)."""
    r = random.Random(77)
    genes = _rand_genes(r, 7, 5000, 7000, ACGT)
    out = _run_child(genes, {"NWK_ORDER": order, "NWK_BITS_WIN": "0"})
    for (pxy, pgap), o in zip(((3, 2), (5, 1)), out):
        assert o["mode"] == 8 and o["batches"] > 1
        _, opens, ohs = oracle.all_pairs(genes, pxy, pgap)
        assert o["pen"] == opens
        assert o["hs"] == ohs


@pytest.mark.parametrize("win", ["auto", "48", "700", "3000"])
def test_bits_windowed_storage_and_full_rerun(win):
    """nw_align_bits windowed storage (only steps within W columns of each
    pair's diagonal are stored; nwk_runtime.cpp): a path that leaves the
    window is caught by the traceback and the pair re-runs with full storage
    (window_retries).  Ragged pairs (slopes far from 1), mutated copies and
    multi-band lengths, with a workspace too small for full storage (so the
    automatic window engages); results bit-exact vs the oracle for any W."""
    r = random.Random(4242)
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in (700, 2500, 4100, 6000)]
    genes += _mutants(r, bytes(r.choice(ACGT) for _ in range(5000)), 3, ACGT)
    # swapped halves: the optimal path runs ~3500 columns off the diagonal
    P, Q = (bytes(r.choice(ACGT) for _ in range(3500)) for _ in range(2))
    genes += [P + Q, Q + P]
    env = {} if win == "auto" else {"NWK_BITS_WIN": win}
    out = _run_child(genes, env, ws=24 << 20)
    for (pxy, pgap), o in zip(((3, 2), (5, 1)), out):
        assert o["mode"] == 8
        _, opens, ohs = oracle.all_pairs(genes, pxy, pgap)
        assert o["pen"] == opens
        assert o["hs"] == ohs
        if win == "48":
            assert o["retries"] > 0, "a 48-column window must send some pairs to the full re-run"


_AFF_WIN_SCRIPT = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import seqalign
genes = [bytes.fromhex(g) for g in json.loads(sys.stdin.read())]
k = len(genes)
out = []
for pxy, go, ge in ((3, 3, 1), (4, 2, 2)):
    with seqalign.Engine(device=0, workspace_bytes=int(sys.argv[2])) as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs_affine(np.arange(k * (k - 1) // 2, dtype=np.int64), pxy, go, ge)
        st = e.stats()
    out.append({"mode": st["mode"], "batches": st["batches"], "retries": st["window_retries"],
                "pen": [int(v) for v in pen], "hs": [x.tobytes().hex() for x in hs]})
print(json.dumps(out))
"""


@pytest.mark.parametrize("win", ["auto", "40", "600", "2000"])
def test_affine_packed_windowed_storage_and_full_rerun(win):
    """nw_align_pka windowed storage: band pair p stores only the 64-step
    super-blocks pka_sb_lo(p) .. + nsb - 1 around the diagonal (nwk_internal.h);
    a traceback that leaves them flags the pair and it re-runs with full
    storage.  Ragged lengths (multi band-pair, slopes far from 1), mutated
    copies and swapped halves (paths ~3000 columns off the diagonal), with a
    workspace too small for full storage; bit-exact vs the oracle for any W."""
    import json
    import sys

    r = random.Random(5151)
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in (900, 2600, 4100, 5200)]
    genes += _mutants(r, bytes(r.choice(ACGT) for _ in range(4500)), 2, ACGT)
    P, Q = (bytes(r.choice(ACGT) for _ in range(3000)) for _ in range(2))
    genes += [P + Q, Q + P]
    # (NWK_GOTOH=0: these scorings run on nw_align_gotoh by default, test_gpu_gotoh.py)
    env = dict(os.environ, NWK_GOTOH="0", **({} if win == "auto" else {"NWK_BITS_WIN": win}))
    res = subprocess.run([sys.executable, "-c", _AFF_WIN_SCRIPT, os.path.dirname(seqalign.__file__), str(40 << 20)],
                         input=json.dumps([g.hex() for g in genes]).encode(), env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert res.returncode == 0, res.stderr.decode()[-2000:]
    out = json.loads(res.stdout.decode().strip().splitlines()[-1])
    for (pxy, go, ge), o in zip(((3, 3, 1), (4, 2, 2)), out):
        assert o["mode"] == 7, "nw_align_pka expected"
        _, opens, ohs = oracle.all_pairs_affine(genes, pxy, go, ge)
        assert o["pen"] == opens
        assert o["hs"] == ohs
        if win == "40":
            assert o["retries"] > 0, "a 40-column window must send some pairs to the full re-run"


_AFF_WIDEN_SCRIPT = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import seqalign, workloads
genes = workloads.synth(2, 20000)
out = []
for ws in (150 << 20, 4 << 30):
    with seqalign.Engine(device=0, workspace_bytes=ws) as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs_affine(np.arange(1, dtype=np.int64), 3, 3, 1)
        st = e.stats()
    out.append({"mode": st["mode"], "batches": st["batches"], "retries": st["window_retries"],
                "pen": [int(v) for v in pen], "hs": [x.tobytes().hex() for x in hs]})
print(json.dumps(out))
"""


def test_affine_window_rerun_widens_when_full_storage_does_not_fit():
    """A windowed nw_align_pka pair whose trace leaves its window re-runs
    with full storage -- or, when full storage does not fit the budget (affine
    has no linear-space path), with the widest doubled window that does.  A
    20k x 20k pair forced to a 32-column window (NWK_BITS_WIN) under a 150 MiB
    budget (full storage ~206 MB, a 4096-column window ~101 MB) must still align, identically to the same pair
    re-run in full under 4 GiB, with the oracle's O(n)-memory affine score."""
    import json
    import sys

    import workloads

    env = dict(os.environ, NWK_BITS_WIN="32", NWK_GOTOH="0")
    res = subprocess.run([sys.executable, "-c", _AFF_WIDEN_SCRIPT, os.path.dirname(seqalign.__file__)],
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert res.returncode == 0, res.stderr.decode()[-2000:]
    small, big = json.loads(res.stdout.decode().strip().splitlines()[-1])
    assert small["mode"] == 7 and small["retries"] >= 1 and big["retries"] >= 1
    assert small["pen"] == big["pen"] and small["hs"] == big["hs"]
    genes = workloads.synth(2, 20000)
    assert small["pen"] == [oracle.score_affine(genes[1], genes[0], 3, 3, 1)]


def test_subset_and_order_of_pair_ids(engine):
    r = random.Random(5)
    genes = _rand_genes(r, 7, 50, 900, ACGT)
    engine.set_sequences(genes)
    ids = np.array([20, 3, 0, 17, 9], dtype=np.int64)
    pen, hs = engine.align_pairs(ids, 3, 2)
    _, opens, ohs = oracle.all_pairs(genes, 3, 2)
    assert [int(v) for v in pen] == [opens[i] for i in ids]
    assert [x.tobytes().hex() for x in hs] == [ohs[i] for i in ids]


def test_multi_batch_workspace():
    """A small HBM budget forces several fill/traceback batches."""
    r = random.Random(9)
    genes = _rand_genes(r, 8, 800, 1500, ACGT)
    with seqalign.Engine(device=0, workspace_bytes=3 << 20) as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(_all_ids(len(genes)), 3, 2)
        assert e.stats()["batches"] > 1
    _, opens, ohs = oracle.all_pairs(genes, 3, 2)
    assert [int(v) for v in pen] == opens
    assert [x.tobytes().hex() for x in hs] == ohs


@pytest.mark.parametrize("m,n", [(1, 1), (1, 9), (9, 1), (700, 30), (30, 700), (2000, 2100), (3000, 64)])
def test_single_pair_strings(engine, m, n):
    r = random.Random(m * 1000 + n)
    x = bytes(r.choice(ACGT) for _ in range(m))
    y = bytes(r.choice(ACGT) for _ in range(n))
    for pxy, pgap in ((3, 2), (5, 1), (-1, 2)):
        got = engine.get_minimum_penalty(x, y, pxy, pgap)
        assert got == oracle.pair(x, y, pxy, pgap)


def test_get_minimum_penalties_api(golden):
    c = golden["mseq1"]
    pxy, pgap, genes = case_input(c)
    pens = [0] * len(c["penalties"])
    h = seqalign.getMinimumPenalties(genes, len(genes), pxy, pgap, pens)
    assert h == c["hash"] and pens == c["penalties"]


@pytest.mark.skipif(not os.path.exists(os.path.join(PKG, "bin", "seqalkway")), reason="driver not built")
@pytest.mark.parametrize("name", ["mseq", "mseq1", "xulin_test", "k1", "k0"])
def test_driver_stdout_contract(golden, name):
    c = golden[name]
    if "file" in c:
        text = open(os.path.join(GOLDEN_DIR, "data", c["file"]), "rb").read()
    else:
        text = c["input"].encode("latin-1")
    out = subprocess.run([os.path.join(PKG, "bin", "seqalkway")], input=text, stdout=subprocess.PIPE,
                         check=True, timeout=300).stdout.decode()
    lines = out.split("\n")
    assert lines[0].startswith("Time: ") and lines[0].endswith(" us")
    assert lines[1] == c["hash"]
    assert lines[2] == "".join("%d " % p for p in c["penalties"])


def test_multi_gpu_allgather_inprocess(golden):
    if seqalign.device_count() < 2:
        pytest.skip("needs >= 2 devices for the in-process RCCL path")
    c = golden["xulin_test"]
    pxy, pgap, genes = case_input(c)
    pens = [0] * len(c["penalties"])
    h = seqalign.getMinimumPenalties(genes, len(genes), pxy, pgap, pens, ngpus=2)
    assert h == c["hash"] and pens == c["penalties"]


@pytest.mark.parametrize("name", ["xulin_test", "big13"])
def test_inprocess_rccl_allgather_one_gpu(golden, name):
    """The in-process multi-GPU path of nwk_get_minimum_penalties (one host
    thread per device, ncclCommInitAll + ONE ncclAllGather of 72-byte records,
    rank-0 chain; replaces sub:296-350) forced at one device (opts.collective),
    so the RCCL code runs on a 1-GPU box: the reference's published answers."""
    c = golden[name]
    pxy, pgap, genes = case_input(c)
    pens = [0] * len(c["penalties"])
    h = seqalign.getMinimumPenalties(genes, len(genes), pxy, pgap, pens, ngpus=1, collective=True)
    assert h == c["hash"] and pens == c["penalties"]


def test_sharded_union_equals_unsharded(engine, golden):
    """Emulated G-way shard: shards run one after another on one GPU."""
    pxy, pgap, genes = case_input(golden["xulin_test"])
    engine.set_sequences(genes)
    lengths = [len(g) for g in genes]
    P = len(genes) * (len(genes) - 1) // 2
    pen = np.zeros(P, dtype=np.int32)
    hs = np.zeros((P, 64), dtype=np.uint8)
    for r in range(8):
        ids = seqalign.shard_pairs(lengths, r, 8)
        p, h = engine.align_pairs(ids, pxy, pgap)
        pen[ids] = p
        hs[ids] = h
    assert seqalign.chain_hash(hs) == golden["xulin_test"]["hash"]


# ---------------------------------------------------------------------------
# Affine-gap variant.  Pinned to the reference only through
# go=0, ge=pgap (must reproduce every linear golden vector, big13 included);
# go > 0 is checked bit-exact against the oracle's restatement (parity
# unpinned by the reference).
# ---------------------------------------------------------------------------
AFFINE_GOLDEN = [c for c in GOLDEN if min(case_input(c)[:2]) >= 0]


@pytest.mark.parametrize("case", AFFINE_GOLDEN, ids=[c["name"] for c in AFFINE_GOLDEN])
def test_affine_degenerate_golden(engine, case):
    pxy, pgap, genes = case_input(case)
    engine.set_sequences(genes)
    pen, hs = engine.align_pairs_affine(_all_ids(len(genes)), pxy, 0, pgap)
    assert [int(v) for v in pen] == case["penalties"]
    assert seqalign.chain_hash(hs) == case["hash"]


AFFINE_PARAMS = [(3, 4, 1), (1, 2, 2), (0, 5, 0), (7, 0, 3), (4, 10, 1), (2, 1, 1)]


@pytest.mark.parametrize("pxy,go,ge", AFFINE_PARAMS)
def test_affine_random_vs_oracle(engine, pxy, go, ge):
    r = random.Random(pxy * 100 + go * 10 + ge)
    genes = _rand_genes(r, 5, 1, 700, ACGT) + _mutants(r, bytes(r.choice(ACGT) for _ in range(650)), 3, ACGT)
    genes += [bytes(r.choice(b"AC_x") for _ in range(L)) for L in (63, 64, 65, 511, 512, 513)]
    engine.set_sequences(genes)
    pen, hs = engine.align_pairs_affine(_all_ids(len(genes)), pxy, go, ge)
    h, opens, ohs = oracle.all_pairs_affine(genes, pxy, go, ge)
    assert [int(v) for v in pen] == opens
    assert [x.tobytes().hex() for x in hs] == ohs
    assert seqalign.chain_hash(hs) == h


# Packed affine fill (nw_align_pka, mode 7): ACGT-only sets with admissible
# penalties run on it by default where nw_align_gotoh has no instantiation
# (opts.kernel = "nw_align_pk2" pins it); every result must equal the oracle
# and the unpacked nw_align_affine (opts.kernel = "nw_align" forces the latter).


@pytest.fixture(scope="module")
def pka_engine():
    e = seqalign.Engine(device=0, kernel="nw_align_pk2")
    yield e
    e.close()
PKA_PARAMS = [(3, 3, 1), (1, 2, 2), (0, 5, 0), (7, 0, 3), (2, 1, 1), (5, 0, 0), (0, 0, 0), (9, 3, 2), (6, 6, 0)]
PKA_LENS = [1, 2, 63, 64, 65, 511, 512, 513, 1023, 1024, 1025, 2100]


@pytest.mark.parametrize("pxy,go,ge", PKA_PARAMS)
def test_affine_packed_vs_oracle(pka_engine, pxy, go, ge):
    r = random.Random(7000 + pxy * 100 + go * 10 + ge)
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in PKA_LENS]
    genes += _mutants(r, bytes(r.choice(ACGT) for _ in range(1500)), 3, ACGT)
    pka_engine.set_sequences(genes)
    pen, hs = pka_engine.align_pairs_affine(_all_ids(len(genes)), pxy, go, ge)
    assert pka_engine.stats()["mode"] == 7, "nw_align_pka expected"
    h, opens, ohs = oracle.all_pairs_affine(genes, pxy, go, ge)
    assert [int(v) for v in pen] == opens
    assert [x.tobytes().hex() for x in hs] == ohs


@pytest.mark.parametrize("seed", range(3))
def test_affine_packed_equals_unpacked(seed):
    """Multi-band(-pair) pairs (3k-7k): nw_align_gotoh, nw_align_pka and
    nw_align_affine, bit-exact against each other."""
    r = random.Random(8100 + seed)
    base = bytes(r.choice(ACGT) for _ in range(5000))
    genes = _rand_genes(r, 3, 3000, 7000, ACGT) + _mutants(r, base, 3, ACGT) + [b"A" * 4000, b"C" * 2500]
    pxy, go, ge = [(3, 3, 1), (4, 2, 1), (2, 4, 2)][seed]
    out = []
    for kernel in ("nw_align_gotoh", "nw_align_pk2", "nw_align"):
        with seqalign.Engine(device=0, kernel=kernel) as e:
            e.set_sequences(genes)
            h, pen, hs = e.align_all(pxy, None, affine=(go, ge))
            out.append((e.stats()["mode"], h, [int(v) for v in pen], hs.tobytes()))
    assert [o[0] for o in out] == [11, 7, 3]
    assert out[0][1:] == out[1][1:] == out[2][1:]


def test_affine_packed_big13_degenerate(pka_engine, golden):
    """big13 at full size on nw_align_pka with go=0, ge=pgap: the reference's published answer."""
    c = golden["big13"]
    pxy, pgap, genes = case_input(c)
    pka_engine.set_sequences(genes)
    pen, hs = pka_engine.align_pairs_affine(_all_ids(len(genes)), pxy, 0, pgap)
    assert pka_engine.stats()["mode"] == 7
    assert [int(v) for v in pen] == c["penalties"]
    assert seqalign.chain_hash(hs) == c["hash"]


def test_affine_packed_not_used_where_inadmissible(engine):
    """go + ge too large for the int16 window, or > 4 symbols: nw_align_affine runs."""
    r = random.Random(91)
    genes = _rand_genes(r, 4, 100, 900, ACGT)
    engine.set_sequences(genes)
    pen, _ = engine.align_pairs_affine(_all_ids(4), 4, 10, 1)
    assert engine.stats()["mode"] == 3
    assert [int(v) for v in pen] == oracle.all_pairs_affine(genes, 4, 10, 1)[1]
    genes5 = genes + [b"ACGTN" * 50]
    engine.set_sequences(genes5)
    pen, _ = engine.align_pairs_affine(_all_ids(5), 3, 3, 1)
    assert engine.stats()["mode"] == 3
    assert [int(v) for v in pen] == oracle.all_pairs_affine(genes5, 3, 3, 1)[1]


@pytest.mark.parametrize("m,n", [(1, 1), (1, 9), (9, 1), (700, 30), (30, 700), (1100, 1030), (2000, 64)])
def test_affine_single_pair_strings(engine, m, n):
    r = random.Random(m * 7 + n)
    x = bytes(r.choice(ACGT) for _ in range(m))
    y = bytes(r.choice(ACGT) for _ in range(n))
    for pxy, go, ge in ((3, 4, 1), (2, 0, 2), (5, 8, 0)):
        assert engine.get_minimum_penalty_affine(x, y, pxy, go, ge) == oracle.pair_affine(x, y, pxy, go, ge)


@pytest.mark.parametrize("kernel,mode", [("auto", 11), ("nw_align_pk2", 7), ("nw_align", 3)])
def test_affine_multi_batch_and_api(golden, kernel, mode):
    """Multi-batch workspaces on nw_align_gotoh (default for ACGT and 3/4/1),
    nw_align_pka and nw_align_affine."""
    r = random.Random(21)
    genes = _rand_genes(r, 7, 600, 1300, ACGT)
    with seqalign.Engine(device=0, workspace_bytes=(12 << 20) if mode == 11 else (3 << 20), kernel=kernel) as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs_affine(_all_ids(len(genes)), 3, 4, 1)
        st = e.stats()
        assert st["batches"] > 1 and st["mode"] == mode
        if kernel == "auto":  # a budget below one pair's nw_align_gotoh storage: the job runs on nw_align_pka
            e2 = seqalign.Engine(device=0, workspace_bytes=3 << 20)
            e2.set_sequences(genes)
            p2, h2 = e2.align_pairs_affine(_all_ids(len(genes)), 3, 4, 1)
            assert e2.stats()["mode"] == 7 and [int(v) for v in p2] == [int(v) for v in pen]
            assert [x.tobytes() for x in h2] == [x.tobytes() for x in hs]
            e2.close()
    h, opens, ohs = oracle.all_pairs_affine(genes, 3, 4, 1)
    assert [int(v) for v in pen] == opens and [x.tobytes().hex() for x in hs] == ohs
    pens = [0] * len(opens)
    assert seqalign.getMinimumPenaltiesAffine(genes, len(genes), 3, 4, 1, pens) == h and pens == opens
    with pytest.raises(seqalign.NwkError):
        seqalign.getMinimumPenaltiesAffine(genes, len(genes), -1, 4, 1, pens)


@pytest.mark.parametrize("name", ["mseq1", "xulin_test", "big13", "k1", "k0", "k2_same"])
def test_align_all_pipelined_chain(engine, golden, name):
    """nwk_align_all: the chain runs while batches are in flight; same answer."""
    c = golden[name]
    pxy, pgap, genes = case_input(c)
    engine.set_sequences(genes)
    h, pen, hs = engine.align_all(pxy, pgap)
    assert h == c["hash"] and [int(v) for v in pen] == c["penalties"]


def test_align_all_multi_batch_affine():
    r = random.Random(33)
    genes = _rand_genes(r, 8, 500, 1200, ACGT)
    with seqalign.Engine(device=0, workspace_bytes=3 << 20) as e:
        e.set_sequences(genes)
        h, pen, hs = e.align_all(3, 2)
        assert e.stats()["batches"] > 2
        ha, pena, _ = e.align_all(3, None, affine=(4, 1))
    oh, opens, _ = oracle.all_pairs(genes, 3, 2)
    assert h == oh and [int(v) for v in pen] == opens
    ah, apens, _ = oracle.all_pairs_affine(genes, 3, 4, 1)
    assert ha == ah and [int(v) for v in pena] == apens


# --- device finalize (nw_hash): rows, penalty and SHA-512 on the GPU

@pytest.fixture(scope="module")
def dev_engine():
    e = seqalign.Engine(device=0, finalize="device")
    yield e
    e.close()


@pytest.mark.parametrize("case", [c for c in GOLDEN if c["name"] != "big13-2"], ids=lambda c: c["name"])
def test_device_finalize_golden(dev_engine, case):
    pxy, pgap, genes = case_input(case)
    dev_engine.set_sequences(genes)
    pen, hs = dev_engine.align_pairs(_all_ids(len(genes)), pxy, pgap)
    assert [int(v) for v in pen] == case["penalties"]
    if "pairs" in case:
        assert [h.tobytes().hex() for h in hs] == [p["problemhash"] for p in case["pairs"]]
    assert seqalign.chain_hash(hs) == case["hash"]
    underscore = any(b"_" in g for g in genes)
    st = dev_engine.stats()
    if len(genes) > 1 and any(len(g) for g in genes):
        assert st["device_finalized"] == (0 if underscore else st["batches"]), \
            "device finalize must run on every batch (and only without '_' inputs)"


@pytest.mark.parametrize("seed", range(4))
def test_device_finalize_random_vs_oracle(dev_engine, seed):
    r = random.Random(100 + seed)
    # ragged lengths incl. 1-char and empty rows, long rows crossing many 128-byte SHA blocks
    genes = _rand_genes(r, 9, 0, 3000, b"ACGT") + [b"A", b"", bytes(r.choice(b"ACGT") for _ in range(5000))]
    for pxy, pgap in ((3, 2), (5, 1), (1, 4)):
        dev_engine.set_sequences(genes)
        pen, hs = dev_engine.align_pairs(_all_ids(len(genes)), pxy, pgap)
        oh, opens, ohs = oracle.all_pairs(genes, pxy, pgap)
        assert [int(v) for v in pen] == opens
        assert [h.tobytes().hex() for h in hs] == ohs


@pytest.mark.parametrize("go,ge", [(3, 1), (0, 2), (5, 2)])
def test_device_finalize_affine_vs_oracle(dev_engine, go, ge):
    r = random.Random(7 + go)
    genes = _rand_genes(r, 7, 1, 2500, b"ACGT")
    dev_engine.set_sequences(genes)
    pen, hs = dev_engine.align_pairs_affine(_all_ids(len(genes)), 3, go, ge)
    h, opens, ohs = oracle.all_pairs_affine(genes, 3, go, ge)
    assert [int(v) for v in pen] == opens
    assert [x.tobytes().hex() for x in hs] == ohs
    assert dev_engine.stats()["device_finalized"] == 1


def test_device_finalize_big13(dev_engine):
    case = next(c for c in GOLDEN if c["name"] == "big13")
    pxy, pgap, genes = case_input(case)
    dev_engine.set_sequences(genes)
    pen, hs = dev_engine.align_pairs(_all_ids(len(genes)), pxy, pgap)
    assert [int(v) for v in pen] == case["penalties"]
    assert seqalign.chain_hash(hs) == case["hash"]


def test_driver_fasta_and_dump(golden, tmp_path):
    """--fasta gives the same stdout as the token input; --dump rows match the oracle."""
    c = golden["mseq1"]
    text = open(os.path.join(GOLDEN_DIR, "data", c["file"]), "rb").read()
    pxy, pgap, genes = seqalign.parse_input(text)
    fa = tmp_path / "mseq1.fa"
    # wrapped at 7 columns, with headers and a blank line
    fa.write_bytes(b"".join(b">seq%d\n" % i + b"\n".join(g[k:k + 7] for k in range(0, len(g), 7)) + b"\n\n"
                            for i, g in enumerate(genes)))
    dump = tmp_path / "pairs.txt"
    out = subprocess.run([os.path.join(PKG, "bin", "seqalkway"), "--fasta", str(fa), "--pxy", str(pxy),
                          "--pgap", str(pgap), "--dump", str(dump)], stdout=subprocess.PIPE, check=True,
                         timeout=300).stdout.decode().split("\n")
    assert out[1] == c["hash"] and out[2] == "".join("%d " % p for p in c["penalties"])
    lines = dump.read_bytes().split(b"\n")
    p = 0
    for i in range(1, len(genes)):
        for j in range(i):
            pen, a1, a2 = oracle.pair(genes[i], genes[j], pxy, pgap)
            assert lines[3 * p] == b"%d %d %d" % (i, j, pen)
            assert lines[3 * p + 1] == a1 and lines[3 * p + 2] == a2
            p += 1


# --- progressive SoP MSA (build-defined; oracle/msa_oracle.c nwo_msa)

MSA_K2 = [c for c in GOLDEN if len(case_input(c)[2]) == 2 and min(case_input(c)[:2]) >= 0
          and b"_" not in b"".join(case_input(c)[2])]


@pytest.mark.parametrize("case", MSA_K2, ids=[c["name"] for c in MSA_K2])
def test_msa_k2_golden(engine, case):
    """k = 2: the MSA is the reference's alignment of pair (1, 0) and its SoP the golden penalty."""
    pxy, pgap, genes = case_input(case)
    engine.set_sequences(genes)
    rows, s = engine.msa(pxy, pgap)
    assert s == case["penalties"][0]
    assert (rows, s) == oracle.msa(genes, pxy, pgap)


@pytest.mark.parametrize("seed", range(8))
def test_msa_random_vs_oracle(engine, seed):
    r = random.Random(500 + seed)
    alpha = [b"ACGT", b"AC", b"ACGTN"][seed % 3]
    pxy, pgap = [(3, 2), (5, 1), (1, 3), (0, 2), (4, 0), (7, 7), (2, 1), (9, 4)][seed]
    k = r.randint(3, 9)
    if seed % 2:
        genes = _mutants(r, _rand_genes(r, 1, 200, 1400, alpha)[0], k, alpha)
    else:
        genes = _rand_genes(r, k, 1, 1300, alpha)
    genes = [g or alpha[:1] for g in genes]
    engine.set_sequences(genes)
    rows, s = engine.msa(pxy, pgap)
    want_rows, want_s = oracle.msa(genes, pxy, pgap)
    assert s == want_s
    assert rows == want_rows
    assert oracle.sop(rows, pxy, pgap) == s


@pytest.mark.parametrize("pxy,pgap,force", [(3, 2, None), (3, 2, "4"), (3, 2, "2"), (3, 2, "0"), (150, 90, None),
                                            (40000, 30000, None)],
                         ids=["auto", "dot4-forced", "dot2-forced", "mad-forced", "dot2-natural", "mad-natural"])
def test_msa_profile_packings(engine, monkeypatch, pxy, pgap, force):
    """nw_profile<DOT>: the one-hot (v_perm: levels whose columns are single sequences), u8 x 4
    (v_dot4), u16 x 2 (v_dot2) and plain (v_mad_u24) profile forms give the oracle's MSA.  Large
    costs pick the wider forms by themselves (rc = members x cost >= 256, >= 65536);
    NWK_PROF_DOT caps the form on small costs."""
    if force is not None:
        monkeypatch.setenv("NWK_PROF_DOT", force)
    r = random.Random(900 + pxy)
    L = 90 if pxy > 1000 else 700
    genes = _mutants(r, _rand_genes(r, 1, L, L, b"ACGT")[0], 5, b"ACGT")
    engine.set_sequences(genes)
    rows, s = engine.msa(pxy, pgap)
    assert (rows, s) == oracle.msa(genes, pxy, pgap)
    assert oracle.sop(rows, pxy, pgap) == s


def test_msa_many_sequences_vs_oracle(engine):
    """20 mutants of one 2,000-base sequence: a deep guide tree whose levels cross every
    nw_profile form in one call -- one-hot leaf columns (v_perm), multi-member columns
    (v_dot4), the walk's diagonal runs (merges of <= 16 sequences) and the plain walk
    (wider merges); bit-exact against the oracle's MSA and SoP."""
    r = random.Random(2024)
    genes = _mutants(r, bytes(r.choice(ACGT) for _ in range(2000)), 20, ACGT)
    engine.set_sequences(genes)
    rows, s = engine.msa(3, 2)
    st = engine.stats()
    assert st["fill_launches"] >= 5, st
    assert (rows, s) == oracle.msa(genes, 3, 2)


@pytest.mark.parametrize("L", [255, 256, 257, 511, 512, 513, 1023, 1025])
def test_msa_band_edges_vs_oracle(engine, L):
    """Profile lengths on either side of nw_profile's band edges (64 lanes x kProfRows = 4
    rows: 256-row bands; 512 with 8 rows): the row above a band, the last band's H(m, n)
    capture and the walk's band switches, bit-exact against the oracle."""
    r = random.Random(7000 + L)
    genes = [bytes(r.choice(ACGT) for _ in range(L))]
    genes += [bytes(r.choice(ACGT) for _ in range(L + d)) for d in (0, -1)]
    engine.set_sequences(genes)
    rows, s = engine.msa(3, 2)
    assert (rows, s) == oracle.msa(genes, 3, 2)
    assert oracle.sop(rows, 3, 2) == s


def test_msa_small_and_edge_sets(engine):
    for genes in ([b"ACGT"], [b"A", b"A"], [b"A", b"C"], [b"AC", b"A", b"C", b"CA"], [b"A" * 600, b"C"]):
        engine.set_sequences(genes)
        assert engine.msa(3, 2) == oracle.msa(genes, 3, 2)


def test_msa_rejects_what_it_cannot_align(engine):
    engine.set_sequences([b"AC_G", b"ACG"])
    with pytest.raises(seqalign.NwkError):
        engine.msa(3, 2)
    engine.set_sequences([b"ACG", b"AG"])
    with pytest.raises(seqalign.NwkError):
        engine.msa(-1, 2)
    engine.set_sequences([b"ABCDEF", b"AB"])
    with pytest.raises(seqalign.NwkError):
        engine.msa(3, 2)


# --- linear-space traceback: boundary rows only, bands recomputed per group

SMALL_GOLDEN = [c for c in GOLDEN if sum(len(g) for g in case_input(c)[2]) < 100000]


@pytest.mark.parametrize("g", [1, 3])
@pytest.mark.parametrize("case", SMALL_GOLDEN, ids=[c["name"] for c in SMALL_GOLDEN])
def test_linear_space_golden(g, case):
    pxy, pgap, genes = case_input(case)
    with seqalign.Engine(device=0, linear_space=g) as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(_all_ids(len(genes)), pxy, pgap)
        st = e.stats()
    assert [int(v) for v in pen] == case["penalties"]
    assert seqalign.chain_hash(hs) == case["hash"]
    assert st["linear_space_pairs"] == sum(1 for i in range(len(genes)) for j in range(i)
                                           if len(genes[i]) and len(genes[j]))


@pytest.mark.parametrize("g", [1, 2, 5])
def test_linear_space_random_vs_oracle(g):
    r = random.Random(900 + g)
    genes = _rand_genes(r, 3, 1, 3000, ACGT) + _mutants(r, _rand_genes(r, 1, 2500, 2600, ACGT)[0], 2, ACGT)
    with seqalign.Engine(device=0, linear_space=g) as e:
        e.set_sequences(genes)
        for pxy, pgap in ((3, 2), (5, 1), (1, 0), (40000, 30000)):
            pen, hs = e.align_pairs(_all_ids(len(genes)), pxy, pgap)
            h, want, _ = oracle.all_pairs(genes, pxy, pgap)
            assert [int(v) for v in pen] == want, (pxy, pgap)
            assert seqalign.chain_hash(hs) == h, (pxy, pgap)


def test_linear_space_single_pair_rows():
    r = random.Random(77)
    x, y = (bytes(r.choice(ACGT) for _ in range(n)) for n in (2600, 1900))
    with seqalign.Engine(device=0, linear_space=2) as e:
        assert e.get_minimum_penalty(x, y, 3, 2) == oracle.pair(x, y, 3, 2)


def test_linear_space_when_the_matrix_does_not_fit():
    """Automatic: a pair whose stored matrix exceeds the HBM budget goes through f2
    (nw_align_bits pinned: nw_align_col's write-saving window fits this pair in 8 MB)."""
    r = random.Random(5)
    genes = [bytes(r.choice(ACGT) for _ in range(6000)) for _ in range(2)] + [b"ACGT" * 10]
    with seqalign.Engine(device=0, workspace_bytes=8 << 20, kernel="nw_align_bits") as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(_all_ids(3), 3, 2)
        st = e.stats()
    h, want, _ = oracle.all_pairs(genes, 3, 2)
    assert [int(v) for v in pen] == want and seqalign.chain_hash(hs) == h
    assert st["linear_space_pairs"] >= 1


def test_linear_space_big13(golden, monkeypatch):
    """Full size (2.785e11 cells) through the linear-space path: the reference's published hash."""
    c = golden["big13"]
    pxy, pgap, genes = case_input(c)
    monkeypatch.setenv("NWK_VERBOSE", "3")  # batch compositions on stderr (shown on failure)
    with seqalign.Engine(device=0, linear_space=16) as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(_all_ids(len(genes)), pxy, pgap)
        st = e.stats()
    bad = [q for q in range(len(pen)) if int(pen[q]) != c["penalties"][q]]
    if bad:  # diagnostics: the failing pairs, the run's batching, and the same pairs again on a fresh engine
        ij = [seqalign.pair_ij(q) for q in bad]
        with seqalign.Engine(device=0, linear_space=16) as e2:
            e2.set_sequences(genes)
            again, _ = e2.align_pairs(np.array(bad, dtype=np.int64), pxy, pgap)
        pytest.fail("pairs %s (i, j %s; m x n %s) got %s want %s; stats %s; the same pairs alone: %s" % (
            bad, ij, [(len(genes[i]), len(genes[j])) for i, j in ij], [int(pen[q]) for q in bad],
            [c["penalties"][q] for q in bad], st, [int(v) for v in again]))
    assert seqalign.chain_hash(hs) == c["hash"]


def test_driver_msa_fasta(golden, tmp_path):
    """--msa writes the progressive SoP MSA as FASTA; rows and score equal the oracle's; stdout unchanged."""
    c = golden["mseq1"]
    text = open(os.path.join(GOLDEN_DIR, "data", c["file"]), "rb").read()
    pxy, pgap, genes = seqalign.parse_input(text)
    out_fa = tmp_path / "msa.fa"
    out = subprocess.run([os.path.join(PKG, "bin", "seqalkway"), "--msa", str(out_fa)], input=text,
                         stdout=subprocess.PIPE, check=True, timeout=300).stdout.decode().split("\n")
    assert out[1] == c["hash"] and out[2] == "".join("%d " % p for p in c["penalties"])
    rows, sop = oracle.msa(genes, pxy, pgap)
    recs = seqalign.parse_fasta(out_fa.read_bytes())
    assert recs == rows
    assert out_fa.read_bytes().split(b"\n")[0] == b">seq0 sop=%d" % sop


# --- fused device finalize + streamed records (nwk_align_pairs_poll) --------------------


@pytest.mark.gpu
@pytest.mark.parametrize("kernel,order", [("nw_align_bits", 1), ("nw_align_bits", 2), ("nw_align_strip", 0)])
def test_fused_finalize_streamed_poll_vs_oracle(kernel, order):
    """The bits kernels finalize each pair in the wave that traced it (rows,
    penalty, problemhash -> host-mapped records); Engine.align_pairs_poll hands
    out the final prefix while the call runs.  Every record against the oracle,
    the prefix monotone, the end() result identical."""
    r = random.Random(31 if kernel == "nw_align_bits" else 32)
    lo, hi = (300, 3000) if kernel == "nw_align_bits" else (4100, 5200)  # strips: n / 64 >= 63
    k = 24 if kernel == "nw_align_bits" else 6
    genes = _rand_genes(r, k, lo, hi, ACGT)
    ids = _all_ids(k)
    with seqalign.Engine(device=0, finalize="fused", kernel=kernel, task_order=order) as e:
        e.set_sequences(genes)
        for pxy, pgap in ((3, 2), (5, 1)):
            e.align_pairs_begin(ids, pxy, pgap)
            pen = np.zeros(len(ids), dtype=np.int32)
            hs = np.zeros((len(ids), 64), dtype=np.uint8)
            got, seen = 0, []
            while got < len(ids):
                u, p_, h_ = e.align_pairs_poll(got)
                assert u >= got
                pen[got:u], hs[got:u] = p_, h_
                if u > got:
                    seen.append(u)
                got = u
            pe, he = e.align_pairs_end()
            st = e.stats()
            assert st["device_finalized"] == st["batches"]
            oh, opens, ohs = oracle.all_pairs(genes, pxy, pgap)
            assert [int(v) for v in pen] == opens
            assert [h.tobytes().hex() for h in hs] == ohs
            assert (pe == pen).all() and (he == hs).all()
            assert seen[-1] == len(ids)

