"""GPU parity at BASELINE.json's full sizes (C3, C4, C5) and at the int16 edge.

Fixtures (tests/golden/large/, made by tests/golden/make_golden_large.py in the
build container; the inputs are regenerated here bit-for-bit by workloads.synth
and tests/golden/gen_inputs.py):
  c3.json                  answer hash + all penalties from oracle/_ref/sub, the
                           reference's own submitted program, on the full config
                           (the reference's evidence model: testing3/sequential.txt:2-3)
  c4.json                  the same from oracle/_ref/skel_debug, the reference's own
                           skeleton, every pair as a two-sequence job (6 processes,
                           3,538 s): the answer is skel:159's chain over its 32,640
                           per-pair problemhashes (all equal to the oracle
                           restatement's); sub's singleton rank would need ~9 h
  c3_pairs / c4_pairs      per-pair penalty + problemhash of the first 36 canonical
                           pairs from skel_debug (skel:158-169)
  c5_scores.json           affine go=3 ge=1 (and linear) penalties of pairs 0 and 1
                           from the oracle's O(n)-memory restatement -- the affine
                           variant has no reference (parity unpinned
                           beyond its degenerate case go=0, ge=pgap)
  edge16.json              long ragged pairs at the 4-bit / packed-int16 penalty
                           limits (1,7) (0,7) (15,0) (13,1), from skel_debug
Bar: bit-exact.
"""
import json
import os

import numpy as np
import pytest

import seqalign
import workloads
from conftest import GOLDEN_DIR

pytestmark = pytest.mark.gpu

LARGE = os.path.join(GOLDEN_DIR, "large")


def _fixture(name):
    f = os.path.join(LARGE, name + ".json")
    if not os.path.exists(f):
        pytest.fail("fixture %s missing (tests/golden/make_golden_large.py)" % f)
    return json.load(open(f))


@pytest.fixture(scope="module")
def engine():
    if seqalign.device_count() < 1:
        pytest.fail("no HIP device visible for a -m gpu run")
    e = seqalign.Engine(device=0)
    yield e
    e.close()


def _ids(n):
    return np.arange(n, dtype=np.int64)


@pytest.mark.parametrize("cfg", ["c3", "c4"])
def test_full_config_answer_vs_reference(engine, cfg):
    """All pairs of C3 (2,016 x 50k^2) / C4 (32,640 x 8k^2): the answer hash and
    every penalty equal the reference program's (oracle/_ref/sub)."""
    g = _fixture(cfg)
    _, k, L, pxy, pgap, _ = workloads.SYNTH[cfg]
    genes = workloads.synth(k, L)
    engine.set_sequences(genes)
    h, pen, _ = engine.align_all(pxy, pgap)
    assert [int(v) for v in pen] == g["penalties"]
    assert h == g["hash"]


@pytest.mark.parametrize("cfg", ["c3", "c4"])
@pytest.mark.parametrize("finalize", ["host", "device"])
def test_first_pairs_problemhash_vs_skel(cfg, finalize):
    """Per-pair problemhash of the first 36 canonical pairs vs skel_debug, with
    the host and the device (nw_hash) finalize."""
    g = _fixture(cfg + "_pairs")
    _, _, L, pxy, pgap, _ = workloads.SYNTH[cfg]
    genes = workloads.synth(g["k"], L)
    with seqalign.Engine(device=0, finalize=finalize) as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(_ids(len(g["pairs"])), pxy, pgap)
    assert [int(v) for v in pen] == [p["penalty"] for p in g["pairs"]]
    assert [x.tobytes().hex() for x in hs] == [p["problemhash"] for p in g["pairs"]]
    assert seqalign.chain_hash(hs) == g["hash"]


def test_c5_affine_degenerate_equals_linear_full_size(engine):
    """C5 at full size (496 pairs x 200k^2): affine go=0, ge=pgap must reproduce
    the linear path's penalties and problem hashes exactly."""
    _, k, L, pxy, pgap, _ = workloads.SYNTH["c5"]
    genes = workloads.synth(k, L)
    engine.set_sequences(genes)
    hl, pl, hsl = engine.align_all(pxy, pgap)
    ha, pa, hsa = engine.align_all(pxy, None, affine=(0, pgap))
    assert (pa == pl).all()
    assert (hsa == hsl).all()
    assert ha == hl


def test_c5_affine_scores_vs_oracle(engine):
    """C5 go=3 ge=1 (the bench's affine config): pairs 0 and 1 (200k x 200k) vs the
    oracle's O(n)-memory score restatement; linear 3/2 on the same pairs too."""
    g = _fixture("c5_scores")
    _, k, L, pxy, pgap, (go, ge) = workloads.SYNTH["c5"]
    genes = workloads.synth(3, L)
    engine.set_sequences(genes)
    ids = np.array([s["pair"] for s in g["scores"]], dtype=np.int64)
    pa, _ = engine.align_pairs_affine(ids, pxy, go, ge)
    assert [int(v) for v in pa] == [s["affine_penalty"] for s in g["scores"]]
    pl, _ = engine.align_pairs(ids, pxy, pgap)
    assert [int(v) for v in pl] == [s["linear_penalty"] for s in g["scores"]]


@pytest.mark.skipif(not os.path.exists(os.path.join(LARGE, "c5_pen.json")), reason="c5_pen.json not generated")
def test_c5_affine_all_penalties_vs_oracle(engine):
    """C5 at full size with its affine scoring (go=3, ge=1: the bench's config),
    every one of the 496 penalties against the oracle's O(n)-memory Gotoh scorer
    (tests/golden/large/c5_pen.json; the affine variant has no reference, SURVEY
    §8 a9), through getMinimumPenalties on the engine: nw_align_gotoh, W = 8192
    windowed storage, the fill-vs-walk guard on every pair."""
    g = _fixture("c5_pen")
    _, k, L, pxy, pgap, (go, ge) = workloads.SYNTH["c5"]
    assert (g["k"], g["L"], g["pxy"], g["go"], g["ge"]) == (k, L, pxy, go, ge)
    genes = workloads.synth(k, L)
    engine.set_sequences(genes)
    _, pen, _ = engine.align_all(pxy, None, affine=(go, ge))
    st = engine.stats()
    assert [int(v) for v in pen] == g["penalties"]
    assert st["mode"] == 11 and st.get("guard_reruns", 0) == 0


def test_affine_window_choice_at_a_large_budget():
    """nw_align_pka's storage window at a budget above 2^33 B (the runtime used
    to multiply the budget by 2^30 and overflow there): k=8 x 30k affine needs
    ~13 GB at full storage, so a 9 GiB budget must pick W = 8192 (one batch, no
    re-runs); pairs 0 and 1 against the oracle's O(n)-memory affine score."""
    import oracle

    genes = workloads.synth(8, 30000)
    with seqalign.Engine(device=0, workspace_bytes=9 << 30) as e:
        e.set_sequences(genes)
        pa, _ = e.align_pairs_affine(np.arange(28, dtype=np.int64), 3, 3, 1)
        st = e.stats()
    assert st["mode"] in (7, 11) and st["window"] == 8192, st  # nw_align_gotoh / nw_align_pka
    assert st["batches"] == 1 and st["window_retries"] == 0, st
    for p in (0, 1):
        i, j = seqalign.pair_ij(p)
        assert int(pa[p]) == oracle.score_affine(genes[i], genes[j], 3, 3, 1)


def _edge_cases():
    f = os.path.join(LARGE, "edge16.json")
    return json.load(open(f))["cases"] if os.path.exists(f) else []


@pytest.mark.parametrize("kernel", ["auto", "nw_align_pk", "nw_align_pk2", "nw_align", "nw_align_bits"])
@pytest.mark.parametrize("case", _edge_cases(), ids=lambda c: "pxy%d_pgap%d" % (c["pxy"], c["pgap"]))
def test_int16_edge_penalties_long_ragged(case, kernel):
    """20k-60k ragged pairs at 2*pgap + pxy = 14..15 (the W = 4 limit) with every
    linear fill kernel forced: the packed int16-relative kernels must hold G's span."""
    import sys

    sys.path.insert(0, GOLDEN_DIR)
    import gen_inputs

    genes = gen_inputs.edge16_genes(case["pxy"], case["pgap"])
    assert [len(x) for x in genes] == case["lengths"]
    with seqalign.Engine(device=0, kernel=kernel) as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(_ids(len(case["pairs"])), case["pxy"], case["pgap"])
        mode = e.stats()["mode"]
    assert [int(v) for v in pen] == [p["penalty"] for p in case["pairs"]]
    assert [x.tobytes().hex() for x in hs] == [p["problemhash"] for p in case["pairs"]]
    assert seqalign.chain_hash(hs) == case["hash"]
    uniform = (-2 * case["pgap"] < 0) == (case["pxy"] - 2 * case["pgap"] < 0)
    want = {"nw_align_pk": 4, "nw_align_pk2": 5}.get(kernel)
    if want is not None:
        assert mode == (want if uniform else 0), "packed kernel only where its profile bytes sign-extend uniformly"
    if kernel == "nw_align_bits":
        assert (mode == 8) == (case["pgap"] in (1, 2)), "bit planes exactly where pgap is 1 or 2"
