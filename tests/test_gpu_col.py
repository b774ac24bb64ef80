"""GPU parity of nw_align_col (csrc/nwk_col.hip): the column-wise bit-parallel
fill + its traceback, forced with kernel="nw_align_col", bit-exact against the
oracle (oracle/nw_oracle.c, the skel restatement pinned to the reference's
golden vectors) and the reference's published answers.

The kernel resolves 32 rows of one column per lane-step with carry chains
(v_addc_co_u32, the carries hopping lane to lane as SGPR masks), so the edge
cases are the 32-row lane words, the 2048-row bands (lane 0's carry in from
the band above's last row, 32-column granules), the first 64 steps (columns
< 0 masked) and the last 32-column word of a row.
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
from conftest import GOLDEN_DIR, case_input, load_golden

pytestmark = pytest.mark.gpu

ACGT = b"ACGT"
COL_PENALTIES = [(p, 2) for p in range(0, 6)] + [(p, 1) for p in range(0, 4)] + [(9, 2), (7, 1)]


def _ids(k):
    return np.arange(k * (k - 1) // 2, dtype=np.int64)


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


def _check(genes, pxy, pgap, ids=None, **kw):
    k = len(genes)
    ids = _ids(k) if ids is None else ids
    with seqalign.Engine(device=0, kernel="nw_align_col", **kw) as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(ids, pxy, pgap)
        st = e.stats()
    assert st["mode"] == 10, "nw_align_col expected"
    _, opens, ohs = oracle.all_pairs(genes, pxy, pgap)
    want_p = [opens[i] for i in ids]
    got_p = [int(v) for v in pen]
    bad = [(int(i), seqalign.pair_ij(int(i)), got_p[q], want_p[q]) for q, i in enumerate(ids) if got_p[q] != want_p[q]]
    assert not bad, "penalties differ (id, (i, j), got, want): %s" % bad[:8]
    assert [x.tobytes().hex() for x in hs] == [ohs[i] for i in ids]
    return st


@pytest.mark.parametrize("pxy,pgap", COL_PENALTIES)
def test_col_every_mismatch_level(pxy, pgap):
    """Every thermometer level SR = 2 pgap - pxy of the mismatch score, on
    lengths straddling 32-row words, 32-column words and 2048-row bands, plus
    mutated copies (long diagonal runs, paths off the diagonal)."""
    r = random.Random(pxy * 41 + pgap)
    lens = [1, 31, 32, 33, 95, 2047, 2048, 2049, 4200]
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in lens]
    genes += _mutants(r, bytes(r.choice(ACGT) for _ in range(3000)), 2, ACGT)
    _check(genes, pxy, pgap)


@pytest.mark.parametrize("case", [c for c in load_golden()], ids=lambda c: c["name"])
def test_col_golden_cases(case):
    """Every golden case through kernel="nw_align_col" (cases outside its
    domain -- more than 4 symbols, pgap not 1 or 2, negative penalties -- run on
    the fallback kernel and must still match)."""
    pxy, pgap, genes = case_input(case)
    if case["name"] in ("big13", "big13_2"):
        pytest.skip("full big13 runs in test_col_big13_published_hash")
    with seqalign.Engine(device=0, kernel="nw_align_col") as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(_ids(len(genes)), pxy, pgap)
    assert [int(v) for v in pen] == case["penalties"]
    assert seqalign.chain_hash(hs) == case["hash"]


def test_col_big13_published_hash():
    """big13 (78 pairs, 30k-90k, 2.785e11 cells): the reference's published
    answer (testing3/sequential.txt:2-3) through nw_align_col."""
    gold = {c["name"]: c for c in load_golden()}["big13"]
    pxy, pgap, genes = case_input(gold)
    with seqalign.Engine(device=0, kernel="nw_align_col") as e:
        e.set_sequences(genes)
        h, pen, _ = e.align_all(pxy, pgap)
        assert e.stats()["mode"] == 10
    assert [int(v) for v in pen] == gold["penalties"]
    assert h == gold["hash"]


@pytest.mark.parametrize("pxy,pgap", [(3, 2), (5, 1)])
def test_col_many_bands_and_ragged(pxy, pgap):
    """Pairs of up to 5 bands with a ragged last band, very wide and very tall
    pairs (slopes far from 1: long U or L runs in the traceback), swapped halves
    (a path ~2500 columns off the diagonal)."""
    r = random.Random(1234 + pxy)
    P, Q = (bytes(r.choice(ACGT) for _ in range(2500)) for _ in range(2))
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in (9000, 6145, 300, 70)] + [P + Q, Q + P]
    genes += _mutants(r, bytes(r.choice(ACGT) for _ in range(7000)), 2, ACGT)
    _check(genes, pxy, pgap)


_CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import seqalign
genes = [bytes.fromhex(g) for g in json.loads(sys.stdin.read())]
ws = int(sys.argv[2])
k = len(genes)
out = []
for pxy, pgap in ((3, 2), (5, 1)):
    with seqalign.Engine(device=0, workspace_bytes=ws, kernel="nw_align_col") as e:
        e.set_sequences(genes)
        pen, hs = e.align_pairs(np.arange(k * (k - 1) // 2, dtype=np.int64), pxy, pgap)
        st = e.stats()
    out.append({"mode": st["mode"], "batches": st["batches"], "retries": st["window_retries"],
                "window": st["window"], "pen": [int(v) for v in pen], "hs": [x.tobytes().hex() for x in hs]})
print(json.dumps(out))
"""


@pytest.mark.parametrize("seg", ["0", "1"])
def test_col_segmented_traceback_on_off(seg):
    """Segmented traceback (trace_col: a speculative segment per band but the
    last, merged into by the pair's own walk) forced off (NWK_COL_SEG=0, whole
    walks) and on, in a child: related many-band pairs whose segments merge,
    swapped halves whose segments never meet the path, ragged last bands."""
    r = random.Random(977)
    base = bytes(r.choice(ACGT) for _ in range(9000))
    genes = _mutants(r, base, 3, ACGT) + [base[:6100], base[2500:]]
    P, Q = (bytes(r.choice(ACGT) for _ in range(3000)) for _ in range(2))
    genes += [P + Q, Q + P]
    env = dict(os.environ, NWK_COL_SEG=seg)
    res = subprocess.run([sys.executable, "-c", _CHILD, os.path.dirname(seqalign.__file__), str(0)],
                         input=json.dumps([g.hex() for g in genes]).encode(), env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert res.returncode == 0, res.stderr.decode()[-2000:]
    out = json.loads(res.stdout.decode().strip().splitlines()[-1])
    for (pxy, pgap), o in zip(((3, 2), (5, 1)), out):
        assert o["mode"] == 10
        _, opens, ohs = oracle.all_pairs(genes, pxy, pgap)
        assert o["pen"] == opens
        assert o["hs"] == ohs


@pytest.mark.parametrize("win", ["auto", "48", "700", "3000"])
def test_col_windowed_storage_and_full_rerun(win):
    """Windowed storage (NWK_BITS_WIN, read once per process: a child) with a
    workspace too small for full storage: a path that leaves the stored steps is
    caught by the traceback and re-runs with full storage (window_retries);
    results bit-exact for any W, several batches reusing the granule region."""
    r = random.Random(4243)
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in (700, 2500, 4100, 6000)]
    genes += _mutants(r, bytes(r.choice(ACGT) for _ in range(5000)), 3, ACGT)
    P, Q = (bytes(r.choice(ACGT) for _ in range(3500)) for _ in range(2))
    genes += [P + Q, Q + P]
    env = dict(os.environ)
    if win != "auto":
        env["NWK_BITS_WIN"] = win
    res = subprocess.run([sys.executable, "-c", _CHILD, os.path.dirname(seqalign.__file__), str(24 << 20)],
                         input=json.dumps([g.hex() for g in genes]).encode(), env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert res.returncode == 0, res.stderr.decode()[-2000:]
    out = json.loads(res.stdout.decode().strip().splitlines()[-1])
    for (pxy, pgap), o in zip(((3, 2), (5, 1)), out):
        assert o["mode"] == 10
        _, opens, ohs = oracle.all_pairs(genes, pxy, pgap)
        assert o["pen"] == opens
        assert o["hs"] == ohs
        if win == "48":
            assert o["retries"] > 0, "a 48-column window must send some pairs to the full re-run"


@pytest.mark.parametrize("order", [1, 2])
def test_col_fused_finalize_streamed(order):
    """The fused device finalize inside the nw_align_col launch (records
    streaming to the host as pairs are hashed, nwk_align_pairs_poll), pair-major
    and band-major task order: every record equals the oracle's."""
    r = random.Random(31 + order)
    genes = [bytes(r.choice(ACGT) for _ in range(r.randint(300, 3000))) for _ in range(24)]
    k = len(genes)
    ids = _ids(k)
    with seqalign.Engine(device=0, kernel="nw_align_col", finalize="fused", task_order=order) as e:
        e.set_sequences(genes)
        e.align_pairs_begin(ids, 3, 2)
        got = 0
        pen = np.zeros(len(ids), np.int32)
        hs = np.zeros((len(ids), 64), np.uint8)
        while got < len(ids):
            u, p_, h_ = e.align_pairs_poll(got)
            pen[got:u], hs[got:u] = p_, h_
            got = u
        pe, he = e.align_pairs_end()
        assert e.stats()["mode"] == 10
    _, opens, ohs = oracle.all_pairs(genes, 3, 2)
    assert [int(v) for v in pen] == opens and [int(v) for v in pe] == opens
    assert [x.tobytes().hex() for x in hs] == ohs
    assert (he == hs).all()


_HSTREAM_SCRIPT = r"""
import json, sys, time
import numpy as np
sys.path.insert(0, sys.argv[1])
import seqalign
genes = [bytes.fromhex(g) for g in json.loads(sys.stdin.read())]
k = len(genes)
ids = np.arange(k * (k - 1) // 2, dtype=np.int64)
out = {}
with seqalign.Engine(device=0, kernel="nw_align_col", finalize="host", workspace_bytes=int(sys.argv[2])) as e:
    e.set_sequences(genes)
    if sys.argv[3] == "bad":  # a failed walk: nothing of it may be reported
        e.align_pairs_begin(ids, 3, 2)
        ups = []
        t0 = time.time()
        while time.time() - t0 < 60:
            try:
                u, _, _ = e.align_pairs_poll(0)
            except seqalign.NwkError as x:
                ups.append(-x.code)
                break
            ups.append(u)
            time.sleep(0.001)
        try:
            e.align_pairs_end()
            out["end"] = "ok"
        except seqalign.NwkError as x:
            out["end"] = x.code
        out["ups"] = sorted(set(ups))
    else:
        pen, hs = e.align_pairs(ids, 3, 2)
        st = e.stats()
        out["sync"] = {"pen": [int(v) for v in pen], "hs": [x.tobytes().hex() for x in hs],
                       "retries": st["window_retries"], "batches": st["batches"], "mode": st["mode"]}
        e.align_pairs_begin(ids, 3, 2)
        got = 0
        while got < len(ids):
            got, _, _ = e.align_pairs_poll(0)
            time.sleep(0.0005)
        pen2, hs2 = e.align_pairs_end()
        out["async"] = {"pen": [int(v) for v in pen2], "hs": [x.tobytes().hex() for x in hs2]}
print(json.dumps(out))
"""


def _hstream_genes():
    r = random.Random(4711)
    base = bytes(r.choice(ACGT) for _ in range(6000))
    genes = [base, _mutants(r, base, 1, ACGT)[0]]  # pair 0 (1, 0): the largest
    genes += [bytes(r.choice(ACGT) for _ in range(L)) for L in (700, 2100, 3300, 4000)]
    P, Q = (bytes(r.choice(ACGT) for _ in range(2400)) for _ in range(2))
    genes += [P + Q, Q + P]  # paths ~2400 columns off the diagonal
    return genes


def _run_hstream(genes, mode, ws, **env):
    res = subprocess.run([sys.executable, "-c", _HSTREAM_SCRIPT, os.path.dirname(seqalign.__file__), str(ws), mode],
                         input=json.dumps([g.hex() for g in genes]).encode(), env=dict(os.environ, **env),
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert res.returncode == 0, res.stderr.decode()[-2000:]
    return json.loads(res.stdout.decode().strip().splitlines()[-1])


def test_col_streamed_host_finalize_window_reruns_and_poll():
    """The streamed host finalize (nw_align_col with host finalize: the walk
    writes its moves to host-mapped memory and flags each pair; host threads
    finalize during the launch) under forced window re-runs (NWK_BITS_WIN=48)
    and several batches, through align_pairs and align_pairs_begin / poll / end:
    bit-exact vs the oracle both ways."""
    genes = _hstream_genes()
    out = _run_hstream(genes, "ok", 120 << 20, NWK_BITS_WIN="48")
    _, opens, ohs = oracle.all_pairs(genes, 3, 2)
    s = out["sync"]
    assert s["mode"] == 10 and s["retries"] > 0 and s["batches"] >= 2, s
    assert s["pen"] == opens and s["hs"] == ohs
    assert out["async"]["pen"] == opens and out["async"]["hs"] == ohs


def test_col_streamed_host_finalize_failed_walk_never_reported():
    """A walk that fails (NWK_DBG_BADWALK=1 marks slot 0's walk -- pair 0, the
    batch's largest -- as failed, as a walk running past m + n would be) is
    published with length -2: the host never finalizes, reports or chains it,
    so poll never gets past pair 0, and the call ends with NWK_EKERNEL."""
    genes = _hstream_genes()
    out = _run_hstream(genes, "bad", 8 << 30, NWK_DBG_BADWALK="1")
    assert out["end"] == -4, out
    assert all(u <= 0 or u == 4 for u in out["ups"]), out  # upto stayed 0 (or the poll raised EKERNEL)
