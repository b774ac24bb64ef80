"""The fill-vs-walk guard (skel:274: the reference's penalty IS the fill's
dp[m][n]; sub:560 the same).  The engine's penalty is the cost summed along
the walked path, which equals dp[m][n] only when the walk read the codes the
fill stored.  Every guarded fill kernel (nw_align_col, nw_align_gotoh,
nw_align_pka) accumulates its own H(m, n) per pair (FillArgs::endv), and
every finalize -- host threads, the streamed host finalize, nw_rows, the fused
in-launch finalize -- compares it with the walked path's cost.  A pair that
disagrees is never published: it re-runs with full storage (stats
guard_reruns), and a second disagreement fails the call with NWK_EKERNEL.

NWK_DBG_CORRUPT = slot + 1 flips the stored code of cell (m, n) of one pair in
the call's first batch just before its walk (NWK_DBG_CORRUPT_ALL: in every
batch).  The sequences share a 24-symbol tail, so (m, n) ends a long run of
matches and the flipped code sends the walk onto a strictly dearer path.
Bar: the corrupted call's answers equal the oracle's bit for bit, with one
re-run; a corruption that recurs ends in NWK_EKERNEL.
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

_CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import seqalign
cfg = json.loads(sys.stdin.read())
genes = [bytes.fromhex(g) for g in cfg["genes"]]
k = len(genes)
ids = np.arange(k * (k - 1) // 2, dtype=np.int64)
out = {}
try:
    with seqalign.Engine(device=0, kernel=cfg["kernel"], finalize=cfg["finalize"],
                         workspace_bytes=cfg.get("ws", 0)) as e:
        e.set_sequences(genes)
        if cfg["affine"]:
            pen, hs = e.align_pairs_affine(ids, *cfg["scoring"])
        else:
            pen, hs = e.align_pairs(ids, *cfg["scoring"])
        out = {"pen": [int(v) for v in pen], "hs": [x.tobytes().hex() for x in hs], "stats": e.stats()}
except seqalign.NwkError as x:
    out = {"err": x.code, "msg": str(x)}
print(json.dumps(out))
"""


def _run(genes, kernel, finalize, scoring, affine=False, ws=0, **env):
    cfg = {"genes": [g.hex() for g in genes], "kernel": kernel, "finalize": finalize, "scoring": list(scoring),
           "affine": affine, "ws": ws}
    res = subprocess.run([sys.executable, "-c", _CHILD, os.path.dirname(seqalign.__file__)],
                         input=json.dumps(cfg).encode(), env=dict(os.environ, **env),
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert res.returncode == 0, res.stderr.decode()[-2000:]
    return json.loads(res.stdout.decode().strip().splitlines()[-1]), res.stderr.decode()


def _genes(seed, n=6, lo=1500, hi=5000):
    r = random.Random(seed)
    tail = bytes(r.choice(ACGT) for _ in range(24))
    return [bytes(r.choice(ACGT) for _ in range(r.randint(lo, hi))) + tail for _ in range(n)]


def _want(genes, scoring, affine):
    if affine:
        _, p, h = oracle.all_pairs_affine(genes, *scoring)
    else:
        _, p, h = oracle.all_pairs(genes, *scoring)
    return p, h


# (finalize, extra env): the host finalize threads, the streamed host finalize
# (nw_align_col's default for host finalize), nw_rows + nw_hash, the fused one
COL_PATHS = [("host", {"NWK_HOST_STREAM": "0"}), ("host", {}), ("device", {}), ("fused", {})]


@pytest.mark.parametrize("fin,env", COL_PATHS, ids=["host", "host-stream", "device", "fused"])
def test_guard_col_corrupt_code_reruns(fin, env):
    genes = _genes(11)
    out, err = _run(genes, "nw_align_col", fin, (3, 2), NWK_DBG_CORRUPT="1", NWK_GUARD_LOG="1", **env)
    assert "err" not in out, out
    p, h = _want(genes, (3, 2), False)
    assert out["pen"] == p and out["hs"] == h
    st = out["stats"]
    assert st["mode"] == 10 and st["guard_checked"] >= len(p)
    assert st["guard_reruns"] == 1, (st, err[-1500:])
    assert "nwk guard: pair" in err


@pytest.mark.parametrize("fin", ["host", "device"])
@pytest.mark.parametrize("kernel,mode", [("nw_align_gotoh", 11), ("nw_align_pk2", 7)])
def test_guard_affine_corrupt_code_reruns(kernel, mode, fin):
    genes = _genes(12, n=5)
    out, err = _run(genes, kernel, fin, (3, 3, 1), affine=True, NWK_DBG_CORRUPT="1", NWK_GUARD_LOG="1")
    assert "err" not in out, out
    p, h = _want(genes, (3, 3, 1), True)
    assert out["pen"] == p and out["hs"] == h
    st = out["stats"]
    assert st["mode"] == mode and st["guard_reruns"] == 1, (st, err[-1500:])


@pytest.mark.parametrize("kernel,affine,scoring", [("nw_align_col", False, (3, 2)),
                                                   ("nw_align_gotoh", True, (3, 3, 1)),
                                                   ("nw_align_pk2", True, (3, 3, 1))])
def test_guard_recurring_disagreement_fails_loudly(kernel, affine, scoring):
    """A pair whose walk disagrees with its fill again after the full-storage
    re-run is an engine fault: NWK_EKERNEL, no answer."""
    genes = _genes(13, n=2)
    out, _ = _run(genes, kernel, "host", scoring, affine=affine, NWK_DBG_CORRUPT="1", NWK_DBG_CORRUPT_ALL="1")
    assert out.get("err") == -4, out
    assert "again after a full-storage re-run" in out["msg"]


# every guarded fill kernel, each at its own end-value capture: the bit-plane
# column sums (nw_align_col, nw_align_bits, nw_align_gotoh) and the captured
# cell of the value kernels (nw_align in its three modes, the int16 packed
# nw_align_pk / nw_align_pk2 / nw_align_pka, the int32 nw_align_affine)
CLEAN = [("nw_align_col", False, (3, 2), (10,)), ("nw_align_col", False, (5, 1), (10,)),
         ("nw_align_bits", False, (3, 2), (8,)), ("nw_align_bits", False, (0, 1), (8,)),
         ("nw_align_gotoh", True, (3, 3, 1), (11,)), ("nw_align_gotoh", True, (3, 0, 2), (11,)),
         ("nw_align_pk2", True, (3, 3, 1), (7,)), ("nw_align_pk2", True, (4, 2, 2), (7,)),
         ("nw_align", True, (3, 3, 1), (3,)),
         ("nw_align_pk2", False, (3, 2), (5,)), ("nw_align_pk", False, (3, 2), (4,)),
         ("nw_align", False, (3, 2), (0, 1)), ("nw_align", False, (4, 3), (0, 1)), ("nw_align", False, (-2, 3), (2,))]


@pytest.mark.parametrize("kernel,affine,scoring,mode", CLEAN)
def test_guard_clean_runs_check_every_pair(kernel, affine, scoring, mode):
    """Without corruption every pair is checked and none disagrees: the fill's
    end values equal the oracle's dp[m][n] on ragged pairs crossing bands and
    band pairs (512 / 1024 / 2048 rows)."""
    r = random.Random(77)
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in (1, 31, 513, 1024, 2047, 2049, 4100, 5000)]
    out, err = _run(genes, kernel, "host", scoring, affine=affine)
    assert "err" not in out, out
    p, h = _want(genes, scoring, affine)
    assert out["pen"] == p and out["hs"] == h
    st = out["stats"]
    assert st["mode"] in mode, st
    assert st["guard_checked"] >= len(p) and st["guard_reruns"] == 0, (st, err[-800:])


@pytest.mark.parametrize("fin", ["host", "device"])
def test_guard_bits_device_and_host_finalize(fin):
    """nw_align_bits' column sum through both finalizes, pgap 1 and 2."""
    genes = _genes(15, n=6)
    for scoring in ((3, 2), (1, 1)):
        out, err = _run(genes, "nw_align_bits", fin, scoring)
        p, h = _want(genes, scoring, False)
        assert out["pen"] == p and out["hs"] == h
        assert out["stats"]["guard_checked"] >= len(p) and out["stats"]["guard_reruns"] == 0, err[-800:]


_LIN_MSA = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import seqalign
genes = [bytes.fromhex(g) for g in json.loads(sys.stdin.read())]
k = len(genes)
ids = np.arange(k * (k - 1) // 2, dtype=np.int64)
out = {}
with seqalign.Engine(device=0, linear_space=2) as e:
    e.set_sequences(genes)
    pen, hs = e.align_pairs(ids, 3, 2)
    out["lin"] = {"pen": [int(v) for v in pen], "hs": [x.tobytes().hex() for x in hs], "stats": e.stats()}
with seqalign.Engine(device=0) as e:
    e.set_sequences(genes)
    rows, sop = e.msa(3, 2)
    out["msa"] = {"rows": [r.hex() if isinstance(r, (bytes, bytearray)) else r for r in rows], "sop": int(sop),
                  "stats": e.stats()}
print(json.dumps(out))
"""


def test_guard_linear_space_and_msa():
    """The linear-space traceback (f2: pass 1 gives H(m, n)) and the MSA's
    profile merges (f3: nw_profile's H(m, n) against each merge's path cost)
    are checked too."""
    r = random.Random(99)
    base = bytes(r.choice(ACGT) for _ in range(1800))
    genes = [bytes(r.choice(ACGT) for _ in range(L)) for L in (700, 1500)] + [base, base[:900] + base[950:]]
    res = subprocess.run([sys.executable, "-c", _LIN_MSA, os.path.dirname(seqalign.__file__)],
                         input=json.dumps([g.hex() for g in genes]).encode(), stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, timeout=120)
    assert res.returncode == 0, res.stderr.decode()[-2000:]
    out = json.loads(res.stdout.decode().strip().splitlines()[-1])
    p, h = _want(genes, (3, 2), False)
    assert out["lin"]["pen"] == p and out["lin"]["hs"] == h
    assert out["lin"]["stats"]["linear_space_pairs"] == len(p) and out["lin"]["stats"]["guard_checked"] >= len(p)
    orows, osop = oracle.msa(genes, 3, 2)
    assert out["msa"]["sop"] == osop
    assert out["msa"]["stats"]["guard_checked"] == len(genes) - 1


def test_guard_off_is_unchecked():
    """NWK_GUARD=0 (A/B runs) turns the check off: nothing is counted."""
    genes = _genes(14, n=4)
    out, _ = _run(genes, "nw_align_col", "host", (3, 2), NWK_GUARD="0")
    assert out["stats"]["guard_checked"] == 0
