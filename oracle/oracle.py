"""ctypes binding of oracle/_build/libnworacle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement (oracle/nw_oracle.c) of the reference path; see that
file's header for the reference file:line each function follows.  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker.  The product never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libnworacle.so")
CLI = os.path.join(HERE, "_build", "nw_oracle")
REF_DIR = os.path.join(HERE, "_ref")

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        L.nwo_pair.restype = ctypes.c_int
        L.nwo_pair.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P]
        L.nwo_pair_affine.restype = ctypes.c_int
        L.nwo_pair_affine.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P]
        L.nwo_problem_hash.restype = None
        L.nwo_problem_hash.argtypes = [P, P, ctypes.c_int, P]
        L.nwo_chain.restype = None
        L.nwo_chain.argtypes = [P, ctypes.c_long, P]
        L.nwo_all.restype = ctypes.c_int
        L.nwo_all.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P]
        L.nwo_score.restype = ctypes.c_int
        L.nwo_score.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.nwo_score_affine.restype = ctypes.c_int
        L.nwo_score_affine.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.nwo_sha512_hex.restype = None
        L.nwo_sha512_hex.argtypes = [P, ctypes.c_size_t, P]
        _lib = L
    return _lib


def _b(s):
    return s if isinstance(s, bytes) else s.encode("latin-1")


def pair(x, y, pxy, pgap):
    """skel getMinimumPenalty + trim: (penalty, align1, align2)."""
    x, y = _b(x), _b(y)
    cap = max(len(x) + len(y), 1)
    a1 = ctypes.create_string_buffer(cap)
    a2 = ctypes.create_string_buffer(cap)
    alen = ctypes.c_int()
    pen = lib().nwo_pair(x, len(x), y, len(y), pxy, pgap, a1, a2, ctypes.byref(alen))
    if pen == -2 ** 31:
        raise MemoryError("oracle: DP allocation failed")
    return pen, a1.raw[:alen.value], a2.raw[:alen.value]


def score(x, y, pxy, pgap):
    """dp[m][n] of skel's fill (skel:195-226) in O(n) memory, no traceback."""
    x, y = _b(x), _b(y)
    v = lib().nwo_score(x, len(x), y, len(y), pxy, pgap)
    if v == -2 ** 31:
        raise MemoryError("oracle: row allocation failed")
    return v


def score_affine(x, y, pxy, go, ge):
    """H[m][n] of the affine variant in O(n) memory, no traceback."""
    x, y = _b(x), _b(y)
    v = lib().nwo_score_affine(x, len(x), y, len(y), pxy, go, ge)
    if v == -2 ** 31:
        raise MemoryError("oracle: row allocation failed")
    return v


def pair_affine(x, y, pxy, go, ge):
    """Affine-gap variant (build-defined): (penalty, align1, align2)."""
    x, y = _b(x), _b(y)
    cap = max(len(x) + len(y), 1)
    a1 = ctypes.create_string_buffer(cap)
    a2 = ctypes.create_string_buffer(cap)
    alen = ctypes.c_int()
    pen = lib().nwo_pair_affine(x, len(x), y, len(y), pxy, go, ge, a1, a2, ctypes.byref(alen))
    if pen == -2 ** 31:
        raise MemoryError("oracle: DP allocation failed")
    return pen, a1.raw[:alen.value], a2.raw[:alen.value]


def all_pairs_affine(genes, pxy, go, ge):
    """(hash, penalties, per-pair problemhash hex) of the affine variant, canonical order."""
    pens, hs = [], []
    for i in range(1, len(genes)):
        for j in range(i):
            p, a1, a2 = pair_affine(genes[i], genes[j], pxy, go, ge)
            pens.append(p)
            hs.append(problem_hash(a1, a2))
    return chain(hs), pens, hs


def problem_hash(a1, a2):
    out = ctypes.create_string_buffer(129)
    lib().nwo_problem_hash(_b(a1), _b(a2), len(a1), out)
    return out.value.decode()


def sha512_hex(data):
    d = _b(data)
    out = ctypes.create_string_buffer(129)
    lib().nwo_sha512_hex(d, len(d), out)
    return out.value.decode()


def chain(hex_hashes):
    buf = "".join(hex_hashes).encode()
    out = ctypes.create_string_buffer(129)
    lib().nwo_chain(buf, len(hex_hashes), out)
    return out.value.decode()


def all_pairs(genes, pxy, pgap):
    """skel getMinimumPenalties: (hash, penalties list, per-pair hex hashes)."""
    bs = [_b(g) for g in genes]
    k = len(bs)
    offs = np.zeros(k + 1, dtype=np.int64)
    if k:
        offs[1:] = np.cumsum([len(b) for b in bs])
    data = b"".join(bs) or b"\0"
    P = k * (k - 1) // 2
    pen = np.zeros(max(P, 1), dtype=np.int32)
    hs = ctypes.create_string_buffer(max(P, 1) * 128 + 1)
    out = ctypes.create_string_buffer(129)
    rc = lib().nwo_all(data, offs.ctypes.data_as(ctypes.c_void_p), k, pxy, pgap,
                       pen.ctypes.data_as(ctypes.c_void_p), hs, out)
    if rc != 0:
        raise MemoryError("oracle: allocation failed")
    raw = hs.raw
    return out.value.decode(), [int(v) for v in pen[:P]], [raw[128 * p:128 * p + 128].decode() for p in range(P)]


def profile_align(X, Y, pxy, pgap):
    """Profile-profile NW (msa_oracle.c): X, Y lists of equal-length rows -> (cost, ops 'D'/'U'/'L')."""
    X, Y = [_b(r) for r in X], [_b(r) for r in Y]
    lx, ly = len(X[0]), len(Y[0])
    ops = ctypes.create_string_buffer(lx + ly + 1)
    n = ctypes.c_int()
    lib().nwo_profile_align.restype = ctypes.c_longlong
    c = lib().nwo_profile_align(b"".join(X), len(X), lx, b"".join(Y), len(Y), ly, pxy, pgap, ops, ctypes.byref(n))
    return c, ops.raw[:n.value].decode()


def sop(rows, pxy, pgap):
    """Sum-of-pairs score of equal-length rows."""
    rows = [_b(r) for r in rows]
    lib().nwo_sop.restype = ctypes.c_longlong
    return lib().nwo_sop(b"".join(rows), len(rows), len(rows[0]) if rows else 0, pxy, pgap)


def msa(genes, pxy, pgap, penalties=None):
    """Progressive SoP MSA (build-defined): (rows in input order, SoP score)."""
    bs = [_b(g) for g in genes]
    k = len(bs)
    if penalties is None:
        penalties = all_pairs(bs, pxy, pgap)[1]
    offs = np.zeros(k + 1, dtype=np.int64)
    if k:
        offs[1:] = np.cumsum([len(b) for b in bs])
    cap = max(1, int(offs[-1]))
    rows = ctypes.create_string_buffer(max(k, 1) * cap)
    pen = np.array(list(penalties) or [0], dtype=np.int32)
    ln = ctypes.c_int()
    sp = ctypes.c_longlong()
    rc = lib().nwo_msa(b"".join(bs) or b"\0", offs.ctypes.data_as(ctypes.c_void_p), k, pxy, pgap,
                       pen.ctypes.data_as(ctypes.c_void_p), rows, cap, ctypes.byref(ln), ctypes.byref(sp))
    if rc != 0:
        raise MemoryError("oracle: msa failed")
    raw = rows.raw
    return [raw[r * cap:r * cap + ln.value] for r in range(k)], sp.value


def run_cli(exe, text, timeout=3600, env=None):
    """Runs a program with the reference's stdin/stdout contract.
    Returns (time_us, hash, penalties)."""
    r = subprocess.run([exe], input=_b(text), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=timeout, env=env)
    if r.returncode != 0:
        raise RuntimeError("%s exited %d: %s" % (exe, r.returncode, r.stderr[-2000:].decode("latin-1")))
    lines = r.stdout.decode("latin-1").split("\n")
    ti = max(i for i, l in enumerate(lines) if l.startswith("Time: "))
    us = int(lines[ti].split()[1])
    return us, lines[ti + 1], [int(t) for t in lines[ti + 2].split()]
