"""Host logic and the C-ABI library, without a GPU.

Covers: libnwk.so loads and exports every entry point include/nwk.h declares;
SHA-512 / hash chain (sha512.hh contract, skel:155-159); the LPT shard of
canonical pair ids; result-record packing of the all-gather; stdin parsing;
and that the product fails loudly (no CPU fallback) when no device exists.
"""
import hashlib
import os
import re

import numpy as np
import pytest

import oracle
import seqalign
import dist as nwdist
from conftest import REPO, case_input

HEADER = os.path.join(REPO, "include", "nwk.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(nwk_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    return seqalign.load_library()


def test_library_exports_every_header_symbol(lib):
    syms = header_symbols()
    assert len(syms) >= 13
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(seqalign.SIGNATURES), "ctypes table out of sync with include/nwk.h"


@pytest.mark.parametrize("n", [0, 1, 3, 111, 112, 113, 127, 128, 129, 239, 240, 255, 256, 1000, 70001])
def test_sha512_hex_matches_fips(lib, n):
    data = bytes((i * 131 + 7) & 0xff for i in range(n))
    assert seqalign.sha512_hex(data) == hashlib.sha512(data).hexdigest()
    assert oracle.sha512_hex(data) == hashlib.sha512(data).hexdigest()


def test_chain_hash_matches_reference_stream(golden):
    c = golden["mseq1"]
    hs = np.array([list(bytes.fromhex(p["problemhash"])) for p in c["pairs"]], dtype=np.uint8)
    assert seqalign.chain_hash(hs) == c["hash"]
    assert seqalign.chain_hash(np.zeros((0, 64), dtype=np.uint8)) == ""


@pytest.mark.parametrize("P", [0, 1, 2, 3, 300])
def test_chain_stream_any_order_equals_chain(P):
    """nwk_chain_* (the skel:159 chain advanced by a worker thread as records
    arrive) fed in random chunks and order equals the one-shot chain, which
    equals hashlib's sha512 over the concatenations (skel:155-159 contract)."""
    rnd = np.random.RandomState(P)
    hs = rnd.randint(0, 256, size=(P, 64)).astype(np.uint8)
    pen = rnd.randint(0, 10 ** 6, size=P).astype(np.int32)
    acc = ""
    for p in range(P):
        acc = hashlib.sha512((acc + hs[p].tobytes().hex()).encode()).hexdigest()
    assert seqalign.chain_hash(hs) == acc
    ch = seqalign.ChainStream(P)
    order = rnd.permutation(P)
    for part in np.array_split(order, min(P, 7) or 1):
        ch.feed(part, pen[part], hs[part])
    h, pen2, hs2 = ch.finish()
    ch.close()
    assert h == acc
    assert (pen2 == pen).all() and (hs2 == hs).all()


def test_chain_stream_rejects_missing_and_duplicate_pairs():
    hs = np.zeros((4, 64), dtype=np.uint8)
    ch = seqalign.ChainStream(4)
    ch.feed([0, 2], [0, 0], hs[:2])
    with pytest.raises(seqalign.NwkError):
        ch.feed([2], [0], hs[:1])  # fed twice
    with pytest.raises(seqalign.NwkError):
        ch.feed([4], [0], hs[:1])  # out of range
    with pytest.raises(seqalign.NwkError):
        ch.feed([1, 1], [0, 0], hs[:2])  # twice within one batch
    with pytest.raises(seqalign.NwkError) as e:
        ch.finish()  # pairs 1 and 3 never fed
    assert "never fed" in str(e.value)
    ch.close()


def test_pair_index_roundtrip():
    p = 0
    for i in range(1, 300):
        for j in range(i):
            assert seqalign.pair_index(i, j) == p
            assert seqalign.pair_ij(p) == (i, j)
            p += 1


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_pairs_partition(world):
    rnd = np.random.RandomState(world)
    lengths = list(rnd.randint(0, 5000, size=23))
    k = len(lengths)
    P = k * (k - 1) // 2
    shards = [seqalign.shard_pairs(lengths, r, world) for r in range(world)]
    allids = np.concatenate(shards)
    assert sorted(allids.tolist()) == list(range(P))
    cost = [0.0] * world
    for r, s in enumerate(shards):
        assert list(s) == sorted(s)
        for p in s:
            i, j = seqalign.pair_ij(int(p))
            cost[r] += lengths[i] * lengths[j] + 1
    # LPT bound: makespan <= mean + max single job
    mx = max(lengths[i] * lengths[j] for i in range(k) for j in range(i)) + 1
    assert max(cost) <= sum(cost) / world + mx
    assert [list(x) for x in shards] == [list(seqalign.shard_pairs(lengths, r, world)) for r in range(world)]


def test_big13_shard_balance(golden):
    _, _, genes = case_input(golden["big13"])
    lengths = [len(g) for g in genes]
    for world in (2, 4, 8):
        costs = []
        for r in range(world):
            c = 0
            for p in seqalign.shard_pairs(lengths, r, world):
                i, j = seqalign.pair_ij(int(p))
                c += lengths[i] * lengths[j]
            costs.append(c)
        assert max(costs) / (sum(costs) / world) < 1.06, (world, costs)


def test_records_roundtrip():
    rnd = np.random.RandomState(3)
    P = 17
    ids = rnd.permutation(P)
    pen = rnd.randint(-50, 10 ** 6, size=P).astype(np.int32)
    hs = rnd.randint(0, 256, size=(P, 64)).astype(np.uint8)
    recs = [nwdist.pack_records(ids[a:b], pen[a:b], hs[a:b], 9) for a, b in ((0, 9), (9, 17))]
    p2, h2 = nwdist.unpack_records(np.concatenate(recs), P)
    order = np.argsort(ids)
    assert (p2 == pen[order]).all() and (h2 == hs[order]).all()
    with pytest.raises(RuntimeError):
        nwdist.unpack_records(recs[0], P)


def test_parse_input_matches_cin_tokens():
    pxy, pgap, genes = seqalign.parse_input(b"3 2\n3\nAGGGCT\n AGGCA\tAAAGGGCT extra\n")
    assert (pxy, pgap, genes) == (3, 2, [b"AGGGCT", b"AGGCA", b"AAAGGGCT"])


def test_no_device_fails_loudly(lib):
    if seqalign.device_count() > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(seqalign.NwkError) as e:
        seqalign.Engine()
    assert e.value.code == -3
    with pytest.raises(seqalign.NwkError):
        seqalign.getMinimumPenalties([b"AC", b"CA"], 2, 3, 2, [0])


@pytest.mark.parametrize("field,value", [("kernel", 8), ("kernel", -1), ("finalize", 4), ("bits", 5), ("task_order", 3),
                                         ("task_order", -1)])
def test_ctx_create_rejects_bad_options(lib, field, value):
    """nwk_ctx_create checks its options before looking for a device: a bad
    kernel / finalize / bits value is NWK_EINVAL with or without a GPU."""
    import ctypes

    o = seqalign.Opts()
    lib.nwk_opts_default(ctypes.byref(o))
    setattr(o, field, value)
    ctx = ctypes.c_void_p()
    assert lib.nwk_ctx_create(ctypes.byref(o), ctypes.byref(ctx)) == -1
    assert field in lib.nwk_last_error().decode()
    assert not ctx.value


def test_parse_fasta_records():
    """FASTA input -- records in order, wrapped lines joined, blanks/comments skipped."""
    text = b">s1 first\nACGT\nAC GT\n\n>s2\n;comment\nTTTT\n>empty\n>s4\r\nGG\r\n"
    assert seqalign.parse_fasta(text) == [b"ACGTACGT", b"TTTT", b"", b"GG"]
    assert seqalign.parse_fasta(b"ACG\nT\n>x\nA\n") == [b"ACGT", b"A"]
    assert seqalign.parse_fasta(b"") == []


def test_read_input_detects_fasta(tmp_path):
    p = tmp_path / "in.fa"
    p.write_bytes(b"\n>a\nACGT\n>b\nAGT\n")
    assert seqalign.read_input(str(p), 5, 1) == (5, 1, [b"ACGT", b"AGT"])
    q = tmp_path / "in.txt"
    q.write_bytes(b"3 2 2\nACGT\nAGT\n")
    assert seqalign.read_input(str(q)) == (3, 2, [b"ACGT", b"AGT"])
