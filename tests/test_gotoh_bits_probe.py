"""Bit-sliced Gotoh step (tools/probe/gotoh_bits.h): the planes' algebra against
the oracle's affine variant (oracle/nw_oracle.c nwo_pair_affine).

The probe is the design for a future affine bit-plane kernel.
tools/probe/gotoh_sim.cpp runs its step one cell at a time on the host and
walks nwo_pair_affine's traceback over the four bits the step stores
(D, F-source, E-extend, F-extend), so a pass here pins both the score and the
stored bits, for C5's scoring (pxy 3, go 3, ge 1) and four others (go = 0
included: the linear case)."""
import os
import random
import subprocess

import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCORINGS = [(3, 3, 1), (3, 0, 2), (1, 2, 1), (4, 5, 2), (0, 1, 1)]


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("gotoh") / "gotoh_sim")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools/probe/gotoh_sim.cpp")],
                   check=True)
    return exe


def _pairs(seed, count, maxlen):
    rng = random.Random(seed)
    out = []
    for t in range(count):
        m, n = rng.randint(1, maxlen), rng.randint(1, maxlen)
        x = "".join(rng.choice("ACGT") for _ in range(m))
        if t % 3 == 0:  # a shared prefix: long diagonal runs, then gaps
            y = x[:n] + "".join(rng.choice("ACGT") for _ in range(max(0, n - m)))
        else:  # skewed alphabets: many ties between the three states
            y = "".join(rng.choice("ACGT"[:rng.randint(1, 4)]) for _ in range(n))
        out.append((x, y))
    return out


@pytest.mark.parametrize("pxy,go,ge", SCORINGS)
def test_gotoh_bits_alignment_matches_oracle(sim, pxy, go, ge):
    prs = _pairs(100 * pxy + 10 * go + ge, 120, 80)
    inp = "%d %d %d trace\n" % (pxy, go, ge) + "".join("%s %s\n" % p for p in prs)
    out = subprocess.run([sim], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()
    assert len(out) == len(prs)
    for (x, y), line in zip(prs, out):
        h, a1, a2 = line.split()
        pen, e1, e2 = oracle.pair_affine(x, y, pxy, go, ge)
        assert (int(h), a1.encode(), a2.encode()) == (pen, e1, e2), (x, y)


def test_gotoh_bits_score_longer_pairs(sim):
    """C5's scoring on longer, unrelated pairs (differences spread over the whole range)."""
    prs = _pairs(17, 6, 700)
    inp = "3 3 1\n" + "".join("%s %s\n" % p for p in prs)
    out = subprocess.run([sim], input=inp, capture_output=True, text=True, check=True).stdout.split()
    assert [int(v) for v in out] == [oracle.score_affine(x, y, 3, 3, 1) for x, y in prs]


@pytest.mark.gpu
def test_gotoh_bits_gpu_band_scores():
    """The step in nw_align_bits' anti-diagonal band layout on the GPU
    (tools/probe/gotoh_gpu.hip, built by __graft_entry__.build): H[m][n] of
    one-band pairs (m <= 2048) against the oracle, C5's scoring."""
    exe = os.path.join(ROOT, "tools", "probe", "gotoh_gpu")
    assert os.path.exists(exe), "tools/probe/gotoh_gpu not built (run __graft_entry__.build())"
    rng = random.Random(23)
    prs = []
    for t in range(48):
        m = [1, 2, 31, 32, 33, 2047, 2048][t] if t < 7 else rng.randint(1, 2048)
        n = [1, 5, 64, 65, 3000, 1, 2100][t] if t < 7 else rng.randint(1, 3000)
        x = "".join(rng.choice("ACGT") for _ in range(m))
        if t % 4 == 1:
            y = x[:n] + "".join(rng.choice("ACGT") for _ in range(max(0, n - m)))
        else:
            y = "".join(rng.choice("ACGT"[:rng.randint(2, 4)]) for _ in range(n))
        prs.append((x, y))
    inp = "".join("%s %s\n" % p for p in prs)
    out = subprocess.run([exe, "check"], input=inp, capture_output=True, text=True, timeout=120, check=True)
    got = [int(v) for v in out.stdout.split()]
    assert got == [oracle.score_affine(x, y, 3, 3, 1) for x, y in prs]


@pytest.mark.gpu
def test_gotoh_bits_gpu_chained_bands():
    """The same step with band hand-off (tools/probe/gotoh_chain.hip: each band's
    last row published as {epoch | plane word} granules and polled by the band
    below): pairs of 1-4 bands against the oracle's H[m][n], C5's scoring."""
    exe = os.path.join(ROOT, "tools", "probe", "gotoh_chain")
    assert os.path.exists(exe), "tools/probe/gotoh_chain not built (run __graft_entry__.build())"
    rng = random.Random(29)
    prs = []
    sizes = [(2048, 100), (2049, 100), (4096, 64), (4097, 1), (1, 5000), (6000, 33), (5000, 2500), (7000, 3000)]
    for t in range(24):
        m, n = sizes[t] if t < len(sizes) else (rng.randint(1, 7000), rng.randint(1, 3000))
        x = "".join(rng.choice("ACGT") for _ in range(m))
        if t % 3 == 1:
            y = x[:n] + "".join(rng.choice("ACGT") for _ in range(max(0, n - m)))
        else:
            y = "".join(rng.choice("ACGT"[:rng.randint(2, 4)]) for _ in range(n))
        prs.append((x, y))
    inp = "".join("%s %s\n" % p for p in prs)
    out = subprocess.run([exe, "check"], input=inp, capture_output=True, text=True, timeout=120, check=True)
    got = [int(v) for v in out.stdout.split()]
    assert got == [oracle.score_affine(x, y, 3, 3, 1) for x, y in prs]


@pytest.mark.gpu
def test_gotoh_bits_gpu_stored_bits_walk():
    """Fill + store on the GPU, walk on the host: gotoh_chain `trace` stores every
    cell's four words (D, F-source, E-extend, F-extend) in the probe's 4-step
    block layout and walks nwo_pair_affine's traceback over them; the strings
    must equal the oracle's alignment, band edges and ties included."""
    exe = os.path.join(ROOT, "tools", "probe", "gotoh_chain")
    assert os.path.exists(exe), "tools/probe/gotoh_chain not built (run __graft_entry__.build())"
    rng = random.Random(31)
    prs = []
    sizes = [(2048, 300), (2049, 2049), (4100, 1000), (1, 700), (3000, 1), (5000, 2200)]
    for t in range(16):
        m, n = sizes[t] if t < len(sizes) else (rng.randint(1, 5000), rng.randint(1, 2500))
        x = "".join(rng.choice("ACGT") for _ in range(m))
        if t % 3 == 1:
            y = x[:n] + "".join(rng.choice("ACGT") for _ in range(max(0, n - m)))
        else:
            y = "".join(rng.choice("ACGT"[:rng.randint(2, 4)]) for _ in range(n))
        prs.append((x, y))
    inp = "".join("%s %s\n" % p for p in prs)
    out = subprocess.run([exe, "trace"], input=inp, capture_output=True, text=True, timeout=120, check=True)
    lines = out.stdout.splitlines()
    assert len(lines) == len(prs)
    for (x, y), line in zip(prs, lines):
        h, a1, a2 = line.split()
        pen, e1, e2 = oracle.pair_affine(x, y, 3, 3, 1)
        assert (int(h), a1.encode(), a2.encode()) == (pen, e1, e2), (len(x), len(y))


@pytest.mark.gpu
def test_gotoh_bits_gpu_device_walk():
    """Fill, store and walk all on the GPU (gotoh_chain `dtrace`: gotoh_walk, one
    wave per pair over LDS tiles of the stored words): the alignments equal the
    oracle's.  The probe's walk buffer wants pairs of equal m + n."""
    exe = os.path.join(ROOT, "tools", "probe", "gotoh_chain")
    assert os.path.exists(exe), "tools/probe/gotoh_chain not built (run __graft_entry__.build())"
    rng = random.Random(37)
    prs = []
    for t, m in enumerate([2048, 2049, 4097, 1, 5999, 3000, 100, 4500, 2500, 5000, 1500, 3500]):
        n = 6000 - m
        x = "".join(rng.choice("ACGT") for _ in range(m))
        if t % 3 == 1:
            y = x[:n] + "".join(rng.choice("ACGT") for _ in range(max(0, n - m)))
        else:
            y = "".join(rng.choice("ACGT"[:rng.randint(2, 4)]) for _ in range(n))
        prs.append((x, y))
    inp = "".join("%s %s\n" % p for p in prs)
    out = subprocess.run([exe, "dtrace"], input=inp, capture_output=True, text=True, timeout=120, check=True)
    lines = out.stdout.splitlines()
    assert len(lines) == len(prs)
    for (x, y), line in zip(prs, lines):
        h, a1, a2 = line.split()
        pen, e1, e2 = oracle.pair_affine(x, y, 3, 3, 1)
        assert (int(h), a1.encode(), a2.encode()) == (pen, e1, e2), (len(x), len(y))
