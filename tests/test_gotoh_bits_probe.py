"""Bit-sliced Gotoh step (csrc/nwk_gotoh_planes.h): the planes' algebra against
the oracle's affine variant (oracle/nw_oracle.c nwo_pair_affine).

The step is nw_align_gotoh's (csrc/nwk_gotoh_planes.h; GPU parity in
tests/test_gpu_gotoh.py).  tools/probe/gotoh_sim.cpp runs it one cell at a time on the host and
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
