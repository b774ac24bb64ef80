"""The BASELINE.json workloads C1-C5 as sequence sets (host-side, no GPU).

C1 mseq.dat and C2 mseq-big13-example.txt are the reference's own input
files (kept as fixtures under tests/golden/data/).  C3-C5 are synthetic,
uniform i.i.d. ACGT per SURVEY §8(d): sequence s of a config comes from its
own MT19937 stream seeded with ``seed + s`` (numpy's MT19937 bit generator,
so the bytes are identical on every box with this image).  Penalties are
the reference's 3/2 (mseq*.dat, big13); C5 is the build-defined affine
variant at go=3, ge=1.
"""
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN_DATA = os.path.join(REPO, "tests", "golden", "data")


def synth(k, L, seed=0):
    """k uniform ACGT sequences of length L; sequence s uses seed + s."""
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    out = []
    for s in range(k):
        rng = np.random.Generator(np.random.MT19937(seed + s))
        out.append(acgt[rng.integers(0, 4, L)].tobytes())
    return out


# name -> (description, k, L, pxy, pgap, affine (go, ge) or None)
SYNTH = {
    "c3": ("synthetic k=64 L=50000 ACGT", 64, 50000, 3, 2, None),
    "c4": ("synthetic k=256 L=8000 ACGT", 256, 8000, 3, 2, None),
    "c5": ("synthetic k=32 L=200000 ACGT, affine go=3 ge=1", 32, 200000, 3, 2, (3, 1)),
}


def token_text(pxy, pgap, genes):
    """The reference's stdin format (skel:40-47): pxy, pgap, k, then k tokens."""
    return b"%d\n%d\n%d\n" % (pxy, pgap, len(genes)) + b"\n".join(genes) + b"\n"


def cells(genes, ids=None):
    """Sum of m*n over the canonical pairs ids (all pairs by default)."""
    L = np.array([len(g) for g in genes], dtype=np.int64)
    k = len(L)
    if ids is None:
        # sum_{i>j} L_i L_j = ((sum L)^2 - sum L^2) / 2
        return int((int(L.sum()) ** 2 - int((L * L).sum())) // 2)
    tot = 0
    for p in ids:
        p = int(p)
        i = int((1 + (1 + 8 * p) ** 0.5) // 2)
        while i * (i - 1) // 2 > p:
            i -= 1
        while (i + 1) * i // 2 <= p:
            i += 1
        tot += int(L[i]) * int(L[p - i * (i - 1) // 2])
    return tot
