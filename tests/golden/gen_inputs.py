"""Deterministic inputs for the large golden sets (no reference needed).

edge16: long, ragged pairs at the penalty limits of the 4-bit / packed-int16
kernels (2*pgap + pxy <= 15; SURVEY §8 a2, DESIGN §3.2 int16 headroom).
The set mixes a random ACGT sequence, a two-letter one, a 60k base and a
near-identical mutated copy cut to 47,111 characters -- long diagonal runs
make G = H - (i+j)*pgap fall by 2*pgap per row, the steepest span the
int16-relative fill has to hold, and the cut leaves a 12.9k-column gap run.
"""
import random

EDGE16_PENALTIES = [(1, 7), (0, 7), (15, 0), (13, 1)]


def _rand(r, n, alpha):
    return "".join(r.choice(alpha) for _ in range(n))


def _mutate(r, base, sub, indel, alpha="ACGT"):
    s = []
    for c in base:
        u = r.random()
        if u < indel / 2:
            continue
        if u < indel:
            s.append(r.choice(alpha))
        s.append(r.choice(alpha) if r.random() < sub else c)
    return "".join(s)


def edge16_genes(pxy, pgap):
    r = random.Random(1000 + 31 * pxy + pgap)
    s0 = _rand(r, 20000, "ACGT")
    s1 = _rand(r, 33333, "AC")
    s2 = _rand(r, 60000, "ACGT")
    s3 = _mutate(r, s2, 0.01, 0.002)[:47111]
    return [s.encode() for s in (s0, s1, s2, s3)]
