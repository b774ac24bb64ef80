"""Path deviation from the proportional diagonal for workload pairs (GPU).
For pair (i, j): max over the alignment of |col - row * n / m| (row = x index).
Affine workloads (c5) trace with their (go, ge).
usage: python tools/pathdev.py [workload=c3] [npairs=16]"""
import math
import os
import sys

sys.path.insert(0, "multiple-sequence-alignment-openmp-openmpi_amd")
import seqalign, workloads  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
npairs = int(sys.argv[2]) if len(sys.argv) > 2 else 16
if wl == "big13":  # the reference's own input (testing3), all 78 pairs unless npairs given
    pxy, pgap, genes = seqalign.parse_input(open(os.path.join(workloads.GOLDEN_DATA, "mseq-big13-example.txt"), "rb").read())
    affine = None
    npairs = int(sys.argv[2]) if len(sys.argv) > 2 else 78
else:
    desc, k, L, pxy, pgap, affine = workloads.SYNTH[wl]
    genes = workloads.synth(k, L)
with seqalign.Engine(device=0) as e:
    devs = []
    for p in range(npairs):
        i = int((1 + math.isqrt(1 + 8 * p)) // 2)
        j = p - i * (i - 1) // 2
        x, y = genes[i], genes[j]
        if affine:
            pen, a1, a2 = e.get_minimum_penalty_affine(x, y, pxy, affine[0], affine[1])
        else:
            pen, a1, a2 = e.get_minimum_penalty(x, y, pxy, pgap)
        m, n = len(x), len(y)
        row = col = 0
        worst = 0
        for c1, c2 in zip(a1, a2):
            if c1 != 95: row += 1
            if c2 != 95: col += 1
            worst = max(worst, abs(col - row * n / m))
        devs.append(int(worst))
        print("pair", p, (i, j), (m, n), "penalty", pen, "max |dev|", int(worst), flush=True)
print("max over pairs", max(devs), "sorted", sorted(devs))
