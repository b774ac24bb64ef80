"""Debug probe: progressive MSA through nwk_msa on a few shapes, against the oracle.

Run on the GPU box (NWK_WATCHDOG=<s> reports wave markers of a launch that does not finish).
"""
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle  # noqa: E402
import seqalign  # noqa: E402


def main():
    e = seqalign.Engine(device=0, verbose=int(os.environ.get("PROBE_VERBOSE", "0")))
    for (m, n) in [(1200, 1100), (300, 1100), (1200, 50), (600, 200), (520, 70), (100, 100)]:
        r = random.Random(m * 7 + n)
        genes = [bytes(r.choice(b"ACGT") for _ in range(m)), bytes(r.choice(b"ACGT") for _ in range(n))]
        e.set_sequences(genes)
        rows, s = e.msa(3, 2)
        want_rows, want = oracle.msa(genes, 3, 2)
        print("k=2 %5d x %5d: gpu %d oracle %d rows %s" % (n, m, s, want, "same" if rows == want_rows else "DIFF"),
              flush=True)
    e.close()


if __name__ == "__main__":
    main()
