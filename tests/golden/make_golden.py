#!/usr/bin/env python3
"""Regenerates tests/golden/golden.json -- the golden vectors for the path.

Run in the build container (where /root/reference exists), after
``oracle/build_ref.sh`` has compiled the REFERENCE programs into oracle/_ref/:

    python tests/golden/make_golden.py

Sources of truth, per case (recorded in each entry's "source"):
  * "skel"          oracle/_ref/skel = testing3/seqalign-mpi-skeleton.cpp
                    compiled from the reference sources, run here.
  * "skel_debug"    oracle/_ref/skel_debug = root seqalign-mpi-skeleton.cpp,
                    whose debug prints (skel:158-169) give the per-pair
                    penalty and problemhash stream.
  * "published"     numbers recorded by the reference author
                    (testing3/sequential.txt:2-3, testing15/*.out:2-3,
                    docs/Project2B.pdf p.7) -- copied here as data.

The GPU box never sees /root/reference: only golden.json and the input data
files under tests/golden/data/ travel.
"""
import json
import os
import random
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_BIN = os.path.join(REPO, "oracle", "_ref")
DATA = os.path.join(HERE, "data")


def run_skel(text, debug=False, timeout=3600):
    exe = os.path.join(REF_BIN, "skel_debug" if debug else "skel")
    out = subprocess.run([exe], input=text.encode("latin-1"), stdout=subprocess.PIPE,
                         check=True, timeout=timeout).stdout.decode("latin-1")
    lines = out.split("\n")
    # final three lines: Time, hash, penalties
    ti = max(i for i, l in enumerate(lines) if l.startswith("Time: "))
    h = lines[ti + 1]
    pens = [int(t) for t in lines[ti + 2].split()]
    pairs = None
    if debug:
        pairs = []
        body = lines[:ti]
        i = 0
        while i < len(body):
            if body[i].startswith("< "):
                pen = int(body[i + 1])
                ph = body[i + 2].split(") ", 1)[1]
                pairs.append({"penalty": pen, "problemhash": ph})
                i += 5
            else:
                i += 1
    return h, pens, pairs


def mk_input(pxy, pgap, seqs):
    return "%d\n%d\n%d\n%s\n" % (pxy, pgap, len(seqs), "\n".join(seqs))


def rnd_seqs(seed, k, L, alphabet="ACGT"):
    r = random.Random(seed)
    return ["".join(r.choice(alphabet) for _ in range(L)) for _ in range(k)]


def mutated(seed, base, k, sub=0.1, indel=0.02, alphabet="ACGT"):
    r = random.Random(seed)
    out = []
    for _ in range(k):
        s = []
        for c in base:
            u = r.random()
            if u < indel / 2:
                continue
            if u < indel:
                s.append(r.choice(alphabet))
            s.append(r.choice(alphabet) if r.random() < sub else c)
        out.append("".join(s))
    return out


def main():
    cases = []

    def add(name, text=None, file=None, debug=False, source="skel", expect=None):
        if file is not None:
            text = open(os.path.join(DATA, file), "rb").read().decode("latin-1")
        if expect is None:
            h, pens, pairs = run_skel(text, debug=debug)
        else:
            h, pens = expect
            pairs = None
        e = {"name": name, "hash": h, "penalties": pens, "source": source}
        if file is not None:
            e["file"] = file
        else:
            e["input"] = text
        if pairs is not None:
            e["pairs"] = pairs
        cases.append(e)
        print(name, h[:16], len(pens), file=sys.stderr)

    # Reference data files (inputs copied under data/).
    add("mseq", file="mseq.dat", debug=True, source="skel_debug; Project2B.pdf p.7")
    add("mseq1", file="mseq1.dat", debug=True, source="skel_debug; testing15/mseq1-12node-16-cpt-1-npn-snowy.out:14-15")
    add("xulin_test", file="xulin_test.txt", debug=True, source="skel_debug (submit/xulin_test.txt, pxy=5 pgap=1)")
    add("xulin_mixedcase", file="xulin.dat", source="skel (testing/xulin.dat: ACGT/acgt mixed, L up to 70k)")
    # Published full-size answers (big13: testing3/sequential.txt:2-3; big13-2
    # = big13 with sequences permuted [2..12,1,0]: testing15/big13-2-*.out:2-3).
    seq_txt = open("/root/reference/testing3/sequential.txt").read().split("\n") \
        if os.path.exists("/root/reference/testing3/sequential.txt") else None
    if seq_txt is not None:
        add("big13", file="mseq-big13-example.txt", source="published testing3/sequential.txt:2-3",
            expect=(seq_txt[1].strip(), [int(t) for t in seq_txt[2].split()]))
        b2 = open("/root/reference/testing15/big13-2-12node-16-cpt-1-npn-snowy.out").read().split("\n")
        cases.append({"name": "big13_2", "file": "mseq-big13-example.txt", "permute": [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 1, 0],
                      "hash": b2[1].strip(), "penalties": [int(t) for t in b2[2].split()],
                      "source": "published testing15/big13-2-12node-16-cpt-1-npn-snowy.out:2-3"})

    # Edge cases (inline inputs).
    add("k0", mk_input(3, 2, []))
    add("k1", mk_input(3, 2, ["ACGT"]))
    add("k2_same", mk_input(3, 2, ["ACGT", "ACGT"]), debug=True)
    add("k2_A_C", mk_input(3, 2, ["A", "C"]), debug=True)
    add("k2_A_CC", mk_input(3, 2, ["A", "CC"]), debug=True)
    add("k2_AC_CA_5_1", mk_input(5, 1, ["AC", "CA"]), debug=True)
    add("k2_case", mk_input(3, 2, ["aC", "AC"]), debug=True)
    add("k3_T_GGGG", mk_input(3, 2, ["T", "GGGG", "TGGGG"]), debug=True)
    add("underscore_trim", mk_input(3, 2, ["A_C_", "_A_C", "__", "A__A_", "_"]), debug=True)
    add("zero_pen", mk_input(0, 0, rnd_seqs(11, 5, 40)), debug=True)
    add("pxy0", mk_input(0, 3, rnd_seqs(12, 5, 37)), debug=True)
    add("pgap0", mk_input(4, 0, rnd_seqs(13, 5, 33)), debug=True)
    add("neg_pxy", mk_input(-1, 2, rnd_seqs(14, 5, 30)), debug=True)
    add("neg_pgap", mk_input(3, -1, rnd_seqs(15, 5, 29)), debug=True)
    add("big_pen", mk_input(300, 200, rnd_seqs(16, 6, 90)), debug=True)
    add("huge_pen", mk_input(70000, 40000, rnd_seqs(17, 4, 50)), debug=True)
    add("ragged", mk_input(3, 2, rnd_seqs(18, 1, 1) + rnd_seqs(19, 1, 63) + rnd_seqs(20, 1, 64)
                           + rnd_seqs(21, 1, 65) + rnd_seqs(22, 1, 513) + rnd_seqs(23, 1, 700)), debug=True)
    add("bytes_alpha", mk_input(3, 2, rnd_seqs(24, 6, 120, alphabet="ACGTNacgtn*#~\x7f\x80\xfe")), debug=True)
    add("mutated", mk_input(3, 2, mutated(25, rnd_seqs(26, 1, 900)[0], 6)), debug=True)
    # Survey Appendix A synthetic: random.seed(0), 4 x 10k, choice('ACGT').
    random.seed(0)
    syn = ["".join(random.choice("ACGT") for _ in range(10000)) for _ in range(4)]
    add("syn_k4_L10k", mk_input(3, 2, syn), source="skel (SURVEY App. A synthetic)")

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
