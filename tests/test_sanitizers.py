"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer.

`make asan` builds tests/native/host_selftest and the driver with the host code
of the C-ABI (nwk_runtime.cpp, sha512.cpp, seqalkway_main.cpp) instrumented.
Device code is not instrumented: GPU sanitizers are not available on this pool.
The self-test replays fixtures written here from the golden vectors and the
oracle (SHA-512, the answer-hash chain, the host finalize of traced moves, the
LPT shard, argument checks, the no-device error path); the driver parses token
and FASTA inputs with --print-inputs.  Any sanitizer report fails the test.
"""
import hashlib
import os
import random
import subprocess

import pytest

import oracle
import seqalign
from conftest import PKG, case_input, load_golden

ASAN_DIR = os.path.join(PKG, "build", "asan")
SELFTEST = os.path.join(ASAN_DIR, "host_selftest")
DRIVER = os.path.join(ASAN_DIR, "seqalkway")
# leaks inside the HIP/HSA runtimes' own initialisation are not ours
SUPP = "leak:libamdhip64\nleak:libhsa-runtime64\nleak:librccl\nleak:libhsakmt\n"


@pytest.fixture(scope="module")
def asan_env(tmp_path_factory):
    if not (os.path.exists(SELFTEST) and os.path.exists(DRIVER)):
        subprocess.run(["make", "-s", "-C", PKG, "asan"], check=True, timeout=900)
    supp = tmp_path_factory.mktemp("asan") / "lsan.supp"
    supp.write_text(SUPP)
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "abort_on_error=0:halt_on_error=1:detect_odr_violation=0"
    env["LSAN_OPTIONS"] = "suppressions=%s:print_suppressions=0" % supp
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    return env


def _clean(stderr):
    bad = ("ERROR: AddressSanitizer", "ERROR: LeakSanitizer", "runtime error:")
    return not any(b in stderr for b in bad)


def _fixture():
    lines = []
    for n in (0, 1, 111, 112, 127, 128, 129, 255, 256, 1000, 4097):
        d = bytes((i * 37 + n) & 0xff for i in range(n))
        lines.append("sha %s %s" % (d.hex() or "-", hashlib.sha512(d).hexdigest()))
    golden = load_golden()
    for c in golden:
        if "pairs" in c:
            ph = " ".join(p["problemhash"] for p in c["pairs"])
            lines.append("chain %d %s %s" % (len(c["pairs"]), c["hash"] or "-", ph))
    r = random.Random(17)
    pairs = []
    for c in golden:
        if c["name"] in ("mseq", "mseq1", "xulin_test", "ragged", "k2_A_CC", "k3_T_GGGG", "mutated", "zero_pen"):
            pxy, pgap, genes = case_input(c)
            pairs += [(genes[i], genes[j], pxy, pgap) for i in range(1, len(genes)) for j in range(i)]
    for _ in range(40):
        x = bytes(r.choice(b"ACGT") for _ in range(r.randint(0, 300)))
        y = bytes(r.choice(b"ACGT") for _ in range(r.randint(0, 300)))
        pairs.append((x, y, r.randint(0, 7), r.randint(0, 5)))
    for x, y, pxy, pgap in pairs:
        pen, a1, a2 = oracle.pair(x, y, pxy, pgap)
        mv = seqalign.moves_of(a1, a2, len(x), len(y))
        ph = oracle.problem_hash(a1, a2)
        f = [(v.decode("latin-1") if v else "-") for v in (x, y)]
        lines.append("fin %s %s %d %d %s %d %s %s %s" % (f[0], f[1], pxy, pgap, mv.decode() or "-", pen,
                                                         a1.decode("latin-1") or "-", a2.decode("latin-1") or "-", ph))
    for world in (1, 2, 3, 8):
        ls = [r.randint(0, 5000) for _ in range(r.randint(0, 30))]
        lines.append("shard %d %s" % (world, " ".join(map(str, ls))))
    return "\n".join(lines) + "\n"


def test_host_selftest_under_asan_ubsan(asan_env):
    r = subprocess.run([SELFTEST], input=_fixture().encode("latin-1"), stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, env=asan_env, timeout=600)
    err = r.stderr.decode("latin-1")
    assert r.returncode == 0, err[-4000:]
    assert _clean(err), err[-4000:]
    assert "0 failures" in r.stdout.decode()


FASTA_VARIANTS = [
    b">s1 first\nACGT\nAC GT\n\n>s2\n;comment\nTTTT\n>empty\n>s4\r\nGG\r\n",
    b"\r\n \t\n>a\r\nAC\r\n\r\nGT\r\n>b\nA C G\n",          # CRLF blank lines before the first header
    b"ACG\nT\n>x\nA\n",                                    # text before the first header
    b"  \n\n>only\n\n",
]


@pytest.mark.parametrize("idx", range(len(FASTA_VARIANTS)))
def test_driver_fasta_parser_matches_python(asan_env, tmp_path, idx):
    """The driver's --fasta and seqalign.parse_fasta give the same records (ASan build)."""
    text = FASTA_VARIANTS[idx]
    f = tmp_path / "in.fa"
    f.write_bytes(text)
    out = subprocess.run([DRIVER, "--fasta", str(f), "--print-inputs"], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, env=asan_env, timeout=120)
    assert out.returncode == 0 and _clean(out.stderr.decode("latin-1")), out.stderr[-3000:]
    lines = out.stdout.decode().split("\n")
    genes = seqalign.parse_fasta(text)
    assert int(lines[0]) == len(genes)
    for g, l in zip(genes, lines[1:]):
        assert l == "%d %s" % (len(g), hashlib.sha512(g).hexdigest())


def test_driver_token_input_under_asan(asan_env):
    c = next(c for c in load_golden() if c["name"] == "mseq1")
    text = open(os.path.join(os.path.dirname(__file__), "golden", "data", c["file"]), "rb").read()
    out = subprocess.run([DRIVER, "--print-inputs"], input=text, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         env=asan_env, timeout=120)
    assert out.returncode == 0 and _clean(out.stderr.decode("latin-1"))
    _, _, genes = seqalign.parse_input(text)
    lines = out.stdout.decode().split("\n")
    assert int(lines[0]) == len(genes)
    assert lines[1:1 + len(genes)] == ["%d %s" % (len(g), hashlib.sha512(g).hexdigest()) for g in genes]
