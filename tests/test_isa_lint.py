"""ISA lint of the packed / int32 fill kernels (csrc/nwk_kernels.hip, the file
whose block loops prefetch the next super-block's words and granules): in the
gfx950 assembly no instruction reads a VGPR whose vector-memory load is still
outstanding (tools/vmscan.py).  This is the hazard that gave nw_align_pka its
intermittent wrong penalties through round 5: inline-asm loads waited for by a
counted s_waitcnt, with compiler copies of the in-flight registers placed
before the wait.  CPU only (hipcc cross-compiles, ~10 s)."""
import os
import re
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd", "csrc", "nwk_kernels.hip")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
def test_no_register_read_with_its_load_outstanding(tmp_path):
    s = tmp_path / "k.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-o", str(s), SRC],
                   check=True, capture_output=True, timeout=600)
    text = s.read_text()
    fns = sorted(set(re.findall(r"^(_ZN3nwk\w+):", text, re.M)))
    kernels = [f for f in fns if re.search(r"nw_align|nw_profile|nw_gather", f)]
    assert len(kernels) >= 10, fns
    bad = []
    for fn in kernels:
        out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "vmscan.py"), str(s), fn],
                             capture_output=True, text=True, timeout=300).stdout
        m = re.search(r"issues (\d+)", out)
        assert m, out
        if int(m.group(1)):
            bad.append(out)
    assert not bad, "\n".join(bad)
