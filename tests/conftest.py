import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLDEN_DIR = os.path.join(REPO, "tests", "golden")
for p in (PKG, ORACLE, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- run with -m gpu")


def load_golden():
    with open(os.path.join(GOLDEN_DIR, "golden.json")) as f:
        return json.load(f)["cases"]


def case_input(case):
    """(pxy, pgap, genes as bytes) for a golden case."""
    import seqalign

    if "file" in case:
        text = open(os.path.join(GOLDEN_DIR, "data", case["file"]), "rb").read()
    else:
        text = case["input"].encode("latin-1")
    pxy, pgap, genes = seqalign.parse_input(text)
    if "permute" in case:
        genes = [genes[i] for i in case["permute"]]
    return pxy, pgap, genes


@pytest.fixture(scope="session")
def golden():
    return {c["name"]: c for c in load_golden()}
