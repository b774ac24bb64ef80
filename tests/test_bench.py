"""bench.py's launch contract: --gpus N spawns N ranks (or fails loudly), the
N-rank path runs the HIP aligner end to end, and the JSON line is well formed.

The -m gpu case rehearses the driver's multi-GPU scaling run on a 1-GPU box:
two rank processes share the card (NWK_BENCH_SHARE_GPU=1, gloo for the one
all-gather), each aligns its LPT shard of big13 with the HIP kernels, and rank 0
chains the gathered records into the reference's published answer hash
(testing3/sequential.txt:2-3).
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(kw)
    return env


def test_gpus_beyond_visible_devices_fails_loudly():
    """`bench.py --gpus N` with fewer than N visible GPUs exits non-zero instead
    of measuring one GPU and printing n_gpus 1 (this container has none)."""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("2+ GPUs visible")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=_env(),
                       timeout=300)
    assert r.returncode != 0
    assert b"GPU(s) visible" in r.stderr
    assert r.stdout.strip() == b""


def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--steps", "1"], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, env=_env(WORLD_SIZE="2", RANK="0"), timeout=300)
    assert r.returncode != 0 and b"WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_two_ranks_share_one_gpu_big13_published_hash():
    env = _env(NWK_BENCH_BACKEND="gloo", NWK_BENCH_SHARE_GPU="1", NWK_BENCH_WS_GB="110")
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "2", "--workload", "big13", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.decode().strip().split("\n")[-1])
    assert line["n_gpus"] == 2
    assert line["answer_hash_ok"] is True
    assert line["kernel"]["name"].startswith("nw_align")
