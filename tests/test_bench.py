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


def test_rank_launcher_stops_peers_on_first_failure():
    """bench.wait_ranks: the first rank to fail (rank 2 here, while ranks 0 and
    1 would block for a minute, as in a collective whose peer died) ends the
    launch with its exit code; the peers are terminated and reaped."""
    import time

    import bench

    procs = [subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"]) for _ in range(2)]
    procs.append(subprocess.Popen([sys.executable, "-c", "import sys, time; time.sleep(0.5); sys.exit(3)"]))
    t0 = time.time()
    assert bench.wait_ranks(procs, grace_s=5.0) == 3
    assert time.time() - t0 < 30
    assert all(p.returncode is not None for p in procs)
    ok = [subprocess.Popen([sys.executable, "-c", "pass"]) for _ in range(3)]
    assert bench.wait_ranks(ok) == 0


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


@pytest.mark.gpu
def test_bench_nccl_all_gather_at_world_one():
    """The driver's multi-GPU bench path with the real backend: RCCL through the
    library's communicator (nwk_comm_*: ncclCommInitRank after a file
    rendezvous on the node), LPT shard, the all-gather of the 72-byte records
    and the max-over-ranks all-reduce, forced at WORLD_SIZE 1
    (NWK_BENCH_FORCE_DIST) so it runs on a 1-GPU box; big13's published hash.
    The rank process never imports torch: it maps exactly one HIP runtime,
    one HSA runtime and one RCCL (the ones libnwk.so links)."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = _env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               NWK_BENCH_FORCE_DIST="1", NWK_BENCH_WS_GB="110")
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "1", "--workload", "big13", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.decode().strip().split("\n")[-1])
    assert line["answer_hash_ok"] is True
    assert line["collective"]["backend"].startswith("rccl")
    libs = line["runtime_libs"]
    print("runtime libraries mapped:", libs)
    for name in ("librccl", "libamdhip64", "libhsa-runtime64"):
        assert len([x for x in libs if name in os.path.basename(x)]) == 1, (name, libs)
    out = os.path.join(REPO, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "bench_nccl_world1.json"), "w") as f:
            f.write(json.dumps(line) + "\n")


@pytest.mark.gpu
@pytest.mark.parametrize("node", ["records", "1", "0"])
def test_two_ranks_streamed_records_big13_published_hash(node):
    """One launch per rank (the engine's default task order: largest pairs
    first, so records arrive in size order, not in canonical order), the
    records handed to rank 0's chain -- every record as soon as it is out,
    through node shared memory (node=records: dist.NodeStream, the default on
    one node since round 6), or four pieces each once all of its records have
    arrived, through node shared memory (node=1: dist.NodeRecords) or one
    all-gather per piece (node=0) -- and one all-gather of the whole shards
    after the launches; the line records when the chain took its first record,
    or when each piece was ready."""
    env = _env(NWK_BENCH_BACKEND="gloo", NWK_BENCH_SHARE_GPU="1", NWK_BENCH_WS_GB="110",
               NWK_BENCH_STREAM="1", NWK_BENCH_CHUNKS="4", NWK_NODE_RECORDS="0" if node == "0" else "1",
               NWK_BENCH_RECORDS="1" if node == "records" else "0")
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "2", "--workload", "big13",
                        "--steps", "1", "--warmup", "0", "--no-cpu-baseline"], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.decode().strip().split("\n")[-1])
    assert line["n_gpus"] == 2 and line["answer_hash_ok"] is True
    assert "streamed" in line["config"]["parallelism"]
    if node == "records":
        assert len(line["collective"]["first_record_ms"]) == 1
        assert line["collective"]["piece_exchange"].startswith("every record through node shared memory")
        assert line["collective"]["all_gathers_per_step"] == 1
        return
    ready = line["collective"]["piece_ready_ms"]
    assert len(ready) == 4 and ready == sorted(ready)
    assert line["collective"]["piece_exchange"].startswith("node" if node == "1" else "one all-gather per piece")
    assert line["collective"]["all_gathers_per_step"] == (1 if node == "1" else 4)
