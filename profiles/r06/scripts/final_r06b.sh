#!/usr/bin/env bash
# Round-6 final session B: C4 and big13 -- bench, rocprofv3 kernel stats, PMC
# passes; then C3 at 8 ranks and C4 at 8 ranks (per-rank emulation).
set -uo pipefail
cd "$(dirname "$0")/../../.."
TAG=r06c4 WL=c4 BSTEPS=5 BENCH_ARGS=--no-cpu-baseline STEPS="bench prof pmc" bash tools/gpu_round.sh || exit 1
TAG=r06big13 WL=big13 BSTEPS=5 BENCH_ARGS=--no-cpu-baseline STEPS="bench prof pmc" bash tools/gpu_round.sh || exit 1
mkdir -p gpurun_out/r06shard
timeout -k 10 400 python -u tools/shardtime.py c3 1 8 > gpurun_out/r06shard/c3.out 2>&1 || exit 1
timeout -k 10 400 python -u tools/shardtime.py c4 --records 1 8 > gpurun_out/r06shard/c4.out 2>&1 || exit 1
tail -n 3 gpurun_out/r06shard/c3.out gpurun_out/r06shard/c4.out
