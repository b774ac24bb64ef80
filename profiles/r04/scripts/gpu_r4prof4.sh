#!/usr/bin/env bash
# Round 4: C4 profiles again (automatic fused finalize: the launch now hashes in-kernel).
set -uo pipefail
cd "$(dirname "$0")/.."
TAG=r4prof4 WL=c4 STEPS="bench prof pmc" BSTEPS=3 BENCH_ARGS=--no-cpu-baseline tools/gpu_round.sh
