#!/usr/bin/env bash
# Round-6 final session A: C3 (the default bench line, with the CPU baseline)
# and C5 -- bench, rocprofv3 kernel stats, and the PMC passes bench.py's
# roofline reads (tools/gpu_round.sh; separate --pmc passes, kernel-trace only).
set -uo pipefail
cd "$(dirname "$0")/../../.."
TAG=r06c3 WL=c3 BSTEPS=5 STEPS="bench prof pmc" bash tools/gpu_round.sh || exit 1
TAG=r06c5 WL=c5 BSTEPS=1 BENCH_ARGS=--no-cpu-baseline STEPS="bench prof pmc" bash tools/gpu_round.sh || exit 1
