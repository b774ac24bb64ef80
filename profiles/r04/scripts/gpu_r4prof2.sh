#!/usr/bin/env bash
# Round 4 profiles, part 2: c4 and big13 (nw_align_col), bench without the CPU leg.
set -uo pipefail
cd "$(dirname "$0")/.."
for wl in c4 big13; do
  TAG=r4prof WL=$wl STEPS="bench prof pmc" BSTEPS=3 BENCH_ARGS=--no-cpu-baseline tools/gpu_round.sh || exit $?
done
