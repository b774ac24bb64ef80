#!/usr/bin/env bash
# Round 4 profiles: bench + rocprofv3 kernel stats + PMC passes for the default (c3,
# nw_align_bits), c4 and big13 (nw_align_col) -- tools/gpu_round.sh per workload.
set -uo pipefail
cd "$(dirname "$0")/.."
for wl in c3 c4 big13; do
  TAG=r4prof WL=$wl STEPS="bench prof pmc" BSTEPS=3 tools/gpu_round.sh || exit $?
done
