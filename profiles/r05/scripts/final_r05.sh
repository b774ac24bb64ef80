#!/usr/bin/env bash
# Round-5 final session: C3 bench line (with the CPU baseline), rocprof + PMC for
# the column kernel on C3 / C4 / big13, then the shard emulations.
set -uo pipefail
cd "$(dirname "$0")/../../.."
TAG=r05c3 WL=c3 BSTEPS=5 STEPS="bench prof pmc" bash tools/gpu_round.sh || exit 1
TAG=r05c4 WL=c4 STEPS="prof pmc" bash tools/gpu_round.sh || exit 1
TAG=r05big13 WL=big13 STEPS="prof pmc" bash tools/gpu_round.sh || exit 1
bash profiles/r05/scripts/final_shard.sh || exit 1
