#!/usr/bin/env bash
# Round 4 session r: C4 rank-0 shard timeline (W=8, fused streamed launch).
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4r}
mkdir -p $O
timeout -k 10 200 python3 tools/c4shard_tl.py auto 8 > $O/tl.out 2> $O/tl.err; rc=$?; tail -2 $O/tl.out; exit $rc
