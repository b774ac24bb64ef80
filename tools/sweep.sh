#!/usr/bin/env bash
# usage: VAR=NWK_LAG tools/sweep.sh 2 4 8 16   -- big13 timing (+ timeline summary) per value
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in "$@"; do
  echo "== ${VAR}=$v"
  env ${VAR}=$v timeout -k 10 120 python3 tools/timeit.py > gpurun_out/sweep_$v.log 2>&1 || { tail -20 gpurun_out/sweep_$v.log; exit 1; }
  grep -E "all bands|timeit|nwk batch" gpurun_out/sweep_$v.log | tail -4
done
