#!/usr/bin/env bash
set -euo pipefail
cd "$(dirname "$0")/.."
for e in "$@"; do
  env $e V=2 REPS=2 timeout -k 10 120 python3 tools/timeit.py > gpurun_out/tl2.log 2>&1 || { tail gpurun_out/tl2.log; exit 1; }
  echo "[$e]"; grep -E "first pair filled [0-9]|all bands|timeit" gpurun_out/tl2.log | tail -4; cp gpurun_out/tl2.log "gpurun_out/tl2_$(echo $e | tr " =" "_-").log"
done
