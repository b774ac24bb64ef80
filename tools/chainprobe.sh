#!/usr/bin/env bash
# Chain-free fill rate (independent 512-row bands, no traceback) vs big13, per waves/SIMD.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for b in ${BPCS:-1 2 3 4}; do
  echo "== BPC=$b"
  NWK_BPC=$b NWK_NOTRACE=1 timeout -k 10 120 python3 tools/indep.py 512 60000 4096 2>&1 | tail -1
  NWK_BPC=$b V=2 REPS=2 timeout -k 10 120 python3 tools/timeit.py > gpurun_out/tl_$b.log 2>&1 || { tail gpurun_out/tl_$b.log; exit 1; }
  grep -E "all bands|timeit" gpurun_out/tl_$b.log | tail -2
done
