#!/usr/bin/env bash
# GPU parity tests, then big13 timeline (BPC=${BPC:-2}) and default timing.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
NWK_BPC=${BPC:-2} V=2 REPS=2 timeout -k 10 120 python3 tools/timeit.py > gpurun_out/tl.log 2>&1 || { tail gpurun_out/tl.log; exit 1; }
grep -A4 "nwk timeline" gpurun_out/tl.log | tail -4; grep -B3 "all bands" gpurun_out/tl.log | tail -4
for b in ${BPCS:-2 3}; do NWK_BPC=$b REPS=4 timeout -k 10 120 python3 tools/timeit.py 2>&1 | grep timeit | sed "s/^/bpc=$b /"; done
