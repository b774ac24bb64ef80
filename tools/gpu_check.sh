#!/usr/bin/env bash
# GPU parity + short bench (+ optional A/B against NWK_PACKED=0).
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
echo "== bench"
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ "${AB:-0}" = 1 ]; then
  echo "== bench NWK_PACKED=0"
  NWK_PACKED=0 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_old.json 2>> gpurun_out/bench.err
  cat gpurun_out/bench_old.json
fi
