#!/usr/bin/env bash
# First GPU contact: smoke, gpu tests, short bench, kernel trace.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== smoke"; timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/smoke.log
echo "== pytest gpu"; timeout -k 10 540 python -m pytest tests/ -q -m gpu --durations=15 > gpurun_out/pytest_gpu.log 2>&1 || { tail -50 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
echo "== bench"; timeout -k 10 200 python bench.py --steps 3 --warmup 1 --verbose > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo "== rocprof"; timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { tail -30 gpurun_out/prof.err; exit 1; }
find gpurun_out/prof -name "*stats*" | head
