#!/usr/bin/env bash
# C3/C4 workloads on one GPU (multi-batch at scale) + big13.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WORKLOADS:-big13 c4 c3}; do
  echo "== $w"
  timeout -k 10 ${TLIM:-420} python bench.py --workload $w --steps ${STEPS:-2} --warmup 1 --verbose --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -30 gpurun_out/bench_$w.err; exit 1; }
  cat gpurun_out/bench_$w.json
done
