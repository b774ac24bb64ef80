#!/usr/bin/env bash
# Round-6 final session D: repeat bench lines on the final tree (box-to-box spread).
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06rep; mkdir -p $O
for w in c3 c3 c4 big13 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline >> $O/bench_$w.jsonl 2>> $O/bench.err || exit 1
done
tail -n 1 $O/bench_*.jsonl | cut -c1-160
