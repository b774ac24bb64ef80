#!/usr/bin/env bash
# col hop change: column-kernel parity, then the C3 / C4 bench lines, then the shard emulations.
set -uo pipefail
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/colhop
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_col.py tests/test_gpu_shard.py > gpurun_out/colhop/tests.txt 2>&1 || { tail -20 gpurun_out/colhop/tests.txt; exit 1; }
tail -1 gpurun_out/colhop/tests.txt
timeout -k 10 300 python3 bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/colhop/bench_c3.json 2> gpurun_out/colhop/bench_c3.err || exit 1
timeout -k 10 300 python3 bench.py --workload c4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/colhop/bench_c4.json 2> gpurun_out/colhop/bench_c4.err || exit 1
timeout -k 10 300 python3 bench.py --workload big13 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/colhop/bench_big13.json 2> gpurun_out/colhop/bench_big13.err || exit 1
for w in c3 c4 big13; do python3 -c "import json;d=json.load(open('gpurun_out/colhop/bench_$w.json'));print('$w', d['value'], d['ms_per_step'], d['answer_hash_ok'], d['kernel']['fill_ms'])"; done
