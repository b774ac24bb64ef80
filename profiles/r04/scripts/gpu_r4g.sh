#!/usr/bin/env bash
# Round 4 session g: torch-free RCCL rank path (single runtime), big13 path deviation, window policy.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4g
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 2 $O/$n.out | cut -c1-240; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 20 $O/$n.err; exit $rc; }; }
run tbench 400 python -u -m pytest tests/test_bench.py -x -q -m gpu --timeout 240 --timeout-method thread
run pathdev 300 python3 tools/pathdev.py big13
B="--steps 3 --warmup 1 --no-cpu-baseline --kernel nw_align_col"
run big13_full 200 env NWK_COL_WIN=0 python3 bench.py --workload big13 $B
run big13_8k 200 env NWK_COL_WIN=8192 python3 bench.py --workload big13 $B
echo done
