#!/usr/bin/env bash
# Round 4 session f: nw_align_col with lane-windowed storage (auto write-saving window).
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4f
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 2 $O/$n.out | cut -c1-240; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 20 $O/$n.err; exit $rc; }; }
run tests 600 python -u -m pytest tests/test_gpu_col.py -x -q --timeout 240 --timeout-method thread
B="--steps 3 --warmup 1 --no-cpu-baseline --kernel nw_align_col"
run big13 200 python3 bench.py --workload big13 $B
run c3 200 python3 bench.py --workload c3 $B
run c4 200 python3 bench.py --workload c4 $B
run c4shard 200 python3 tools/c4shard_tl.py nw_align_col
run big13_v 200 python3 bench.py --workload big13 --steps 1 --warmup 1 --no-cpu-baseline --kernel nw_align_col --verbose
run st_c3 400 env NWK_ST_KERNEL=nw_align_col python3 tools/shardtime.py c3 8
run st_c4 400 env NWK_ST_KERNEL=nw_align_col python3 tools/shardtime.py c4 --stream 8
echo done
