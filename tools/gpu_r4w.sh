#!/usr/bin/env bash
# Round 4 session w: nw_align_col on the transposed matrix for wide pairs: col tests, big13, shards.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4w}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 2 $O/$n.out | cut -c1-250; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 30 $O/$n.err; exit $rc; }; }
run tests 600 python -u -m pytest tests/test_gpu_col.py tests/test_gpu_shard.py tests/test_gpu_large.py -x -q --timeout 240 --timeout-method thread
B="--workload big13 --steps 5 --warmup 1 --no-cpu-baseline"
run big13 200 python3 bench.py $B
run big13_notr 200 env NWK_COL_TR=0 python3 bench.py $B
run tl 200 python3 tools/wl_tl.py big13 auto
run st_big13 300 python3 tools/shardtime.py big13 1 2 4 8
echo done
