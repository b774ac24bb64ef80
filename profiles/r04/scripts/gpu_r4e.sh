#!/usr/bin/env bash
# Round 4 session e: nw_align_col with trace / long-pair priority (default build) vs no trace priority vs 6 waves/SIMD.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4e
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 2 $O/$n.out | cut -c1-240; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 20 $O/$n.err; exit $rc; }; }
B="--steps 3 --warmup 1 --no-cpu-baseline --kernel nw_align_col"
run big13 200 python3 bench.py --workload big13 $B
run big13_noprio 200 env NWK_COL_PRIO=0 python3 bench.py --workload big13 $B
run c4 200 python3 bench.py --workload c4 $B
run c4_notprio 200 env NWK_LIB=tools/abv/notprio/libnwk.so python3 bench.py --workload c4 $B
run c4_wpe6 200 env NWK_LIB=tools/abv/wpe6/libnwk.so python3 bench.py --workload c4 $B
run c3 200 python3 bench.py --workload c3 $B
run c3_wpe6 200 env NWK_LIB=tools/abv/wpe6/libnwk.so python3 bench.py --workload c3 $B
run c4shard 200 python3 tools/c4shard_tl.py nw_align_col
run c4shard_wpe6 200 env NWK_LIB=tools/abv/wpe6/libnwk.so python3 tools/c4shard_tl.py nw_align_col
run st_c3_wpe6 400 env NWK_LIB=tools/abv/wpe6/libnwk.so NWK_ST_KERNEL=nw_align_col python3 tools/shardtime.py c3 8
run st_c4 400 env NWK_ST_KERNEL=nw_align_col python3 tools/shardtime.py c4 --stream 8
echo done
