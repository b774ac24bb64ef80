#!/usr/bin/env bash
# Round 4 session d: nw_align_col timelines (lone-pair traces, big13, one C4 shard).
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4d
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -2 $O/$n.out | cut -c1-300; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -20 $O/$n.err; exit $rc; }; }
run tp_col 200 env NWK_TP_KERNEL=nw_align_col python3 tools/trace_probe.py 8192 50000
run tp_bits 200 env NWK_TP_KERNEL=nw_align_bits python3 tools/trace_probe.py 8192 50000
run big13_col_v 200 python3 bench.py --workload big13 --steps 1 --warmup 1 --no-cpu-baseline --kernel nw_align_col --verbose
run c4shard_col_v 200 python3 tools/c4shard_tl.py nw_align_col
for v in wpe5 wpe6; do
  run c3_col_$v 300 env NWK_LIB=tools/abv/$v/libnwk.so python3 bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --kernel nw_align_col
  run big13_col_$v 300 env NWK_LIB=tools/abv/$v/libnwk.so python3 bench.py --workload big13 --steps 3 --warmup 1 --no-cpu-baseline --kernel nw_align_col
done
run st_c3_col_wpe6 400 env NWK_LIB=tools/abv/wpe6/libnwk.so NWK_ST_KERNEL=nw_align_col python3 tools/shardtime.py c3 8
echo done
