#!/usr/bin/env bash
# Round 4 session c: nw_align_col vs nw_align_bits on C3, big13, C4; sharded emulation with col.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4c
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -2 $O/$n.out | cut -c1-600; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -20 $O/$n.err; exit $rc; }; }
run c3_col 300 python3 bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline --kernel nw_align_col
run c3_bits 300 python3 bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline --kernel nw_align_bits
run big13_col 300 python3 bench.py --workload big13 --steps 5 --warmup 1 --no-cpu-baseline --kernel nw_align_col
run big13_auto 300 python3 bench.py --workload big13 --steps 5 --warmup 1 --no-cpu-baseline
run c4_col 300 python3 bench.py --workload c4 --steps 5 --warmup 1 --no-cpu-baseline --kernel nw_align_col
run st_c4_col 400 env NWK_ST_KERNEL=nw_align_col python3 tools/shardtime.py c4 --stream 8
run st_c3_col 400 env NWK_ST_KERNEL=nw_align_col python3 tools/shardtime.py c3 1 8
echo done
