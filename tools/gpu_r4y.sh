#!/usr/bin/env bash
# Round 4 session y: transpose threshold 1.15 x critical span: big13 W=1 and shards.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4y}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 4 $O/$n.out | cut -c1-250; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 30 $O/$n.err; exit $rc; }; }
B="--workload big13 --steps 5 --warmup 1 --no-cpu-baseline"
run big13 200 python3 bench.py $B
run st_big13 300 python3 tools/shardtime.py big13 1 2 4 8
echo done
