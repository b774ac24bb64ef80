#!/usr/bin/env bash
# Round 4 per-rank times (tools/shardtime.py, answers checked): C3 1/2/4/8, C4 streamed 1/2/4/8, big13 1/2/4/8.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4sched}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; cat $O/$n.out | cut -c1-300; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 30 $O/$n.err; exit $rc; }; }
run st_c3 500 python3 tools/shardtime.py c3 1 2 4 8
run st_c4 500 python3 tools/shardtime.py c4 --stream 1 2 4 8
run st_big13 500 python3 tools/shardtime.py big13 1 2 4 8
echo done
