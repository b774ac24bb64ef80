#!/usr/bin/env bash
# Round 4 session p: auto kernel choice (nw_align_col per job): full GPU suite, benches, sharded times.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4p}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 2 $O/$n.out | cut -c1-250; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 30 $O/$n.err; exit $rc; }; }
run tests 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread
B="--steps 3 --warmup 1 --no-cpu-baseline"
for wl in c3 c4 big13; do run bench_$wl 300 python3 bench.py --workload $wl $B; done
run st_c4 400 python3 tools/shardtime.py c4 --stream 8
run st_c3 400 python3 tools/shardtime.py c3 8
echo done
