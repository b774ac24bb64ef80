#!/usr/bin/env bash
# Round 4 session v: big13 finish-time priority tiers (NWK_COL_PRIO_HI / _LO).
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4v}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 1 $O/$n.out | cut -c1-200; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 30 $O/$n.err; exit $rc; }; }
B="--workload big13 --steps 5 --warmup 1 --no-cpu-baseline"
run d 200 python3 bench.py $B
run h90 200 env NWK_COL_PRIO_HI=0.9 NWK_COL_PRIO_LO=0.8 python3 bench.py $B
run h80 200 env NWK_COL_PRIO_HI=0.8 NWK_COL_PRIO_LO=0.6 python3 bench.py $B
run old 200 env NWK_COL_PRIO_HI=0.7 NWK_COL_PRIO_LO=0.7 python3 bench.py $B
run off 200 env NWK_COL_PRIO=0 python3 bench.py $B
echo done
