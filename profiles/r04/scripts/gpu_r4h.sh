#!/usr/bin/env bash
# Round 4 session h: big13 timeline with nw_align_col (write-bound window policy).
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4h
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 2 $O/$n.out | cut -c1-240; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 20 $O/$n.err; exit $rc; }; }
run tl_big13 200 python3 tools/wl_tl.py big13 nw_align_col
run tl_big13_bits 200 python3 tools/wl_tl.py big13 auto
B="--steps 3 --warmup 1 --no-cpu-baseline --kernel nw_align_col"
run big13 200 python3 bench.py --workload big13 $B
run c4 200 python3 bench.py --workload c4 $B
echo done
