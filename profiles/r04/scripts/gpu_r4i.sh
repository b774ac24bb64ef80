#!/usr/bin/env bash
# Round 4 session i: nw_align_col traceback: horizontal runs, tile reuse across key windows, top-exit prefetch.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4i}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 2 $O/$n.out | cut -c1-240; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 20 $O/$n.err; exit $rc; }; }
run tests 600 python -u -m pytest tests/test_gpu_col.py -x -q --timeout 240 --timeout-method thread
run tl_big13 200 python3 tools/wl_tl.py big13 nw_align_col
B="--steps 3 --warmup 1 --no-cpu-baseline --kernel nw_align_col"
run big13 200 python3 bench.py --workload big13 $B
run c3 200 python3 bench.py --workload c3 $B
run tp 200 env NWK_TP_KERNEL=nw_align_col python3 tools/trace_probe.py
echo done
