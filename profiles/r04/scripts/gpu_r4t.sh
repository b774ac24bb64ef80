#!/usr/bin/env bash
# Round 4 session t: trace without the undefined-phi load wait (unwindowed pairs): tests, big13/c4, phases.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4t}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 1 $O/$n.out | cut -c1-250; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 30 $O/$n.err; exit $rc; }; }
run tests 600 python -u -m pytest tests/test_gpu_col.py -x -q --timeout 240 --timeout-method thread
B="--steps 3 --warmup 1 --no-cpu-baseline"
run big13 300 python3 bench.py --workload big13 $B
run c4 300 python3 bench.py --workload c4 $B
run tprof_big13 200 env NWK_LIB=tools/abv/tprof/libnwk.so python3 tools/wl_tl.py big13 auto
run tprof_lone 200 env NWK_LIB=tools/abv/tprof/libnwk.so NWK_TP_KERNEL=nw_align_col python3 tools/trace_probe.py 8192 50000
echo done
