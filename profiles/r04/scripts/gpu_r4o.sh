#!/usr/bin/env bash
# Round 4 session o: streamed host finalize (nw_align_col): GPU tests, big13 bench + host phases.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4o}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 1 $O/$n.out | cut -c1-200; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 20 $O/$n.err; exit $rc; }; }
run tests 600 python -u -m pytest tests/test_gpu_col.py -x -q --timeout 240 --timeout-method thread
B="--steps 3 --warmup 1 --no-cpu-baseline --kernel nw_align_col"
run big13 200 python3 bench.py --workload big13 $B
run big13_nostream 200 env NWK_HOST_STREAM=0 python3 bench.py --workload big13 $B
run big13_v 200 python3 bench.py --workload big13 --steps 2 --warmup 1 --no-cpu-baseline --kernel nw_align_col --verbose
echo done
