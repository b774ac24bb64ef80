#!/usr/bin/env bash
# Round 4 session n: segments on/off on C3/C4/big13 (nw_align_col), big13 trace phases under load, host phases.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4n}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 1 $O/$n.out | cut -c1-200; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 20 $O/$n.err; exit $rc; }; }
run tests 600 python -u -m pytest tests/test_gpu_col.py -x -q --timeout 240 --timeout-method thread -k "segmented or big13 or golden"
B="--steps 3 --warmup 1 --no-cpu-baseline --kernel nw_align_col"
for wl in c4 c3 big13; do
  run ${wl}_seg 200 python3 bench.py --workload $wl $B
  run ${wl}_noseg 200 env NWK_COL_SEG=0 python3 bench.py --workload $wl $B
done
run big13_v 200 python3 bench.py --workload big13 --steps 1 --warmup 1 --no-cpu-baseline --kernel nw_align_col --verbose
run tprof_big13 200 env NWK_LIB=tools/abv/tprof/libnwk.so python3 tools/wl_tl.py big13 nw_align_col
echo done
