#!/usr/bin/env bash
# Round 4 session s: big13 trace phases under load (segments off), lone 8k/50k.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4s}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 1 $O/$n.out | cut -c1-300; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 30 $O/$n.err; exit $rc; }; }
run tprof_big13 200 env NWK_LIB=tools/abv/tprof/libnwk.so python3 tools/wl_tl.py big13 auto
run tprof_lone 200 env NWK_LIB=tools/abv/tprof/libnwk.so NWK_TP_KERNEL=nw_align_col python3 tools/trace_probe.py 8192 50000
echo done
