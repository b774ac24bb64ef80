#!/usr/bin/env bash
# Round 4 session q: first-piece priority for streamed nw_align_col ranks (C4 W=8), C3 W=8.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4q}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 1 $O/$n.out | cut -c1-300; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 30 $O/$n.err; exit $rc; }; }
run st_c4 400 python3 tools/shardtime.py c4 --stream 8
run st_c4_noprio 400 env NWK_PIECE_PRIO=0 python3 tools/shardtime.py c4 --stream 8
run st_c3s 400 python3 tools/shardtime.py c3 --stream 8
echo done
