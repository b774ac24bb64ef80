#!/usr/bin/env bash
# Round-6 session b: C4 at 8 ranks by per-record streaming (tools/shardtime.py
# --records) against the 16-piece replay; C5's storage window vs batch count.
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06b; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -4 $O/$name.out; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step c4_pieces 300 python -u tools/shardtime.py c4 --stream 1 8
step c4_records 300 python -u tools/shardtime.py c4 --records 1 8
for w in 8192 6144 5120; do
  NWK_BITS_WIN=$w step c5_win$w 240 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline
done
step c5_timeline 240 python -u tools/c5_timeline.py
