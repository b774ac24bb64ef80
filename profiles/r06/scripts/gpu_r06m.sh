#!/usr/bin/env bash
# Round-6 session m: C4 at 8 ranks, per-record chain, priority tiers
# (NWK_PIECE_TOP = first tier's priority, one lower per np/NWK_PIECE_DIV pairs).
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06m; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -1 $O/$name.out | cut -c1-330; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step top2_div8 300 python -u tools/shardtime.py c4 --records 8
NWK_PIECE_TOP=3 step top3_div8 300 python -u tools/shardtime.py c4 --records 8
NWK_PIECE_TOP=3 NWK_PIECE_DIV=12 step top3_div12 300 python -u tools/shardtime.py c4 --records 8
NWK_PIECE_TOP=3 NWK_PIECE_DIV=16 step top3_div16 300 python -u tools/shardtime.py c4 --records 8
step top2_div8b 300 python -u tools/shardtime.py c4 --records 8
