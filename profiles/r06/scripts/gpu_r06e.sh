#!/usr/bin/env bash
# Round-6 session e: nw_align_gotoh with its segment loop split in three (no
# per-segment spills) at 4 / 5 waves per SIMD, 8-byte vs per-step 4-byte
# stores; C4 per-record chain with the first 1/8 + 1/8 of the shard prioritised.
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06e; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -3 $O/$name.out; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step ab_main0 200 python -u tools/ab_wl.py multiple-sequence-alignment-openmp-openmpi_amd/lib c5 2
step ab_main 200 python -u tools/ab_wl.py multiple-sequence-alignment-openmp-openmpi_amd/lib c5 2
for v in gw4s1 gw5s1 gw5s0; do step ab_$v 200 python -u tools/ab_wl.py abv6/$v c5 2; done
step ab_main2 200 python -u tools/ab_wl.py multiple-sequence-alignment-openmp-openmpi_amd/lib c5 2
NWK_PIECE_DIV=8 step c4_div8 300 python -u tools/shardtime.py c4 --records 8
NWK_PIECE_DIV=6 step c4_div6 300 python -u tools/shardtime.py c4 --records 8
step c4_div16 300 python -u tools/shardtime.py c4 --records 8
