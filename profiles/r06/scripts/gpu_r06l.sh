#!/usr/bin/env bash
# Round-6 session l: C5 task order A/B (NWK_ORDER: 1 band-major = default for
# nw_align_gotoh, g >= 2 groups of g pairs band-major inside).
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06l; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -1 $O/$name.out | cut -c1-200; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for o in 1 62 31 16 8; do NWK_ORDER=$o step c5_order$o 200 python -u tools/ab_wl.py multiple-sequence-alignment-openmp-openmpi_amd/lib c5 1; done
