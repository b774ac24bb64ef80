#!/usr/bin/env bash
# Round-6 session i: C5 band-chain slack experiment (NWK_GOTOH_SLACK = chunks a
# band below starts behind the band above, beyond the minimum 64).
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06i; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -2 $O/$name.out | cut -c1-300; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for sk in 0 32 96 192; do
  NWK_GOTOH_SLACK=$sk step c5_slack$sk 200 python -u tools/ab_wl.py multiple-sequence-alignment-openmp-openmpi_amd/lib c5 1
done
NWK_GOTOH_SLACK=96 step tl_slack96 200 python -u tools/c5_timeline.py
