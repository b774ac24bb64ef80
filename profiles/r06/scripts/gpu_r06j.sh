#!/usr/bin/env bash
# Round-6 session j: MSA with the packed-lane walk -- per-level walk share (k64 x 5k) and a repeat of msa_bench.
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06j; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -4 $O/$name.out | cut -c1-300; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }

step levels_k64 200 python -u tools/msa_bench.py --reps 1 --sets 64:5000 --levels

