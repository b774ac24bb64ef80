#!/usr/bin/env bash
# Round-6 session n: MSA host time per level (k64 x 5k, verbose 2): as built vs with
# glibc's mmap threshold raised (freed level buffers reused without page faults).
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06h; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -1 $O/$name.out | cut -c1-300; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step levels_a 200 python -u tools/msa_bench.py --reps 1 --sets 64:5000 --levels
MALLOC_MMAP_THRESHOLD_=1073741824 MALLOC_TRIM_THRESHOLD_=1073741824 step levels_b 200 python -u tools/msa_bench.py --reps 1 --sets 64:5000 --levels
step levels_a2 200 python -u tools/msa_bench.py --reps 1 --sets 64:5000 --levels
MALLOC_MMAP_THRESHOLD_=1073741824 MALLOC_TRIM_THRESHOLD_=1073741824 step levels_b2 200 python -u tools/msa_bench.py --reps 1 --sets 64:5000 --levels
