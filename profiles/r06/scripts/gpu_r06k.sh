#!/usr/bin/env bash
# Round-6 session k: nw_profile's walk one run at a time (NWK_PROF_RUNWALK=1,
# the tree) vs one move at a time (abv6/pk): MSA tests, per-level walk phases, msa_bench.
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06k; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -3 $O/$name.out | cut -c1-300; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step msa_tests 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_guard.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "msa or profile"
step levels_run 200 python -u tools/msa_bench.py --reps 1 --sets 64:5000 --levels
NWK_LIB=abv6/pk/libnwk.so step levels_pk 200 python -u tools/msa_bench.py --reps 1 --sets 64:5000 --levels
step bench_run 300 python -u tools/msa_bench.py --reps 3
NWK_LIB=abv6/pk/libnwk.so step bench_pk 300 python -u tools/msa_bench.py --reps 3
# C5 against all 496 oracle penalties (tests/golden/large/c5_pen.json)
step c5_pen_test 300 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k c5_affine_all_penalties
step bench_c5 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline
