#!/usr/bin/env bash
# Round-6 session n: MSA A/B runs: the tree vs abv6/base = the tree built with -DNWK_POLL_SLEEP_MAX=4 (shorter granule-poll sleeps).
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06n; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -2 $O/$name.out | cut -c1-300; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step msa_tests 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_guard.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "msa or profile"
step levels_new 200 python -u tools/msa_bench.py --reps 1 --sets 64:5000 --levels
NWK_LIB=abv6/base/libnwk.so step levels_base 200 python -u tools/msa_bench.py --reps 1 --sets 64:5000 --levels
step bench_new 300 python -u tools/msa_bench.py --reps 3 --sets 64:5000,8:50000,256:2000
NWK_LIB=abv6/base/libnwk.so step bench_base 300 python -u tools/msa_bench.py --reps 3 --sets 64:5000,8:50000,256:2000
