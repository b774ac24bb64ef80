#!/usr/bin/env bash
# Round-6 session h: nw_profile changes (MSA tests
# against the oracle, msa_bench): the min3 chain (not kept), then the packed-lane walk.
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06h; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -5 $O/$name.out | cut -c1-400; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step msa_tests 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_guard.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "msa or profile"
step msa_bench 300 python -u tools/msa_bench.py --reps 3
