#!/usr/bin/env bash
# Round-6 session c2: the guard without loop-carried VGPRs (col / gotoh END
# capture by v_readlane) -- guard tests, C3 and C5 bench lines.
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06c2; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -4 $O/$name.out; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step guard_tests 400 python -u -m pytest tests/test_gpu_guard.py tests/test_gpu_gotoh.py tests/test_gpu_col.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider
step bench_c3 300 python -u bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline
step bench_c5 300 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline
