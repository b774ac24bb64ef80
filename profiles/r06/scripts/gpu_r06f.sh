#!/usr/bin/env bash
# Round-6 session f: nw_align_gotoh at 5 waves/SIMD as the default (tests, C5
# bench x2); C4 per-record chain with the 1/8 + 1/8 priority tiers; big13
# occupancy knobs (span-bound: fewer waves per SIMD beside the long bands).
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06f; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -2 $O/$name.out | cut -c1-700; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step gotoh_tests 400 python -u -m pytest tests/test_gpu_gotoh.py tests/test_gpu_guard.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider
step bench_c5a 200 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline
step bench_c5b 200 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline
step c4_records 300 python -u tools/shardtime.py c4 --records 1 8
step big13_base 200 python -u bench.py --workload big13 --steps 5 --warmup 1 --no-cpu-baseline
NWK_BPC=3 step big13_bpc3 200 python -u bench.py --workload big13 --steps 5 --warmup 1 --no-cpu-baseline
NWK_COL_WPE_HI=0 step big13_wpe4 200 python -u bench.py --workload big13 --steps 5 --warmup 1 --no-cpu-baseline
NWK_BPC=2 step big13_bpc2 200 python -u bench.py --workload big13 --steps 5 --warmup 1 --no-cpu-baseline
