#!/usr/bin/env bash
# Round-6 session d: C4 at 8 ranks, per-record streaming with and without the
# first pieces hashed at once by their tracing wave (NWK_EARLY_HASH); the
# bench's streamed paths (gloo ranks sharing the GPU).
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06d; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -4 $O/$name.out; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step c4_records_early 300 python -u tools/shardtime.py c4 --records 1 8
NWK_EARLY_HASH=0 step c4_records_noearly 300 python -u tools/shardtime.py c4 --records 8
step c4_records_early2 300 python -u tools/shardtime.py c4 --records 8
step bench_tests 600 python -u -m pytest tests/test_bench.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu
