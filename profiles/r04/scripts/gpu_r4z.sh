#!/usr/bin/env bash
# Round 4 session z: automatic fused finalize for large nw_align_col align_all calls (C4).
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4z}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 1 $O/$n.out | cut -c1-200; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 30 $O/$n.err; exit $rc; }; }
B="--workload c4 --steps 3 --warmup 1 --no-cpu-baseline"
run c4_fuse 300 python3 bench.py $B
run c4_nofuse 300 env NWK_AUTO_FUSE=0 python3 bench.py $B
run c4_fuse_v 300 python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline --verbose
run tests 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_col.py -x -q --timeout 240 --timeout-method thread
echo done
