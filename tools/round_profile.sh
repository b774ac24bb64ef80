#!/usr/bin/env bash
# Round measurement: bench lines (big13 default + c3/c4/c5), rocprofv3 kernel
# stats of the default bench, and the HBM-traffic PMC passes (FETCH_SIZE and
# WRITE_SIZE in separate passes, MI355X_MICROARCH.md "HBM").
set -uo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/round
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, seconds, cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 $lim "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?
  tail -2 $OUT/$name.out
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -20 $OUT/$name.err; exit $rc; fi
}
run bench_big13 300 python3 bench.py --steps 10 --warmup 2
run prof_big13 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
run pmc_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc_fetch -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
run pmc_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_write -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
run bench_c4 300 python3 bench.py --workload c4 --steps 3 --warmup 1
run bench_c3 400 python3 bench.py --workload c3 --steps 2 --warmup 1
#run bench_c5 500 python3 bench.py --workload c5 --steps 1 --warmup 1
echo done
