#!/usr/bin/env bash
# One GPU-box session: host probe, GPU parity tests, bench lines, rocprofv3
# kernel stats and the PMC passes the bench's roofline reads (separate passes,
# kernel-trace only; MI355X_MICROARCH.md "HBM").  Every GPU step has its own
# time limit and the steps are chained: the first failure ends the script.
#   STEPS="probe tests bench prof pmc"  WL=c3  PYTEST_K=<-k expr>
set -uo pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-round}
mkdir -p "$OUT"
export TMPDIR=/tmp
WL=${WL:-c3}
STEPS=${STEPS:-probe tests bench prof pmc}
BENCH_ARGS=${BENCH_ARGS:-}

run() {  # name seconds cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  tail -3 "$OUT/$name.out"
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -30 "$OUT/$name.err"; exit $rc; fi
}

for s in $STEPS; do
  case $s in
    probe)
      { nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo;
        grep "physical id" /proc/cpuinfo | sort -u | wc -l; free -g; which mpirun mpiexec 2>&1;
        ls /opt/conda/bin/mpirun 2>&1; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-}"; rocm-smi --showuse 2>&1 | head -20; } > "$OUT/host.txt" 2>&1
      ;;
    tests)
      run pytest_gpu 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 150 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
      ;;
    bench)
      run bench_$WL 600 python3 bench.py --workload "$WL" --steps "${BSTEPS:-5}" --warmup 1 $BENCH_ARGS
      ;;
    prof)
      run prof_$WL 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$WL" -o run --output-format csv -- python3 bench.py --workload "$WL" --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS
      ;;
    pmc)
      run pmc_valu_$WL 300 timeout -s KILL 280 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE -d "$OUT/pmc_valu_$WL" -o p --output-format csv -- python3 bench.py --workload "$WL" --steps 1 --warmup 1 --no-cpu-baseline $BENCH_ARGS
      run pmc_fetch_$WL 300 timeout -s KILL 280 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$WL" -o p --output-format csv -- python3 bench.py --workload "$WL" --steps 1 --warmup 1 --no-cpu-baseline $BENCH_ARGS
      run pmc_write_$WL 300 timeout -s KILL 280 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write_$WL" -o p --output-format csv -- python3 bench.py --workload "$WL" --steps 1 --warmup 1 --no-cpu-baseline $BENCH_ARGS
      ;;
  esac
done
echo "done $(date +%T)"
