#!/usr/bin/env bash
# Round 4: lone-pair traceback times (current tree), and the C3 clock at lower occupancy
# (one PMC pass per occupancy: NWK_BPC=2 and 1 blocks of 4 waves per CU).
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4clk}
mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 2 $O/$n.out | cut -c1-200; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 20 $O/$n.err; exit $rc; }; }
run tp 200 python3 tools/trace_probe.py 8192 50000
run tp_col 200 env NWK_TP_KERNEL=nw_align_col python3 tools/trace_probe.py 8192 50000
for b in 2 1; do
  export NWK_BPC=$b
  run pmc_bpc$b 300 timeout -s KILL 280 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $O/pmc_bpc$b -o p --output-format csv -- python3 bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline
  unset NWK_BPC
done
echo done
