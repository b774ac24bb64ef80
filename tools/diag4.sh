# nw_align_bits under rocprofv3 --kernel-trace: bench big13 (chained bands).
set -o pipefail
export TMPDIR=/tmp NWK_WATCHDOG=20 PYTHONFAULTHANDLER=1
O=gpurun_out/d4b; mkdir -p $O
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt -o p --output-format csv -- python3 -u bench.py --workload big13 --steps 2 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1
echo rc=$?
grep -v "^\s*wave" $O/kt.log | tail -n 12
grep "^\s*wave" $O/kt.log | awk '{print $3}' | sort | uniq -c | sort -rn | head -20
