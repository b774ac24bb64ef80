#!/usr/bin/env bash
# Round 4 final check: full GPU suite, smoke(), default bench (C3 with the CPU leg).
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4final}
mkdir -p $O
run() { local n=$1 lim=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $lim "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -n 2 $O/$n.out | cut -c1-400; [ $rc -eq 0 ] || { echo "$n failed rc=$rc"; tail -n 30 $O/$n.err; exit $rc; }; }
run tests 1000 python -u -m pytest tests/ -q -m gpu --timeout 200 --timeout-method thread
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python3 -u bench.py
run c4 300 python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline
run big13 300 python3 bench.py --workload big13 --steps 5 --warmup 1 --no-cpu-baseline
echo done
