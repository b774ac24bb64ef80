#!/usr/bin/env bash
# Round-6 session o: the tree rebuilt in a re-created container -- full -m gpu suite, smoke, default bench.
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06o; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -2 $O/$name.out | cut -c1-300; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python -u bench.py
