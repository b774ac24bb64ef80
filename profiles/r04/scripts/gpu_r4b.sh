#!/usr/bin/env bash
# Round 4 session b: VALU/SALU issue probe, nw_align_col parity, full-size sharded answers.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 120 ./tools/probe/col_probe > $O/col_probe.txt 2>&1 || { echo "probe failed"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_col.py -x -v --timeout 240 --timeout-method thread > $O/pytest_col.log 2>&1
rc=$?
echo "col tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 300 --timeout-method thread > $O/pytest_shard.log 2>&1
echo "shard tests rc=$?"
