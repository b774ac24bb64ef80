#!/usr/bin/env bash
# usage: VAR=NWK_PARK tools/sweep2.sh v1 v2 ...  -- HEAD lib vs working lib, same box
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
echo "== head"; timeout -k 10 120 python3 tools/timeit.py tools/libvariants/head 2>&1 | grep timeit
for v in "$@"; do
  echo "== ${VAR}=$v"
  env ${VAR}=$v timeout -k 10 120 python3 tools/timeit.py multiple-sequence-alignment-openmp-openmpi_amd/lib > gpurun_out/sweep_$v.log 2>&1 || { tail -20 gpurun_out/sweep_$v.log; exit 1; }
  grep -E "all bands|timeit|queue:" gpurun_out/sweep_$v.log | tail -4
done
echo "== head"; timeout -k 10 120 python3 tools/timeit.py tools/libvariants/head 2>&1 | grep timeit
