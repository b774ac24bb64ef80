#!/usr/bin/env bash
# Traceback phase cycles (tools/abv/tprof: nw_align_col built with NWK_TRACE_PROF=1), lone pairs.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-tprof}
mkdir -p $O
timeout -k 10 200 env NWK_LIB=tools/abv/tprof/libnwk.so NWK_TP_KERNEL=nw_align_col python3 tools/trace_probe.py 8192 50000 > $O/tp.out 2> $O/tp.err
rc=$?; grep trace_col $O/tp.out | tail -4; exit $rc
