#!/usr/bin/env bash
# Fill-only (NWK_NOTRACE) big13 and independent-chain rates for the packed kernels.
set -euo pipefail
cd "$(dirname "$0")/.."
for e in "$@"; do
  env $e NWK_NOTRACE=1 REPS=3 timeout -k 10 120 python3 tools/timeit.py 2>&1 | grep timeit | sed "s/^/[$e notrace] /"
done
for b in 1 2; do
  NWK_PACKED=1 NWK_BPC=$b NWK_NOTRACE=1 timeout -k 10 120 python3 tools/indep.py 512 60000 4096 | sed "s/^/[pk bpc=$b] /"
  NWK_PACKED=2 NWK_BPC=$b NWK_NOTRACE=1 timeout -k 10 120 python3 tools/indep.py 1024 60000 2048 | sed "s/^/[pk2 bpc=$b] /"
done
