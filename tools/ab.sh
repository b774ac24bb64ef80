#!/usr/bin/env bash
# A/B of lib variants on big13 (kernel ms), plus fill-only (NWK_NOTRACE) for the first variant.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export REPS=${REPS:-4} ROUNDS=${ROUNDS:-2}
for b in ${BPCS:-2}; do
  echo "== BPC=$b"
  NWK_BPC=$b timeout -k 10 300 python3 tools/fill_timeit.py "$@" 2>&1 | grep timeit
  [ -n "${NOTRACE:-}" ] && NWK_NOTRACE=1 NWK_BPC=$b ROUNDS=1 timeout -k 10 120 python3 tools/fill_timeit.py "$1" 2>&1 | grep timeit | sed 's/^/notrace /'
done
