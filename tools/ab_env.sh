#!/usr/bin/env bash
# A/B of env settings on big13 in one lib: ab_env.sh "NWK_PACKED=1" "NWK_PACKED=2" ...
set -euo pipefail
cd "$(dirname "$0")/.."
for r in 1 2; do for e in "$@"; do
  env $e REPS=${REPS:-4} timeout -k 10 120 python3 tools/fill_timeit.py 2>&1 | grep timeit | sed "s/^/[$e] /"
done; done
