#!/usr/bin/env bash
# per-rank big13 shard time at world sizes $WS under env settings
set -euo pipefail
cd "$(dirname "$0")/.."
for e in "$@"; do env $e timeout -k 10 200 python3 tools/shardtime.py ${WS:-8} | sed "s/^/[$e] /"; done
