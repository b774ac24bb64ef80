#!/usr/bin/env bash
# Round-5 final per-rank emulations: C3 W = 1/2/4/8, C4 streamed W = 8, big13 W = 8.
set -uo pipefail
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/r05shard
mkdir -p "$OUT"
timeout -k 10 500 python3 -u tools/shardtime.py c3 1 2 4 8 > "$OUT/shard_c3.txt" 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/shardtime.py c4 --stream --chunks 16 1 8 > "$OUT/shard_c4.txt" 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/shardtime.py big13 1 8 > "$OUT/shard_big13.txt" 2>&1 || exit 1
echo done
