# C4 8-rank streamed shards at 2 / 3 / 4 strip waves per SIMD: fewer pairs in flight
# finish sooner, so the chain can start before the whole shard is aligned
set -uo pipefail
O=gpurun_out/r3q4; mkdir -p $O
for B in 2 3 4; do
  NWK_BPC=$B NWK_STRIP=1 timeout -k 10 240 python3 -u tools/shardtime.py c4 --stream --chunks 16 8 > $O/st_bpc$B.txt 2>&1 || { tail -5 $O/st_bpc$B.txt; exit 1; }
  echo bpc$B; tail -1 $O/st_bpc$B.txt
done
