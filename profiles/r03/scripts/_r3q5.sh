# C4 8-rank streamed shards: the first H of 16 pieces as band tasks (shorter per-pair
# latency) in a launch beside the strips, so the chain starts earlier
set -uo pipefail
O=gpurun_out/r3q5; mkdir -p $O
for H in 1 2 4; do
  NWK_ST_KERNEL=nw_align_strip timeout -k 10 240 python3 -u tools/shardtime.py c4 --stream --hybrid $H --chunks 16 8 > $O/st_h$H.txt 2>&1 || { tail -5 $O/st_h$H.txt; exit 1; }
  echo h$H; tail -1 $O/st_h$H.txt
done
