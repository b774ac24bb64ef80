# A/B: C4 8-rank streamed shards, strip tasks issued at priority 3..0 by quarter of the
# given (canonical) order, so the first records reach the chain earlier
set -uo pipefail
O=gpurun_out/r3q3; mkdir -p $O
for V in idp base; do
  L=tools/abv/$V/libnwk.so; [ $V = base ] && L=multiple-sequence-alignment-openmp-openmpi_amd/lib/libnwk.so
  NWK_ST_LIB=$L timeout -k 10 240 python3 -u tools/shardtime.py c4 --stream --chunks 16 8 > $O/st_$V.txt 2>&1 || { tail -5 $O/st_$V.txt; exit 1; }
  echo $V; tail -1 $O/st_$V.txt
done
