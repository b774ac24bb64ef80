set -uo pipefail
TAG=r3z STEPS="tests" PYTEST_K="bits or strip or golden or random or strings or c3 or c4 or fused or window or single_pair or edge or driver" bash tools/gpu_round.sh || exit 1
mkdir -p gpurun_out/r3z
for V in base2 trace2; do
  NWK_LIB=tools/abv/$V/libnwk.so timeout -k 10 120 python3 -u tools/trace_probe.py 8192 50000 > gpurun_out/r3z/tp_$V.txt 2>&1 || exit 1
  grep -E "^ +0 " gpurun_out/r3z/tp_$V.txt | tail -1 | sed "s/^/$V /"
done
for V in base2 trace2; do
  timeout -k 10 200 python3 -u tools/ab_wl.py tools/abv/$V c3 3 2>&1 | grep "^ab" || exit 1
done
