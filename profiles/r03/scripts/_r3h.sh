set -uo pipefail
for i in 1 2; do timeout 60 tools/probe/chain_probe2 || exit 1; done
grep -m1 "model name" /proc/cpuinfo
mkdir -p gpurun_out/r3h
for V in base3 w5nb1 w5nb2 base3; do
  timeout -k 10 200 python3 -u tools/ab_wl.py tools/abv/$V c3 3 2>&1 | grep "^ab" || exit 1
done
for V in base3 w5nb1; do
  timeout -k 10 200 python3 -u tools/ab_wl.py tools/abv/$V c4 3 2>&1 | grep "^ab" || exit 1
  NWK_LIB=tools/abv/$V/libnwk.so timeout -k 10 120 python3 -u tools/trace_probe.py 50000 > gpurun_out/r3h/tp_$V.txt 2>&1 || exit 1
  grep -E "^ +0 " gpurun_out/r3h/tp_$V.txt | tail -1 | sed "s/^/$V /"
done
TAG=r3g STEPS="tests" bash tools/gpu_round.sh || exit 1
