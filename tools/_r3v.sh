set -uo pipefail
mkdir -p gpurun_out/r3v
NWK_LIB=tools/abv/tprof/libnwk.so timeout -k 10 120 python3 -u tools/trace_probe.py 8192 50000 > gpurun_out/r3v/trace_prof.txt 2>&1 || exit 1
grep -E "^ +0 " gpurun_out/r3v/trace_prof.txt | tail -3
TAG=r3v STEPS="bench" WL=c5 BSTEPS=2 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
NWK_STRIP=0 TAG=r3v_band STEPS="bench" WL=c4 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3v_strip STEPS="bench" WL=c4 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
