set -uo pipefail
TAG=r3f3 STEPS="tests" PYTEST_K="c4 or strip or stream or fused or golden or window" bash tools/gpu_round.sh || exit 1
TAG=r3f3 STEPS="bench" WL=c4 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3f3 WL=c4 STEPS="prof pmc" bash tools/gpu_round.sh || exit 1
mkdir -p gpurun_out/r3f3
timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 16 --stream 1 8 > gpurun_out/r3f3/st_c4_stream16.txt 2>&1 || exit 1
tail -2 gpurun_out/r3f3/st_c4_stream16.txt
TAG=r3f3 STEPS="bench" WL=c5 BSTEPS=2 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
