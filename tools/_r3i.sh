set -uo pipefail
TAG=r3i STEPS="tests" PYTEST_K="strip or bits or c4 or c3 or window or edge or golden or random or single_pair or strings" bash tools/gpu_round.sh || exit 1
mkdir -p gpurun_out/r3i
timeout -k 10 120 python -u tools/shard_tl.py 8 0 c3 > gpurun_out/r3i/tl_c3_w8.txt 2>&1 || exit 1
grep -E "timeline: first|nwk:" gpurun_out/r3i/tl_c3_w8.txt | tail -2
grep -E "^ +[0-9]+ +[0-9]+ x" gpurun_out/r3i/tl_c3_w8.txt | tail -3
TAG=r3i STEPS="bench" WL=c3 BSTEPS=3 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3i STEPS="bench" WL=c4 BSTEPS=3 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3i STEPS="bench" WL=big13 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
