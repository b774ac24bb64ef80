set -uo pipefail
TAG=r3g STEPS="tests" PYTEST_K="strip or bits or c4 or c3 or window or edge or golden or random or single_pair or strings" bash tools/gpu_round.sh || exit 1
TAG=r3g STEPS="bench" WL=c4 BSTEPS=3 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3g STEPS="bench" WL=c3 BSTEPS=3 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3g STEPS="bench" WL=big13 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
mkdir -p gpurun_out/r3g
timeout -k 10 300 python -u tools/shardtime.py c4 --chunks 1 1 8 > gpurun_out/r3g/shard_c4.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/shardtime.py c3 --chunks 1 1 8 > gpurun_out/r3g/shard_c3.txt 2>&1 || exit 1
cat gpurun_out/r3g/shard_c4.txt gpurun_out/r3g/shard_c3.txt | grep -v amdgpu.ids
