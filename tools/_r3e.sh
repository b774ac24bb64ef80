set -uo pipefail
TAG=r3e STEPS="tests" PYTEST_K="strip or bits_kernel or c4 or c3 or window" bash tools/gpu_round.sh || exit 1
TAG=r3e STEPS="bench" WL=c4 BSTEPS=3 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3e STEPS="bench" WL=c3 BSTEPS=3 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
mkdir -p gpurun_out/r3e
NWK_VERBOSE=1 timeout -k 10 300 python -u tools/shardtime.py c4 --chunks 1 1 8 > gpurun_out/r3e/shard_c4_ch1.txt 2> gpurun_out/r3e/shard_c4_ch1.err || exit 1
timeout -k 10 300 python -u tools/shardtime.py c4 --chunks 2 8 > gpurun_out/r3e/shard_c4_ch2.txt 2>&1 || exit 1
cat gpurun_out/r3e/shard_c4_ch*.txt; grep "nwk" gpurun_out/r3e/shard_c4_ch1.err | tail -8
WL=c4 TAG=r3e STEPS="pmc" BENCH_ARGS="" bash tools/gpu_round.sh || exit 1
