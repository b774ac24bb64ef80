set -uo pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
TAG=r3d STEPS="tests" PYTEST_K="strip or bits or c4 or c3 or window or edge or bench or rccl or chain" bash tools/gpu_round.sh || exit 1
TAG=r3d STEPS="bench" WL=c4 BSTEPS=3 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3d STEPS="bench" WL=c3 BSTEPS=3 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
mkdir -p gpurun_out/r3d
timeout -k 10 300 python -u tools/shardtime.py c4 --chunks 1 1 8 > gpurun_out/r3d/shard_c4_ch1.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/shardtime.py c4 --chunks 2 8 > gpurun_out/r3d/shard_c4_ch2.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/shardtime.py c4 --chunks 3 8 > gpurun_out/r3d/shard_c4_ch3.txt 2>&1 || exit 1
cat gpurun_out/r3d/shard_c4_ch*.txt
