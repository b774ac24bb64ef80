set -uo pipefail
TAG=r3y STEPS="probe tests" bash tools/gpu_round.sh || exit 1
TAG=r3y STEPS="bench" WL=c3 BSTEPS=5 bash tools/gpu_round.sh || exit 1
TAG=r3y STEPS="bench" WL=c4 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
mkdir -p gpurun_out/r3y
timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 16 --stream 1 8 > gpurun_out/r3y/st_c4_stream16.txt 2>&1 || exit 1
tail -2 gpurun_out/r3y/st_c4_stream16.txt
timeout -k 10 300 python3 -u tools/shardtime.py c3 1 2 4 8 > gpurun_out/r3y/st_c3.txt 2>&1 || exit 1
tail -4 gpurun_out/r3y/st_c3.txt
