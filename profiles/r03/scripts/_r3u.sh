set -uo pipefail
TAG=r3u STEPS="tests" bash tools/gpu_round.sh || exit 1
TAG=r3u STEPS="bench" WL=c3 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3u STEPS="bench" WL=c4 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3u STEPS="bench" WL=big13 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
mkdir -p gpurun_out/r3u
timeout -k 10 120 python3 -u tools/trace_probe.py 8192 50000 > gpurun_out/r3u/trace_probe.txt 2>&1 || exit 1
grep -E "^ +0 " gpurun_out/r3u/trace_probe.txt | tail -2
timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 8 --stream 1 8 > gpurun_out/r3u/st_stream8.txt 2>&1 || exit 1
tail -2 gpurun_out/r3u/st_stream8.txt
timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 16 --stream 8 > gpurun_out/r3u/st_stream16.txt 2>&1 || exit 1
tail -1 gpurun_out/r3u/st_stream16.txt
