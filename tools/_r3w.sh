set -uo pipefail
TAG=r3w STEPS="tests" bash tools/gpu_round.sh || exit 1
TAG=r3w STEPS="bench" WL=c3 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3w STEPS="bench" WL=c4 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
NWK_STRIP=0 TAG=r3w_band STEPS="bench" WL=c4 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3w STEPS="bench" WL=big13 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
mkdir -p gpurun_out/r3w
timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 16 --stream 1 8 > gpurun_out/r3w/st_stream16_pm.txt 2>&1 || exit 1
tail -2 gpurun_out/r3w/st_stream16_pm.txt
NWK_ST_ORDER=2 timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 16 --stream 8 > gpurun_out/r3w/st_stream16_bm.txt 2>&1 || exit 1
tail -1 gpurun_out/r3w/st_stream16_bm.txt
NWK_ST_KERNEL=nw_align_strip NWK_ST_ORDER=0 timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 16 --stream 8 > gpurun_out/r3w/st_stream16_strip.txt 2>&1 || exit 1
tail -1 gpurun_out/r3w/st_stream16_strip.txt
NWK_STRIP=0 timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 1 8 > gpurun_out/r3w/st_band1.txt 2>&1 || exit 1
tail -1 gpurun_out/r3w/st_band1.txt
