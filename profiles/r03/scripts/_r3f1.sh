set -uo pipefail
TAG=r3f STEPS="probe tests" bash tools/gpu_round.sh || exit 1
mkdir -p gpurun_out/r3f
timeout -k 10 120 python3 -u tools/trace_probe.py 8192 50000 > gpurun_out/r3f/trace_probe.txt 2>&1 || exit 1
grep -E "^ +0 " gpurun_out/r3f/trace_probe.txt | tail -1
timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 16 --stream 1 8 > gpurun_out/r3f/st_c4_stream16.txt 2>&1 || exit 1
tail -2 gpurun_out/r3f/st_c4_stream16.txt
for wl in c3 c4; do
  TAG=r3f WL=$wl STEPS="prof pmc" bash tools/gpu_round.sh || exit 1
done
