set -uo pipefail
mkdir -p gpurun_out/r3h
{ nproc; grep -m1 "model name" /proc/cpuinfo; grep MHz /proc/cpuinfo | head -3; } > gpurun_out/r3h/cpu.txt
for i in 1 2 3; do timeout 60 tools/probe/chain_probe >> gpurun_out/r3h/chain_probe.txt; done
timeout -k 10 120 python -u tools/shard_tl.py 8 0 c3 > gpurun_out/r3h/tl_c3_w8.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/shard_tl.py 8 0 c4 > gpurun_out/r3h/tl_c4_w8.txt 2>&1 || exit 1
cat gpurun_out/r3h/cpu.txt gpurun_out/r3h/chain_probe.txt
grep -E "timeline|all bands|nwk:" gpurun_out/r3h/tl_c3_w8.txt | tail -6
grep -E "timeline|all bands|nwk:" gpurun_out/r3h/tl_c4_w8.txt | tail -6
