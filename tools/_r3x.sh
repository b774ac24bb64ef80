set -uo pipefail
mkdir -p gpurun_out/r3x
NWK_STRIP=0 timeout -k 10 120 python3 -u tools/c4_check.py > gpurun_out/r3x/c4_band.txt 2>&1; rc=$?; cat gpurun_out/r3x/c4_band.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/c4_check.py > gpurun_out/r3x/c4_strip.txt 2>&1; rc=$?; cat gpurun_out/r3x/c4_strip.txt; [ $rc -eq 0 ] || exit $rc
