set -o pipefail
mkdir -p gpurun_out/d2
t() { timeout -k 10 180 "$@"; }
t python3 tools/indep.py 2048 50000 1024 2048 50000 3072 > gpurun_out/d2/indep_bits.txt 2>&1 &&
t python3 tools/fill_timeit.py > gpurun_out/d2/big13_bits.txt 2>&1 &&
NWK_NOTRACE=1 t python3 tools/fill_timeit.py > gpurun_out/d2/big13_bits_notrace.txt 2>&1 &&
t python3 -u -m pytest tests/test_gpu.py -x -q --timeout 150 --timeout-method thread -k "golden or random or big13" > gpurun_out/d2/tests.txt 2>&1
rc=$?
tail -3 gpurun_out/d2/*.txt
exit $rc
