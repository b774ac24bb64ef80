set -o pipefail
mkdir -p gpurun_out/d1
t() { timeout -k 10 180 "$@"; }
t python3 tools/indep.py 2048 50000 3072 2048 50000 1024 > gpurun_out/d1/indep_bits.txt 2>&1 &&
NWK_BITS=0 t python3 tools/indep.py 1024 50000 3072 > gpurun_out/d1/indep_pk2.txt 2>&1 &&
NWK_NOTRACE=1 t python3 tools/fill_timeit.py > gpurun_out/d1/big13_bits_notrace.txt 2>&1 &&
NWK_BITS=0 NWK_NOTRACE=1 t python3 tools/fill_timeit.py > gpurun_out/d1/big13_pk2_notrace.txt 2>&1 &&
t python3 tools/fill_timeit.py > gpurun_out/d1/big13_bits.txt 2>&1 &&
NWK_BITS=0 t python3 tools/fill_timeit.py > gpurun_out/d1/big13_pk2.txt 2>&1
rc=$?
cat gpurun_out/d1/*.txt
exit $rc
