set -o pipefail
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread -k "bits or golden or big13 or c3_pairs or single_pair or random" > gpurun_out/t12.log 2>&1; rc=$?; tail -n 3 gpurun_out/t12.log; [ $rc -eq 0 ] || exit $rc
for v in tools/libvariants/nobop3 multiple-sequence-alignment-openmp-openmpi_amd/lib; do
  NWK_NOTRACE=1 LIB=$v timeout -k 10 100 python3 tools/indep.py 2048 50000 3072 | sed "s|^|$v |" || exit 1
  timeout -k 10 100 python3 tools/ab_wl.py $v c3 2 || exit 1
done
