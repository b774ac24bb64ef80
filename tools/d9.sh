# parity subset (unless NOTEST=1), then C3 / big13 / C4 bench lines (tools/diag5.sh)
set -o pipefail
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread \
    -k "(bits_kernel or golden or random or big13 or single_pair or c3) and not full_config" > gpurun_out/t9.log 2>&1
  rc=$?; tail -n 5 gpurun_out/t9.log; [ $rc -eq 0 ] || exit $rc
fi
source tools/diag5.sh
run c3 c3 A=1 && run big13 big13 A=1 && run c4 c4 A=1
