set -e
mkdir -p gpurun_out
for a in "${@}"; do
  echo "== $a"; timeout -k 10 200 python tools/c3dbg.py $a
done
