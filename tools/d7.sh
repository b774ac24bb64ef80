set -o pipefail
for v in base half4 half4_wps4; do
  timeout -k 10 120 python3 tools/ab_wl.py tools/libvariants/$v c3 3 || exit 1
done
for v in base half4 half4_wps4; do
  LIB=tools/libvariants/$v timeout -k 10 120 python3 tools/indep.py 2048 50000 3072 | sed "s/^/$v /" || exit 1
done
