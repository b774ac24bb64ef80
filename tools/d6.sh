set -o pipefail
# (NWK_NOTRACE with single-band pairs hangs the bits kernel -- under investigation)
for v in base nostore; do
  LIB=tools/libvariants/$v timeout -k 10 120 python3 tools/indep.py 2048 50000 3072 2048 50000 1024 | sed "s/^/$v /" || exit 1
done
