set -o pipefail
t() { timeout -k 10 100 "$@"; }
NWK_NOTRACE=1 t python3 tools/indep.py 2048 50000 3072 2048 50000 1024 | sed "s/^/notrace /" &&
NWK_NOTRACE=1 LIB=tools/libvariants/nostore t python3 tools/indep.py 2048 50000 3072 2048 50000 1024 | sed "s/^/nostore-notrace /" &&
t python3 tools/indep.py 2048 50000 3072 | sed "s/^/trace /" &&
NWK_NOTRACE=1 t python3 tools/ab_wl.py multiple-sequence-alignment-openmp-openmpi_amd/lib c3 2 | sed "s/^/notrace /" &&
NWK_NOTRACE=1 t python3 tools/ab_wl.py tools/libvariants/nostore c3 2 | sed "s/^/nostore-notrace /"
