set -o pipefail
source tools/diag5.sh
run c3 c3 A=1 && run c3_w0 c3 NWK_BITS_WIN=0 && run c4 c4 A=1 && run big13 big13 A=1 && NWK_VERBOSE=1 timeout -k 10 100 python3 tools/ab_wl.py multiple-sequence-alignment-openmp-openmpi_amd/lib c3 1 2>&1 | grep -E "nwk:|nwk host|^ab" | tail -4
