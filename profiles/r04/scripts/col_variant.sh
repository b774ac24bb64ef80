#!/usr/bin/env bash
# A/B variant of nw_align_col only: compiles csrc/nwk_col.hip with extra flags and links it with
# the main build's other objects into tools/abv/<name>/libnwk.so (use with NWK_LIB=...).
# usage: tools/col_variant.sh <name> <flags...>
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
P=multiple-sequence-alignment-openmp-openmpi_amd
out=tools/abv/$name
mkdir -p $out
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result "$@" -c $P/csrc/nwk_col.hip -o $out/nwk_col.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/libnwk.so $P/build/nwk_kernels.o $P/build/nwk_bits.o \
  $out/nwk_col.o $P/build/nwk_hash.o $P/build/nwk_runtime.o $P/build/sha512.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $out/libnwk.so
