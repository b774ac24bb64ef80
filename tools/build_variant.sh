#!/usr/bin/env bash
# Builds a libnwk.so variant with extra compile flags into tools/libvariants/<name>/ (for tools/fill_timeit.py A/B).
# usage: tools/build_variant.sh <name> <flags...>
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
out=${VARIANT_DIR:-tools/libvariants}/$name
mkdir -p $out/obj
P=multiple-sequence-alignment-openmp-openmpi_amd
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 $*"
/opt/rocm/bin/hipcc $F -c $P/csrc/nwk_kernels.hip -o $out/obj/k.o
/opt/rocm/bin/hipcc $F -c $P/csrc/nwk_hash.hip -o $out/obj/h.o
/opt/rocm/bin/hipcc $F -c $P/csrc/nwk_bits.hip -o $out/obj/b.o
/opt/rocm/bin/hipcc $F -c $P/csrc/nwk_runtime.cpp -o $out/obj/r.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -c $P/csrc/sha512.cpp -o $out/obj/s.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/libnwk.so $out/obj/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $out/libnwk.so
