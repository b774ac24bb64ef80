#!/usr/bin/env bash
# Builds a libnwk.so variant with extra compile flags into tools/libvariants/<name>/
# (A/B runs: NWK_LIB / NWK_ST_LIB point seqalign / tools/shardtime.py at it).
# usage: tools/build_variant.sh <name> <flags...>
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
out=${VARIANT_DIR:-tools/libvariants}/$name
mkdir -p $out/obj
P=multiple-sequence-alignment-openmp-openmpi_amd
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result $*"
# ONLY="nwk_gotoh ...": rebuild just these sources with the flags, the other
# objects are the main build's ($P/build)
for f in nwk_kernels nwk_hash nwk_bits nwk_col nwk_gotoh; do
  if [ -n "${ONLY:-}" ] && [[ " $ONLY " != *" $f "* ]]; then cp $P/build/$f.o $out/obj/$f.o; continue; fi
  /opt/rocm/bin/hipcc $F -c $P/csrc/$f.hip -o $out/obj/$f.o &
done
if [ -n "${ONLY:-}" ]; then cp $P/build/nwk_runtime.o $P/build/sha512.o $out/obj/; else
/opt/rocm/bin/hipcc $F -c $P/csrc/nwk_runtime.cpp -o $out/obj/nwk_runtime.o &
g++ -O3 -march=x86-64-v3 -std=c++17 -fPIC -c $P/csrc/sha512.cpp -o $out/obj/sha512.o &
fi
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/libnwk.so $out/obj/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $out/libnwk.so
