#!/usr/bin/env bash
# Compiles the REFERENCE programs from their sources where they lie under
# /root/reference (read-only) into oracle/_ref/.  Test infrastructure only:
# the outputs validate oracle/nw_oracle.c and serve as bench.py's CPU
# baseline ("kind": "reference").  Nothing is copied into the repository.
#
#   _ref/skel  testing3/seqalign-mpi-skeleton.cpp   (sequential oracle)
#   _ref/sub   submit/xuliny-seqalkway.cpp          (submitted MPI+OpenMP)
#   _ref/skel_debug  seqalign-mpi-skeleton.cpp (root copy: prints the
#              per-pair penalty / problemhash / chain lines, skel:158-169)
#
# Needs MPICH (found at /opt/conda in this image).  The conda mpicxx wrapper
# names a compiler that does not exist, so g++ is called directly with the
# MPICH include/lib paths; libstdc++ is linked statically because the conda
# libstdc++ is older than g++ 11's.
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
MPI=${MPI_HOME:-/opt/conda}
if [ ! -d "$REF" ]; then echo "build_ref: $REF absent, skipping"; exit 0; fi
if [ ! -f "$MPI/include/mpi.h" ]; then echo "build_ref: no MPI headers under $MPI, skipping"; exit 0; fi
mkdir -p "$OUT"
CXXFLAGS="-std=c++14 -O3 -fopenmp -I$MPI/include"
LDFLAGS="-L$MPI/lib -lmpi -Wl,-rpath,$MPI/lib -static-libstdc++ -static-libgcc"
# -I the source's own directory so its sha512.hh is found next to it.
g++ $CXXFLAGS -I"$REF/testing3" -o "$OUT/skel" "$REF/testing3/seqalign-mpi-skeleton.cpp" $LDFLAGS
g++ $CXXFLAGS -I"$REF/submit" -o "$OUT/sub" "$REF/submit/xuliny-seqalkway.cpp" $LDFLAGS
g++ $CXXFLAGS -I"$REF" -o "$OUT/skel_debug" "$REF/seqalign-mpi-skeleton.cpp" $LDFLAGS
echo "build_ref: built $OUT/skel $OUT/sub"
