#!/bin/bash
# nw_profile A/B: the committed library (tools/varlib/libnwk_head.so, built from
# the previous commit) against the in-tree build, then the in-tree build's
# forced profile forms and a kernel trace.  Output under gpurun_out/msa/.
# The baseline library (not kept): git archive 1b9d9fe multiple-sequence-alignment-openmp-openmpi_amd include
# | tar -x -C /tmp/old && make -C /tmp/old/multiple-sequence-alignment-openmp-openmpi_amd, then copy its
# lib/libnwk.so to tools/varlib/libnwk_head.so.
set -e
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/msa
timeout -k 10 200 python -u tools/msa_bench.py --sets 16:10000,64:5000,8:50000,256:2000 > gpurun_out/msa/new.jsonl
NWK_LIB=tools/varlib/libnwk_head.so timeout -k 10 200 python -u tools/msa_bench.py --sets 16:10000,64:5000,8:50000,256:2000 > gpurun_out/msa/head.jsonl
NWK_PROF_DOT=0 timeout -k 10 200 python -u tools/msa_bench.py --sets 64:5000,256:2000 > gpurun_out/msa/new_mad.jsonl
NWK_PROF_DOT=2 timeout -k 10 200 python -u tools/msa_bench.py --sets 64:5000,256:2000 > gpurun_out/msa/new_dot2.jsonl
timeout -k 10 200 python -u tools/msa_bench.py --reps 1 --sets 64:5000,256:2000 --levels > gpurun_out/msa/levels.jsonl 2> gpurun_out/msa/levels.txt
