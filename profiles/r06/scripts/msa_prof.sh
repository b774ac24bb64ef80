#!/bin/bash
# (round 6) nw_profile kernel trace + PMC passes on the k=64 x 5k MSA (tools/msa_bench.py),
# one counter set per pass.  Output under gpurun_out/msaprof/.
set -e
cd "$(dirname "$0")/../../.."
O=gpurun_out/msaprof6
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
A="tools/msa_bench.py --reps 1 --sets 64:5000"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o msa --output-format csv -- python3 $A > $O/trace.log 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $O/pmc_valu_msa_k64 -o p --output-format csv -- python3 $A > $O/valu.log 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch_msa_k64 -o p --output-format csv -- python3 $A > $O/fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write_msa_k64 -o p --output-format csv -- python3 $A > $O/write.log 2>&1
