#!/usr/bin/env bash
# Round-6 final session C: the whole -m gpu suite on the final tree, the MSA
# bench and its nw_profile trace + PMC passes.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/${TAG:-r06final}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.out 2>&1 || { tail -30 $O/pytest_gpu.out; exit 1; }
tail -2 $O/pytest_gpu.out
# (msa_bench: run separately)

# (msa_prof: run separately, profiles/r06/scripts/msa_prof.sh)
echo done
