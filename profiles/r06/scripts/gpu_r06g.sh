#!/usr/bin/env bash
# Round-6 session g: C3 at 8 ranks by rounds (tools/c3_rounds.py); big13's
# span-critical pairs vs the rest, each alone, at default and reduced occupancy.
set -u
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06g; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -6 $O/$name.out | cut -c1-400; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step c3_rounds 400 python -u tools/c3_rounds.py 8
step b13_all 200 python -u tools/big13_split.py all
step b13_crit 200 python -u tools/big13_split.py crit
NWK_BPC=1 step b13_crit_bpc1 200 python -u tools/big13_split.py crit
NWK_BPC=2 step b13_crit_bpc2 200 python -u tools/big13_split.py crit
step b13_rest 200 python -u tools/big13_split.py rest
NWK_CU_RESERVE=112 step b13_rest_cu144 200 python -u tools/big13_split.py rest
NWK_CU_RESERVE=64 step b13_rest_cu192 200 python -u tools/big13_split.py rest
