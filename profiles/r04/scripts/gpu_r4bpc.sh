#!/usr/bin/env bash
# A/B: big13 under nw_align_col at 1/2/3 blocks of 4 waves per CU (NWK_BPC) vs default.
set -uo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${SESSION:-r4bpc}
mkdir -p $O
for cfg in def 1 2 3 def; do
  if [ $cfg = def ]; then unset NWK_BPC; else export NWK_BPC=$cfg; fi
  echo "== bpc=$cfg $(date +%T)"
  timeout -k 10 240 python3 bench.py --workload big13 --steps 10 --warmup 2 --no-cpu-baseline > $O/big13_$cfg.out 2> $O/big13_$cfg.err || { echo "failed rc=$?"; tail -n 20 $O/big13_$cfg.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('$O/big13_$cfg.out').read().strip().splitlines()[-1]);print('bpc=$cfg', d['ms_per_step'], d['value'])" | tee -a $O/summary.txt
done
echo done
