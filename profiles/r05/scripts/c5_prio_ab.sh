#!/usr/bin/env bash
# C5 A/B: gotoh band issue priority (NWK_BAND_PRIO=1) vs off, alternating, same box.
set -uo pipefail
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/c5prio
for rep in 1 2; do
  for v in 0 1; do
    NWK_BAND_PRIO=$v timeout -k 10 200 python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5prio/b.json 2> gpurun_out/c5prio/b.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c5prio/b.json'));print('prio $v', d['value'], d['ms_per_step'], d['kernel']['fill_ms'])" | tee -a gpurun_out/c5prio/ab.txt
  done
done
