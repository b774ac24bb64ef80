#!/usr/bin/env bash
# same-box A/B of the column kernel's hop order: base (tree) vs NWK_LIB=tools/varlib/hopfwd.so, alternating.
set -uo pipefail
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out/colab2
for rep in 1 2; do
  for v in base fwd; do
    for w in c3 c4 big13; do
      if [ $v = fwd ]; then export NWK_LIB=tools/varlib/hopfwd.so; else unset NWK_LIB; fi
      timeout -k 10 300 python3 bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/colab2/b.json 2> gpurun_out/colab2/b.err || exit 1
      python3 -c "import json;d=json.load(open('gpurun_out/colab2/b.json'));print('$v $w', d['value'], d['ms_per_step'], d['answer_hash_ok'], d['kernel']['fill_ms'])" | tee -a gpurun_out/colab2/ab.txt
    done
  done
done
