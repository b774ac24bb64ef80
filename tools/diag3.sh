# C3/big13 bench under task-order and occupancy knobs (one process per setting).
set -o pipefail
mkdir -p gpurun_out/d3
for wl in ${WLS:-c3}; do
for o in ${ORDERS:-0 64 128 256 1}; do
  NWK_ORDER=$o timeout -k 10 120 python3 bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/d3/$wl.o$o.json 2> gpurun_out/d3/$wl.o$o.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/d3/$wl.o$o.json').read().strip().splitlines()[-1]);print('$wl order $o', d['value'], d['kernel']['fill_ms'], d.get('answer_hash_ok'))"
done
done
