# Source me: run TAG WORKLOAD [ENV=VAL ...] -> one bench line (no CPU baseline) per call, summary on stdout.
set -o pipefail
mkdir -p gpurun_out/runs
run() { # tag wl env...
  local tag=$1 wl=$2; shift 2
  env "$@" timeout -k 10 ${BT:-150} python3 bench.py --workload $wl --steps ${BS:-2} --warmup 1 --no-cpu-baseline > gpurun_out/runs/$tag.json 2> gpurun_out/runs/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/runs/$tag.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/runs/$tag.json').read().strip().splitlines()[-1]);print('$tag', d['value'], d['ms_per_step'], d['kernel']['fill_ms'], d['kernel']['batches'], d.get('answer_hash_ok'))"
}
