set -o pipefail
mkdir -p gpurun_out/c5ab
for cfg in "NWK_X=0" "NWK_LIB=tools/varlib/gwpe6.so" "NWK_X=1"; do
  echo "== $cfg" >> gpurun_out/c5ab/ab.txt
  env $cfg timeout -k 10 200 python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5ab/last.json 2>> gpurun_out/c5ab/err.txt || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c5ab/last.json'));k=d['kernel'];print(d['value'],d['ms_per_step'],k['batches'],k['window_retries'],k['window'],k['fill_ms'])" >> gpurun_out/c5ab/ab.txt
done
