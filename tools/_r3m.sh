set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3m; mkdir -p $O
for m in 0 1 2 3; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/m$m -o p --output-format csv -- tools/probe/store_probe $m > $O/m$m.out 2>&1 || exit 1
  cat $O/m$m.out | grep mode
done
python3 - <<'PY'
import csv, glob
for m in range(4):
    for f in glob.glob("gpurun_out/r3m/m%d/**/*counter_collection.csv" % m, recursive=True):
        for r in csv.DictReader(open(f)):
            if "store_kernel" in r["Kernel_Name"]:
                print("mode", m, r["Dispatch_Id"], "WRITE_SIZE %.4g GB" % (float(r["Counter_Value"]) * 1024 / 1e9))
PY
