set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3j; mkdir -p $O
for W in 0 8192; do
  NWK_BITS_WIN=$W timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/w$W -o p --output-format csv -- python3 tools/pka_write_probe.py 4 20000 > $O/w$W.out 2>&1 || exit 1
  cat $O/w$W.out | grep rep
done
NWK_BITS_WIN=0 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/f0 -o p --output-format csv -- python3 tools/pka_write_probe.py 4 20000 > $O/f0.out 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
for d in ("w0", "w8192", "f0"):
    for f in glob.glob("gpurun_out/r3j/%s/**/*counter_collection.csv" % d, recursive=True):
        for r in csv.DictReader(open(f)):
            if "pka" in r["Kernel_Name"]:
                print(d, r["Dispatch_Id"], r["Counter_Name"], "%.4g GB" % (float(r["Counter_Value"]) * 1024 / 1e9))
PY
