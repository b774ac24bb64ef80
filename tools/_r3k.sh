set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3k; mkdir -p $O
NWK_BITS_WIN=8192 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/w8 -o p --output-format csv -- python3 tools/pka_write_probe.py 8 200000 > $O/w8.out 2>&1 || exit 1
grep rep $O/w8.out
timeout -s KILL 280 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/w32 -o p --output-format csv -- python3 tools/pka_write_probe.py 32 200000 > $O/w32.out 2>&1 || exit 1
grep rep $O/w32.out
python3 - <<'PY'
import csv, glob
for d in ("w8", "w32"):
    for f in glob.glob("gpurun_out/r3k/%s/**/*counter_collection.csv" % d, recursive=True):
        for r in csv.DictReader(open(f)):
            if "pka" in r["Kernel_Name"] or "fill" in r["Kernel_Name"]:
                print(d, r["Dispatch_Id"], r["Kernel_Name"][:40], r["Counter_Name"], "%.4g GB" % (float(r["Counter_Value"]) * 1024 / 1e9),
                      "%.1f ms" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
PY
