set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3l; mkdir -p $O
for V in base poll32; do
  LIBV=""; [ $V != base ] && LIBV=tools/abv/$V/libnwk.so
  NWK_LIB=${LIBV:-multiple-sequence-alignment-openmp-openmpi_amd/lib/libnwk.so} NWK_BITS_WIN=8192 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/$V -o p --output-format csv -- python3 tools/pka_write_probe.py 8 200000 > $O/$V.out 2>&1 || exit 1
  grep rep $O/$V.out | sed "s/^/$V /"
done
python3 - <<'PY'
import csv, glob
for d in ("base", "poll32"):
    for f in glob.glob("gpurun_out/r3l/%s/**/*counter_collection.csv" % d, recursive=True):
        for r in csv.DictReader(open(f)):
            if "pka" in r["Kernel_Name"]:
                print(d, r["Dispatch_Id"], r["Counter_Name"], "%.4g GB" % (float(r["Counter_Value"]) * 1024 / 1e9),
                      "%.1f ms" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
PY
