# nw_align_pka WRITE_SIZE at two storage windows: the slope against the stored
# code bytes separates the code stores from the per-launch rest (granules, polls, ops)
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3p; mkdir -p $O
for W in 8192 16384; do
  NWK_BITS_WIN=$W timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/w$W -o p --output-format csv -- python3 tools/pka_write_probe.py 8 200000 > $O/w$W.out 2>&1 || exit 1
  grep rep $O/w$W.out | sed "s/^/W=$W /"
done
python3 - <<'PY'
import csv, glob
for W in (8192, 16384):
    for f in glob.glob("gpurun_out/r3p/w%d/**/*counter_collection.csv" % W, recursive=True):
        for r in csv.DictReader(open(f)):
            if "pka" in r["Kernel_Name"]:
                print("W=%d" % W, "dispatch", r["Dispatch_Id"], "WRITE_SIZE %.4g GB" % (float(r["Counter_Value"]) * 1024 / 1e9))
PY
