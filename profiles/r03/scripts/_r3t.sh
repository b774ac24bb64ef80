set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r3t; mkdir -p $O
# nw_align_pka writes with one-lane sentinel polls (was: whole-wave atomic re-reads)
NWK_BITS_WIN=8192 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pw -o p --output-format csv -- python3 tools/pka_write_probe.py 8 200000 > $O/pw.out 2>&1 || exit 1
grep rep $O/pw.out
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r3t/pw/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "pka" in r["Kernel_Name"]:
            print("pka", r["Dispatch_Id"], r["Counter_Name"], "%.4g GB" % (float(r["Counter_Value"]) * 1024 / 1e9),
                  "%.1f ms" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
PY
# C4 8-rank emulation: band tasks in 4 / 8 pieces against strips in 2
NWK_STRIP=0 timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 4 1 8 > $O/st_band4.txt 2>&1 || exit 1
tail -2 $O/st_band4.txt
NWK_STRIP=0 timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 8 8 > $O/st_band8.txt 2>&1 || exit 1
tail -1 $O/st_band8.txt
NWK_STRIP=0 NWK_ORDER=0 timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 4 8 > $O/st_band4_pm.txt 2>&1 || exit 1
tail -1 $O/st_band4_pm.txt
timeout -k 10 300 python3 -u tools/shardtime.py c4 --chunks 1 8 > $O/st_strip1.txt 2>&1 || exit 1
tail -1 $O/st_strip1.txt
# occupancy A/B: nw_align_bits / nw_align_strip at 5 waves/SIMD (96 VGPRs, spills only outside the step loop)
for V in base wpe5; do
  timeout -k 10 200 python3 -u tools/ab_wl.py tools/abv/$V c3 3 2>&1 | grep "^ab" || exit 1
  timeout -k 10 200 python3 -u tools/ab_wl.py tools/abv/$V c4 3 2>&1 | grep "^ab" || exit 1
done
