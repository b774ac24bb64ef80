#!/usr/bin/env bash
# PMC passes over tools/indep.py (chain-free bands), one pass per counter set.
#   TAG=<out dir>  ARGS="m n pairs"  PT=<seconds per pass>  NSETS=<how many sets>
set -o pipefail
OUT=gpurun_out/${TAG:-dpmc}
mkdir -p $OUT
export TMPDIR=/tmp NWK_NOTRACE=${NWK_NOTRACE:-1}
ARGS=${ARGS:-2048 50000 1024}
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
      "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
      "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC")
for ((i = 0; i < ${NSETS:-3}; i++)); do
  timeout -s KILL ${PT:-100} rocprofv3 --kernel-trace --pmc ${SETS[$i]} --output-format csv -d $OUT/p$i -o p -- python3 -u tools/indep.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True)):
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in rows:
        if "nw_align" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f, {k: "%.4g" % (v / max(1, n[k])) for k, v in agg.items()}, "launches", max(n.values()) if n else 0)
PY
