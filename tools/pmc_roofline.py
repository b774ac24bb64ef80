#!/usr/bin/env python3
"""Per-launch counters of the dominant fill kernel -> profiles/<round>/pmc_<workload>.json.

Reads the rocprofv3 --pmc passes of tools/gpu_round.sh (separate passes:
SQ_INSTS_VALU/SQ_ACTIVE_INST_VALU/SQ_WAVES/GRBM_GUI_ACTIVE, FETCH_SIZE,
WRITE_SIZE) and averages each counter over the kernel's dispatches.

  HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024: on gfx950 FETCH_SIZE
  tallies 128-B read requests at 64 B (MI355X_MICROARCH.md "HBM"), WRITE_SIZE
  reads exact for streaming stores.
  VALU issue fraction = SQ_INSTS_VALU x 2 cycles / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8):
  a wave64 VALU instruction issues over 2 cycles (MI355X_MICROARCH.md), and
  GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles.

usage: python tools/pmc_roofline.py <gpurun_out/TAG> <workload> <kernel> <round, e.g. r02> [suffix]
"""
import collections
import csv
import glob
import json
import os
import sys

src, wl, kernel, rnd = sys.argv[1:5]
suffix = sys.argv[5] if len(sys.argv) > 5 else ""
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "multiple-sequence-alignment-openmp-openmpi_amd"))
import seqalign  # noqa: E402  (kernel_source_id: no library load)


def per_dispatch(pattern):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for f in glob.glob(os.path.join(src, pattern, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if ("::%s(" % kernel) not in name and ("::%s<" % kernel) not in name:
                continue  # "nwk::nw_align_pk2(nwk::FillArgs)", "void nwk::nw_align<0, 4>(...)"
            d = r["Dispatch_Id"]
            vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return vals, dur


def mean(xs):
    xs = list(xs)
    return sum(xs) / len(xs) if xs else None


valu, dur = per_dispatch("pmc_valu_" + wl + suffix)
fetch, _ = per_dispatch("pmc_fetch_" + wl + suffix)
write, _ = per_dispatch("pmc_write_" + wl + suffix)
out = {
    "workload": wl + suffix,
    "kernel": kernel,
    # the kernel build these counters belong to (bench.py reports frac null on a mismatch);
    # run this script on the tree the passes ran on
    "kernel_source_id": seqalign.kernel_source_id(kernel),
    "launches_measured": [len(valu), len(fetch), len(write)],
    "sq_insts_valu_per_launch": mean(v["SQ_INSTS_VALU"] for v in valu.values()),
    "sq_active_inst_valu_per_launch": mean(v["SQ_ACTIVE_INST_VALU"] for v in valu.values()),
    "sq_waves_per_launch": mean(v["SQ_WAVES"] for v in valu.values()),
    "grbm_gui_active_per_launch": mean(v["GRBM_GUI_ACTIVE"] for v in valu.values()),
    "duration_ns_per_launch": mean(dur.values()),
    "fetch_size_kib_per_launch": mean(v["FETCH_SIZE"] for v in fetch.values()),
    "write_size_kib_per_launch": mean(v["WRITE_SIZE"] for v in write.values()),
}
if out["fetch_size_kib_per_launch"] is not None and out["write_size_kib_per_launch"] is not None:
    out["hbm_bytes_per_launch"] = int((2 * out["fetch_size_kib_per_launch"] + out["write_size_kib_per_launch"]) * 1024)
if out["sq_insts_valu_per_launch"] and out["grbm_gui_active_per_launch"]:
    cyc = out["grbm_gui_active_per_launch"] / 8.0
    out["valu_issue_frac"] = out["sq_insts_valu_per_launch"] * 2 / 1024 / cyc
    out["clock_ghz"] = cyc / out["duration_ns_per_launch"]
    out["hbm_frac_at_pmc_duration"] = out.get("hbm_bytes_per_launch", 0) / (out["duration_ns_per_launch"] * 1e-9) / 8e12
# PMC_CMD: the profiled command when it is not bench.py (e.g. profiles/r05/scripts/msa_prof.sh)
cmd = os.environ.get("PMC_CMD") or ("'bench.py --workload %s --steps 1 --warmup 1 --no-cpu-baseline' "
                                    "(tools/gpu_round.sh)" % wl)
out["method"] = ("rocprofv3 --kernel-trace --pmc in three separate passes over %s; per-launch means over the "
                 "kernel's dispatches; traffic = (2 x FETCH_SIZE + WRITE_SIZE) KiB; valu_issue_frac = "
                 "SQ_INSTS_VALU x 2 / 1024 / (GRBM_GUI_ACTIVE / 8)" % cmd)
dst = os.path.join(REPO, "profiles", rnd, "pmc_%s%s.json" % (wl, suffix))
os.makedirs(os.path.dirname(dst), exist_ok=True)
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
