#!/usr/bin/env python3
"""Per-launch SQ counters of one kernel from a rocprofv3 --pmc (+ --kernel-trace) run, as the JSON
bench.py reads to put the issue side of the roofline beside the HBM side:
  python scripts/pmc_sq.py <rocprof dir> <literals> <workload> <kernel substring>
Counters are summed over the chip per dispatch and averaged over dispatches. Derived fractions use
the kernel-trace durations of the same run and the 2.4 GHz peak clock (MI355X_MICROARCH.md: a wave64
VALU instruction occupies a SIMD-32 for 2 cycles; 1,024 SIMDs; LDS_IDX_ACTIVE counts LDS-array cycles
of the 256 CUs), so they are lower bounds when the chip runs below 2.4 GHz."""
import collections
import csv
import glob
import json
import os
import sys

root, literals, workload = sys.argv[1], int(sys.argv[2]), sys.argv[3]
kname = sys.argv[4] if len(sys.argv) > 4 else "hpk_decode12"
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
durs = []
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
mean = {k: sum(v) / len(v) for k, v in vals.items()}
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402

out = {"kernel": kname, "workload": workload, "literals": literals, "src_sha16": bench.source_hash(),
       "dispatches": {k: len(v) for k, v in vals.items()}, "per_launch": mean}
CLK, SIMDS, CUS = 2.4e9, 1024, 256
if durs:
    t = sorted(durs)[len(durs) // 2]
    out["median_launch_us_profiled"] = t * 1e6
    if "SQ_INSTS_VALU" in mean:
        out["valu_issue_frac"] = mean["SQ_INSTS_VALU"] * 2 / (SIMDS * CLK * t)
    if "SQ_LDS_IDX_ACTIVE" in mean:
        out["lds_active_frac"] = mean["SQ_LDS_IDX_ACTIVE"] / (CUS * CLK * t)
    if "SQ_LDS_BANK_CONFLICT" in mean and "SQ_LDS_IDX_ACTIVE" in mean:
        out["lds_conflict_share"] = mean["SQ_LDS_BANK_CONFLICT"] / max(1.0, mean["SQ_LDS_IDX_ACTIVE"])
out["basis"] = ("valu_issue_frac = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x 2.4 GHz x t); lds_active_frac = "
                "SQ_LDS_IDX_ACTIVE / (256 CUs x 2.4 GHz x t); t = median kernel-trace duration of the same run")
print(json.dumps(out, indent=1))
