#!/usr/bin/env python3
"""Per-launch HBM traffic of hpk_decode_kernel from rocprofv3 --pmc CSVs (gpu_pmc_traffic.sh).

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB per dispatch. On gfx950 FETCH_SIZE
counts a 128-B fabric read request as 64 B (MI355X_MICROARCH.md, HBM section), so the read
bytes are doubled; the raw EA request counters are kept beside it as a cross-check
(RDREQ: 64-B requests; RDREQ_32B: the 32-B subset; WRREQ: requests, WRREQ_64B: the 64-B subset).
"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
literals = int(sys.argv[2]) if len(sys.argv) > 2 else None
workload = sys.argv[3] if len(sys.argv) > 3 else None
kname = sys.argv[4] if len(sys.argv) > 4 else "hpk_decode"
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if kname not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
mean = {k: sum(v) / len(v) for k, v in vals.items()}
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from loona_amd import _lib  # noqa: E402

out = {"kernel": kname, "workload": workload, "kernel_version": _lib.lib().hpk_version().decode(),
       "src_sha16": bench.source_hash(), "literals": literals, "dispatches": {k: len(v) for k, v in vals.items()},
       "raw_mean": mean}
if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
    rd = mean["FETCH_SIZE"] * 1024 * 2
    wr = mean["WRITE_SIZE"] * 1024
    out.update({"read_bytes_per_launch": rd, "write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
                "correction": "FETCH_SIZE(KiB)*1024*2 (gfx950 half-count) + WRITE_SIZE(KiB)*1024"})
if "TCC_EA0_RDREQ_sum" in mean:
    r32 = mean.get("TCC_EA0_RDREQ_32B_sum", 0.0)
    out["ea_read_bytes_per_launch_128B_requests"] = (mean["TCC_EA0_RDREQ_sum"] - r32) * 128 + r32 * 32
if "TCC_EA0_WRREQ_sum" in mean:
    w64 = mean.get("TCC_EA0_WRREQ_64B_sum", 0.0)
    out["ea_write_bytes_per_launch"] = w64 * 64 + (mean["TCC_EA0_WRREQ_sum"] - w64) * 32
print(json.dumps(out, indent=1))
