#!/usr/bin/env python3
"""Split the small synchronous calls of scripts/lat_trace.py into their parts from a rocprofv3
--hip-trace --kernel-trace run: `python scripts/lat_split.py <rocprof dir> <reps>`. Per decode
launch (the calls of lat_trace.py, in order: 20 warm + reps at 1k literals, then at 5k): the HIP
API time by function between the previous call's synchronisation and this one's, the launch API,
launch-API end -> kernel start, the kernel, kernel end -> synchronisation return, and the host time
outside any HIP call. Medians per batch size, microseconds; one JSON line each."""
import csv
import glob
import json
import os
import statistics
import sys

root, reps = sys.argv[1], int(sys.argv[2])


def rows(pat):
    out = []
    for f in glob.glob(os.path.join(root, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


api = sorted(rows("*hip_api_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
ker = [r for r in rows("*kernel_trace.csv") if "hpk_decode" in r["Kernel_Name"]]
ker.sort(key=lambda r: int(r["Start_Timestamp"]))
by_corr = {r["Correlation_Id"]: r for r in api}
calls = []
for k in ker:
    la = by_corr.get(k["Correlation_Id"])
    if la is None:
        continue
    calls.append((k, la))
groups = {1000: calls[20:20 + reps], 5000: calls[40 + reps:40 + 2 * reps]}
for n, g in groups.items():
    parts = {}
    for i, (k, la) in enumerate(g):
        tid = la["Thread_Id"]
        l0, l1 = int(la["Start_Timestamp"]), int(la["End_Timestamp"])
        k0, k1 = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
        # this call's API records: from the end of the previous call's sync to the end of its own
        sync = next((r for r in api if r["Thread_Id"] == tid and "Synchronize" in r["Function"]
                     and int(r["Start_Timestamp"]) >= l1), None)
        if sync is None:
            continue
        s1 = int(sync["End_Timestamp"])
        prev_end = parts.setdefault("_prev", None)
        lo = prev_end if prev_end is not None else l0
        mine = [r for r in api if r["Thread_Id"] == tid and lo <= int(r["Start_Timestamp"]) <= s1]
        by_fn = {}
        for r in mine:
            by_fn[r["Function"]] = by_fn.get(r["Function"], 0) + int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        api_sum = sum(by_fn.values())
        rec = {"call": s1 - lo, "launch_api": l1 - l0, "launch_to_kernel": k0 - l1, "kernel": k1 - k0,
               "kernel_to_sync_return": s1 - k1, "host_outside_hip": (s1 - lo) - api_sum}
        for f, v in by_fn.items():
            rec["api:" + f] = v
        for key, v in rec.items():
            parts.setdefault(key, []).append(v)
        parts["_prev"] = s1
    parts.pop("_prev", None)
    out = {"literals": n, "calls": len(parts.get("call", []))}
    for key, v in parts.items():
        out[key + "_us"] = round(statistics.median(v) / 1e3, 2)
    print(json.dumps(out))
