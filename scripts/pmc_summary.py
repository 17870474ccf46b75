#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per kernel (template args shortened), mean per dispatch and
per wave of every counter."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1]
data = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        m = re.search(r"hpk_decode_kernel<(.*?)>|hpk_decode_kernelILi(\d+)ELi(\d+)ELi(\d+)E|hpk_decode_kernelILi(\d+)E", k)
        if "decode" not in k:
            continue
        if m and m.group(1):
            name = m.group(1)
        elif m and m.group(2):
            name = f"{m.group(2)},{m.group(3)},{m.group(4)}"
        else:
            name = k[:40]
        data[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, ctrs in data.items():
    waves = sum(ctrs["SQ_WAVES"]) / max(1, len(ctrs["SQ_WAVES"])) if "SQ_WAVES" in ctrs else 4096
    print("==", name, "waves", waves)
    for c in sorted(ctrs):
        v = ctrs[c]
        mean = sum(v) / len(v)
        print(f"   {c:28s} {mean:14.4g}  per-wave {mean / waves:10.4g}")
