#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per kernel (template args shortened), mean per dispatch and
per wave of every counter."""
import collections
import csv
import os
import glob
import re
import sys

root = sys.argv[1]
data = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if os.environ.get("PMC_FILTER", "decode") not in k:
            continue
        m = re.search(r"(hpk_(?:de|en)code\w*?)I((?:Li\d+E)+)", k)
        if m:
            name = m.group(1) + "<" + ",".join(re.findall(r"Li(\d+)E", m.group(2))) + ">"
        else:
            m = re.search(r"(hpk_decode\w*<[^>]*>)", k)
            name = m.group(1) if m else k[:60]
        data[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, ctrs in data.items():
    waves = sum(ctrs["SQ_WAVES"]) / max(1, len(ctrs["SQ_WAVES"])) if "SQ_WAVES" in ctrs else 4096
    print("==", name, "waves", waves)
    for c in sorted(ctrs):
        v = ctrs[c]
        mean = sum(v) / len(v)
        print(f"   {c:28s} {mean:14.4g}  per-wave {mean / waves:10.4g}")
