#!/usr/bin/env python
"""Average PMC counters per kernel from rocprofv3 --pmc csv runs: python scripts/pmc_summary.py DIR [filter]"""
import collections
import csv
import glob
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
flt = sys.argv[2] if len(sys.argv) > 2 else "bcfl"
for f in sorted(glob.glob(sys.argv[1] + "/p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if flt not in n:
            continue
        m = re.search(r"::(\w+<[^>]*>)", n)   # the full template argument list
        k = m.group(1) if m else n[:50]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[k]["dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, d in agg.items():
    print(f"## {k}")
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):.4g}")
