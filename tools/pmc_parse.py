#!/usr/bin/env python3
"""Average rocprofv3 PMC counters per kernel over the dispatches of a run dir."""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        ctr = row.get("Counter_Name", "")
        try:
            v = float(row.get("Counter_Value", "nan"))
        except ValueError:
            continue
        acc[name][(ctr, row.get("Dispatch_Id", row.get("Correlation_Id", "")))].append(v)
out = {}
for name, d in acc.items():
    per = defaultdict(list)
    for (ctr, disp), vals in d.items():
        per[ctr].append(sum(vals))  # sum over instances (XCD/SE dimensions) of one dispatch
    out[name[:120]] = {c: sum(v) / len(v) for c, v in per.items()}
    out[name[:120]]["_dispatches"] = max(len(v) for v in per.values())
json.dump(out, sys.stdout, indent=1)
