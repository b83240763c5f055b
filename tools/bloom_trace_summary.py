#!/usr/bin/env python3
"""Per-kernel averages and the median per-call span of rm_bloom from a
rocprofv3 kernel trace of tools/post_probe.py bloom (tools/sess_x.sh).
Usage: bloom_trace_summary.py TRACE_DIR [LABEL]"""
import csv
import glob
import json
import sys

d = sys.argv[1]
label = sys.argv[2] if len(sys.argv) > 2 else d
stats = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
trace = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
kern = {}
for r in csv.DictReader(open(stats)):
    if "bloom" in r["Name"] or "mip" in r["Name"]:
        kern[r["Name"].split("(")[0].replace("void ", "")] = {"calls": int(r["Calls"]),
                                                               "avg_us": float(r["AverageNs"]) / 1e3}
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "bloom_min" in r["Kernel_Name"]]
spans = []
for i in ends[1:]:
    j = i
    while j > 0 and any(k in rows[j - 1]["Kernel_Name"] for k in ("mip", "poly", "runs")):
        j -= 1
    spans.append((int(rows[i]["End_Timestamp"]) - int(rows[j]["Start_Timestamp"])) / 1e3)
spans.sort()
print(json.dumps({"label": label, "call_span_us_median": spans[len(spans) // 2] if spans else None,
                  "kernels": kern}))
