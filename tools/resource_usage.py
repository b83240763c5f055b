#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output per kernel."""
import re
import sys

txt = open(sys.argv[1] if len(sys.argv) > 1 else "raymarching_amd/build/resource_usage.txt").read()
KEYS = [("VGPR", r"VGPRs"), ("AGPR", r"AGPRs"), ("SGPR", r"TotalSGPRs"), ("occ", r"Occupancy \[waves/SIMD\]"),
        ("scratch", r"ScratchSize \[bytes/lane\]"), ("sgpr_spill", r"SGPRs Spill"), ("vgpr_spill", r"VGPRs Spill"),
        ("lds", r"LDS Size \[bytes/block\]")]
for b in re.split(r"Function Name: ", txt)[1:]:
    name = b.split()[0]
    vals = []
    for k, pat in KEYS:
        m = re.search(pat + r": (\d+)", b)
        vals.append(f"{k}={m.group(1) if m else '?'}")
    print(f"{name[:70]:70s} " + " ".join(vals))
