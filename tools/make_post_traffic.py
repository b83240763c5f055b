#!/usr/bin/env python3
"""profiles/pmc_post.json entry from a tools/pmc_post.sh summary: the HBM
bytes one post pass moves, per kernel (2 FETCH_SIZE + WRITE_SIZE, KiB
counters, FETCH doubled for gfx950's wide reads as MI355X_MICROARCH.md's HBM
section prescribes), averaged over the run's dispatches and summed over the
pass's kernels.  The probe's own frame render and dispatch-order kernels, the
buffer fills, and bloom's run tables (built once per frame size,
rm_bloom_runs_kernel) are not part of a pass.  bench.py reports the total as
the pass's `traffic` beside its algorithmic bytes (bench.post_bytes).
usage: make_post_traffic.py SUMMARY.json fxaa|bloom|chain W H [OUT]"""
import json
import os
import sys

SKIP = ("rm_render_direct", "rm_sched_", "fillBuffer", "rm_bloom_runs_kernel")
SHORT = (("rm_fxaa", "fxaa"), ("rm_mip_pyramid", "mips"), ("rm_mip_down", "mips"), ("rm_bloom_poly", "poly"),
         ("rm_bloom_min", "bloom_min"), ("rm_bloom_kernel", "bloom"))


def entry(summ, which, W, H):
    d = json.load(open(summ))
    kern = {}
    for name, v in d.items():
        if any(s in name for s in SKIP) or "FETCH_SIZE" not in v or "WRITE_SIZE" not in v:
            continue
        short = next((s for k, s in SHORT if k in name), name)
        kern[short] = kern.get(short, 0.0) + (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024
    return f"{which}_{W}x{H}", {"hbm_bytes": sum(kern.values()), "kernels": kern, "source": os.path.relpath(summ)}


def main():
    summ, which, W, H = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else "profiles/pmc_post.json"
    key, e = entry(summ, which, W, H)
    allj = json.load(open(out)) if os.path.exists(out) else {}
    allj[key] = e
    json.dump(allj, open(out, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(e))


if __name__ == "__main__":
    main()
