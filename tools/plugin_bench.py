#!/usr/bin/env python3
"""Scene plugins vs the compiled-in scenes: frame time of one render launch
(HIP events around the kernel, rm_stats.kernel_ms) at 4096^2, RGBA8 out.

usage: python tools/plugin_bench.py [--size 4096] [--max-steps 512] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raymarching_amd as rm  # noqa: E402

CASES = [("O builtin", "output_shader.frag"), ("O plugin", "output_shader.hip"),
         ("MB plugin", "mandelbulb.hip"), ("SC plugin", "showcase.hip")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--max-steps", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--pose", default="P0")
    ap.add_argument("--cases", default="", help="comma-separated case-name prefixes (default: all)")
    a = ap.parse_args()
    import torch
    r = rm.Renderer(0)
    pose = rm.POSES[a.pose]
    out = torch.empty((a.size, a.size), dtype=torch.int32, device="cuda:0")
    for name, f in CASES:
        if a.cases and not any(name.startswith(c) for c in a.cases.split(",")):
            continue
        path = f if f.endswith(".frag") else os.path.join(rm.SCENES_DIR, f)
        t0 = time.time()
        r.load_scene(path)
        load_s = time.time() - t0
        r.set_pose(pose["pos"], pose["mouse"], pose["time"])
        r.set_params(max_steps=a.max_steps, shadow_max_steps=0, count_evals=1, kernel="auto")
        _, st = r.render_rgba8(a.size, a.size, out=out, stats=True)
        evals = st["evals"]
        r.set_params(count_evals=0)
        t_end = time.time() + 0.3  # clock ramp, and the adaptive order settles
        while time.time() < t_end:
            r.render_rgba8(a.size, a.size, out=out)
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            _, st = r.render_rgba8(a.size, a.size, out=out, stats=True)
            ms.append(st["kernel_ms"])
        best = sorted(ms)[len(ms) // 2]  # (median)
        print(json.dumps(dict(lib=os.path.basename(os.environ.get("RM_LIB", "librm.so")), case=name, file=f, size=a.size, max_steps=a.max_steps, pose=a.pose,
                              load_s=round(load_s, 3), kernel_ms=round(best, 4), kernel_ms_all=[round(x, 4) for x in ms],
                              evals=evals, ray_steps_per_s=evals / (best * 1e-3))), flush=True)
    r.close()


if __name__ == "__main__":
    main()
