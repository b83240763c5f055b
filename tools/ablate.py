#!/usr/bin/env python3
"""Time the T render at 4096^2 with the shadow loop capped / marches capped, to
apportion kernel time between shadow steps, march steps and the fixed work."""
import json
import sys

import torch

sys.path.insert(0, ".")
import raymarching_amd as rm  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "T"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 256
W = H = 4096
r = rm.Renderer(0)
r.load_scene(rm.SCENE_FILES[scene])
p = rm.POSES["P0"]
r.set_pose(p["pos"], p["mouse"], p["time"])
buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
for ms_, sh in ((steps, 0), (steps, 1), (steps, 4), (8, 0), (8, 1), (1, 1)):
    r.set_params(max_steps=ms_, shadow_max_steps=sh, count_evals=1)
    _, st = r.render(W, H, out=buf, stats=True)
    r.set_params(count_evals=0)
    ts = []
    for _ in range(6):
        _, s2 = r.render(W, H, out=buf, stats=True)
        ts.append(s2["kernel_ms"])
    ts.sort()
    print(json.dumps(dict(scene=scene, max_steps=ms_, shadow_cap=sh, evals_px=st["evals"] / W / H,
                          ms=ts[len(ts) // 2])), flush=True)
