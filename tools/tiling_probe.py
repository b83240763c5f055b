#!/usr/bin/env python3
"""Kernel time of the 16x16 vs 8x8-pixel workgroup tilings on full frames and 1/8 shards."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import raymarching_amd as rm  # noqa: E402

r = rm.Renderer(0)
r.set_stream(torch.cuda.current_stream())
for scene, W, steps, pn, nsh in (("T", 4096, 256, "P0", 1), ("T", 4096, 256, "P0", 8), ("T", 1920, 128, "P1", 1),
                                 ("O", 4096, 512, "P0", 1), ("O", 8192, 512, "P0", 8)):
    H = W if W != 1920 else 1080
    p = rm.POSES[pn]
    r.load_scene(rm.SCENE_FILES[scene])
    r.set_uniform("u_resolution", W, H)
    r.set_pose(p["pos"], p["mouse"], p["time"])
    n = rm.shard_rows(H, 16, nsh, 0)
    buf = torch.empty((n, W, 4), dtype=torch.float32, device="cuda")
    res = {}
    for k in ("tile16", "tile8", "tile16x4"):
        r.set_params(max_steps=steps, kernel=k)
        r.render_band(W, H, 16, nsh, 0, out=buf)
        ts = [r.render_band(W, H, 16, nsh, 0, out=buf, stats=True)[1]["kernel_ms"] for _ in range(5)]
        res[k] = float(np.median(ts))
    print(json.dumps(dict(scene=scene, W=W, H=H, pose=pn, nshards=nsh, **res)), flush=True)
