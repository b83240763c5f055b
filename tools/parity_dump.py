#!/usr/bin/env python3
"""Dump HIP renders for offline parity analysis (gpurun_out/parity_<tag>.npz)."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
import raymarching_amd as rm  # noqa: E402
from raymarching_amd import POSES  # noqa: E402

tag = sys.argv[1]
r = rm.Renderer(0)
res = {}
for sc, W, H, pn, steps in [("O", 64, 64, "P0", 128), ("O", 96, 54, "P2", 128), ("O", 64, 64, "P6", 128),
                            ("O", 128, 128, "P0", 128), ("T", 64, 64, "P0", 128), ("OG", 96, 54, "P2", 128)]:
    p = POSES[pn]
    r.load_scene(rm.SCENE_FILES[sc])
    r.set_pose(p["pos"], p["mouse"], p["time"])
    r.set_params(max_steps=steps, count_evals=1)
    img, st = r.render(W, H, stats=True)
    res[f"{sc}_{W}x{H}_{pn}"] = img.cpu().numpy()
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(f"gpurun_out/parity_{tag}.npz", **res)
print("ok", tag)
