#!/usr/bin/env python3
"""Dump one HIP render to gpurun_out/dump_<tag>.npy: dump_img.py TAG SCENE W H POSE STEPS"""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
import raymarching_amd as rm  # noqa: E402

tag, sc, W, H, pn, steps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], int(sys.argv[6])
r = rm.Renderer(0)
p = rm.S0_POSE if pn == "S0" else rm.POSES[pn]
r.load_scene(rm.SCENE_FILES[sc])
r.set_pose(p["pos"], p["mouse"], p["time"])
r.set_params(max_steps=steps)
img = r.render(W, H).cpu().numpy()
os.makedirs("gpurun_out", exist_ok=True)
np.save(f"gpurun_out/dump_{tag}.npy", img)
print("saved", tag, img.shape)
