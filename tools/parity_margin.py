#!/usr/bin/env python3
"""Parity statistics (HIP vs oracle) per scene and pose, to see the margin a
kernel change leaves against tests/parity.py's POLICY; one JSON line per case."""
import json
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import oracle  # noqa: E402  (checker)
import raymarching_amd as rm  # noqa: E402
from parity import diff_stats  # noqa: E402

r = rm.Renderer(0)
scenes = sys.argv[1:] or ["T", "O"]
for sc in scenes:
    for pn, p in rm.POSES.items():
        W, H, steps = 96, 54, 128
        r.load_scene(rm.SCENE_FILES[sc])
        r.set_uniform("u_resolution", W, H)
        r.set_pose(p["pos"], p["mouse"], p["time"])
        r.set_params(max_steps=steps, count_evals=1)
        img, st = r.render(W, H, stats=True)
        ref, ev = oracle.render(sc, W, H, pos=p["pos"], mouse=p["mouse"], time=p["time"], max_steps=steps)
        d = diff_stats(img.cpu().numpy(), ref)
        d.update(scene=sc, pose=pn, evals=st["evals"], evals_ref=int(ev.sum()))
        print(json.dumps(d), flush=True)
