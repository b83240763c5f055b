#!/usr/bin/env python3
"""Cost of a renderer leaving and re-entering a frame stream every frame (the
pattern DistributedFrame/DeltaFrame use with two frame streams: ADVICE r4).
Small scene-T frames back to back on one stream, with and without a
set_stream(frame) / set_stream(caller) pair around each render; wall time per
frame over `frames` frames (median of 5).  Usage: stream_switch_probe.py [W] [frames]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raymarching_amd as rm  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 512
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 400
r = rm.Renderer(0)
r.load_scene(rm.SCENE_FILES["T"])
p = rm.POSES["P0"]
r.set_pose(p["pos"], p["mouse"], p["time"])
r.set_params(max_steps=256, count_evals=0)
caller = torch.cuda.current_stream()
st = torch.cuda.Stream()
out = torch.empty((W, W), dtype=torch.int32, device="cuda")


def run(switch):
    with torch.cuda.stream(st):
        r.set_stream(st)
        for _ in range(20):
            r.render_rgba8(W, W, out=out)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(frames):
            if switch:
                r.set_stream(st)
            r.render_rgba8(W, W, out=out)
            if switch:
                r.set_stream(caller)
        torch.cuda.synchronize()
        r.set_stream(caller)
        return (time.perf_counter() - t0) / frames * 1e3


res = {"stay": [], "switch": []}
for _ in range(5):
    res["stay"].append(run(False))
    res["switch"].append(run(True))
med = {k: sorted(v)[2] for k, v in res.items()}
print(json.dumps({"W": W, "frames": frames, "ms_per_frame_stay": med["stay"], "ms_per_frame_switch": med["switch"],
                  "switch_cost_us": (med["switch"] - med["stay"]) * 1e3}))
