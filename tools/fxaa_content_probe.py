"""FXAA time at 4096^2 by frame content (the short-span rows of rm_fxaa.hip
output their centre texel, so smooth frames run faster): scene T and scene O
frames at P0, uniform random bytes (no short-span rows), a constant frame.
Median of 7 batches of 20 passes; one JSON line per frame (tools/; analysis)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import raymarching_amd as rm  # noqa: E402

W = H = 4096
r = rm.Renderer(0)
p = rm.POSES["P0"]
frames = {}
for name, scene, steps in (("T_P0", "T", 256), ("O_P0", "O", 512)):
    r.load_scene(rm.SCENE_FILES[scene])
    r.set_pose(p["pos"], p["mouse"], p["time"])
    r.set_params(max_steps=steps, count_evals=0)
    frames[name] = r.render_rgba8(W, H).clone()
g = torch.Generator(device="cuda").manual_seed(5)
frames["random"] = torch.randint(0, 2**31 - 1, (H, W), dtype=torch.int32, device="cuda", generator=g)
frames["constant"] = torch.full((H, W), 0x7f4080ff - 2**32 if 0x7f4080ff >= 2**31 else 0x7f4080ff,
                                dtype=torch.int32, device="cuda")
out = torch.empty((H, W), dtype=torch.int32, device="cuda")
for name, f in frames.items():
    ms = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            r.fxaa(f, out=out)
        e1.record()
        e1.synchronize()
        ms.append(e0.elapsed_time(e1) / 20)
    print(json.dumps({"frame": name, "W": W, "H": H, "fxaa_ms": sorted(ms)[3]}), flush=True)
r.close()
