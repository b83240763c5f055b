"""Debug aid: frames of every kernel kind against tile8 (bit equality), then
single persistent-wave launches of growing scene-O sizes, timed."""
import sys
import time
import numpy as np
import torch
sys.path.insert(0, ".")
import raymarching_amd as rm
from raymarching_amd import POSES, S0_POSE

r = rm.Renderer(0)
for scene, W, H in (("S0", 77, 45), ("T", 77, 45), ("T", 256, 128), ("O", 64, 48), ("O", 200, 136)):
    r.load_scene(rm.SCENE_FILES[scene])
    p = S0_POSE if scene == "S0" else POSES["P3"]
    r.set_pose(p["pos"], p["mouse"], p["time"])
    r.set_params(max_steps=128, count_evals=1, kernel="tile8", schedule=0)
    a, sa = r.render_rgba8(W, H, stats=True)
    A = a.cpu().numpy()
    for k in ("tile16", "tile16x4", "persist", "persist", "persist"):
        r.set_params(kernel=k)
        b, sb = r.render_rgba8(W, H, stats=True)
        torch.cuda.synchronize()
        B = b.cpu().numpy()
        bad = np.argwhere(A != B)
        print(scene, W, H, k, "evals", sa["evals"], sb["evals"], "bad px", len(bad),
              "first", bad[:3].tolist(), flush=True)
r.load_scene(rm.SCENE_FILES["O"])
r.set_params(max_steps=512, count_evals=0, kernel="persist", schedule=1)
for n in (256, 1024, 2048, 4096):
    for rep in range(3):
        t = time.time()
        _, st = r.render_rgba8(n, n, stats=True)
        print("O persist", n, rep, "kernel_ms", round(st["kernel_ms"], 3), "wall_s", round(time.time() - t, 3), flush=True)
r.close()
