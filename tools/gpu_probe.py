#!/usr/bin/env python3
"""Quick GPU probe: HIP vs oracle parity stats per scene/pose + a timing line."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import oracle  # noqa: E402
import raymarching_amd as rm  # noqa: E402
from raymarching_amd import POSES, S0_POSE  # noqa: E402


def stats(a, b):
    d = np.abs(a[..., :3].astype(np.float64) - b[..., :3]).max(-1)
    d = np.where(np.isnan(d), 1.0, d)
    return dict(max=float(d.max()), mean=float(d.mean()), f2e3=float(np.mean(d <= 2e-3)),
                f1e2=float(np.mean(d <= 1e-2)))


def main():
    kernel = sys.argv[1] if len(sys.argv) > 1 else "auto"
    r = rm.Renderer(0)
    out = {}
    cases = [("S0", 256, 256, S0_POSE, 64), ("T", 256, 256, POSES["P0"], 128), ("T", 192, 108, POSES["P1"], 128),
             ("T", 160, 160, POSES["P4"], 256), ("O", 128, 128, POSES["P0"], 128), ("O", 160, 90, POSES["P2"], 128),
             ("OG", 128, 128, POSES["P0"], 128)]
    for sc, W, H, pose, steps in cases:
        r.load_scene(rm.SCENE_FILES[sc])
        r.set_pose(pose["pos"], pose["mouse"], pose["time"])
        r.set_params(max_steps=steps, count_evals=1, kernel=kernel)
        img, st = r.render(W, H, stats=True)
        img = img.cpu().numpy()
        ref, ev = oracle.render(sc, W, H, pos=pose["pos"], mouse=pose["mouse"], time=pose["time"], max_steps=steps)
        s = stats(img, ref)
        s["evals_gpu"] = st["evals"] / (W * H)
        s["evals_cpu"] = float(ev.mean())
        out[f"{sc}_{W}x{H}"] = s
        print(sc, W, H, json.dumps(s), flush=True)
    # timing: 4096^2 T 256 steps P0
    for sc, steps in (("T", 256), ("O", 512)):
        r.load_scene(rm.SCENE_FILES[sc])
        p = POSES["P0"]
        r.set_pose(p["pos"], p["mouse"], p["time"])
        r.set_params(max_steps=steps, count_evals=1, kernel=kernel)
        W = H = 4096
        buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        _, st = r.render(W, H, out=buf, stats=True)
        evals = st["evals"]
        r.set_params(count_evals=0)
        for _ in range(2):
            r.render(W, H, out=buf)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            _, s2 = r.render(W, H, out=buf, stats=True)
            ts.append(s2["kernel_ms"])
        ms = float(np.median(ts))
        print(json.dumps(dict(scene=sc, W=W, steps=steps, evals=evals, evals_px=evals / W / H, ms=ms,
                              steps_per_s=evals / ms * 1e3,
                              tflops=evals * rm.FLOP_PER_EVAL[sc] / ms / 1e9)), flush=True)


if __name__ == "__main__":
    t = time.time()
    main()
    print("probe done in", time.time() - t)
