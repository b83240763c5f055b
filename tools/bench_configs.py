#!/usr/bin/env python3
"""Single-GPU timing of every BASELINE.json config (C1-C5) plus the oracle's CPU
rate on the same workload sample; one JSON line per case -> stdout.

C4/C5 are 8-GPU configs: here they run as one GPU's share (rows dealt in
bands of 16 to shard 0 of 8), which is what each rank renders before the
gather.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import oracle  # noqa: E402  (CPU rate only)
import raymarching_amd as rm  # noqa: E402

F = rm.FLOP_PER_EVAL


def gpu_case(r, scene, W, H, steps, pose, band=None, nshards=1, reps=5):
    r.load_scene(rm.SCENE_FILES[scene])
    r.set_uniform("u_resolution", W, H)
    r.set_pose(pose["pos"], pose["mouse"], pose["time"])
    r.set_params(max_steps=steps, count_evals=1)
    band = band or H
    n = rm.shard_rows(H, band, nshards, 0)
    buf = torch.empty((n, W, 4), dtype=torch.float32, device="cuda")
    _, st = r.render_band(W, H, band, nshards, 0, out=buf, stats=True)
    r.set_params(count_evals=0)
    ts = []
    for _ in range(reps):
        _, s2 = r.render_band(W, H, band, nshards, 0, out=buf, stats=True)
        ts.append(s2["kernel_ms"])
    ms = float(np.median(ts))
    return st["evals"], st["flop"], ms, n


def cpu_rate(scene, W, H, steps, pose, rows):
    t0 = time.perf_counter()
    _, ev = oracle.render_rows(scene, W, H, rows, fast=True, pos=pose["pos"], mouse=pose["mouse"],
                               time=pose["time"], max_steps=steps)
    dt = time.perf_counter() - t0
    return float(ev.sum()) / dt


def main():
    r = rm.Renderer(0)
    r.set_stream(torch.cuda.current_stream())
    cases = [("C1", "S0", 256, 256, 64, "S0", None, 1)]
    cases += [("C2", "T", 1920, 1080, 128, p, None, 1) for p in rm.POSES]
    cases += [("C3", "T", 4096, 4096, 256, "P0", None, 1),
              ("C4-share", "T", 4096, 4096, 256, "P0", 16, 8),
              ("C5-share", "O", 8192, 8192, 512, "P0", 16, 8),
              ("O-4096", "O", 4096, 4096, 512, "P0", None, 1)]
    for name, scene, W, H, steps, pn, band, nsh in cases:
        pose = rm.S0_POSE if pn == "S0" else rm.POSES[pn]
        evals, flop, ms, n = gpu_case(r, scene, W, H, steps, pose, band, nsh)
        rows = np.arange(0, H, max(1, H // 32), dtype=np.int32) if H > 64 else np.arange(H, dtype=np.int32)
        cpu = cpu_rate(scene, W, H, steps, pose, rows) if os.environ.get("NO_CPU") is None else None
        print(json.dumps(dict(config=name, scene=scene, W=W, H=H, max_steps=steps, pose=pn, rows=n,
                              kernel_ms=ms, ray_steps=evals, ray_steps_per_px=evals / (W * n),
                              ray_steps_per_s=evals / ms * 1e3, frames_per_s_share=1e3 / ms,
                              tflops_counted=flop / ms / 1e9, flop_per_ray_step=flop / max(evals, 1),
                              tflops_reference_tally=evals * F[scene] / ms / 1e9,
                              cpu_ray_steps_per_s=cpu, cpu_threads=oracle.lib(True).oracle_num_threads())),
              flush=True)


if __name__ == "__main__":
    main()
