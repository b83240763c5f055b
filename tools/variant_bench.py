#!/usr/bin/env python3
"""Time the render kernel of librm.so builds side by side (A/B of RM_OPT
variants, tools/build_variants.sh) on the configurations the bench and the
verdict quote: one JSON line per (library, config).  Each library runs in its
own process (RM_LIB).  Usage: variant_bench.py lib.so [lib.so ...]"""
import json
import os
import subprocess
import sys

CONFIGS = [  # name, scene, W, H, steps, pose, band, nshards, shard
    ("C3", "T", 4096, 4096, 256, "P0", 4096, 1, 0),
    ("C4share", "T", 4096, 4096, 256, "P0", 16, 8, 0),
    ("C2P1", "T", 1920, 1080, 128, "P1", 1080, 1, 0),
    ("O4096", "O", 4096, 4096, 512, "P0", 4096, 1, 0),
    ("C5frame", "O", 8192, 8192, 512, "P0", 8192, 1, 0),
    ("C5share", "O", 8192, 8192, 512, "P0", 16, 8, 0),
    # other poses (select with CONFIGS=...)
    ("C2P0", "T", 1920, 1080, 128, "P0", 1080, 1, 0),
    ("C2P3", "T", 1920, 1080, 128, "P3", 1080, 1, 0),
    ("C2P8", "T", 1920, 1080, 128, "P8", 1080, 1, 0),
    ("C4shareP1", "T", 4096, 4096, 256, "P1", 16, 8, 0),
    ("C4shareP3", "T", 4096, 4096, 256, "P3", 16, 8, 0),
    ("C4share7", "T", 4096, 4096, 256, "P0", 16, 8, 7),
]

CHILD = r'''
import json, os, sys, time, torch
sys.path.insert(0, ".")
import raymarching_amd as rm
cfgs = json.loads(sys.argv[1])
r = rm.Renderer(0)
for (name, scene, W, H, steps, pose, band, n, shard), sched in [(c, s) for c in cfgs for s in (0, 1)]:
    p = rm.POSES[pose]
    r.load_scene(rm.SCENE_FILES[scene])
    r.set_uniform("u_resolution", W, H)
    r.set_pose(p["pos"], p["mouse"], p["time"])
    r.set_params(max_steps=steps, shadow_max_steps=0, count_evals=1, schedule=sched,
                 kernel=os.environ.get("RM_KERNEL", "auto"))
    rows = rm.shard_rows(H, band, n, shard)
    out = torch.empty((rows, W), dtype=torch.int32, device="cuda")
    _, st = r.render_band_rgba8(W, H, band, n, shard, out=out, stats=True)
    evals = st["evals"]
    r.set_params(count_evals=0)
    t_end = time.time() + 0.4
    while time.time() < t_end:  # clock ramp
        r.render_band_rgba8(W, H, band, n, shard, out=out)
    torch.cuda.synchronize()
    ms = sorted(r.render_band_rgba8(W, H, band, n, shard, out=out, stats=True)[1]["kernel_ms"] for _ in range(15))
    print(json.dumps(dict(lib=sys.argv[2], kernel=os.environ.get("RM_KERNEL", "auto"), config=name, schedule=sched, kernel_ms=ms[len(ms) // 2], min_ms=ms[0],
                          ray_steps=evals, rate=evals / (ms[len(ms) // 2] / 1e3))), flush=True)
'''


def main():
    libs = sys.argv[1:] or ["raymarching_amd/librm.so"]
    only = os.environ.get("CONFIGS")
    cfgs = [c for c in CONFIGS if not only or c[0] in only.split(",")]
    for lib in libs:
        env = dict(os.environ, RM_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, "-c", CHILD, json.dumps(cfgs), os.path.basename(lib)], env=env,
                           timeout=600)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
