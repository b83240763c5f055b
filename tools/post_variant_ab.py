#!/usr/bin/env python3
"""Time a post pass (FXAA, or bloom with POST=bloom) of librm.so builds side by
side (tools/build_variants.sh variants; one process per library, RM_LIB) over
one 4096^2 scene-T RGBA8 frame: median of 7 batches of 20 passes.
FRAME=random: a frame of uniform random bytes instead.
Usage: [POST=bloom] [FRAME=random] post_variant_ab.py lib.so ..."""
import os
import subprocess
import sys

CHILD = r'''
import os, sys, torch
sys.path.insert(0, ".")
import raymarching_amd as rm
r = rm.Renderer(0)
r.load_scene(rm.SCENE_FILES["T"])
p = rm.POSES["P0"]; r.set_pose(p["pos"], p["mouse"], p["time"]); r.set_params(max_steps=256)
f = r.render_rgba8(4096, 4096)
if os.environ.get("FRAME") == "random":  # uniform random bytes: no short-span blocks
    g = torch.Generator(device="cuda").manual_seed(5)
    f = torch.randint(0, 2**31 - 1, f.shape, dtype=torch.int32, device="cuda", generator=g)
out = torch.empty_like(f)
fn = getattr(r, sys.argv[2])
ref = fn(f).clone()
ms = []
for _ in range(7):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn(f, out=out)
    e1.record(); e1.synchronize()
    ms.append(e0.elapsed_time(e1) / 20)
import hashlib
print(sys.argv[1], os.environ.get("FRAME", "T_P0"), sys.argv[2] + "_ms", sorted(ms)[3], "same_as_first", bool(torch.equal(out, ref)),
      "sha", hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16], flush=True)
'''
for lib in sys.argv[1:]:
    subprocess.run([sys.executable, "-c", CHILD, os.path.basename(lib), os.environ.get("POST", "fxaa")],
                   env=dict(os.environ, RM_LIB=os.path.abspath(lib)), timeout=120, check=True)
