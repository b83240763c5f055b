"""Post-pass driver for rocprofv3 runs: one 4096^2 scene-T RGBA8 frame, then
`reps` passes of `fxaa`, `bloom` or `post_chain` (FXAA then bloom of its
output, rm_post_chain) over it (tools/; not part of the product).  FRAME=random
replaces the rendered frame by uniform noise (FXAA's worst content: no short
spans).  Usage: post_probe.py fxaa|bloom|post_chain|fxaa_bloom [W] [H] [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import raymarching_amd as rm  # noqa: E402

which = sys.argv[1]
W = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
H = int(sys.argv[3]) if len(sys.argv) > 3 else W
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
r = rm.Renderer(0)
r.load_scene("template.frag")
r.set_pose(*[rm.POSES["P0"][k] for k in ("pos", "mouse", "time")])
r.set_params(max_steps=256, count_evals=0)
frame = r.render_rgba8(W, H)
if os.environ.get("FRAME") == "random":
    g = torch.Generator(device="cuda").manual_seed(7)
    frame = torch.randint(-2**31, 2**31 - 1, (H, W), dtype=torch.int32, device="cuda", generator=g)
out = torch.empty_like(frame)
mid = torch.empty_like(frame)
for _ in range(reps):
    if which == "post_chain":
        r.post_chain(frame, mid=mid, out=out)
    elif which == "fxaa_bloom":  # the two passes as separate calls (rm_fxaa, then rm_bloom of its output)
        r.fxaa(frame, out=mid)
        r.bloom(mid, out=out)
    else:
        getattr(r, which)(frame, out=out)
torch.cuda.synchronize()
print("post probe done", which, W, H, reps)
r.close()
