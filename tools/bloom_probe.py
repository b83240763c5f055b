"""Bloom-only driver for rocprofv3 runs: one 4096^2 scene-T RGBA8 frame, then
`reps` bloom passes over it (tools/; not part of the product)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import raymarching_amd as rm  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
H = int(sys.argv[2]) if len(sys.argv) > 2 else W
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
r = rm.Renderer(0)
r.load_scene("template.frag")
r.set_pose(*[rm.POSES["P0"][k] for k in ("pos", "mouse", "time")])
r.set_params(max_steps=256, count_evals=0)
frame = r.render_rgba8(W, H)
out = torch.empty_like(frame)
for _ in range(reps):
    r.bloom(frame, out=out)
torch.cuda.synchronize()
print("bloom probe done", W, H, reps)
r.close()
