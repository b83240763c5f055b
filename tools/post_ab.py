#!/usr/bin/env python3
"""Time the post passes (bloom, FXAA: bench.py's timers) of librm.so builds
side by side on one 4096^2 scene-T RGBA8 frame and check that every build's
output is identical to the first one's.  Each library runs in its own process
(RM_LIB).  Usage: post_ab.py lib.so [lib.so ...]   (tools/; A/B only)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import hashlib, json, sys, torch
sys.path.insert(0, ".")
import bench, raymarching_amd as rm
W = int(sys.argv[2])
r = rm.Renderer(0)
r.load_scene("template.frag")
r.set_pose(*[rm.POSES["P0"][k] for k in ("pos", "mouse", "time")])
r.set_params(max_steps=256)
frame = r.render_rgba8(W, W)
st = torch.cuda.current_stream()
r.set_stream(st)
b = bench.time_bloom(r, frame, st, reps=40)
f = bench.time_fxaa(r, frame, st, reps=40)
out = torch.empty_like(frame)
r.bloom(frame, out=out)
h = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
print(json.dumps(dict(lib=sys.argv[1], size=W, bloom_ms=b["ms"], fxaa_ms=f["ms"], bloom_sha=h)), flush=True)
'''


def main():
    size = os.environ.get("SIZE", "4096")
    for lib in sys.argv[1:]:
        env = dict(os.environ, RM_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, "-c", CHILD, os.path.basename(lib), size], env=env, timeout=300)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
