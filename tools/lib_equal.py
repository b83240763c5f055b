#!/usr/bin/env python3
"""Bit-identity of librm.so builds: each library (RM_LIB, own process) renders
the same frames (float4 image + per-pixel ray-step map) and writes their
SHA-256; the parent compares them to the first library's.  Used to show that a
kernel restructuring leaves pixels and step maps unchanged.
Per frame: the instrumented kernel's image and step map, the timed kernels'
frames (float4; RGBA8 with the adaptive order), and whether the timed float4
frame equals the instrumented one.
Usage: lib_equal.py lib.so [lib.so ...]   (SCENES=O,OG,T, SIZE=512)"""
import hashlib
import json
import os
import subprocess
import sys

CHILD = r'''
import hashlib, json, os, sys, torch
sys.path.insert(0, ".")
import raymarching_amd as rm
r = rm.Renderer(0)
size = int(os.environ.get("SIZE", "512"))
out = {}
for scene in os.environ.get("SCENES", "O,OG,T").split(","):
    for pn, pose in rm.POSES.items():
        r.load_scene(rm.SCENE_FILES[scene])
        r.set_pose(pose["pos"], pose["mouse"], pose["time"])
        steps = 512 if scene == "O" else 128
        r.set_params(max_steps=steps, shadow_max_steps=0, count_evals=1, schedule=0)
        img, ev, st = r.render_step_map(size, size * 9 // 16)
        h = hashlib.sha256(img.cpu().numpy().tobytes() + ev.cpu().numpy().tobytes()).hexdigest()
        # the timed (uninstrumented) kernel: float4 and RGBA8, row-major and adaptive order
        r.set_params(count_evals=0)
        timed = [r.render(size, size * 9 // 16).cpu().numpy().tobytes()]
        r.set_params(schedule=1)
        for _ in range(3):
            timed.append(r.render_rgba8(size, size * 9 // 16).cpu().numpy().tobytes())
        ht = hashlib.sha256(b"".join(timed)).hexdigest()
        same = timed[0] == img.cpu().numpy().tobytes()
        out[f"{scene}/{pn}"] = [h, st["evals"], ht, same]
print(json.dumps(out))
'''


def main():
    res = []
    for lib in sys.argv[1:]:
        env = dict(os.environ, RM_LIB=os.path.abspath(lib))
        p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=900)
        if p.returncode:
            print(p.stderr[-3000:])
            sys.exit(p.returncode)
        res.append(json.loads(p.stdout.strip().splitlines()[-1]))
    ok = all(v[3] for v in res[0].values())
    print(json.dumps(dict(lib=os.path.basename(sys.argv[1]), timed_eq_instrumented=ok)))
    for lib, r in zip(sys.argv[2:], res[1:]):
        diff = [k for k in res[0] if r.get(k) != res[0][k]]
        ok &= not diff and all(v[3] for v in r.values())
        print(json.dumps(dict(lib=os.path.basename(lib), vs=os.path.basename(sys.argv[1]), frames=len(r),
                              identical=not diff, differ=diff, timed_eq_instrumented=all(v[3] for v in r.values()))))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
