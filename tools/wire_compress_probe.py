"""How compressible is the RGB8 wire of a rendered frame?  Renders the C3
(T 4096^2, 256 steps, P0) and C5 (O 8192^2, 512 steps, P0; top-left 4096^2)
frames and estimates, per 64-pixel row segment (one wave's store), the bytes
of a fixed-width delta code: left-neighbour differences per channel, zig-zag,
the segment's maximal bit width per channel, 64 * bits + a 2-byte header.
Also zlib level 1 of the whole RGB8 frame for scale.  (tools/; not product.)"""
import json
import os
import sys
import zlib

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

import raymarching_amd as rm  # noqa: E402


def estimate(rgba):
    rgb = rgba.view(np.uint8).reshape(rgba.shape[0], rgba.shape[1], 4)[..., :3].astype(np.int16)
    H, W, _ = rgb.shape
    seg = rgb.reshape(H, W // 64, 64, 3)
    d = np.diff(seg, axis=2, prepend=seg[:, :, :1, :] * 0)
    d[:, :, 0, :] = 0  # the first pixel is sent raw
    z = np.where(d >= 0, 2 * d, -2 * d - 1)
    bits = np.ceil(np.log2(z.max(axis=2) + 1)).astype(np.int64)  # per segment, per channel
    seg_bytes = 3 + 2 + (63 * bits.sum(-1) + 7) // 8
    raw = H * W * 3
    flat = float(np.mean(bits.sum(-1) == 0))
    comp = zlib.compress(np.ascontiguousarray(rgb.astype(np.uint8)).tobytes(), 1)
    return dict(raw_bytes=raw, delta_code_bytes=int(seg_bytes.sum()), ratio=raw / float(seg_bytes.sum()),
                flat_segments=flat, zlib1_ratio=raw / len(comp),
                bits_hist=np.bincount(bits.sum(-1).ravel(), minlength=25)[:25].tolist())


r = rm.Renderer(0)
out = {}
for name, scene, W, H, steps in (("C3", "T", 4096, 4096, 256), ("C5", "O", 8192, 8192, 512)):
    r.load_scene(rm.SCENE_FILES[scene])
    r.set_uniform("u_resolution", W, H)
    p = rm.POSES["P0"]
    r.set_pose(p["pos"], p["mouse"], p["time"])
    r.set_params(max_steps=steps, count_evals=0)
    f = r.render_rgba8(W, H)[:4096, :4096].cpu().numpy()
    out[name] = estimate(f)
    print(json.dumps({name: out[name]}), flush=True)
r.close()
