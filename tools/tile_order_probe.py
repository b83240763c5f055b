#!/usr/bin/env python3
"""Does the dispatch order of the render's tiles move the tail of a launch?
For each configuration: per-pixel ray-step map (rm_render_step_map) -> per
8x8-tile cost (max and sum of the tile's sceneSDF calls) -> the tiles sorted
costliest first (rm_set_tile_order) -> kernel time against the identity order
(median of 15 launches after a clock ramp).  One JSON line per config/order."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import raymarching_amd as rm  # noqa: E402
from raymarching_amd.frame import ShardPlan  # noqa: E402

CONFIGS = [  # name, scene, W, H, steps, pose, band, nshards, shard
    ("C4share", "T", 4096, 4096, 256, "P0", 16, 8, 0),
    ("C2P1", "T", 1920, 1080, 128, "P1", 1080, 1, 0),
    ("C2P0", "T", 1920, 1080, 128, "P0", 1080, 1, 0),
    ("C3", "T", 4096, 4096, 256, "P0", 4096, 1, 0),
    ("C5share", "O", 8192, 8192, 512, "P0", 16, 8, 0),
]


def timed(r, W, H, band, n, shard, out, reps=15):
    t_end = time.time() + 0.3
    while time.time() < t_end:
        r.render_band_rgba8(W, H, band, n, shard, out=out)
    torch.cuda.synchronize()
    ms = sorted(r.render_band_rgba8(W, H, band, n, shard, out=out, stats=True)[1]["kernel_ms"] for _ in range(reps))
    return ms[len(ms) // 2]


def main():
    r = rm.Renderer(0)
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
    for name, scene, W, H, steps, pose, band, n, shard in CONFIGS:
        if only and name not in only:
            continue
        p = rm.POSES[pose]
        r.load_scene(rm.SCENE_FILES[scene])
        r.set_uniform("u_resolution", W, H)
        r.set_pose(p["pos"], p["mouse"], p["time"])
        r.set_params(max_steps=steps, shadow_max_steps=0, count_evals=0)
        _, ev, _ = r.render_step_map(W, H)
        ev = ev.cpu().numpy()
        rows = ShardPlan(W, H, band, n).rows(shard)
        ev = ev[rows]
        tx, ty = r.tile_grid(W, len(rows))
        pad = np.zeros((ty * 8, tx * 8), np.int64)
        pad[: ev.shape[0], : ev.shape[1]] = ev
        tiles = pad.reshape(ty, 8, tx, 8).transpose(0, 2, 1, 3).reshape(ty * tx, 64)
        out = torch.empty((len(rows), W), dtype=torch.int32, device="cuda")
        r.set_tile_order(None)
        ref = r.render_band_rgba8(W, H, band, n, shard, out=out.clone())
        res = {"identity": timed(r, W, H, band, n, shard, out)}
        for key, cost in (("max", tiles.max(1)), ("sum", tiles.sum(1))):
            order = np.argsort(-cost, kind="stable").astype(np.uint32)
            r.set_tile_order(order)
            res[key] = timed(r, W, H, band, n, shard, out)
            assert torch.equal(out, ref), "tile order changed pixels"
        r.set_tile_order(None)
        print(json.dumps(dict(config=name, tiles=tx * ty, max_tile_evals=int(tiles.max()),
                              mean_tile_evals=float(tiles.mean()), **{k + "_ms": v for k, v in res.items()})),
              flush=True)


if __name__ == "__main__":
    main()
