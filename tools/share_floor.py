#!/usr/bin/env python3
"""The single-chain floor of a per-rank share: rank 0's packed
rows of an N-GPU frame rendered 8 rows (one tile row) per launch; the longest
such launch is bounded below by the costliest tile's duration (all of a tile
row's tiles run at once), so it is the share's floor whatever the dispatch
order.  Prints the share's per-launch time (adaptive order, latency tiles, as
bench.py renders it) and the per-tile-row launch times.
Usage: share_floor.py [scene W H steps band nshards shard pose]"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import raymarching_amd as rm  # noqa: E402

a = sys.argv[1:]
scene, W, H, steps, band, n, shard, pose = (a + [None] * 8)[:8]
scene = scene or "T"
W, H = int(W or 4096), int(H or 4096)
steps, band, n, shard = int(steps or 256), int(band or 16), int(n or 8), int(shard or 0)
pose = rm.POSES[pose or "P0"]
r = rm.Renderer(0)
r.load_scene(rm.SCENE_FILES[scene])
r.set_uniform("u_resolution", W, H)
r.set_pose(pose["pos"], pose["mouse"], pose["time"])
r.set_params(max_steps=steps, shadow_max_steps=0, count_evals=0, schedule=1)
rows = rm.shard_rows(H, band, n, shard)
out = torch.empty((rows, W), dtype=torch.int32, device="cuda")


def med(f, k=9):
    return float(np.median([f() for _ in range(k)]))


for _ in range(200):  # clock ramp + the adaptive order of the whole share
    r.render_band_rgba8(W, H, band, n, shard, out=out)
torch.cuda.synchronize()
share = med(lambda: r.render_band_rgba8(W, H, band, n, shard, out=out, stats=True)[1]["kernel_ms"])
r.set_params(schedule=0)
share_rm = med(lambda: r.render_band_rgba8(W, H, band, n, shard, out=out, stats=True)[1]["kernel_ms"])
chunk = []
for j0 in range(0, rows, 8):
    c = min(8, rows - j0)
    chunk.append(med(lambda: r.render_rows(W, H, band, n, shard, j0, c, out[j0:j0 + c], stats=True)[1]["kernel_ms"], 5))
empty = med(lambda: r.render_rows(W, H, band, n, shard, 0, 1, out[0:1], stats=True)[1]["kernel_ms"])
i = int(np.argmax(chunk))
print(json.dumps(dict(scene=scene, W=W, H=H, steps=steps, band=band, nshards=n, shard=shard, share_rows=rows,
                      share_ms_adaptive=share, share_ms_rowmajor=share_rm, tile_row_launches=len(chunk),
                      longest_tile_row_ms=chunk[i], longest_tile_row=i, median_tile_row_ms=float(np.median(chunk)),
                      one_row_launch_ms=empty, floor_frac_of_share=chunk[i] / share)))
