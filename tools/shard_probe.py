#!/usr/bin/env python3
"""Per-rank work of an N-GPU frame, timed on one GPU: the render of each
shard's rows (RGBA8), its RGB8 pack, and the root's de-interleave of the
gathered wire.  The gather itself needs N GPUs (the driver's scaling run).
usage: shard_probe.py [W] [scene] [max_steps]"""
import json
import sys

import torch

sys.path.insert(0, ".")
import raymarching_amd as rm  # noqa: E402
from raymarching_amd.frame import ShardPlan  # noqa: E402

W = H = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
scene = sys.argv[2] if len(sys.argv) > 2 else "T"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 256
r = rm.Renderer(0)
r.load_scene(rm.SCENE_FILES[scene])
p = rm.POSES["P0"]
r.set_pose(p["pos"], p["mouse"], p["time"])
r.set_params(max_steps=steps, shadow_max_steps=0, count_evals=0)
stream = torch.cuda.current_stream()
r.set_stream(stream)


def timed(fn, reps=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


full = torch.empty((H, W), dtype=torch.int32, device="cuda")
t1 = timed(lambda: r.render_rgba8(W, H, out=full))
print(json.dumps({"n": 1, "frame_ms": t1}), flush=True)
for n in (2, 4, 8):
    plan = ShardPlan(W, H, 16, n)
    rps = plan.rows_per_shard
    band = torch.empty((rps, W), dtype=torch.int32, device="cuda")
    wire = torch.empty((rps, 3 * W), dtype=torch.uint8, device="cuda")
    per = [timed(lambda s=s: r.render_rows(W, H, 16, n, s, 0, plan.count(s), band[: plan.count(s)]))
           for s in range(n)]
    pack = timed(lambda: r.pack_rgb8(band, out=wire))
    g = torch.zeros((n, rps, 3 * W), dtype=torch.uint8, device="cuda")
    dein = timed(lambda: r.deinterleave(W, H, 16, n, rps, g, out=full))
    wire_mib = (n - 1) * rps * 3 * W / 2 ** 20
    print(json.dumps({"n": n, "render_ms_per_shard": per, "render_ms_max": max(per), "pack_ms": pack,
                      "deinterleave_ms": dein, "root_inbound_MiB": wire_mib,
                      "ideal_ms": t1 / n}), flush=True)
r.close()

# frames overlapped on two streams: frame k+1's waves fill the SIMDs while
# frame k's longest waves (the grazing shadow marches) finish
r = rm.Renderer(0)
r.load_scene(rm.SCENE_FILES[scene])
r.set_pose(p["pos"], p["mouse"], p["time"])
r.set_params(max_steps=steps, shadow_max_steps=0, count_evals=0)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
for n in (1, 2, 4, 8):
    plan = ShardPlan(W, H, 16, n)
    cnt = plan.count(0)
    bufs = [torch.empty((cnt, W), dtype=torch.int32, device="cuda") for _ in range(2)]
    res = {"n": n}
    for ns in (1, 2):
        def frames(k):
            for i in range(k):
                st = streams[i % ns]
                r.set_stream(st)
                r.render_rows(W, H, 16, n, 0, 0, cnt, bufs[i % 2])
        frames(4)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(streams[0])
        for st in streams[1:]:
            st.wait_event(e0)
        reps = 20
        frames(reps)
        for st in streams[1:ns]:
            ev = torch.cuda.Event()
            ev.record(st)
            streams[0].wait_event(ev)
        e1.record(streams[0])
        e1.synchronize()
        res[f"ms_per_frame_{ns}stream"] = e0.elapsed_time(e1) / reps
    print(json.dumps(res), flush=True)
r.close()
