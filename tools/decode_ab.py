"""A/B of the compressed wire's root decode (rm_wire_decode_parts) on the C3
frame: every non-root part of an even N-rank split encoded by the render
epilogue, then all of them decoded into the frame in one launch, timed with
events on the stream the renderer is bound to; the frame is checked against
rm_render_rgba8.  One JSON line per N (DEC_NS, default 2,8).  Run once per
library (RM_LIB=...).
(tools/; not product.)"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import raymarching_amd as rm  # noqa: E402
from raymarching_amd.frame import ShardPlan  # noqa: E402

W = H = 4096
r = rm.Renderer(0)
r.set_stream(torch.cuda.current_stream())
r.load_scene(rm.SCENE_FILES["T"])
r.set_uniform("u_resolution", W, H)
p = rm.POSES["P0"]
r.set_pose(p["pos"], p["mouse"], p["time"])
r.set_params(max_steps=256, count_evals=0, schedule=1)
ref = r.render_rgba8(W, H)
for N in [int(x) for x in os.environ.get("DEC_NS", "2,8").split(",")]:
    plan = ShardPlan(W, H, 16, N)
    frame = torch.zeros((H, W), dtype=torch.int32, device="cuda")
    msgs = []
    for q in range(1, N):
        n = plan.count(q)
        msg = torch.empty(rm.wire_capacity(W, n), dtype=torch.uint8, device="cuda")
        ws = torch.empty(rm.wire_workspace_bytes(W, n), dtype=torch.uint8, device="cuda")
        size = torch.zeros(1, dtype=torch.int64, device="cuda")
        r.render_cycle_rows_wire(W, H, plan.cycle, plan.offsets[q], 16, 0, n, msg, ws, size)
        msgs.append(msg)
    loc = torch.empty((plan.count(0), W), dtype=torch.int32, device="cuda")
    r.render_cycle_rows(W, H, plan.cycle, plan.offsets[0], 16, 0, plan.count(0), loc)
    r.scatter_part_rgba8(W, H, plan.cycle, plan.offsets[0], 16, plan.count(0), loc, frame)
    args = (W, H, plan.cycle, [plan.offsets[q] for q in range(1, N)], [16] * (N - 1),
            [plan.count(q) for q in range(1, N)], msgs, frame)
    r.wire_decode_parts(*args)
    torch.cuda.synchronize()
    ok = torch.equal(frame, ref)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(40):
        r.wire_decode_parts(*args)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"lib": os.path.basename(os.environ.get("RM_LIB", "librm.so")), "N": N,
                      "decode_ms": e0.elapsed_time(e1) / 40, "frame_equal": ok}), flush=True)
r.close()
