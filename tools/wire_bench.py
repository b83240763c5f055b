"""Time the compressed wire on one GPU: for each config and N, every
non-root part's render to RGBA8 rows, its render straight into the message
(rm_render_cycle_rows_wire: the encode in the render kernel's epilogue, plus
the scan and compaction), the rows encoder (rm_wire_encode), its message size
against the RGB8 wire, and the root's decode of all of them
(rm_wire_decode_parts) plus the copy of its own rows (rm_scatter_part_rgba8)
-- what DeltaFrame adds per frame.  One JSON line per (config, N); the times are host-bound
for small parts (Python enqueue), so run it under rocprofv3 --kernel-trace
--stats for the kernels' own durations.  (tools/; not product.)"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import raymarching_amd as rm  # noqa: E402
from raymarching_amd.frame import ShardPlan  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


r = rm.Renderer(0)
for name, scene, W, H, steps in (("C3", "T", 4096, 4096, 256), ("C5", "O", 8192, 8192, 512)):
    r.load_scene(rm.SCENE_FILES[scene])
    r.set_uniform("u_resolution", W, H)
    p = rm.POSES["P0"]
    r.set_pose(p["pos"], p["mouse"], p["time"])
    r.set_params(max_steps=steps, count_evals=0, schedule=1)
    for N in (2, 4, 8):
        plan = ShardPlan(W, H, 16, N)
        frame = torch.zeros((H, W), dtype=torch.int32, device="cuda")
        enc_ms, sizes, msgs, locs, rows_ms, fused_ms = [], [], [], [], [], []
        for q in range(N):
            n = plan.count(q)
            loc = torch.empty((n, W), dtype=torch.int32, device="cuda")
            r.render_rows(W, H, 16, N, q, 0, n, loc)
            locs.append(loc)
            if q == 0:
                continue
            msg = torch.empty(rm.wire_capacity(W, n), dtype=torch.uint8, device="cuda")
            ws = torch.empty(rm.wire_workspace_bytes(W, n), dtype=torch.uint8, device="cuda")
            size = torch.zeros(1, dtype=torch.int64, device="cuda")
            rows_ms.append(timed(lambda: r.render_rows(W, H, 16, N, q, 0, n, loc)))
            fused_ms.append(timed(lambda: r.render_cycle_rows_wire(W, H, plan.cycle, plan.offsets[q], 16, 0, n, msg,
                                                                   ws, size)))
            enc_ms.append(timed(lambda: r.wire_encode(loc, msg, ws, size)))
            sizes.append(int(size.item()))
            msgs.append(msg)

        def root():
            r.scatter_part_rgba8(W, H, plan.cycle, plan.offsets[0], 16, plan.count(0), locs[0], frame)
            r.wire_decode_parts(W, H, plan.cycle, [plan.offsets[q] for q in range(1, N)], [16] * (N - 1),
                                [plan.count(q) for q in range(1, N)], msgs, frame)

        dec_ms = timed(root)
        dec_only_ms = timed(lambda: r.wire_decode_parts(W, H, plan.cycle, [plan.offsets[q] for q in range(1, N)],
                                                        [16] * (N - 1), [plan.count(q) for q in range(1, N)], msgs,
                                                        frame))
        ok = torch.equal(frame, r.render_rgba8(W, H))
        raw = plan.count(1) * W * 3
        print(json.dumps({"config": name, "N": N, "share_rows_ms_max": max(rows_ms),
                          "share_render_to_message_ms_max": max(fused_ms), "rows_encode_ms_max": max(enc_ms),
                          "root_scatter_decode_ms": dec_ms, "root_decode_ms": dec_only_ms,
                          "msg_bytes_max": max(sizes), "rgb8_bytes": raw, "ratio_min": raw / max(sizes),
                          "root_ingress_bytes": sum(sizes), "frame_equal": ok}), flush=True)
r.close()
