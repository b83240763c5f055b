"""The reference's whole frame (render -> FXAA -> bloom of the FXAA frame,
main.cpp:196-214) on one GPU, timed two ways after 0.3 s of untimed frames
each: serial on one stream (bench.py's pipeline leg) and overlapped (frame k's
post passes on a second stream while frame k + 1 renders, two frame buffers).
The overlapped frames are checked against rm_fxaa then rm_bloom.  One JSON
line per pass.  (tools/; not product.)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import raymarching_amd as rm  # noqa: E402
from raymarching_amd.frame import concurrent_streams  # noqa: E402

W = H = 4096
REPS = 40
r = rm.Renderer(0)
main = torch.cuda.current_stream()
r.set_stream(main)
r.load_scene(rm.SCENE_FILES["T"])
r.set_uniform("u_resolution", W, H)
p = rm.POSES["P0"]
r.set_pose(p["pos"], p["mouse"], p["time"])
r.set_params(max_steps=256, count_evals=0, schedule=1)
bufs = [torch.empty((H, W), dtype=torch.int32, device="cuda") for _ in range(2)]
mids = [torch.empty_like(bufs[0]) for _ in range(2)]
outs = [torch.empty_like(bufs[0]) for _ in range(2)]


def serial(k):
    r.render_rgba8(W, H, out=bufs[0])
    r.post_chain(bufs[0], mid=mids[0], out=outs[0])


s_render, s_post = concurrent_streams(torch.device("cuda:0"), 2)
rendered = [torch.cuda.Event(), torch.cuda.Event()]
posted = [torch.cuda.Event(), torch.cuda.Event()]


def overlapped(k):
    a = k % 2
    r.set_stream(s_render, kept=True)
    s_render.wait_event(posted[a])
    r.render_rgba8(W, H, out=bufs[a])
    rendered[a].record(s_render)
    s_post.wait_event(rendered[a])
    r.set_stream(s_post, kept=True)
    r.post_chain(bufs[a], mid=mids[a], out=outs[a])
    posted[a].record(s_post)


def timed(step, first, last):
    t_end = time.time() + 0.3
    k = 0
    while time.time() < t_end:
        step(k)
        k += 1
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(first)
    for j in range(REPS):
        step(k + j)
    if last is not first:
        first.wait_stream(last)
    e1.record(first)
    e1.synchronize()
    return e0.elapsed_time(e1) / REPS, k + REPS - 1


for rep in range(2):
    ser, _ = timed(serial, main, main)
    r.set_stream(main)
    ov, klast = timed(overlapped, s_render, s_post)
    r.set_stream(main)
    torch.cuda.synchronize()
    a = klast % 2
    ref = r.bloom(r.fxaa(bufs[a]))
    torch.cuda.synchronize()
    print(json.dumps({"serial_ms": ser, "overlapped_ms": ov, "overlapped_equal": bool(torch.equal(ref, outs[a]))}),
          flush=True)
r.close()
