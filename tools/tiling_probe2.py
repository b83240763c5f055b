import sys, torch
sys.path.insert(0, ".")
import raymarching_amd as rm
r = rm.Renderer(0); r.load_scene("template.frag")
p = rm.POSES["P0"]; r.set_pose(p["pos"], p["mouse"], p["time"])
out = torch.empty((4096, 4096), dtype=torch.int32, device="cuda")
for k in (2, 3, 1, 2, 3):
    r.set_params(max_steps=256, count_evals=0, kernel=k)
    ts = []
    for _ in range(8):
        _, st = r.render_rgba8(4096, 4096, out=out, stats=True) if False else (None, None)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); r.render_rgba8(4096, 4096, out=out); e1.record(); e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort(); print("kernel", k, "ms", round(ts[len(ts)//2], 4), flush=True)
