import json, sys, torch
sys.path.insert(0, ".")
import raymarching_amd as rm
r = rm.Renderer(0)
for scene, W, H, steps, pose in (("T", 4096, 4096, 256, "P0"), ("T", 4096, 4096, 256, "P1"), ("O", 8192, 8192, 512, "P0")):
    r.load_scene(rm.SCENE_FILES[scene]); r.set_uniform("u_resolution", W, H)
    p = rm.POSES[pose]; r.set_pose(p["pos"], p["mouse"], p["time"])
    r.set_params(max_steps=steps, shadow_max_steps=0, count_evals=1)
    _, ev, _ = r.render_step_map(W, H)
    row = ev.double().sum(1)
    tot = row.sum().item()
    srt = torch.sort(row, descending=True).values.cumsum(0) / tot
    fr = {f"{q}": round(srt[int(q * H) - 1].item(), 3) for q in (0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7)}
    # coarse profile: cost share of each 1/16 of the frame, top to bottom
    prof = [round(x, 3) for x in (row.view(16, -1).sum(1) / tot).tolist()]
    print(json.dumps({"scene": scene, "pose": pose, "top_rows_cost_share": fr, "profile16": prof}), flush=True)
