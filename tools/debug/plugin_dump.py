"""Render the plugin goldens' configurations and save the images (debugging)."""
import glob, json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import raymarching_amd as rm
from tests.parity import diff_stats
SC = {"O": "output_shader.hip", "MB": "mandelbulb.hip", "SC": "showcase.hip"}
r = rm.Renderer(0)
out = {}
for p in sorted(glob.glob("tests/golden/*.npz")):
    nm = os.path.basename(p)[:-4]
    if not nm.startswith(("MB_", "SC_", "O_")):
        continue
    z = np.load(p, allow_pickle=False)
    m = json.loads(str(z["meta"]))
    r.load_scene(os.path.join(rm.SCENES_DIR, SC[m["scene"]]))
    r.set_pose(m["pos"], m["mouse"], m["time"])
    r.set_params(max_steps=m["max_steps"], shadow_max_steps=0, count_evals=1, kernel="auto")
    img, st = r.render(m["W"], m["H"], stats=True)
    img = img.cpu().numpy()
    out[nm] = img
    print(nm, diff_stats(img, z["rgba"]), st["evals"], int(z["evals"].sum()), flush=True)
np.savez_compressed("gpurun_out/plugin_dump.npz", **out)
