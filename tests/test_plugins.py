"""Scene plugins: scene sources compiled with hiprtc
into gfx950 code objects and loaded by rm_load_scene, the analogue of the
reference's "Reload scene shader" (main.cpp:134-139 ->
ShaderLoader::loadFromFile, source/shader_loader.cpp:8-20).

CPU tests compile (hiprtc needs no GPU) and check the diagnostics; GPU tests
check the scene library against SwiftShader known answers of the reference's
common.frag (LIB_kat.npz, cases in golden/lib_kat_cases.py) and plugin
renders against SwiftShader renders of the same scene text (MB_*, SC_*) and
against the compiled-in scene O."""
import glob
import json
import os

import numpy as np
import pytest

import raymarching_amd as rm
from tests.golden import lib_kat_cases as kat
from tests.parity import assert_parity

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
SCENES = {"O": "output_shader.hip", "MB": "mandelbulb.hip", "SC": "showcase.hip"}
PLUGIN_GOLDEN = sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
                       if os.path.basename(p).startswith(("MB_", "SC_")))


def scene_path(name):
    return os.path.join(rm.SCENES_DIR, SCENES[name])


@pytest.fixture(scope="module")
def kat_file(tmp_path_factory):
    p = tmp_path_factory.mktemp("kat") / "lib_kat.hip"
    p.write_text(kat.plugin_source())
    return str(p)


# ------------------------------------------------------------ CPU (hiprtc)


@pytest.mark.parametrize("name", sorted(SCENES))
def test_example_scene_compiles(name):
    ok, log = rm.compile_scene(scene_path(name))
    assert ok, log


def test_known_answer_plugin_compiles(kat_file):
    ok, log = rm.compile_scene(kat_file)
    assert ok, log


def test_compile_error_is_reported_with_the_file_name(tmp_path):
    p = tmp_path / "broken.hip"
    p.write_text("SdResult sceneSDF(vec3 p)\n{\n    return SdResult(sphere(p), undefined_material);\n}\n")
    ok, log = rm.compile_scene(str(p))
    assert not ok
    assert "broken.hip:3" in log, log


def test_glsl_float_literals_are_float(tmp_path):
    # 0.5 is a GLSL float; the translated source must not compute in double
    p = tmp_path / "literals.hip"
    p.write_text("static_assert(sizeof(0.5) == 4, \"literal\");\nconst float kE = 1e-3;\n"
                 "SdResult sceneSDF(vec3 p)\n{\n    return SdResult(length(p) - 1.0 + kE, Material(vec3(0.5), "
                 "vec3(0.0), 1.0, 0.0, 0.0, vec3(0.0), 1.0, vec3(0.0)));\n}\n")
    ok, log = rm.compile_scene(str(p))
    assert ok, log


def test_swizzles_and_qualifiers_translate(tmp_path):
    p = tmp_path / "swz.hip"
    p.write_text("void bump(inout vec3 q, in float a, out float b) { q.x += a; b = q.y; }\n"
                 "SdResult sceneSDF(vec3 p)\n{\n    vec4 v = vec4(p.zyx, 1.0);\n    float b;\n"
                 "    vec3 q = v.xyz;\n    bump(q, v.w, b);\n    vec2 t = q.xz + p.yx;\n"
                 "    return SdResult(length(t) - b, Material(q.zzz, vec3(0.0), 1.0, 0.0, 0.0, vec3(0.0), 1.0, "
                 "vec3(0.0)));\n}\n")
    ok, log = rm.compile_scene(str(p))
    assert ok, log


def test_missing_file_and_include_raise(tmp_path):
    with pytest.raises(rm.RmError):
        rm.compile_scene(str(tmp_path / "absent.hip"))
    p = tmp_path / "inc.hip"
    p.write_text('#include "not_there.hip"\nSdResult sceneSDF(vec3 p) { return SdResult(0.0, Material()); }\n')
    with pytest.raises(rm.RmError):
        rm.compile_scene(str(p))


def test_include_is_inlined(tmp_path, monkeypatch):
    # include names resolve against the process CWD, as in
    # ShaderLoader::preprocess (source/shader_loader.cpp:24,65)
    monkeypatch.chdir(tmp_path)
    (tmp_path / "mats.hip").write_text("const Material kInc = Material(vec3(0.1), vec3(0.0), 1.0, 0.0, 0.0, "
                                       "vec3(0.0), 1.0, vec3(0.0));\n")
    p = tmp_path / "main.hip"
    p.write_text('#include "mats.hip"\nSdResult sceneSDF(vec3 p)\n{\n    return SdResult(length(p) - 1.0, kInc);'
                 "\n}\n")
    ok, log = rm.compile_scene(str(p))
    assert ok, log


def test_kat_cases_match_the_golden_layout():
    z = np.load(os.path.join(GOLDEN, "LIB_kat.npz"), allow_pickle=False)
    m = json.loads(str(z["meta"]))
    assert m["cases"] == [c[0] for c in kat.CASES]
    assert z["dist"].shape == (len(kat.CASES), kat.N_POINTS)
    assert z["mat"].shape == (len(kat.CASES), kat.N_POINTS, 16)
    assert not np.isnan(z["dist"]).any()


# ------------------------------------------------------------ GPU


@pytest.fixture(scope="module")
def R(torch_cuda):
    r = rm.Renderer(0)
    yield r
    r.close()


def _within(a, b, rel, ab):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b) <= ab + rel * np.abs(b)


@pytest.mark.gpu
def test_scene_library_known_answers(R, kat_file):
    """Every case of lib_kat_cases.py through the plugin's rm_scene_eval vs
    the reference common.frag run by SwiftShader."""
    z = np.load(os.path.join(GOLDEN, "LIB_kat.npz"), allow_pickle=False)
    pts = z["points"]
    R.load_scene(kat_file)
    bad = []
    for i, (name, _, cls) in enumerate(kat.CASES):
        R.set_uniform("u_time", float(i))
        dist, mat = R.scene_eval(pts, material=True)
        rel, ab, allowed = kat.TOL[cls]
        exact = float(np.mean((dist == z["dist"][i]) & (mat == z["mat"][i]).all(-1)))
        if exact < 1.0:
            print(f"LIB_kat {name}: {exact:.3f} of points bit-exact, max |d dist| "
                  f"{float(np.max(np.abs(dist - z['dist'][i]))):.3g}")
        ok = _within(dist, z["dist"][i], rel, ab) & _within(mat, z["mat"][i], rel, ab).all(-1)
        if int((~ok).sum()) > allowed:
            j = int(np.argmin(ok))
            bad.append(f"{name}: {int((~ok).sum())} points off, e.g. p={pts[j]} dist {dist[j]} vs "
                       f"{z['dist'][i][j]}, mat {mat[j][:4]} vs {z['mat'][i][j][:4]}")
    assert not bad, "\n".join(bad)


@pytest.mark.gpu
def test_eval_only_plugin_refuses_to_render(R, kat_file):
    R.load_scene(kat_file)
    with pytest.raises(rm.RmError):
        R.render(16, 16)


def _setup(r, path, m):
    r.load_scene(path)
    r.set_pose(m["pos"], m["mouse"], m["time"])
    r.set_params(max_steps=m["max_steps"], shadow_max_steps=0, count_evals=1, kernel="auto")


@pytest.mark.gpu
@pytest.mark.parametrize("path", PLUGIN_GOLDEN, ids=[os.path.basename(p)[:-4] for p in PLUGIN_GOLDEN])
def test_plugin_matches_reference_glsl_golden(R, path):
    z = np.load(path, allow_pickle=False)
    m = json.loads(str(z["meta"]))
    _setup(R, scene_path(m["scene"]), m)
    img, evmap, st = R.render_step_map(m["W"], m["H"])
    s = assert_parity(m["scene"], img.cpu().numpy(), z["rgba"], label="plugin vs golden")
    exact = float(np.mean(evmap.cpu().numpy() == z["evals"]))
    print(f"{os.path.basename(path)}: plugin vs golden {s}, step map exact {exact:.4f}")
    assert exact >= 0.95, exact
    tot = int(z["evals"].sum(dtype=np.uint64))
    assert abs(st["evals"] - tot) <= 5e-3 * tot + 4, (st["evals"], tot)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["O_64_P0", "O_96x54_P2", "O_72x40_P3_512"])
def test_output_shader_plugin_matches_golden(R, name):
    """scenes/output_shader.hip renders scene O through the generic plugin
    path (no sponge-space rays, no exact early exits)."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    m = json.loads(str(z["meta"]))
    _setup(R, scene_path("O"), m)
    img, evmap, st = R.render_step_map(m["W"], m["H"])
    s = assert_parity("O", img.cpu().numpy(), z["rgba"], label="plugin O vs golden")
    exact = float(np.mean(evmap.cpu().numpy() == z["evals"]))
    print(f"{name}: plugin O vs golden {s}, step map exact {exact:.4f}")
    assert exact >= 0.95, exact
    tot = int(z["evals"].sum(dtype=np.uint64))
    assert abs(st["evals"] - tot) <= 5e-3 * tot + 4, (st["evals"], tot)


@pytest.mark.gpu
def test_output_shader_plugin_matches_builtin_scene_eval(R):
    rng = np.random.default_rng(7)
    pts = rng.uniform([-8, -1, -8], [8, 7, 8], (4096, 3)).astype(np.float32)
    R.load_scene("output_shader.frag")
    R.set_uniform("u_time", 3.5)
    d0, m0 = R.scene_eval(pts, material=True)
    R.load_scene(scene_path("O"))
    R.set_uniform("u_time", 3.5)
    d1, m1 = R.scene_eval(pts, material=True)
    assert np.mean(_within(d1, d0, 1e-5, 1e-5)) >= 0.999
    assert np.mean(_within(m1, m0, 1e-5, 1e-5).all(-1)) >= 0.999


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["S0", "T", "O"])
def test_builtin_scene_eval_matches_oracle(R, scene):
    import oracle
    rng = np.random.default_rng(11)
    pts = rng.uniform([-6, -1, -6], [6, 6, 6], (2048, 3)).astype(np.float32)
    R.load_scene(rm.SCENE_FILES[scene])
    R.set_uniform("u_time", 1.25)
    d = R.scene_eval(pts)
    o = oracle.scene_dist(scene, pts, time=1.25)
    assert np.mean(_within(d, o, 1e-5, 1e-5)) >= 0.999, np.abs(d - o).max()


@pytest.mark.gpu
def test_failed_reload_keeps_the_previous_scene(R, tmp_path):
    p = tmp_path / "broken.hip"
    p.write_text("SdResult sceneSDF(vec3 p) { return nope; }\n")
    R.load_scene(scene_path("SC"))
    R.set_pose((2.0, 3.0, 3.0), (0.0, 0.0), 0.0)
    R.set_params(max_steps=64, count_evals=0)
    a = R.render(32, 32).cpu().numpy()
    with pytest.raises(rm.RmError):
        R.load_scene(str(p))
    b = R.render(32, 32).cpu().numpy()
    assert np.array_equal(a, b)


# ------------------------------------- reload of the reference's scene files

REF = "/root/reference"  # build container only; these tests skip elsewhere


def _ref_tree(tmp_path, edit_scene=None, edit_pipeline=None, edit_common=None):
    """Copies of the reference's output_shader.frag + common.frag (+ template.frag)
    in tmp_path, optionally edited the way a user edits them before pressing
    "Reload scene shader" (main.cpp:134-139)."""
    src = open(os.path.join(REF, "output_shader.frag")).read()
    lib = open(os.path.join(REF, "common.frag")).read()
    if edit_scene:
        src = edit_scene(src)
    if edit_pipeline:
        src = edit_pipeline(src)
    if edit_common:
        lib = edit_common(lib)
    (tmp_path / "output_shader.frag").write_text(src)
    (tmp_path / "common.frag").write_text(lib)
    (tmp_path / "template.frag").write_text(open(os.path.join(REF, "template.frag")).read())
    return tmp_path


needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree absent (GPU box)")


@needs_ref
def test_reference_scene_files_load_the_compiled_in_scenes(tmp_path, monkeypatch):
    monkeypatch.chdir(_ref_tree(tmp_path))
    ok, log = rm.compile_scene("output_shader.frag")
    assert ok and log == "compiled-in scene O", log
    ok, log = rm.compile_scene("template.frag")
    assert ok and log == "compiled-in scene T", log
    # line endings and indentation do not matter
    (tmp_path / "output_shader.frag").write_text(open(os.path.join(REF, "output_shader.frag")).read()
                                                 .replace("\n", "\r\n").replace("\t", "    "))
    ok, log = rm.compile_scene("output_shader.frag")
    assert ok and log == "compiled-in scene O", log


@needs_ref
def test_edited_scene_part_is_compiled_as_a_plugin(tmp_path, monkeypatch):
    """The reference's workflow: swap the sponge for the commented mandelbulb
    line of sceneSDF (output_shader.frag:41-42) and reload."""
    def edit(s):
        s = s.replace("\t//SdResult dist0 = SdResult(mandelbulb(", "\tSdResult dist0 = SdResult(mandelbulb(", 1)
        return s.replace("\tSdResult dist0 = SdResult(mengersponge(", "\t//SdResult dist0 = SdResult(mengersponge(", 1)
    monkeypatch.chdir(_ref_tree(tmp_path, edit_scene=edit))
    ok, log = rm.compile_scene("output_shader.frag")
    assert ok, log
    assert "compiled-in" not in log
    # a syntax error in the edited scene is reported with the file's name
    (tmp_path / "output_shader.frag").write_text(edit(open(os.path.join(REF, "output_shader.frag")).read())
                                                 .replace("return sminCubic(dist0", "return sminCubic(dist0 +", 1))
    ok, log = rm.compile_scene("output_shader.frag")
    assert not ok and "output_shader.frag" in log


@needs_ref
@pytest.mark.parametrize("what", ["pipeline", "common", "template"])
def test_edits_outside_the_scene_part_are_refused(tmp_path, monkeypatch, what):
    kw = {}
    if what == "pipeline":
        kw["edit_pipeline"] = lambda s: s.replace("float SSSAmbient     = 0.3;", "float SSSAmbient     = 0.5;", 1)
    elif what == "common":
        kw["edit_common"] = lambda s: s.replace("const float ZFAR = 50;", "const float ZFAR = 60;", 1)
    monkeypatch.chdir(_ref_tree(tmp_path, **kw))
    if what == "template":
        (tmp_path / "template.frag").write_text(open(os.path.join(REF, "template.frag")).read() + "\n// edit\nint x;\n")
    ok, log = rm.compile_scene("template.frag" if what == "template" else "output_shader.frag")
    assert not ok, log


@pytest.mark.gpu
def test_reload_right_after_an_asynchronous_render(R, torch_cuda):
    """rm_load_scene unloads the previous plugin's code object: it must first
    wait for kernels of that module still queued on the context's stream."""
    torch = torch_cuda
    R.load_scene(scene_path("SC"))
    R.set_pose((2.0, 3.0, 3.0), (0.0, 0.0), 0.0)
    R.set_params(max_steps=128, count_evals=0)
    a = torch.empty((192, 256, 4), dtype=torch.float32, device="cuda")
    R.render(256, 192, out=a)          # asynchronous: no stats
    R.load_scene(scene_path("MB"))     # unloads SC's module right away
    R.render(64, 64)
    R.load_scene(scene_path("SC"))
    b = R.render(256, 192)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.gpu
def test_plugin_adaptive_dispatch_order_keeps_pixels(R, torch_cuda):
    """Scene plugins record their tile durations and run costliest first from
    the second launch on (rm_params.schedule), with the same pixels."""
    torch = torch_cuda
    R.load_scene(scene_path("SC"))
    R.set_pose((2.0, 3.0, 3.0), (0.3, 0.1), 1.5)
    R.set_params(max_steps=128, count_evals=0, schedule=0)
    ref = R.render_rgba8(160, 96)
    R.set_params(schedule=1)
    for _ in range(3):
        assert torch.equal(R.render_rgba8(160, 96), ref)
