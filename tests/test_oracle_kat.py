"""Closed-form known-answer tests of the oracle's SDF library (GLSL
semantics of common.frag).  No reference fixtures exist for these; values are
exact by construction."""
import math
import os

import numpy as np
import pytest

import oracle


@pytest.fixture(scope="module")
def L():
    return oracle.lib()


def test_glsl_mod_is_floor_based(L):
    # GLSL mod(x, y) = x - y * floor(x / y): result has the sign of y
    assert L.oracle_glsl_mod(-0.5, 2.0) == pytest.approx(1.5)
    assert L.oracle_glsl_mod(3.5, 2.0) == pytest.approx(1.5)
    assert L.oracle_glsl_mod(-4.0, 2.0) == 0.0
    assert math.fmod(-0.5, 2.0) == -0.5  # C fmod differs


def test_smoothstep(L):
    assert L.oracle_glsl_smoothstep(0.0, 1.0, -1.0) == 0.0
    assert L.oracle_glsl_smoothstep(0.0, 1.0, 2.0) == 1.0
    assert L.oracle_glsl_smoothstep(0.0, 1.0, 0.5) == pytest.approx(0.5)
    assert L.oracle_glsl_smoothstep(0.15, 1.1, 0.15) == 0.0


def test_sphere_and_boxes(L):
    assert L.oracle_sphere(0, 1, -1, 0, 1, -3, 1) == pytest.approx(1.0)
    assert L.oracle_sphere(0, 1, -3, 0, 1, -3, 1) == pytest.approx(-1.0)
    # cube: exact euclidean box distance; inside -> negative max component
    assert L.oracle_cube(-5, 4, 8, -5, 4, 5, 1) == pytest.approx(2.0)
    assert L.oracle_cube(-3, 6, 5, -5, 4, 5, 1) == pytest.approx(math.sqrt(2.0))
    assert L.oracle_cube(-5, 4, 5, -5, 4, 5, 1) == pytest.approx(-1.0)
    # sdBox (common.frag:595-600) is min(max-component, outside length)
    assert L.oracle_sdbox(3, 0, 0, 1, 1, 1) == pytest.approx(2.0)
    assert L.oracle_sdbox(3, 3, 0, 1, 1, 1) == pytest.approx(2.0)  # min(2, 2.83)
    assert L.oracle_sdbox(0, 0, 0, 1, 1, 1) == pytest.approx(-1.0)


def test_menger_sponge(L):
    # far outside: the bounding box term dominates
    assert L.oracle_menger(5, 0, 0) == pytest.approx(4.0)
    # the centre lies in the first-level cross hole: distance (1-1/3*... ) > 0
    assert L.oracle_menger(0, 0, 0) > 0.0
    # a corner of the cube is solid (inside, d < 0)
    assert L.oracle_menger(0.95, 0.95, 0.95) < 0.0


def test_smin_cubic(L):
    # |a-b| >= k: plain min
    assert L.oracle_smin_cubic(1.0, 3.0, 0.5) == 1.0
    assert L.oracle_smin_cubic(3.0, 1.0, 0.5) == 1.0
    # a == b: min - k/6
    assert L.oracle_smin_cubic(1.0, 1.0, 0.6) == pytest.approx(1.0 - 0.6 / 6.0, rel=1e-6)


def test_sphere_scene_normal_points_outward():
    pts = np.array([[0, 2, -3], [1, 1, -3], [0, 1, -2]], np.float32)
    n = oracle.normal("S0", pts)
    exp = np.array([[0, 1, 0], [1, 0, 0], [0, 0, 1]], np.float32)
    np.testing.assert_allclose(n, exp, atol=2e-3)


def test_scene_distances_consistent():
    pts = np.array([[0, 3, 0], [3, 2, 3], [-5, 4, 5], [10, 0.5, 10]], np.float32)
    dT = oracle.scene_dist("T", pts, time=0.0)
    dO = oracle.scene_dist("O", pts, time=0.0)
    assert dT[0] == pytest.approx(float(oracle.lib().oracle_menger(0, 0, 0)), abs=1e-6)
    assert dO[1] < 0 and dO[2] < 0  # inside sphere / cube
    assert dO[3] == pytest.approx(0.5, abs=1e-6)  # floor plane


def test_hash11_range(L):
    v = [L.oracle_hash11(float(i)) for i in range(32)]
    assert all(0.0 <= x < 1.0 for x in v)
    assert len(set(v)) > 28


def test_step_counts_and_exhaustion():
    # scene T, 1 step: each of the 2 marches makes exactly 1 call, plus the
    # normal (4), AO (4) and >= 1 shadow step
    img1, ev1 = oracle.render("T", 16, 16, max_steps=1)
    assert ev1.min() >= 2 + 4 + 4 + 1
    assert np.isfinite(img1).all()
    # step-exhausted castRayD returns the last SDF value as the hit distance
    # (common.frag:900): the image changes with the cap
    img2, _ = oracle.render("O", 16, 16, max_steps=2)
    img3, _ = oracle.render("O", 16, 16, max_steps=128)
    assert np.abs(img2 - img3).max() > 1e-2


def test_row_subsets_equal_full_frame():
    full, ev = oracle.render("O", 24, 20)
    part, evp = oracle.render("O", 24, 20, row0=7, nrows=5)
    np.testing.assert_array_equal(part, full[7:12])
    rows, evr = oracle.render_rows("O", 24, 20, [3, 19, 0])
    np.testing.assert_array_equal(rows, full[[3, 19, 0]])
    np.testing.assert_array_equal(evr, ev[[3, 19, 0]])


def test_shadow_cap_only_shortens():
    _, ev0 = oracle.render("T", 32, 32, shadow_max_steps=0)
    _, ev1 = oracle.render("T", 32, 32, shadow_max_steps=8)
    assert ev1.sum() <= ev0.sum()


def test_sdbox_equals_componentwise_max(L):
    """The HIP path evaluates sdBox(p, vec3(1)) (common.frag:595-600) as
    max(|p|-1) without the sqrt: min(mc, length(max(di,0))) == mc exactly
    (the rounded length of a vector whose largest component is mc > 0 is >= mc).
    Checked bit for bit against the restatement on random points."""
    rng = np.random.default_rng(7)
    pts = np.concatenate([rng.uniform(-3, 3, (6000, 3)), rng.uniform(-1.2, 1.2, (6000, 3)),
                          rng.normal(0, 1e-3, (2000, 3)) + 1.0]).astype(np.float32)
    for x, y, z in pts:
        ref = L.oracle_sdbox(x, y, z, 1.0, 1.0, 1.0)
        mc = max(np.float32(abs(x)) - np.float32(1), np.float32(abs(y)) - np.float32(1),
                 np.float32(abs(z)) - np.float32(1))
        assert np.float32(ref) == np.float32(mc), (x, y, z, ref, mc)


def test_oracle_under_address_and_undefined_behaviour_sanitizers():
    """oracle/selftest.c over every scene, the diagnostic channels, FXAA and
    bloom at ragged sizes, built with -fsanitize=address,undefined (SURVEY.md
    section 5: sanitizers on the CPU restatement)."""
    import subprocess
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    b = subprocess.run(["make", "-C", here, "sanitize"], capture_output=True, text=True)
    if b.returncode != 0 and "sanitize" in b.stderr and "cannot find" in b.stderr:
        pytest.skip("no sanitizer runtime")
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, OMP_NUM_THREADS="4", ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(here, "build", "selftest_asan")], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "selftest ok" in r.stdout


def test_render_pixels_equals_rows():
    """oracle.render_pixels (column-strided full-size samples) renders a pixel
    exactly as render_rows does: colour and ray-step count."""
    import numpy as np

    from raymarching_amd import POSES
    kw = {k: POSES["P2"][k] for k in ("pos", "mouse", "time")}
    rows = np.array([7, 100], np.int32)
    o, ev = oracle.render_rows("O", 320, 200, rows, max_steps=128, **kw)
    xs = np.tile(np.arange(320), 2)
    ys = np.repeat(rows, 320)
    o2, ev2 = oracle.render_pixels("O", 320, 200, xs, ys, max_steps=128, **kw)
    assert np.array_equal(o.reshape(-1, 4), o2)
    assert np.array_equal(ev.ravel(), ev2)
    with pytest.raises(ValueError):
        oracle.render_pixels("O", 320, 200, [320], [0])


@pytest.mark.parametrize("scene,steps", [("T", 256), ("O", 512)])
def test_shadow_settle_rule_never_changes_a_result(scene, steps):
    """once the settle rule holds on a soft-shadow march, no
    later step of the reference's march lowers res or occludes -- checked on
    every step of every march of frames at all poses (the oracle runs the
    reference's full loop and tests the rule beside it)."""
    from raymarching_amd import POSES
    tot = dict(steps=0, after=0, violations=0, refl_after=0, back_steps=0)
    for pose in POSES.values():
        r = oracle.shadow_settle(scene, 96, 64, pos=pose["pos"], mouse=pose["mouse"], time=pose["time"],
                                 max_steps=steps)
        for k in tot:
            tot[k] += r[k]
    assert tot["violations"] == 0, tot
    # (`after` counts the marches of points that face the light; the others'
    # steps are back_steps, which the kernels skip whole)
    assert tot["after"] > 0.02 * tot["steps"], tot
    assert tot["after"] + tot["back_steps"] > 0.1 * tot["steps"], tot
