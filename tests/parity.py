"""Image comparison helpers and the tolerance policy of the parity tests.

The oracle (oracle/rm_oracle.c) is pinned against SwiftShader renders of the
reference GLSL (tests/golden).  GLSL leaves transcendental and division
precision to the implementation (parity is unpinned at the ulp level), and
sphere tracing amplifies ulp differences at silhouettes, step-exhausted rays
and in the ``fract(x * 443.897)`` hashes of output_shader.frag:54-66, so
images are compared per pixel with a tolerance on the channel difference and
a bound on the fraction of pixels outside it (DESIGN.md "Parity policy").
"""
import numpy as np


def diff_stats(a, b):
    a = np.asarray(a, np.float64)[..., :3]
    b = np.asarray(b, np.float64)[..., :3]
    d = np.abs(a - b)
    both_nan = np.isnan(a) & np.isnan(b)
    d = np.where(both_nan, 0.0, d)
    d = np.where(np.isnan(d), 1.0, d).max(-1)
    return dict(max=float(d.max()), mean=float(d.mean()), f2e3=float(np.mean(d <= 2e-3)),
                f1e2=float(np.mean(d <= 1e-2)), f5e2=float(np.mean(d <= 5e-2)))


# Per scene: minimal fraction of pixels within 2e-3 / within 1e-2, max mean |d|.
POLICY = {
    "S0": dict(f2e3=0.999, f1e2=1.0, mean=1e-4),
    "T": dict(f2e3=0.99, f1e2=0.995, mean=1e-3),
    # SURVEY.md 8(c)'s policy (99 % within 2e-3, mean <= 1e-3); the residual
    # of round 1 was attributed and removed
    "O": dict(f2e3=0.99, f1e2=0.999, mean=1e-3),
    "OG": dict(f2e3=0.99, f1e2=0.999, mean=1e-3),
    # scene plugins (raymarching_amd/scenes): the mandelbulb's pow/atan/acos
    # orbit is the most ulp-sensitive SDF of the library
    "MB": dict(f2e3=0.9, f1e2=0.97, mean=5e-3),
    # showcase.hip: its library calls (transformTR, opSmoothUnion, sminCubic,
    # pMod1, ...) round as the reference GLSL's since mix() is evaluated in the
    # fixture renderer's form (measured: 100 %, max 7.7e-7)
    "SC": dict(f2e3=0.99, f1e2=0.999, mean=1e-3),
}


# Full-size frames (C2/C3/C5, tests/test_gpu_parity.py full_size_parity): the
# levels the HIP path achieves there (round 4: C3 f2e3 0.999997, C2 >= 0.99998,
# C5 1.0), ratcheted so that a regression moving 0.01 % of a frame (1.7 k
# pixels at 4096^2) fails; the small golden frames keep POLICY above.
FULL_SIZE_POLICY = {
    "T": dict(f2e3=0.9999, f1e2=0.99995, mean=1e-4),
    "O": dict(f2e3=0.9999, f1e2=0.99995, mean=1e-4),
}
# per-pixel ray-step maps at full size: fraction of pixels whose sceneSDF call
# count equals the oracle's (achieved: T 0.9985-0.9999, O 1.00000)
FULL_SIZE_STEP_MAP = {"T": 0.998, "O": 0.9999}


def assert_parity(scene, a, b, policy=None, label=""):
    p = dict(POLICY[scene] if policy is None else policy)
    s = diff_stats(a, b)
    msg = f"{label} {scene}: {s} vs policy {p}"
    assert s["f2e3"] >= p["f2e3"], msg
    assert s["f1e2"] >= p["f1e2"], msg
    assert s["mean"] <= p["mean"], msg
    return s
