"""oracle -- TEST INFRASTRUCTURE ONLY.

ctypes binding for the CPU restatement in ``oracle/rm_oracle.c`` of the
reference's per-pixel ray-march pass (common.frag + output_shader.frag +
template.frag of cahekp/Raymarching).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import this
package, and only as the checker / CPU baseline: the product path
(``raymarching_amd``) never touches it.

Pinning: see DESIGN.md "Oracle" -- the restatement is checked against golden
images that SwiftShader rendered from the reference GLSL in the build
container (``tests/golden/``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

SCENES = {"S0": 0, "T": 1, "O": 2, "OG": 3}


class OracleUniforms(ctypes.Structure):
    """Mirror of ``oracle_uniforms`` (rm_oracle.c)."""

    _fields_ = [
        ("res_x", ctypes.c_float), ("res_y", ctypes.c_float),
        ("mouse_x", ctypes.c_float), ("mouse_y", ctypes.c_float),
        ("pos_x", ctypes.c_float), ("pos_y", ctypes.c_float), ("pos_z", ctypes.c_float),
        ("time", ctypes.c_float),
        ("max_steps", ctypes.c_int32),
        ("shadow_max_steps", ctypes.c_int32),
        ("jit_x", ctypes.c_float), ("jit_y", ctypes.c_float),
    ]


_LIBS: dict[str, ctypes.CDLL] = {}


def build(quiet: bool = True) -> None:
    """Compile oracle/liboracle*.so with the committed Makefile."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


def lib(fast: bool = False) -> ctypes.CDLL:
    name = "liboracle_fast.so" if fast else "liboracle.so"
    if name not in _LIBS:
        path = os.path.join(HERE, name)
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        f32p = ctypes.POINTER(ctypes.c_float)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        i32p = ctypes.POINTER(ctypes.c_int32)
        up = ctypes.POINTER(OracleUniforms)
        L.oracle_render.argtypes = [ctypes.c_int, up, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, f32p, u32p]
        L.oracle_render.restype = ctypes.c_int
        L.oracle_render_rows.argtypes = [ctypes.c_int, up, ctypes.c_int, ctypes.c_int, i32p,
                                         ctypes.c_int, f32p, u32p]
        L.oracle_render_rows.restype = ctypes.c_int
        L.oracle_render_pixels.argtypes = [ctypes.c_int, up, ctypes.c_int, ctypes.c_int, i32p, ctypes.c_int, f32p,
                                           u32p]
        L.oracle_render_pixels.restype = ctypes.c_int
        for fn in ("oracle_scene_dist", "oracle_normal"):
            getattr(L, fn).argtypes = [ctypes.c_int, up, f32p, ctypes.c_int, f32p]
            getattr(L, fn).restype = ctypes.c_int
        for fn, n in (("oracle_glsl_mod", 2), ("oracle_glsl_smoothstep", 3), ("oracle_sdbox", 6),
                      ("oracle_sphere", 7), ("oracle_cube", 7), ("oracle_menger", 3),
                      ("oracle_smin_cubic", 3), ("oracle_hash11", 1)):
            getattr(L, fn).argtypes = [ctypes.c_float] * n
            getattr(L, fn).restype = ctypes.c_float
        L.oracle_fxaa.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_fxaa.restype = ctypes.c_int
        L.oracle_bloom.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_bloom.restype = ctypes.c_int
        L.oracle_mip_down.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_mip_down.restype = ctypes.c_int
        L.oracle_bloom_levels.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                                          ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.oracle_bloom_levels.restype = ctypes.c_int
        L.oracle_render_diag.argtypes = [ctypes.c_int, up, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, f32p, f32p]
        L.oracle_render_diag.restype = ctypes.c_int
        L.oracle_shadow_settle.argtypes = [ctypes.c_int, up, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_void_p]
        L.oracle_shadow_settle.restype = ctypes.c_int
        L.oracle_num_threads.argtypes = []
        L.oracle_num_threads.restype = ctypes.c_int
        _LIBS[name] = L
    return _LIBS[name]


def uniforms(W, H, pos=(2.0, 3.0, 3.0), mouse=(0.0, 0.0), time=0.0, max_steps=128,
             shadow_max_steps=0, res=None, jitter=(0.0, 0.0)) -> OracleUniforms:
    rx, ry = (W, H) if res is None else res
    return OracleUniforms(float(rx), float(ry), float(mouse[0]), float(mouse[1]), float(pos[0]),
                          float(pos[1]), float(pos[2]), float(time), int(max_steps),
                          int(shadow_max_steps), float(jitter[0]), float(jitter[1]))


def seed_jitter(seed1):
    """The sub-pixel offset progressive accumulation renders with (rm.h
    rm_render_accumulate): fract(u_seed1) - 0.5 per axis, GLSL fract, in f32."""
    s = np.asarray(seed1, np.float32)
    return tuple(float(v) for v in (s - np.floor(s)) - np.float32(0.5))


def accumulate(prev, colour, part):
    """mix(u_sample, colour, u_sample_part) as the accumulating pass stores it:
    prev + (colour - prev) * part in f32 (each operation rounded, no FMA); part >= 1
    stores the colour.  RGB of float32 [..., 4] arrays; alpha = 1."""
    part = np.float32(part)
    if part >= 1.0:
        out = colour.astype(np.float32).copy()
    else:
        p = prev.astype(np.float32)
        out = (p + (colour.astype(np.float32) - p) * part).astype(np.float32)
    out[..., 3] = 1.0
    return out


def unpack_rgba8(words):
    """RGBA8 words -> float32 [..., 4] as the accumulating pass reads u_sample:
    b * RN(1/255)."""
    w = np.asarray(words).astype(np.uint32)
    k = np.float32(1.0) / np.float32(255.0)
    return np.stack([((w >> s) & 255).astype(np.float32) * k for s in (0, 8, 16, 24)], -1)


def pack_rgba8(rgba):
    """float32 [..., 4] -> RGBA8 words as the kernels pack them: clamp to [0, 1]
    (NaN -> 0), x * 255 rounded to nearest even."""
    c = np.nan_to_num(np.clip(rgba.astype(np.float32), 0.0, 1.0), nan=0.0)
    b = np.rint(c * np.float32(255.0)).astype(np.uint32)
    return (b[..., 0] | (b[..., 1] << 8) | (b[..., 2] << 16) | (b[..., 3] << 24)).astype(np.uint32)


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def render(scene: str, W: int, H: int, row0: int = 0, nrows: int | None = None, fast=False,
           **kw):
    """Render rows [row0,row0+nrows) -> (rgba f32 [nrows,W,4], evals u32 [nrows,W])."""
    nrows = H - row0 if nrows is None else nrows
    u = uniforms(W, H, **kw)
    out = np.zeros((nrows, W, 4), np.float32)
    ev = np.zeros((nrows, W), np.uint32)
    rc = lib(fast).oracle_render(SCENES[scene], ctypes.byref(u), W, H, row0, nrows,
                                 _p(out, ctypes.c_float), _p(ev, ctypes.c_uint32))
    if rc:
        raise ValueError(f"oracle_render failed rc={rc}")
    return out, ev


def render_rows(scene: str, W: int, H: int, rows, fast=False, **kw):
    rows = np.ascontiguousarray(rows, np.int32)
    u = uniforms(W, H, **kw)
    out = np.zeros((len(rows), W, 4), np.float32)
    ev = np.zeros((len(rows), W), np.uint32)
    rc = lib(fast).oracle_render_rows(SCENES[scene], ctypes.byref(u), W, H, _p(rows, ctypes.c_int32),
                                      len(rows), _p(out, ctypes.c_float), _p(ev, ctypes.c_uint32))
    if rc:
        raise ValueError(f"oracle_render_rows failed rc={rc}")
    return out, ev


def render_pixels(scene: str, W: int, H: int, xs, ys, fast=False, **kw):
    """Pixels (xs[i], ys[i]) of a W x H frame -> (rgba f32 [n, 4], evals u32 [n])."""
    xy = np.ascontiguousarray(np.stack([np.asarray(xs, np.int32).ravel(), np.asarray(ys, np.int32).ravel()], -1))
    n = len(xy)
    u = uniforms(W, H, **kw)
    out = np.zeros((n, 4), np.float32)
    ev = np.zeros(n, np.uint32)
    rc = lib(fast).oracle_render_pixels(SCENES[scene], ctypes.byref(u), W, H, _p(xy, ctypes.c_int32), n,
                                        _p(out, ctypes.c_float), _p(ev, ctypes.c_uint32))
    if rc:
        raise ValueError(f"oracle_render_pixels failed rc={rc}")
    return out, ev


def shadow_settle(scene: str, W: int, H: int, every: int = 1, **kw):
    """Analysis aid: the soft-shadow settle rule tested on
    every `every`-th step of the reference's shadow marches of a W x H frame
    (the kernels test scene O every 8th step, scene T every step) ->
    dict(marches, steps, after, settled, violations); `violations` counts
    changes of res (or occlusions) after a march settled, and scene-T
    reflection marches past depth 3 whose clamp factor is not 1; `refl_after`
    counts scene T's reflection-march steps begun at depth >= 3, `back_steps`
    the shadow-march steps of points facing away from the light (`after`
    counts the other marches' steps only)."""
    u = uniforms(W, H, **kw)
    out = np.zeros(7, np.uint64)
    if lib().oracle_shadow_settle(SCENES[scene], ctypes.byref(u), W, H, 0, H, every, out.ctypes.data):
        raise ValueError("oracle_shadow_settle failed")
    return dict(zip(("marches", "steps", "after", "settled", "violations", "refl_after", "back_steps"),
                    (int(v) for v in out)))


N_DIAG = 7


def render_diag(scene: str, W: int, H: int, **kw):
    """Scene-O diagnostic channels (make_goldens.py diag_edit) -> (diag f32
    [H, W, N_DIAG, 4], rgba f32 [H, W, 4])."""
    u = uniforms(W, H, **kw)
    diag = np.zeros((H, W, N_DIAG, 4), np.float32)
    out = np.zeros((H, W, 4), np.float32)
    rc = lib().oracle_render_diag(SCENES[scene], ctypes.byref(u), W, H, 0, H, _p(diag, ctypes.c_float),
                                  _p(out, ctypes.c_float))
    if rc:
        raise ValueError(f"oracle_render_diag failed rc={rc}")
    return diag, out


def scene_dist(scene: str, pts, **kw):
    pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 3)
    out = np.zeros(len(pts), np.float32)
    u = uniforms(1, 1, **kw)
    lib().oracle_scene_dist(SCENES[scene], ctypes.byref(u), _p(pts, ctypes.c_float), len(pts),
                            _p(out, ctypes.c_float))
    return out


def normal(scene: str, pts, **kw):
    pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 3)
    out = np.zeros((len(pts), 3), np.float32)
    u = uniforms(1, 1, **kw)
    lib().oracle_normal(SCENES[scene], ctypes.byref(u), _p(pts, ctypes.c_float), len(pts),
                        _p(out, ctypes.c_float))
    return out


def fxaa(img_u32):
    """post.frag FXAA over an [H, W] RGBA8 image -> (RGBA8 [H, W], float [H, W, 4])."""
    img = np.ascontiguousarray(img_u32, np.uint32)
    H, W = img.shape
    out = np.zeros((H, W), np.uint32)
    outf = np.zeros((H, W, 4), np.float32)
    rc = lib().oracle_fxaa(W, H, img.ctypes.data, out.ctypes.data, outf.ctypes.data)
    if rc:
        raise ValueError("oracle_fxaa failed")
    return out, outf


def bloom_levels(W, H):
    """(lod, d1, d2) of bloom.frag's textureLod for a W x H image."""
    lod, d1, d2 = ctypes.c_float(), ctypes.c_int(), ctypes.c_int()
    lib().oracle_bloom_levels(int(W), int(H), ctypes.byref(lod), ctypes.byref(d1), ctypes.byref(d2))
    return lod.value, d1.value, d2.value


def mip_down(img_u32):
    """One glGenerateMipmap step: [h, w] RGBA8 -> [max(1, h/2), max(1, w/2)]."""
    img = np.ascontiguousarray(img_u32, np.uint32)
    h, w = img.shape
    out = np.zeros((max(1, h >> 1), max(1, w >> 1)), np.uint32)
    if lib().oracle_mip_down(w, h, img.ctypes.data, out.ctypes.data):
        raise ValueError("oracle_mip_down failed")
    return out


def bloom(img_u32):
    """bloom.frag over an [H, W] RGBA8 image -> (RGBA8 [H, W], [levels 1..d2])."""
    img = np.ascontiguousarray(img_u32, np.uint32)
    H, W = img.shape
    _, _, d2 = bloom_levels(W, H)
    dims, w, h = [], W, H
    for _ in range(d2):
        w, h = max(1, w >> 1), max(1, h >> 1)
        dims.append((h, w))
    mips = np.zeros(max(1, sum(a * b for a, b in dims)), np.uint32)
    out = np.zeros((H, W), np.uint32)
    if lib().oracle_bloom(W, H, img.ctypes.data, out.ctypes.data, mips.ctypes.data):
        raise ValueError("oracle_bloom failed")
    levels, off = [], 0
    for h, w in dims:
        levels.append(mips[off:off + h * w].reshape(h, w))
        off += h * w
    return out, levels
