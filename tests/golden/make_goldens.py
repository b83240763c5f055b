#!/usr/bin/env python3
"""Generate golden images by running the REFERENCE GLSL itself (test data only).

Runs in the build container, never on the GPU box: it reads the reference
shaders from /root/reference, inlines ``#include`` exactly as
``ShaderLoader::preprocess`` does (source/shader_loader.cpp:22-81), applies the
mechanical GLSL-1.30 -> GLSL-ES-3.00 rewrites of SURVEY.md Appendix A (no
semantic change; the ``template.frag`` repair that defines scene T is the one
semantic edit, also Appendix A), compiles the result with the SwiftShader
GLES3 implementation bundled in the ``kaleido`` wheel, renders full-screen
passes into an RGBA32F FBO and stores the pixels.  The adapted shader text
lives only in memory; only the rendered numbers are committed
(``tests/golden/*.npz``).

Each fixture holds:
  rgba   float32 [H,W,4]   pre-quantisation ``gl_FragColor`` (row 0 = tc.y 0.5/H)
  evals  int32   [H,W]     sceneSDF calls per pixel, counting as the build
                           does: the dead ``nr`` normal of getColorReflect
                           (common.frag:995) and phongContribForLight's repeat
                           of the caller's normal (common.frag:733) excluded.
  meta   json string       scene, W, H, pose, max_steps

Usage: python tests/golden/make_goldens.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import re
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)
from raymarching_amd.poses import POSES, S0_POSE  # noqa: E402

SS = "/usr/local/lib/python3.10/dist-packages/kaleido/executable/bin/swiftshader/"

# ----------------------------------------------------------- shader source


def preprocess(path: str, root: str) -> str:
    """Same semantics as ShaderLoader::preprocess: an ``#include`` not preceded
    by ``//`` on its line pulls in the named file (no include guards)."""
    out = []
    with open(path) as f:
        for line in f.read().split("\n"):
            k = line.find("#include")
            if k != -1 and (k == 0 or line.rfind("//", 0, k) == -1):
                m = re.search(r'["<]([^">]*)[">]', line[k + 8:])
                out.append(preprocess(os.path.join(root, m.group(1)), root))
                continue
            out.append(line)
    return "\n".join(out)


def must_sub(pat, rep, s, count=0, regex=False):
    new = re.sub(pat, rep, s, count=count) if regex else s.replace(pat, rep) if count == 0 else s.replace(pat, rep, count)
    if new == s:
        raise RuntimeError(f"rewrite did not apply: {pat!r}")
    return new


def es3_rewrite(src: str) -> str:
    """SURVEY Appendix A mechanical rewrites (GLSL 1.30 leniencies -> ES 3.00)."""
    s = src
    s = re.sub(r"^\s*#version.*$", "", s, flags=re.M)
    s = must_sub("const float ZFAR = 50;", "const float ZFAR = 50.0;", s)
    # default arguments (the reference call sites pass every argument)
    s = must_sub("float k = 32)", "float k)", s)
    s = must_sub("in float h = 0.1)", "in float h)", s)
    s = must_sub("float maxt, float k = 2)", "float maxt, float k)", s)
    s = must_sub("in vec3 be = vec3(2.0), in vec3 bi = vec3(2.0))", "in vec3 be, in vec3 bi)", s)
    s = must_sub("float value = 0.9)", "float value)", s)
    s = must_sub("float value = 0.85)", "float value)", s)
    s = must_sub("float amount = 0.1)", "float amount)", s)
    # implicit int -> float
    s = must_sub(r"\b1/scale", "1.0/scale", s, regex=True)
    s = must_sub("length(max(q, 0)) + min(max(q.x, max(q.y, q.z)), 0)",
                 "length(max(q, 0.0)) + min(max(q.x, max(q.y, q.z)), 0.0)", s)
    s = must_sub("float s = (p<0)?-1:1;", "float s = (p<0.0)?-1.0:1.0;", s)
    s = must_sub("if (t < 0) {", "if (t < 0.0) {", s)
    s = must_sub("(2*t)*planeNormal", "(2.0*t)*planeNormal", s)
    s = must_sub("return (t<0)?-1:1;", "return (t<0.0)?-1.0:1.0;", s)
    s = must_sub("(1 - a) * d2", "(1.0 - a) * d2", s)
    s = must_sub("const float _AOSteps = 4;", "const int _AOSteps = 4;", s)
    s = must_sub("float sum    = 0;", "float sum    = 0.0;", s)
    s = must_sub("float maxSum = 0;", "float maxSum = 0.0;", s)
    s = must_sub("normal * (i+1) * _AOStepSize", "normal * float(i+1) * _AOStepSize", s)
    s = must_sub("1. / pow(2., i) * sceneSDF(p).dist", "1. / pow(2., float(i)) * sceneSDF(p).dist", s)
    s = must_sub("1. / pow(2., i) * (i+1) * _AOStepSize", "1. / pow(2., float(i)) * float(i+1) * _AOStepSize", s)
    # step counting (fixture-only instrumentation): skip the dead nr normal
    # and phong's repeat of the caller's normal, as the build does
    s = must_sub("vec3 N = getNormalFast(p);", "g_cnt_off++; vec3 N = getNormalFast(p); g_cnt_off--;", s)
    s = must_sub("vec3 nr = getNormalFast(pr);\n    \n\t// return simple depth texture",
                 "g_cnt_off++; vec3 nr = getNormalFast(pr); g_cnt_off--;\n    \n\t// return simple depth texture", s)
    return s


HEADER = """#version 300 es
precision highp float;
precision highp int;
in vec2 v_uv;
out vec4 o_col;
int g_evals = 0;
int g_cnt_off = 0;
"""


def count_hook(s: str, sig: str) -> str:
    """Insert the eval counter at the top of the scene's sceneSDF body."""
    k = s.index(sig)
    k = s.index("{", k) + 1
    return s[:k] + "\n\tif (g_cnt_off == 0) g_evals++;" + s[k:]


# gl_TexCoord[0].xy of the ray-march pass: the exact pixel-centre coordinate
# ((x + .5)/W, (y + .5)/H), row 0 first.  A rasterizer interpolates the
# varying to within an ulp of it (SwiftShader's v_uv is 1 ulp off on 1/3 of
# the columns of a 96-wide target); the fixtures feed the
# exact value, which is what the oracle and the HIP path compute.
EXACT_TC = "((vec2(floor(gl_FragCoord.x), u_resolution.y - 1.0 - floor(gl_FragCoord.y)) + 0.5) / u_resolution)"


def main_rewrite(s: str) -> str:
    s = s.replace("gl_TexCoord[0].xy", EXACT_TC)
    head, sep, tail = s.rpartition(f"col = vignette(col, {EXACT_TC});")
    if not sep:
        raise RuntimeError("vignette call not found")
    s = head + f"col = vignette(col, {EXACT_TC}, 0.1);" + tail
    # only the live main() (the last one; common.frag:1124-1188 holds commented-out ones)
    head, sep, tail = s.rpartition("gl_FragColor = vec4(col, 1.0);")
    if not sep:
        raise RuntimeError("main() output not found")
    return (head + "#ifdef COUNT_MODE\n\to_col = vec4(float(g_evals), 0.0, 0.0, 1.0);\n#else\n"
            "\to_col = vec4(col, 1.0);\n#endif" + tail)


def scene_O(ref: str, edit=None) -> str:
    s = preprocess(os.path.join(ref, "output_shader.frag"), ref)
    if edit is not None:
        s = edit(s)
    s = es3_rewrite(s)
    if edit is None or "u_time * 2, 0" in s:
        s = must_sub("vec3(180, u_time * 2, 0)", "vec3(180, u_time * 2.0, 0)", s)
    s = must_sub("sd.mat.transparency > 0 ?", "sd.mat.transparency > 0.0 ?", s)
    s = must_sub("if (sd.mat.reflectivity > 0)", "if (sd.mat.reflectivity > 0.0)", s)
    s = must_sub("if (sd.mat.transparency > 0)", "if (sd.mat.transparency > 0.0)", s)
    s = must_sub("float reflectivity = 0.0)", "float reflectivity)", s)  # output_shader.frag:246
    s = count_hook(s, "SdResult sceneSDF(vec3 p)\n{")
    return HEADER + main_rewrite(s)


# Diagnostic channels (DIAG_* fixtures): intermediate values of scene O's
# render() per pixel, recorded from the reference GLSL so that a parity
# residual can be attributed term by term.  Seven vec4:
#   0 primary hit: normal n, castRayD dist      1 primary light(): thickness, sha, occ, ind
#   2 primary light() colour, fresnel factor     3 reflection hit: normal, dist (-1: miss)
#   4 reflection light(): thickness, sha, occ, ind
#   5 reflection colour (light() or background)  6 render() colour (pre-tonemap)
# Unset channels hold -9.
N_DIAG = 7
DIAG_HEADER = "vec4 g_d[7] = vec4[7](vec4(-9.0), vec4(-9.0), vec4(-9.0), vec4(-9.0), vec4(-9.0), vec4(-9.0), vec4(-9.0));\n" \
              "int g_lvl = 0;\n"


def diag_edit(s: str) -> str:
    """Record the diagnostic channels in output_shader.frag's render()/light()/
    renderReflection() (reference text; lines output_shader.frag:127-176,
    246-262, 348-385).  Values only are copied out; no arithmetic changes."""
    s = must_sub("\t\tvec3 n = getNormalFast(p);\n\t\t\n\t\t// light the surface",
                 "\t\tvec3 n = getNormalFast(p);\n\t\tg_d[0] = vec4(n, sd.dist);\n\t\t\n\t\t// light the surface", s, count=1)
    s = must_sub("\t\tvec3 n = getNormalFast(p);\n\t\t\n        return light(sd.mat, ro, rd, p, n);",
                 "\t\tvec3 n = getNormalFast(p);\n\t\tg_d[3] = vec4(n, sd.dist);\n\t\t\n"
                 "        vec3 lc_ = light(sd.mat, ro, rd, p, n); g_d[5] = vec4(lc_, 0.0); return lc_;", s, count=1)
    s = must_sub("\telse // render background (for example: skybox or gradient)\n\t{\n\t\treturn background(ro, rd);\n\t}\t\n}",
                 "\telse // render background (for example: skybox or gradient)\n\t{\n"
                 "\t\tg_d[3] = vec4(0.0, 0.0, 0.0, -1.0); vec3 bc_ = background(ro, rd); g_d[5] = vec4(bc_, 0.0); return bc_;\n\t}\t\n}",
                 s, count=1)
    s = must_sub("\tfloat thickness = CalculateThickness(p, n);\n",
                 "\tfloat thickness = CalculateThickness(p, n);\n"
                 "\tif (g_lvl == 0) g_d[1] = vec4(thickness, sha, occ, ind); else g_d[4] = vec4(thickness, sha, occ, ind);\n", s)
    s = must_sub("\t\tif (sd.mat.reflectivity > 0)\n\t\t{",
                 "\t\tg_d[2] = vec4(color, reflect_factor); g_lvl = 1;\n\t\tif (sd.mat.reflectivity > 0)\n\t\t{", s, count=1)
    s = must_sub("        return color;\n\t}\n\telse // render background",
                 "        g_d[6] = vec4(color, 0.0); return color;\n\t}\n\telse // render background", s, count=1)
    return s


def scene_O_diag(ref: str) -> str:
    s = scene_O(ref, diag_edit)
    s = must_sub("int g_cnt_off = 0;\n", "int g_cnt_off = 0;\n" + DIAG_HEADER, s, count=1)
    return must_sub("#ifdef COUNT_MODE\n", "#ifdef DIAG_K\n\to_col = g_d[DIAG_K];\n#elif defined(COUNT_MODE)\n", s, count=1)


def scene_OG(ref: str) -> str:
    """output_shader.frag with its blue material made transparent (0.9 in
    place of 0.0 at output_shader.frag:14): the sphere and the cube then drive
    renderRefraction (:298-343) and castRayDI (common.frag:903-925), which the
    reference scene never reaches.  The build's test scene "OG"."""
    def edit(s):
        s = must_sub("vec3(0.02, 0.02, 0.04), 32.0, 0.0, 0.0, vec3(2.0, 2.0, 0.75) * 0.2",
                     "vec3(0.02, 0.02, 0.04), 32.0, 0.0, 0.9, vec3(2.0, 2.0, 0.75) * 0.2", s, count=1)
        return refraction_loop_flags(s)
    return scene_O(ref, edit)


def refraction_loop_flags(s: str) -> str:
    """renderRefraction's two `break`s (output_shader.frag:320,332) as a done
    flag that guards the rest of the body and ends the loop: the same
    control flow.  SwiftShader (the fixture renderer) executes the straight
    sceneSDF calls after a `break` of its unrolled loop for the exited lane
    (getNormalFast and ambientOcclusionReal: +8 counted calls on every
    refracting pixel, measured); the colours were unaffected.  Fixture
    bookkeeping only, the arithmetic is untouched."""
    s = must_sub("\tfor (int i = 0; i < MAX_REFRACTIONS; i++)\n\t{\n\t\tSdResult sd;",
                 "\tbool done_ = false;\n\tfor (int i = 0; i < MAX_REFRACTIONS && !done_; i++)\n\t{\n\t\tSdResult sd;", s,
                 count=1)
    s = must_sub("\t\t\t\tcolor += background(ro, rd);\n\t\t\tbreak;\n\t\t}\n",
                 "\t\t\t\tcolor += background(ro, rd);\n\t\t\tdone_ = true;\n\t\t}\n\t\tif (!done_) {\n", s, count=1)
    s = must_sub("\t\tif (invert > 0.0)\n\t\t\tbreak;\n",
                 "\t\tif (invert > 0.0)\n\t\t\tdone_ = true;\n\t\tif (!done_) {\n", s, count=1)
    return must_sub("\t\tinvert = tif ? invert : invert * -1.0;\n\t}\n",
                    "\t\tinvert = tif ? invert : invert * -1.0;\n\t\t}}\n\t}\n", s, count=1)


def scene_MB(ref: str) -> str:
    """output_shader.frag with the mandelbulb line it keeps commented out
    (output_shader.frag:41) live in place of the Menger sponge (:42) -- the
    scene raymarching_amd/scenes/mandelbulb.hip restates as a plugin."""
    def edit(s):
        s = must_sub("\t//SdResult dist0 = SdResult(mandelbulb(", "\tSdResult dist0 = SdResult(mandelbulb(", s, count=1)
        return must_sub("\tSdResult dist0 = SdResult(mengersponge(", "\t//SdResult dist0 = SdResult(mengersponge(", s,
                        count=1)
    return scene_O(ref, edit)


def scene_SC(ref: str) -> str:
    """output_shader.frag with its sceneSDF replaced by the text of the
    example plugin raymarching_amd/scenes/showcase.hip (written in the
    GLSL subset both accept)."""
    with open(os.path.join(os.path.dirname(os.path.dirname(HERE)), "raymarching_amd", "scenes", "showcase.hip")) as f:
        scene = f.read()

    def edit(s):
        sig = "SdResult sceneSDF(vec3 p)\n{"
        a = s.index(sig)
        b = s.index("\n}\n", a) + 3
        return s[:a] + scene + s[b:]
    return scene_O(ref, edit)


def lib_kat(ref: str) -> str:
    """common.frag with the known-answer cases of lib_kat_cases.py: pixel
    (x=i, y=fn) holds case fn at kat_point(i); POINTS_MODE writes the point."""
    from lib_kat_cases import PRELUDE, kat_function
    s = "#define ALLOW_MATERIAL_BLENDING\n#include \"common.frag\"\n" + PRELUDE + kat_function() + """
SdResult sceneSDF(vec3 p)
{
	return r1(length(p) - 1.0);
}
void main()
{
	int i = int(gl_FragCoord.x);
	int fn = int(gl_FragCoord.y);
	vec3 p = kat_point(i);
	SdResult r = kat(fn, p);
#ifdef POINTS_MODE
	o_col = vec4(p, r.dist);
#else
	o_col = vec4(r.dist, r.mat.diffuse);
#endif
}
"""
    s = _preprocess_text(s, ref)
    s = es3_rewrite(s)
    return HEADER + s


def lib_kat_materials(ref: str) -> str:
    """As lib_kat, writing the material of the case's SdResult instead:
    pass k (0..3) writes floats 4k..4k+3 of the 16-float Material record
    (diffuse, specular, shininess, reflectivity, transparency, absorption,
    ior, emission -- rm_scene_eval's order)."""
    s = lib_kat(ref)
    return must_sub("\to_col = vec4(r.dist, r.mat.diffuse);",
                    "\tMaterial m = r.mat;\n"
                    "\tfloat f[16] = float[16](m.diffuse.x, m.diffuse.y, m.diffuse.z, m.specular.x, m.specular.y, "
                    "m.specular.z, m.shininess, m.reflectivity, m.transparency, m.absorption.x, m.absorption.y, "
                    "m.absorption.z, m.refraction_index, m.emission.x, m.emission.y, m.emission.z);\n"
                    "\to_col = vec4(f[4 * KPASS], f[4 * KPASS + 1], f[4 * KPASS + 2], f[4 * KPASS + 3]);", s)


def scene_T(ref: str) -> str:
    """template.frag repaired as SURVEY Appendix A defines scene T."""
    with open(os.path.join(ref, "template.frag")) as f:
        lines = f.read().split("\n")
    # delete template.frag:3-20 (re-definitions of Material / blendMaterial)
    body = "\n".join(lines[:2] + lines[20:])
    body = must_sub("32.0, 0.0);", "32.0, 0.0, 0.0, vec3(0), 1.0, vec3(0));", body)
    body = must_sub("64., 0.9);", "64., 0.9, 0.0, vec3(0), 1.0, vec3(0));", body)
    body = must_sub("128.0, 0.0);", "128.0, 0.0, 0.0, vec3(0), 1.0, vec3(0));", body)
    body = must_sub("return dist;", "return SdResult(dist, red);", body)
    tmp = "#define ALLOW_MATERIAL_BLENDING\n" + body
    s = _preprocess_text(tmp, ref)
    s = es3_rewrite(s)
    s = must_sub("vec3(180, u_time * 2, 0)", "vec3(180, u_time * 2.0, 0)", s)
    s = count_hook(s, "SdResult sceneSDF(in vec3 p)\n{")
    return HEADER + main_rewrite(s)


def scene_S0(ref: str) -> str:
    """Config 1 scene (defined by this build): the reference
    library with a one-sphere sceneSDF and a lambert render()."""
    s = "#define ALLOW_MATERIAL_BLENDING\n#include \"common.frag\"\n" + """
const Material red = Material(vec3(0.2, 0.02, 0.02), vec3(0.04, 0.02, 0.02), 32.0, 0.0, 0.0, vec3(0), 1.0, vec3(0));
SdResult sceneSDF(vec3 p)
{
	return SdResult(sphere(vec4(0.0, 1.0, -3.0, 1.0), p), red);
}
vec3 background(vec3 ro, vec3 rd)
{
	vec3 color = vec3(0);
	return applyScattering(color, ro, ro + rd * ZFAR, vec3(0.34, 0.435, 0.57), vec3(2.0), vec3(2.0));
}
vec3 render(in vec3 ro, in vec3 rd)
{
	SdResult sd = castRayD(ro, rd);
	if (sd.dist > 0.0)
	{
		vec3 p = ro + rd * sd.dist;
		vec3 n = getNormalFast(p);
		vec3 lightDir = normalize(vec3(20, 50, 0) - p);
		return sd.mat.diffuse * (0.1 + lambert(lightDir, n));
	}
	return background(ro, rd);
}
void main()
{
	vec2 uv = (gl_TexCoord[0].xy - 0.5) * u_resolution / u_resolution.y;
	vec3 rayOrigin = u_pos;
	vec3 rayDirection = normalize(vec3(uv.x, -uv.y, -1.0));
	rayDirection.yz *= rot(-u_mouse.y);
	rayDirection.xz *= rot(u_mouse.x);
	vec3 col = render(rayOrigin, rayDirection);
	col = tonemap(col);
	col = contrast(col);
	col = vignette(col, gl_TexCoord[0].xy);
	gl_FragColor = vec4(col, 1.0);
}
"""
    s = _preprocess_text(s, ref)
    s = es3_rewrite(s)
    s = count_hook(s, "SdResult sceneSDF(vec3 p)\n{")
    return HEADER + main_rewrite(s)


def _preprocess_text(text: str, root: str) -> str:
    out = []
    for line in text.split("\n"):
        k = line.find("#include")
        if k != -1 and (k == 0 or line.rfind("//", 0, k) == -1):
            m = re.search(r'["<]([^">]*)[">]', line[k + 8:])
            out.append(preprocess(os.path.join(root, m.group(1)), root))
            continue
        out.append(line)
    return "\n".join(out)


def set_max_steps(src: str, n: int) -> str:
    if n == 128:  # the reference's own value (common.frag:15)
        return src
    return must_sub("const int MAX_MARCHING_STEPS = 128;", f"const int MAX_MARCHING_STEPS = {n};", src)


# ------------------------------------------------------------- EGL / GLES3

VS = """#version 300 es
out vec2 v_uv;
void main() {
    vec2 p = vec2(float((gl_VertexID << 1) & 2), float(gl_VertexID & 2));
    v_uv = vec2(p.x, 1.0 - p.y);
    gl_Position = vec4(2.0 * p - 1.0, 0.0, 1.0);
}
"""


class GL:
    def __init__(self, W, H):
        self.egl = egl = ctypes.CDLL(SS + "libEGL.so")
        self.gl = gl = ctypes.CDLL(SS + "libGLESv2.so")
        vp = ctypes.c_void_p
        egl.eglGetDisplay.restype = vp
        egl.eglChooseConfig.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp), ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_int)]
        egl.eglCreatePbufferSurface.restype = vp
        egl.eglCreatePbufferSurface.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_int)]
        egl.eglCreateContext.restype = vp
        egl.eglCreateContext.argtypes = [vp, vp, vp, ctypes.POINTER(ctypes.c_int)]
        egl.eglMakeCurrent.argtypes = [vp, vp, vp, vp]
        egl.eglInitialize.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        dpy = egl.eglGetDisplay(vp(0))
        a, b = ctypes.c_int(), ctypes.c_int()
        assert egl.eglInitialize(vp(dpy), ctypes.byref(a), ctypes.byref(b))
        EGL_NONE = 0x3038
        attrs = (ctypes.c_int * 15)(0x3033, 0x0001, 0x3040, 0x0040, 0x3024, 8, 0x3023, 8, 0x3022, 8, 0x3021, 8,
                                    EGL_NONE, 0, 0)
        cfg = vp()
        n = ctypes.c_int()
        assert egl.eglChooseConfig(vp(dpy), attrs, ctypes.byref(cfg), 1, ctypes.byref(n)) and n.value > 0
        sattr = (ctypes.c_int * 5)(0x3057, W, 0x3056, H, EGL_NONE)
        surf = egl.eglCreatePbufferSurface(vp(dpy), cfg, sattr)
        egl.eglBindAPI(0x30A0)
        cattr = (ctypes.c_int * 3)(0x3098, 3, EGL_NONE)
        ctx = egl.eglCreateContext(vp(dpy), cfg, vp(0), cattr)
        assert ctx, "eglCreateContext failed"
        assert egl.eglMakeCurrent(vp(dpy), vp(surf), vp(surf), vp(ctx))
        gl.glGetString.restype = ctypes.c_char_p
        self.renderer = gl.glGetString(0x1F01).decode()
        self.version = gl.glGetString(0x1F02).decode()
        self.W, self.H = W, H
        u = ctypes.c_uint()
        gl.glGenVertexArrays(1, ctypes.byref(u))
        gl.glBindVertexArray(u)
        tex, fbo = ctypes.c_uint(), ctypes.c_uint()
        gl.glGenTextures(1, ctypes.byref(tex))
        gl.glBindTexture(0x0DE1, tex)
        gl.glTexStorage2D(0x0DE1, 1, 0x8814, W, H)  # GL_RGBA32F
        gl.glGenFramebuffers(1, ctypes.byref(fbo))
        gl.glBindFramebuffer(0x8D40, fbo)
        gl.glFramebufferTexture2D(0x8D40, 0x8CE0, 0x0DE1, tex, 0)
        st = gl.glCheckFramebufferStatus(0x8D40)
        assert st == 0x8CD5, hex(st)
        gl.glViewport(0, 0, W, H)
        gl.glGetUniformLocation.argtypes = [ctypes.c_uint, ctypes.c_char_p]
        for fn in ("glUniform1f", "glUniform2f", "glUniform3f"):
            getattr(gl, fn).argtypes = [ctypes.c_int] + [ctypes.c_float] * int(fn[-2])

    def shader(self, kind, src):
        gl = self.gl
        sh = gl.glCreateShader(kind)
        b = src.encode()
        arr = (ctypes.c_char_p * 1)(b)
        ln = (ctypes.c_int * 1)(len(b))
        gl.glShaderSource(sh, 1, arr, ln)
        gl.glCompileShader(sh)
        ok = ctypes.c_int()
        gl.glGetShaderiv(sh, 0x8B81, ctypes.byref(ok))
        if not ok.value:
            buf = ctypes.create_string_buffer(65536)
            gl.glGetShaderInfoLog(sh, 65536, None, buf)
            raise RuntimeError("compile failed:\n" + buf.value.decode())
        return sh

    def program(self, fs_src):
        gl = self.gl
        p = gl.glCreateProgram()
        gl.glAttachShader(p, self.shader(0x8B31, VS))
        gl.glAttachShader(p, self.shader(0x8B30, fs_src))
        gl.glLinkProgram(p)
        ok = ctypes.c_int()
        gl.glGetProgramiv(p, 0x8B82, ctypes.byref(ok))
        if not ok.value:
            buf = ctypes.create_string_buffer(65536)
            gl.glGetProgramInfoLog(p, 65536, None, buf)
            raise RuntimeError("link failed:\n" + buf.value.decode())
        return p

    def draw(self, prog, pose, res):
        gl = self.gl
        gl.glUseProgram(prog)

        def loc(n):
            return gl.glGetUniformLocation(prog, n.encode())
        gl.glUniform2f(loc("u_resolution"), float(res[0]), float(res[1]))
        gl.glUniform3f(loc("u_pos"), *[float(v) for v in pose["pos"]])
        gl.glUniform2f(loc("u_mouse"), *[float(v) for v in pose["mouse"]])
        gl.glUniform1f(loc("u_time"), float(pose["time"]))
        gl.glDrawArrays(0x0004, 0, 3)
        gl.glFinish()
        buf = np.zeros((self.H, self.W, 4), np.float32)
        gl.glReadPixels(0, 0, self.W, self.H, 0x1908, 0x1406, buf.ctypes.data_as(ctypes.c_void_p))
        err = gl.glGetError()
        assert err == 0, hex(err)
        return buf[::-1].copy()  # GL rows bottom-up -> row 0 = tc.y 0.5/H


    def post(self, prog, img_u32, res):
        """Run a post pass reading `img_u32` (H x W RGBA8 words, row 0 first)
        as u_main_tex with the sampler state of an sf::RenderTexture that was
        never setSmooth()ed or setRepeated(): NEAREST, CLAMP_TO_EDGE; render
        into an RGBA8 target and read the bytes back (row 0 = tc.y 0.5/H)."""
        gl = self.gl
        H, W = img_u32.shape
        src = ctypes.c_uint()
        gl.glGenTextures(1, ctypes.byref(src))
        gl.glActiveTexture(0x84C0)
        gl.glBindTexture(0x0DE1, src)
        for pname, val in ((0x2801, 0x2600), (0x2800, 0x2600), (0x2802, 0x812F), (0x2803, 0x812F)):
            gl.glTexParameteri(0x0DE1, pname, val)  # MIN/MAG NEAREST, WRAP_S/T CLAMP_TO_EDGE
        data = np.ascontiguousarray(img_u32, np.uint32)
        gl.glTexImage2D(0x0DE1, 0, 0x8058, W, H, 0, 0x1908, 0x1401, data.ctypes.data_as(ctypes.c_void_p))  # RGBA8
        dst, fbo = ctypes.c_uint(), ctypes.c_uint()
        gl.glGenTextures(1, ctypes.byref(dst))
        gl.glBindTexture(0x0DE1, dst)
        gl.glTexStorage2D(0x0DE1, 1, 0x8058, W, H)
        gl.glGenFramebuffers(1, ctypes.byref(fbo))
        gl.glBindFramebuffer(0x8D40, fbo)
        gl.glFramebufferTexture2D(0x8D40, 0x8CE0, 0x0DE1, dst, 0)
        assert gl.glCheckFramebufferStatus(0x8D40) == 0x8CD5
        gl.glBindTexture(0x0DE1, src)
        gl.glViewport(0, 0, W, H)
        gl.glUseProgram(prog)
        gl.glUniform2f(gl.glGetUniformLocation(prog, b"u_resolution"), float(res[0]), float(res[1]))
        gl.glUniform1i(gl.glGetUniformLocation(prog, b"u_main_tex"), 0)
        gl.glDrawArrays(0x0004, 0, 3)
        gl.glFinish()
        out = np.zeros((H, W), np.uint32)
        gl.glReadPixels(0, 0, W, H, 0x1908, 0x1401, out.ctypes.data_as(ctypes.c_void_p))
        assert gl.glGetError() == 0
        return out[::-1].copy()


    def bloom(self, prog, img_u32, res):
        """bloom.frag over `img_u32` as PostBloom::apply sees postTexture after
        setSmooth(true) + generateMipmap() (main.cpp:212-214): MIN
        LINEAR_MIPMAP_LINEAR, MAG LINEAR, CLAMP_TO_EDGE, the mip chain built by
        glGenerateMipmap.  Returns (output RGBA8 row 0 = tc.y 0.5/H, [mip levels
        1.. as stored, row 0 = t 0.5/h])."""
        gl = self.gl
        H, W = img_u32.shape
        src = ctypes.c_uint()
        gl.glGenTextures(1, ctypes.byref(src))
        gl.glActiveTexture(0x84C0)
        gl.glBindTexture(0x0DE1, src)
        for pname, val in ((0x2801, 0x2703), (0x2800, 0x2601), (0x2802, 0x812F), (0x2803, 0x812F)):
            gl.glTexParameteri(0x0DE1, pname, val)
        data = np.ascontiguousarray(img_u32, np.uint32)
        gl.glTexImage2D(0x0DE1, 0, 0x8058, W, H, 0, 0x1908, 0x1401, data.ctypes.data_as(ctypes.c_void_p))
        gl.glGenerateMipmap(0x0DE1)
        mips = []
        fbo = ctypes.c_uint()
        gl.glGenFramebuffers(1, ctypes.byref(fbo))
        gl.glBindFramebuffer(0x8D40, fbo)
        k = 1
        while True:
            w, h = max(1, W >> k), max(1, H >> k)
            gl.glFramebufferTexture2D(0x8D40, 0x8CE0, 0x0DE1, src, k)
            assert gl.glCheckFramebufferStatus(0x8D40) == 0x8CD5
            m = np.zeros((h, w), np.uint32)
            gl.glReadPixels(0, 0, w, h, 0x1908, 0x1401, m.ctypes.data_as(ctypes.c_void_p))
            mips.append(m)
            if w == 1 and h == 1:
                break
            k += 1
        dst = ctypes.c_uint()
        gl.glGenTextures(1, ctypes.byref(dst))
        gl.glBindTexture(0x0DE1, dst)
        gl.glTexStorage2D(0x0DE1, 1, 0x8058, W, H)
        gl.glFramebufferTexture2D(0x8D40, 0x8CE0, 0x0DE1, dst, 0)
        assert gl.glCheckFramebufferStatus(0x8D40) == 0x8CD5
        gl.glBindTexture(0x0DE1, src)
        gl.glViewport(0, 0, W, H)
        gl.glUseProgram(prog)
        gl.glUniform2f(gl.glGetUniformLocation(prog, b"u_resolution"), float(res[0]), float(res[1]))
        gl.glUniform1i(gl.glGetUniformLocation(prog, b"u_main_tex"), 0)
        gl.glDrawArrays(0x0004, 0, 3)
        gl.glFinish()
        out = np.zeros((H, W), np.uint32)
        gl.glReadPixels(0, 0, W, H, 0x1908, 0x1401, out.ctypes.data_as(ctypes.c_void_p))
        assert gl.glGetError() == 0
        return out[::-1].copy(), mips


def post_bloom(ref: str) -> str:
    """shaders/post/bloom.frag with the ES 3.00 header swap."""
    with open(os.path.join(ref, "shaders", "post", "bloom.frag")) as f:
        s = f.read()
    s = re.sub(r"^\s*#version.*$", "", s, flags=re.M)
    s = must_sub("gl_TexCoord[0]", "vec4(v_uv, 0.0, 0.0)", s)
    s = must_sub("gl_FragColor = vec4(color, 1.0);", "o_col = vec4(color, 1.0);", s)
    s = must_sub("vec2(x * iaspect, y)", "vec2(float(x) * iaspect, y)", s)  # implicit int -> float
    return ("#version 300 es\nprecision highp float;\nprecision highp int;\nprecision highp sampler2D;\n"
            "in vec2 v_uv;\nout vec4 o_col;\n" + s)


def bloom_inputs():
    """(name, H x W RGBA8) inputs: FXAA outputs of two ray-march goldens (the
    reference's bloom input is post.frag's output) and synthetic bright
    patterns at power-of-two and odd sizes."""
    out = []
    for nm in ("FXAA_T_64_P0", "FXAA_O_96x54_P2"):
        z = np.load(os.path.join(HERE, nm + ".npz"), allow_pickle=False)
        out.append(("BLOOM_" + nm[5:], z["output"]))
    rng = np.random.default_rng(20261016)
    for H, W in ((64, 128), (37, 61), (256, 256)):
        yy, xx = np.mgrid[0:H, 0:W]
        img = np.zeros((H, W, 4), np.float32)
        img[..., 3] = 1.0
        img[..., 0] = np.clip(1.2 - np.hypot(xx - W * 0.3, yy - H * 0.4) / (0.15 * H), 0, 1)   # a bright disc
        img[..., 1] = ((xx // 7 + yy // 5) % 2) * 0.9                                        # blocks
        img[..., 2] = rng.uniform(0, 1, (H, W))                                               # noise
        out.append((f"BLOOM_synthetic_{W}x{H}", unorm8(img)))
    return out


def post_fxaa(ref: str) -> str:
    """post.frag (FXAA main, post.frag:135-144) with the ES 3.00 header swap."""
    with open(os.path.join(ref, "post.frag")) as f:
        s = f.read()
    s = re.sub(r"^\s*#version.*$", "", s, flags=re.M)
    s = must_sub("gl_TexCoord[0]", "vec4(v_uv, 0.0, 0.0)", s)
    s = must_sub("gl_FragColor = color;", "o_col = color;", s)
    return ("#version 300 es\nprecision highp float;\nprecision highp int;\nprecision highp sampler2D;\n"
            "in vec2 v_uv;\nout vec4 o_col;\n" + s)


def unorm8(rgba):
    q = np.clip(np.rint(np.clip(np.nan_to_num(rgba, nan=0.0), 0.0, 1.0) * 255.0), 0, 255).astype(np.uint32)
    return q[..., 0] | (q[..., 1] << 8) | (q[..., 2] << 16) | (q[..., 3] << 24)


def fxaa_inputs():
    """(name, H x W RGBA8) inputs: two ray-march goldens and a synthetic edge pattern."""
    out = []
    for nm in ("T_64_P0", "O_96x54_P2"):
        z = np.load(os.path.join(HERE, nm + ".npz"), allow_pickle=False)
        out.append(("FXAA_" + nm, unorm8(z["rgba"])))
    rng = np.random.default_rng(20261015)
    H, W = 37, 61
    yy, xx = np.mgrid[0:H, 0:W]
    img = np.zeros((H, W, 4), np.float32)
    img[..., 3] = 1.0
    img[..., 0] = (xx * 0.7 + yy * 1.3 > 30).astype(np.float32)          # a slanted edge
    img[..., 1] = ((xx // 5 + yy // 4) % 2).astype(np.float32) * 0.8     # blocks
    img[..., 2] = rng.uniform(0, 1, (H, W)).astype(np.float32)           # noise
    out.append(("FXAA_synthetic_61x37", unorm8(img)))
    return out


# ------------------------------------------------------------- fixtures

FIXTURES = [
    # name, scene, W, H, pose, max_steps
    ("S0_64_P0", "S0", 64, 64, "S0", 64),
    ("T_64_P0", "T", 64, 64, "P0", 128),
    ("T_96x54_P1", "T", 96, 54, "P1", 128),
    ("T_64_P4_256", "T", 64, 64, "P4", 256),
    ("T_80x48_P7", "T", 80, 48, "P7", 128),
    ("O_64_P0", "O", 64, 64, "P0", 128),
    ("O_96x54_P2", "O", 96, 54, "P2", 128),
    ("O_64_P6", "O", 64, 64, "P6", 128),
    ("O_72x40_P3_512", "O", 72, 40, "P3", 512),
    # the refraction path (blue made transparent): scene OG
    ("OG_96x54_P1", "OG", 96, 54, "P1", 128),
    ("OG_64_P7", "OG", 64, 64, "P7", 128),
    ("OG_72x40_P3", "OG", 72, 40, "P3", 128),
    # scene plugins (raymarching_amd/scenes/*.hip) against the same reference text
    ("MB_64_P0", "MB", 64, 64, "P0", 128),
    ("MB_72x40_P3", "MB", 72, 40, "P3", 128),
    ("SC_64_P0", "SC", 64, 64, "P0", 128),
    ("SC_96x54_P5", "SC", 96, 54, "P5", 128),
]


DIAG_FIXTURES = [
    # name, W, H, pose, max_steps (scene O)
    ("DIAG_O_96x54_P2", 96, 54, "P2", 128),
    ("DIAG_O_64_P6", 64, 64, "P6", 128),
]
DIAG_DOC = ["primary normal.xyz, dist", "primary thickness, sha, occ, ind", "primary light colour.rgb, fresnel",
            "reflection normal.xyz, dist (-1 miss)", "reflection thickness, sha, occ, ind",
            "reflection colour.rgb", "render colour.rgb (pre-tonemap)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    builders = {"O": scene_O, "OG": scene_OG, "T": scene_T, "S0": scene_S0, "MB": scene_MB, "SC": scene_SC}
    for name, scene, W, H, pose_name, steps in FIXTURES:
        if args.only and args.only not in name:
            continue
        pose = S0_POSE if pose_name == "S0" else POSES[pose_name]
        src = set_max_steps(builders[scene](args.ref), steps)
        g = GL(W, H)
        t0 = time.time()
        rgba = g.draw(g.program(src), pose, (W, H))
        cnt = g.draw(g.program(src.replace("precision highp int;\n", "precision highp int;\n#define COUNT_MODE\n", 1)),
                     pose, (W, H))
        dt = time.time() - t0
        meta = dict(scene=scene, W=W, H=H, pose=pose_name, pos=list(pose["pos"]), mouse=list(pose["mouse"]),
                    time=pose["time"], max_steps=steps, renderer=g.renderer, gl_version=g.version,
                    generator="tests/golden/make_goldens.py")
        np.savez_compressed(os.path.join(HERE, name + ".npz"), rgba=rgba, evals=cnt[..., 0].astype(np.int32),
                            meta=json.dumps(meta))
        print(f"{name}: {dt:.2f}s mean={rgba[..., :3].mean():.4f} evals/px={cnt[..., 0].mean():.2f} "
              f"nan={int(np.isnan(rgba).sum())}")
    # scene-O diagnostic channels (diag_edit) at the poses of two O fixtures
    for name, W, H, pose_name, steps in DIAG_FIXTURES:
        if args.only and args.only not in name:
            continue
        pose = POSES[pose_name]
        src = set_max_steps(scene_O_diag(args.ref), steps)
        g = GL(W, H)
        chans = []
        for k in range(N_DIAG):
            chans.append(g.draw(g.program(src.replace("precision highp int;\n",
                                                      f"precision highp int;\n#define DIAG_K {k}\n", 1)), pose, (W, H)))
        rgba = g.draw(g.program(src), pose, (W, H))
        meta = dict(scene="O", W=W, H=H, pose=pose_name, pos=list(pose["pos"]), mouse=list(pose["mouse"]),
                    time=pose["time"], max_steps=steps, renderer=g.renderer, channels=DIAG_DOC,
                    generator="tests/golden/make_goldens.py (diag_edit)")
        np.savez_compressed(os.path.join(HERE, name + ".npz"), diag=np.stack(chans, axis=2), rgba=rgba,
                            meta=json.dumps(meta))
        print(f"{name}: {N_DIAG} channels, primary hits {int(np.sum(chans[0][..., 3] > 0))}")
    # scene-library known answers (lib_kat_cases.py) for the plugin dialect
    if not args.only or args.only in "LIB_kat":
        from lib_kat_cases import CASES, N_POINTS
        g = GL(N_POINTS, len(CASES))
        noop = dict(pos=(0.0, 0.0, 0.0), mouse=(0.0, 0.0), time=0.0)
        src = lib_kat(args.ref)
        res = (N_POINTS, len(CASES))
        pts = g.draw(g.program(src.replace("precision highp int;\n", "precision highp int;\n#define POINTS_MODE\n", 1)),
                     noop, res)[::-1][0, :, :3].copy()
        vals = g.draw(g.program(src), noop, res)[::-1].copy()
        mats = np.concatenate([g.draw(g.program(lib_kat_materials(args.ref).replace(
            "precision highp int;\n", f"precision highp int;\n#define KPASS {k}\n", 1)), noop, res)[::-1]
            for k in range(4)], axis=-1)
        meta = dict(cases=[c[0] for c in CASES], classes=[c[2] for c in CASES], renderer=g.renderer,
                    generator="tests/golden/make_goldens.py (cases: tests/golden/lib_kat_cases.py)")
        np.savez_compressed(os.path.join(HERE, "LIB_kat.npz"), points=pts, dist=vals[..., 0].copy(), mat=mats,
                            meta=json.dumps(meta))
        print(f"LIB_kat: {len(CASES)} cases x {N_POINTS} points, nan={int(np.isnan(vals).sum())}")
    # the FXAA post pass (post.frag), next to the hot path
    for name, img in fxaa_inputs():
        if args.only and args.only not in name:
            continue
        H, W = img.shape
        g = GL(W, H)
        out = g.post(g.program(post_fxaa(args.ref)), img, (W, H))
        meta = dict(pass_="post.frag fxaa", W=W, H=H, sampler="NEAREST, CLAMP_TO_EDGE", renderer=g.renderer,
                    generator="tests/golden/make_goldens.py")
        np.savez_compressed(os.path.join(HERE, name + ".npz"), input=img, output=out, meta=json.dumps(meta))
        print(f"{name}: changed pixels {float(np.mean(out != img[::-1])):.3f}")
    # the bloom post pass (shaders/post/bloom.frag) over its mip chain
    for name, img in bloom_inputs():
        if args.only and args.only not in name:
            continue
        H, W = img.shape
        g = GL(W, H)
        out, mips = g.bloom(g.program(post_bloom(args.ref)), img, (W, H))
        meta = dict(pass_="shaders/post/bloom.frag", W=W, H=H, levels=len(mips) + 1,
                    sampler="LINEAR_MIPMAP_LINEAR / LINEAR, CLAMP_TO_EDGE, glGenerateMipmap", renderer=g.renderer,
                    generator="tests/golden/make_goldens.py")
        arrs = {f"mip{k + 1}": m for k, m in enumerate(mips)}
        np.savez_compressed(os.path.join(HERE, name + ".npz"), input=img, output=out, meta=json.dumps(meta), **arrs)
        print(f"{name}: levels {len(mips) + 1}, mean |out - in| "
              f"{float(np.mean(np.abs((out & 255).astype(int) - (img[::-1] & 255).astype(int)))):.2f}")


if __name__ == "__main__":
    main()
