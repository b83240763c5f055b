#!/usr/bin/env python3
"""Evaluate GLSL expressions of the reference scene under SwiftShader at
explicit input points (build container only; analysis aid for DESIGN.md
section 3, not a test).

Each pixel reads one RGBA32F texel ``P`` of an input texture and writes
``vec4(EXPR)``; the expression may call anything output_shader.frag and
common.frag define (the shader is make_goldens.scene_O's text with its main()
replaced).  ``probe(exprs, pts, time)`` returns {expr: [n, 4] float32}.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests", "golden"))
sys.path.insert(0, os.path.join(HERE, ".."))
import make_goldens as mg  # noqa: E402

MAIN = """
uniform highp sampler2D u_in;
void main()
{
\tvec4 P = texelFetch(u_in, ivec2(gl_FragCoord.xy), 0);
\tvec3 p = P.xyz;
\to_col = vec4(%s);
	// keep sceneSDF's callees referenced (the translator prunes otherwise)
	if (P.w > 1e30) o_col = vec4(sceneSDF(p).dist);
}
"""


def _shader(expr: str, ref: str) -> str:
    s = mg.scene_O(ref)
    k = s.rfind("void main()")
    return s[:k] + MAIN % expr


def probe(exprs, pts, time=0.0, ref="/root/reference"):
    pts = np.asarray(pts, np.float32)
    if pts.shape[-1] == 3:
        pts = np.concatenate([pts, np.zeros(pts.shape[:-1] + (1,), np.float32)], -1)
    n = len(pts)
    W = min(n, 256)
    H = (n + W - 1) // W
    inp = np.zeros((H * W, 4), np.float32)
    inp[:n] = pts
    g = mg.GL(W, H)
    gl = g.gl
    tex = ctypes.c_uint()
    gl.glGenTextures(1, ctypes.byref(tex))
    gl.glActiveTexture(0x84C1)  # unit 1
    gl.glBindTexture(0x0DE1, tex)
    for pname, val in ((0x2801, 0x2600), (0x2800, 0x2600)):
        gl.glTexParameteri(0x0DE1, pname, val)
    gl.glTexImage2D(0x0DE1, 0, 0x8814, W, H, 0, 0x1908, 0x1406, inp.ctypes.data_as(ctypes.c_void_p))
    out = {}
    for e in exprs:
        prog = g.program(_shader(e, ref))
        gl.glUseProgram(prog)
        gl.glUniform1i(gl.glGetUniformLocation(prog, b"u_in"), 1)
        # GL.draw reads rows bottom-up and flips; undo the flip for point order
        res = g.draw(prog, dict(pos=(0.0, 0.0, 0.0), mouse=(0.0, 0.0), time=time), (W, H))[::-1]
        out[e] = res.reshape(-1, 4)[:n].copy()
    return out


if __name__ == "__main__":
    rng = np.random.default_rng(0)
    pts = rng.uniform(-3, 3, (1024, 3)).astype(np.float32)
    r = probe(["sceneSDF(p).dist, 0.0, 0.0, 0.0"], pts, time=10.0)
    print(next(iter(r.values()))[:4])
