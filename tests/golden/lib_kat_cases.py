"""Known-answer cases for the scene library (TEST DATA, not product code).

Each case is a function body that is valid both as GLSL ES 3.00 appended to
the reference's common.frag (make_goldens.py renders it with SwiftShader and
stores the values in LIB_kat.npz) and as a scene plugin over
raymarching_amd/csrc/rm_sdf_lib.h (tests/test_plugins.py evaluates it on the
GPU through rm_scene_eval).  A case returns an SdResult whose dist and
mat.diffuse carry up to four outputs; case i runs at N_POINTS points
(kat_point), selected on the GPU by u_time = i.
"""
N_POINTS = 64

PRELUDE = """
const Material kA = Material(vec3(0.2, 0.02, 0.02), vec3(0.04, 0.02, 0.02), 32.0, 0.0, 0.0, vec3(0.0), 1.0, vec3(0.0));
const Material kB = Material(vec3(0.02, 0.3, 0.5), vec3(0.5, 0.25, 0.125), 64.0, 0.25, 0.5, vec3(0.4, 0.4, 0.15), 1.52, vec3(0.0, 0.0, 4.0));
Material kOut(vec3 v) { return Material(v, vec3(0.0), 0.0, 0.0, 0.0, vec3(0.0), 1.0, vec3(0.0)); }
SdResult r1(float d) { return SdResult(d, kOut(vec3(0.0))); }
SdResult r3(vec3 v) { return SdResult(v.x, kOut(v)); }
SdResult r4(float d, vec3 v) { return SdResult(d, kOut(v)); }
float kSph(vec3 p) { return sphere(vec4(0.5, 1.0, 0.0, 1.0), p); }
float kCub(vec3 p) { return cube(vec4(-1.0, 0.5, 0.5, 0.8), p); }
float kTor(vec3 p) { return torus(p, vec2(1.0, 0.3)); }
vec3 kat_point(int i)
{
    float f = float(i);
    return vec3(2.6 * sin(f * 1.37 + 0.3), 1.0 + 2.2 * cos(f * 0.71), 2.4 * sin(f * 2.13 + 1.1));
}
"""

_POS = "vec3(1.0, -0.5, 2.0)"
_ROT = "vec3(20.0, 35.0, -15.0)"
_SCL = "vec3(1.5, 0.5, 2.0)"

# (name, body, tolerance class)
CASES = [
    ("opUnion", "return r1(opUnion(kSph(p), kCub(p)));", "exact"),
    ("opSubtraction", "return r1(opSubtraction(kSph(p), kCub(p)));", "exact"),
    ("opIntersection", "return r1(opIntersection(kSph(p), kCub(p)));", "exact"),
    ("opSmoothUnion", "return r1(opSmoothUnion(kSph(p), kCub(p), 0.7));", "exact"),
    ("opSmoothSubtraction", "return r1(opSmoothSubtraction(kSph(p), kCub(p), 0.7));", "exact"),
    ("opSmoothIntersection", "return r1(opSmoothIntersection(kSph(p), kCub(p), 0.7));", "exact"),
    ("sdf_blend", "return r1(sdf_blend(kSph(p), kTor(p), 0.3));", "exact"),
    ("smin", "return r1(smin(kSph(p), kCub(p), 0.6));", "exact"),
    ("smin_exp", "return r1(smin_exp(kSph(p), kCub(p), 4.0));", "trans"),
    ("smin_exp32", "return r1(smin_exp(kSph(p) * 0.1, kCub(p) * 0.1, 32.0));", "trans"),
    ("rounding", "return r1(rounding(sdBox(p, vec3(1.0, 0.5, 0.7)), 0.1));", "exact"),
    ("plane_sdPlane", "return r1(plane(p) + 0.5 * sdPlane(p, vec4(normalize(vec3(1.0, 2.0, 3.0)), 0.5)));", "exact"),
    ("sphere", "return r1(sphere(vec4(0.3, -0.2, 0.5, 1.2), p));", "exact"),
    ("cube", "return r1(cube(vec4(-0.4, 0.5, 0.2, 0.9), p));", "exact"),
    ("sdBox", "return r1(sdBox(p, vec3(1.0, 0.5, 0.7)));", "exact"),
    ("cylinder", "return r1(cylinder(p, 0.7));", "exact"),
    ("cone", "return r1(cone(p, normalize(vec2(0.8, 0.6))));", "exact"),
    ("torus", "return r1(kTor(p));", "exact"),
    ("mengersponge", "vec3 m = mengersponge(p * 0.5); return r4(m.x, m);", "exact"),
    ("mandelbulb", "vec4 c; float d = mandelbulb(p * 0.6, c); return r4(d, vec3(c.y, c.z, c.w));", "fractal"),
    ("mandelbulb_m", "vec4 c; float d = mandelbulb(p * 0.6, c); return r1(log(c.x) + 0.0 * d);", "fractal"),
    ("rotatePoint", "vec2 q = vec2(p.x, p.z); rotatePoint(q, 0.7); return r4(q.x, vec3(q.x, q.y, 0.0));", "trans"),
    ("rotatePointX", "return r3(rotatePointX(p, 0.7));", "trans"),
    ("rotatePointY", "return r3(rotatePointY(p, -1.1));", "trans"),
    ("rotatePointZ", "return r3(rotatePointZ(p, 2.3));", "trans"),
    ("translatePoint", "vec3 q = p; translatePoint(q, vec3(0.5, -1.0, 2.0)); return r3(q);", "exact"),
    ("rotationX", "vec4 v = vec4(p, 1.0) * rotationX(33.0); return r4(v.w, vec3(v.x, v.y, v.z));", "trans"),
    ("rotationY", "vec4 v = vec4(p, 1.0) * rotationY(-47.0); return r4(v.w, vec3(v.x, v.y, v.z));", "trans"),
    ("rotationZ", "vec4 v = vec4(p, 1.0) * rotationZ(128.0); return r4(v.w, vec3(v.x, v.y, v.z));", "trans"),
    ("transform", f"return r3(transform(p, {_POS}, {_ROT}, {_SCL}));", "trans"),
    ("transformTR", f"return r3(transformTR(p, {_POS}, {_ROT}));", "trans"),
    ("transformTRX", f"return r3(transformTRX(p, {_POS}, 40.0));", "trans"),
    ("transformTRY", f"return r3(transformTRY(p, {_POS}, 50.0));", "trans"),
    ("transformTRZ", f"return r3(transformTRZ(p, {_POS}, 60.0));", "trans"),
    ("transformTRXS", f"return r3(transformTRXS(p, {_POS}, 40.0, {_SCL}));", "trans"),
    ("transformTRYS", f"return r3(transformTRYS(p, {_POS}, 50.0, {_SCL}));", "trans"),
    ("transformTRZS", f"return r3(transformTRZS(p, {_POS}, 60.0, {_SCL}));", "trans"),
    ("transformTRS1", f"return r3(transformTRS1(p, {_POS}, {_ROT}, 1.7));", "trans"),
    ("transformTRXS1", f"return r3(transformTRXS1(p, {_POS}, 40.0, 1.7));", "trans"),
    ("transformTRYS1", f"return r3(transformTRYS1(p, {_POS}, 50.0, 1.7));", "trans"),
    ("transformTRZS1", f"return r3(transformTRZS1(p, {_POS}, 60.0, 1.7));", "trans"),
    ("transformR", "return r3(transformR(p, vec3(180.0, 33.0, 0.0)));", "trans"),
    ("transformRX", "return r3(transformRX(p, 40.0));", "trans"),
    ("transformRY", "return r3(transformRY(p, 50.0));", "trans"),
    ("transformRZ", "return r3(transformRZ(p, 60.0));", "trans"),
    ("transformRXS", f"return r3(transformRXS(p, 40.0, {_SCL}));", "trans"),
    ("transformRYS", f"return r3(transformRYS(p, 50.0, {_SCL}));", "trans"),
    ("transformRZS", f"return r3(transformRZS(p, 60.0, {_SCL}));", "trans"),
    ("transformRS1", f"return r3(transformRS1(p, {_ROT}, 1.7));", "trans"),
    ("transformRXS1", "return r3(transformRXS1(p, 40.0, 1.7));", "trans"),
    ("transformRYS1", "return r3(transformRYS1(p, 50.0, 1.7));", "trans"),
    ("transformRZS1", "return r3(transformRZS1(p, 60.0, 1.7));", "trans"),
    ("pMod1", "vec3 q = p; float c = pMod1(q.x, 1.5); return r4(c, q);", "exact"),
    ("pMod2", "vec2 q = vec2(p.x, p.z); vec2 c = pMod2(q, vec2(1.5, 0.8)); return r4(c.x, vec3(c.y, q.x, q.y));",
     "exact"),
    ("pMirror", "vec3 q = p; float s = pMirror(q.x, 0.8); return r4(s, q);", "exact"),
    ("pReflect", "vec3 q = p; float s = pReflect(q, normalize(vec3(1.0, -1.0, 0.5)), 0.3); return r4(s, q);", "exact"),
    ("sdUnion", "return sdUnion(SdResult(kSph(p), kA), SdResult(kTor(p), kB));", "exact"),
    ("sminCubic", "return sminCubic(SdResult(kSph(p), kA), SdResult(kTor(p), kB), 0.8);", "exact"),
    ("sminCubic2", "return sminCubic(SdResult(kCub(p), kB), SdResult(kTor(p), kA), vec2(0.5, 1.5));", "exact"),
    ("blendMaterial", "return SdResult(0.0, blendMaterial(kA, kB, clamp(p.x * 0.2 + 0.5, 0.0, 1.0)));", "exact"),
    ("scaleSDF", "return r1(scaleSDF(kTor, p, 1.7));", "exact"),
    ("scaleSDF3", "return r1(scaleSDF3(kTor, p, 1.7, 0.8, 1.2));", "exact"),
]

# per class: (relative, absolute) tolerance and the points allowed outside it
TOL = {"exact": (2e-6, 2e-6, 1), "trans": (5e-5, 5e-5, 1), "fractal": (5e-3, 5e-3, 6)}


def kat_function() -> str:
    """SdResult kat(int fn, vec3 p): case fn at p (GLSL and plugin alike)."""
    body = "\n".join(f"\tif (fn == {i}) {{ {b} }}" for i, (_, b, _) in enumerate(CASES))
    return "SdResult kat(int fn, vec3 p)\n{\n" + body + "\n\treturn r1(0.0);\n}\n"


def plugin_source() -> str:
    """The cases as a scene plugin: sceneSDF(p) = case int(u_time) at p."""
    return ("// generated by tests/golden/lib_kat_cases.py (scene-library known answers)\n"
            "#define RM_PLUGIN_EVAL_ONLY\n" + PRELUDE + kat_function() +
            "SdResult sceneSDF(vec3 p)\n{\n\treturn kat(int(u_time), p);\n}\n")
