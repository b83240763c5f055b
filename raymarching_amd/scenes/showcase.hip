// A scene built from the reference's shape library (common.frag:93-617):
// a spinning torus merged with a rounded box, a row of pillars repeated
// along x, a sphere carved by a cube, and a floor.  It uses only syntax that
// is both GLSL and this plugin dialect, so tests/golden/make_goldens.py
// renders the very same text as output_shader.frag's sceneSDF with the
// reference GLSL (golden SC_*).
const Material gold = Material(vec3(0.25, 0.18, 0.05), vec3(0.3, 0.25, 0.1), 64.0, 0.15, 0.0, vec3(0.0), 1.0, vec3(0.0));
const Material jade = Material(vec3(0.03, 0.15, 0.08), vec3(0.05, 0.08, 0.06), 32.0, 0.0, 0.0, vec3(0.0), 1.0, vec3(0.0));
const Material chalk = Material(vec3(0.2, 0.2, 0.22), vec3(0.02), 16.0, 0.0, 0.0, vec3(0.0), 1.0, vec3(0.0));

SdResult sceneSDF(vec3 p)
{
	vec3 q = transformTR(p, vec3(0.0, 2.0, 0.0), vec3(90.0, u_time * 20.0, 0.0));
	float ring = opSmoothUnion(torus(q, vec2(1.2, 0.3)), rounding(sdBox(q, vec3(0.5)), 0.1), 0.4);
	vec3 r = p - vec3(0.0, 0.0, -4.0);
	float cell = pMod1(r.x, 3.0);
	float pillar = opIntersection(cylinder(transformRX(r, 90.0), 0.35 + 0.05 * cell), r.y - 3.0);
	float carved = opSubtraction(cube(vec4(3.0, 1.2, 2.0, 0.55), p), sphere(vec4(3.0, 1.2, 2.0, 0.8), p));
	SdResult a = SdResult(ring, gold);
	SdResult b = SdResult(pillar, jade);
	SdResult c = SdResult(carved, chalk);
	SdResult fl = SdResult(plane(p), chalk);
	return sminCubic(sdUnion(a, c), sminCubic(b, fl, 0.3), vec2(0.25, 0.5));
}
