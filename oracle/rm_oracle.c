/*
 * oracle/rm_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, scalar CPU restatement of the reference's per-pixel ray-march
 * pass (cahekp/Raymarching: common.frag + output_shader.frag + template.frag),
 * written line by line against the GLSL so that the HIP product path
 * (raymarching_amd/csrc) can be checked against it.  Nothing in the product
 * path links, loads or calls this file: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg use it, and only as the checker / CPU
 * baseline.
 *
 * Pinning: the reference has no tests or fixtures.  This restatement is
 * pinned against golden images rendered in-container by SwiftShader from the
 * reference GLSL itself (tests/golden/make_goldens.py), see DESIGN.md
 * "Oracle".  GLSL built-ins follow the GLSL 1.30 spec definitions
 * (min/max/clamp/mix/mod/fract/smoothstep/reflect/refract/normalize).
 * Transcendentals use libm (the reference's driver precision is unpinned).
 *
 * Build: oracle/Makefile (-O2 -ffp-contract=off for parity; an -O3
 * -march=native variant for the CPU baseline timing).
 *
 * Every function cites the reference file:line it restates.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- types */

typedef struct { float x, y; } vec2;
typedef struct { float x, y, z; } vec3;

/* common.frag:20-35 */
typedef struct {
    vec3 diffuse;
    vec3 specular;
    float shininess;
    float reflectivity;
    float transparency;
    vec3 absorption;
    float refraction_index;
    vec3 emission;
} Material;

/* common.frag:57-61 */
typedef struct {
    float dist;
    Material mat;
} SdResult;

enum { SCENE_S0 = 0, SCENE_T = 1, SCENE_O = 2, SCENE_OG = 3 };

/* Uniforms of common.frag:4-7 plus the run-time knobs that replace the
 * compile-time MAX_MARCHING_STEPS (common.frag:15). Layout mirrored by
 * tests/oracle.py (ctypes). */
typedef struct {
    float res_x, res_y;     /* u_resolution */
    float mouse_x, mouse_y; /* u_mouse      */
    float pos_x, pos_y, pos_z; /* u_pos     */
    float time;             /* u_time       */
    int32_t max_steps;      /* MAX_MARCHING_STEPS (common.frag:15) */
    int32_t shadow_max_steps; /* 0 = unbounded, as common.frag:814 */
    float jit_x, jit_y;     /* progressive accumulation: sub-pixel offset of the fragment
                               (fract(u_seed1) - 0.5; 0 = the pixel centre) */
} oracle_uniforms;

typedef struct {
    int scene;
    oracle_uniforms u;
    /* transformR's three rotations (common.frag:434-441, 190-227) depend on
     * uniforms only; their sin/cos are taken once per frame here exactly as
     * rotationX/Y/Z compute them (radians(), cos(), sin()). */
    float ry_c, ry_s, rx_c, rx_s, rz_c, rz_s;
    uint64_t *evals; /* per-thread counter of sceneSDF calls */
    struct SegRec *rec; /* optional: per-pixel phase/segment recorder (analysis) */
    float *diag;        /* optional: scene-O diagnostic channels, N_DIAG vec4 per pixel */
    int lvl;            /* 0 = primary light(), 1 = inside the reflection bounce */
    struct SettleRec *settle; /* optional: soft-shadow settle analysis (scenes T, O) */
} Ctx;

/* Diagnostic channels of make_goldens.py diag_edit (test aid, values only):
 * 0 primary normal, dist; 1 primary thickness, sha, occ, ind; 2 primary light()
 * colour, fresnel; 3 reflection normal, dist (-1 miss); 4 reflection thickness,
 * sha, occ, ind; 5 reflection colour; 6 render() colour.  Unset = -9. */
#define N_DIAG 7
static inline void diag_set(const Ctx *C, int k, float a, float b, float c, float d) {
    if (!C->diag) return;
    C->diag[4 * k] = a; C->diag[4 * k + 1] = b; C->diag[4 * k + 2] = c; C->diag[4 * k + 3] = d;
}

/* Analysis aid (not part of the restatement): records, per pixel, the
 * sequence of sceneSDF-call segments as (phase, count) pairs, so the SIMD
 * efficiency of lane-per-pixel vs. wave-compacted schedules can be simulated
 * (tools/wave_sim.py).  Phases: 0 march, 1 normal, 2 AO, 3 shadow, 4 SSS. */
enum { PH_MARCH = 0, PH_NORMAL = 1, PH_AO = 2, PH_SHADOW = 3, PH_SSS = 4 };
#define MAX_SEG 24
typedef struct SegRec {
    int phase, fresh, nseg;
    uint16_t *out; /* MAX_SEG x (phase, count) */
} SegRec;
static inline void seg_begin(const Ctx *C, int phase) {
    if (C->rec) { C->rec->phase = phase; C->rec->fresh = 1; }
}
static inline void seg_eval(SegRec *r) {
    if (!r->fresh && r->nseg > 0) { r->out[2 * (r->nseg - 1) + 1]++; return; }
    if (r->nseg < MAX_SEG) {
        r->out[2 * r->nseg] = (uint16_t)r->phase;
        r->out[2 * r->nseg + 1] = 1;
        r->nseg++;
    }
    r->fresh = 0;
}

/* --------------------------------------------------------- GLSL built-ins */

static inline vec3 v3(float x, float y, float z) { vec3 r = {x, y, z}; return r; }
static inline vec3 v3s(float s) { return v3(s, s, s); }
static inline vec3 add(vec3 a, vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline vec3 sub(vec3 a, vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline vec3 mul(vec3 a, vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline vec3 muls(vec3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline vec3 divs(vec3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline vec3 neg(vec3 a) { return v3(-a.x, -a.y, -a.z); }
static inline float dot3(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float length3(vec3 a) { return sqrtf(dot3(a, a)); }
/* GLSL normalize(x) = x / length(x); the pinned implementation (SwiftShader,
 * tests/golden) multiplies by the correctly rounded reciprocal of the length
 * (bit-exact on 8192 vectors, tools/ss_probe.py) */
static inline vec3 normalize3(vec3 a) { return muls(a, 1.0f / length3(a)); }
/* GLSL 1.30 spec 8.3: min(x,y) = y < x ? y : x ; max(x,y) = x < y ? y : x */
static inline float gmin(float x, float y) { return y < x ? y : x; }
static inline float gmax(float x, float y) { return x < y ? y : x; }
static inline float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }
/* GLSL mix(x, y, a) (spec: x(1-a) + ya); the pinned implementation (SwiftShader,
 * tests/golden) evaluates x + (y - x)a (bit-exact on 4096 triples, tools/ss_probe.py) */
static inline float gmix(float x, float y, float a) { return x + (y - x) * a; }
static inline vec3 mix3(vec3 x, vec3 y, float a) { return v3(gmix(x.x, y.x, a), gmix(x.y, y.y, a), gmix(x.z, y.z, a)); }
static inline float gmod(float x, float y) { return x - y * floorf(x / y); }
static inline float gfract(float x) { return x - floorf(x); }
static inline float gsmoothstep(float e0, float e1, float x) {
    float t = gclamp((x - e0) / (e1 - e0), 0.0f, 1.0f);
    return t * t * (3.0f - 2.0f * t);
}
static inline vec3 vabs(vec3 a) { return v3(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
static inline vec3 vmax0(vec3 a) { return v3(gmax(a.x, 0.0f), gmax(a.y, 0.0f), gmax(a.z, 0.0f)); }
/* reflect(I,N) = I - 2.0 * dot(N, I) * N */
static inline vec3 reflect3(vec3 I, vec3 N) { return sub(I, muls(N, 2.0f * dot3(N, I))); }
/* refract(I,N,eta): k = 1 - eta*eta*(1 - dot(N,I)*dot(N,I)); k < 0 -> 0 */
static inline vec3 refract3(vec3 I, vec3 N, float eta) {
    float d = dot3(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return v3s(0.0f);
    return sub(muls(I, eta), muls(N, eta * d + sqrtf(k)));
}
static inline float radians(float deg) { return deg * 0.017453292519943295f; }

/* GLSL sin()/cos().  GLSL leaves their precision to the implementation
 * (parity unpinned at that level); these restate the implementation that
 * renders the golden fixtures (SwiftShader 4.1, tests/golden/make_goldens.py):
 * reduce to y = x/2pi - round(y) in [-1/2, 1/2], evaluate the cos/sin of
 * pi*y by two minimax polynomials, double the angle twice and normalize
 * ("A Fast, Vectorizable Algorithm for Producing Single-Precision Sine-Cosine
 * Pairs"); cos(x) = sin(x + 1.57079632).  Bit-exact against SwiftShader on
 * 8000 arguments in [-400, 400] (tools/ss_probe.py).  The uniform-derived
 * rotations (camera rot(), transformR) and floorMat use them: a ulp of the
 * sponge rotation moves the sampled distances that getNormalFast
 * differentiates, and the normal feeds the Hash33 of CalculateThickness. */
static float glsl_sin(float x) {
    float y = x * 1.59154943e-1f;
    y = y - rintf(y);
    float y2 = y * y;
    float c1 = y2 * (y2 * (y2 * -0.0204391631f + 0.2536086171f) + -1.2336977925f) + 1.0f;
    float s1 = y * (y2 * (y2 * (y2 * -0.0046075748f + 0.0796819754f) + -0.645963615f) + 1.5707963235f);
    float c2 = c1 * c1 - s1 * s1;
    float s2 = 2.0f * s1 * c1;
    return 2.0f * s2 * c2 * (1.0f / (s2 * s2 + c2 * c2));
}
static float glsl_cos(float x) { return glsl_sin(x + 1.57079632f); }

/* ------------------------------------------------------------- constants */

static const float ZNEAR = 0.02f;   /* common.frag:13 */
static const float ZFAR = 50.0f;    /* common.frag:14 */
static const float PI = 3.1416f;    /* common.frag:1108 */

/* ---------------------------------------------------------- materials */

/* common.frag:37-53 with ALLOW_MATERIAL_BLENDING defined (output_shader.frag:9) */
static Material blendMaterial(const Material *a, const Material *b, float k) {
    Material m;
    m.diffuse = mix3(a->diffuse, b->diffuse, k);
    m.specular = mix3(a->specular, b->specular, k);
    m.shininess = gmix(a->shininess, b->shininess, k);
    m.reflectivity = gmix(a->reflectivity, b->reflectivity, k);
    m.transparency = gmix(a->transparency, b->transparency, k);
    m.absorption = mix3(a->absorption, b->absorption, k);
    m.refraction_index = gmix(a->refraction_index, b->refraction_index, k);
    m.emission = mix3(a->emission, b->emission, k);
    return m;
}

static Material make_mat(vec3 d, vec3 s, float sh, float refl, float tr, vec3 ab, float ior, vec3 em) {
    Material m = {d, s, sh, refl, tr, ab, ior, em};
    return m;
}

/* output_shader.frag:12 (red), :14 (blue), :15 (mirror) */
static Material mat_red(void) {
    return make_mat(v3(0.2f, 0.02f, 0.02f), v3(0.04f, 0.02f, 0.02f), 32.0f, 0.0f, 0.0f, v3s(0.0f), 1.0f, v3s(0.0f));
}
static Material mat_blue(int glass) {
    /* glass != 0 is the test-only variant "OG" that exercises the refraction
     * path (renderRefraction, output_shader.frag:298-343), which is dead in
     * the reference scene because every material has transparency 0. */
    return make_mat(v3(0.02f, 0.02f, 0.2f), v3(0.02f, 0.02f, 0.04f), 32.0f, 0.0f, glass ? 0.9f : 0.0f,
                    muls(v3(2.0f, 2.0f, 0.75f), 0.2f), 1.52f, v3(0.0f, 0.0f, 100.0f));
}
static Material mat_mirror(void) {
    return make_mat(v3s(0.1f), v3s(0.09f), 64.0f, 0.25f, 0.0f, v3s(0.0f), 1.0f, v3s(0.0f));
}

/* output_shader.frag:16-28 */
static Material floorMat(vec3 pos) {
    vec3 white = v3s(0.3f);
    vec3 black = v3s(0.025f);
    float smoothstepSize = 0.005f;
    float scale = gmax(10.0f, powf(length3(pos), 1.3f));
    float tx = gsmoothstep(-smoothstepSize, smoothstepSize, sinf(pos.x * PI) / scale);
    float ty = gsmoothstep(-smoothstepSize, smoothstepSize, sinf(pos.z * PI) / scale);
    float tile = gmin(gmax(tx, ty), gmax(1.0f - tx, 1.0f - ty));
    vec3 color = mix3(white, black, tile);
    return make_mat(color, v3s(0.03f), 128.0f, 0.0f, 0.0f, v3s(0.0f), 1.0f, v3s(0.0f));
}

/* -------------------------------------------------------- SDF library */

/* common.frag:72-85 (vec2 k form) called through :87-89 with k = vec2(k) */
static SdResult sminCubic(const SdResult *a, const SdResult *b, float kf) {
    float kx = gmax(kf, 0.0001f), ky = gmax(kf, 0.0001f);
    float ad = fabsf(a->dist - b->dist);
    float hx = gmax(kx - ad, 0.0f) / kx;
    float hy = gmax(ky - ad, 0.0f) / ky;
    float mx = hx * hx * hx * 0.5f;
    float my = hy * hy * hy * 0.5f;
    float sx = mx * kx * (1.0f / 3.0f);
    SdResult res;
    int aCloser = a->dist < b->dist;
    res.dist = (aCloser ? a->dist : b->dist) - sx;
    float blendCoeff = aCloser ? my : 1.0f - my;
    res.mat = blendMaterial(&a->mat, &b->mat, blendCoeff);
    return res;
}

/* common.frag:572-575 */
static float plane(vec3 p) { return p.y; }

/* common.frag:584-587 */
static float sphere(float sx, float sy, float sz, float sw, vec3 p) {
    return length3(sub(p, v3(sx, sy, sz))) - sw;
}

/* common.frag:589-593 */
static float cube(float sx, float sy, float sz, float sw, vec3 p) {
    vec3 q = sub(vabs(sub(p, v3(sx, sy, sz))), v3s(sw));
    return length3(vmax0(q)) + gmin(gmax(q.x, gmax(q.y, q.z)), 0.0f);
}

/* common.frag:595-600 */
static float sdBox(vec3 p, vec3 b) {
    vec3 di = sub(vabs(p), b);
    float mc = gmax(di.x, gmax(di.y, di.z));
    return gmin(mc, length3(vmax0(di)));
}

/* common.frag:654-679; only .x is consumed by the scenes */
static float mengersponge_x(vec3 p) {
    float d = sdBox(p, v3s(1.0f));
    float s = 1.0f;
    for (int m = 0; m < 3; m++) {
        vec3 ps = muls(p, s);
        vec3 a = v3(gmod(ps.x, 2.0f) - 1.0f, gmod(ps.y, 2.0f) - 1.0f, gmod(ps.z, 2.0f) - 1.0f);
        s *= 3.0f;
        vec3 r = vabs(sub(v3s(1.0f), muls(vabs(a), 3.0f)));
        float da = gmax(r.x, r.y);
        float db = gmax(r.y, r.z);
        float dc = gmax(r.z, r.x);
        float c = (gmin(da, gmin(db, dc)) - 1.0f) / s;
        if (c > d) d = c;
    }
    return d;
}

/* common.frag:434-441: (vec4(p,1) * r_y * r_x * r_z).xyz, each factor a
 * row-vector x column-major mat4 product (rotationX/Y/Z, :190-227). The
 * w=1 row contributes exact zeros. */
static vec3 transformR(const Ctx *C, vec3 p) {
    /* v * rotationY: cols (c,0,s,0) (0,1,0,0) (-s,0,c,0) */
    float c = C->ry_c, s = C->ry_s;
    vec3 q = v3(p.x * c + p.y * 0.0f + p.z * s, p.y, p.x * -s + p.y * 0.0f + p.z * c);
    /* v * rotationX: cols (1,0,0,0) (0,c,-s,0) (0,s,c,0) */
    c = C->rx_c; s = C->rx_s;
    q = v3(q.x, q.x * 0.0f + q.y * c + q.z * -s, q.x * 0.0f + q.y * s + q.z * c);
    /* v * rotationZ: cols (c,-s,0,0) (s,c,0,0) (0,0,1,0) */
    c = C->rz_c; s = C->rz_s;
    q = v3(q.x * c + q.y * -s, q.x * s + q.y * c, q.z);
    return q;
}

/* ---------------------------------------------------------- the scenes */

/* Scene S0 (BASELINE config 1): single sphere, red (output_shader.frag:12). */
static SdResult sceneSDF_S0(const Ctx *C, vec3 p) {
    (void)C;
    SdResult r;
    r.dist = sphere(0.0f, 1.0f, -3.0f, 1.0f, p);
    r.mat = mat_red();
    return r;
}

/* Scene T: template.frag:39-43 repaired: the sponge
 * distance with the red material. */
static SdResult sceneSDF_T(const Ctx *C, vec3 p) {
    SdResult r;
    r.dist = mengersponge_x(transformR(C, sub(p, v3(0.0f, 3.0f, 0.0f))));
    r.mat = mat_red();
    return r;
}

/* Scene O: output_shader.frag:38-48 */
static SdResult sceneSDF_O(const Ctx *C, vec3 p) {
    SdResult d0, d1, d2, d3, t1, t2;
    d0.dist = mengersponge_x(transformR(C, sub(p, v3(0.0f, 3.0f, 0.0f))));
    d0.mat = mat_mirror();
    d1.dist = sphere(3.0f, 2.0f, 3.0f, 1.0f, p);
    d1.mat = mat_blue(C->scene == SCENE_OG);
    d2.dist = cube(-5.0f, 4.0f, 5.0f, 1.0f, p);
    d2.mat = mat_blue(C->scene == SCENE_OG);
    d3.dist = plane(p);
    d3.mat = floorMat(p);
    t1 = sminCubic(&d1, &d2, 0.5f);
    t2 = sminCubic(&t1, &d3, 0.5f);
    return sminCubic(&d0, &t2, 0.33f);
}

static SdResult sceneSDF(const Ctx *C, vec3 p) {
    (*C->evals)++;
    if (C->rec) seg_eval(C->rec);
    switch (C->scene) {
    case SCENE_S0: return sceneSDF_S0(C, p);
    case SCENE_T: return sceneSDF_T(C, p);
    default: return sceneSDF_O(C, p);
    }
}

/* ------------------------------------------------------- marching etc. */

/* common.frag:697-708 */
static vec3 getNormalFast(const Ctx *C, vec3 p) {
    seg_begin(C, PH_NORMAL);
    const float h = 0.001f;
    const vec3 k0 = v3(1.0f, -1.0f, -1.0f);
    const vec3 k1 = v3(-1.0f, -1.0f, 1.0f);
    const vec3 k2 = v3(-1.0f, 1.0f, -1.0f);
    const vec3 k3 = v3(1.0f, 1.0f, 1.0f);
    float d0 = sceneSDF(C, add(p, muls(k0, h))).dist;
    float d1 = sceneSDF(C, add(p, muls(k1, h))).dist;
    float d2 = sceneSDF(C, add(p, muls(k2, h))).dist;
    float d3 = sceneSDF(C, add(p, muls(k3, h))).dist;
    return normalize3(add(add(add(muls(k0, d0), muls(k1, d1)), muls(k2, d2)), muls(k3, d3)));
}

/* common.frag:710-713 */
static float lambert(vec3 lightDir, vec3 n) { return gclamp(dot3(n, lightDir), 0.0f, 1.0f); }

/* common.frag:730-754.  N is passed in: the reference recomputes
 * getNormalFast(p) here (:733) at the very p whose normal the caller already
 * holds; a pure function of p, so the value is identical and the 4 repeated
 * sceneSDF calls are elided (and not counted) in both oracle and HIP path. */
static vec3 phongContribForLight(vec3 k_d, vec3 k_s, float alpha, vec3 p, vec3 eye,
                                 vec3 lightPos, vec3 lightIntensity, vec3 N) {
    vec3 L = normalize3(sub(lightPos, p));
    vec3 V = normalize3(sub(eye, p));
    vec3 R = normalize3(reflect3(neg(L), N));
    float dotLN = dot3(L, N);
    float dotRV = dot3(R, V);
    if (dotLN < 0.0f) return v3s(0.0f);
    if (dotRV < 0.0f) return mul(lightIntensity, muls(k_d, dotLN));
    return mul(lightIntensity, add(muls(k_d, dotLN), muls(k_s, powf(dotRV, alpha))));
}

/* common.frag:810-831.  max_steps == 0: unbounded, as the reference. */
/* Analysis aid (not part of the restatement): the soft-shadow "settle" test
 * of DESIGN.md 2.11 evaluated at every step of scene T's shadow marches: the
 * step at which it first holds, the steps after it, and any change of res (or
 * an occlusion) after it -- which the test's proof says cannot happen. */
typedef struct SettleRec {
    uint64_t marches, steps, after, settled, violations;
    int every; /* test on steps every, 2 every, ... of a march (1: every step) */
    uint64_t refl_after; /* scene T: reflection-march steps begun at depth >= 3 */
    int back;            /* the current march shades a point facing away from the light */
    uint64_t back_steps; /* steps of such marches (their result is multiplied by 0) */
} SettleRec;
static int settle_test(const Ctx *C, vec3 p, vec3 rd, float t, float maxt, float res) {
    /* sponge space: q(t) = transformR(p - (0,3,0)), dq/dt = transformR(rd) (linear) */
    vec3 q = transformR(C, sub(p, v3(0.0f, 3.0f, 0.0f))), d = transformR(C, rd);
    float ax = fabsf(q.x), ay = fabsf(q.y), az = fabsf(q.z);
    float m = fmaxf(ax, fmaxf(ay, az)), B = m - 1.0f;
    float sl = ax == m ? (q.x < 0 ? -d.x : d.x) : ay == m ? (q.y < 0 ? -d.y : d.y) : (q.z < 0 ? -d.z : d.z);
    if (!(B >= 0.1f) || !(sl >= 0.0f)) return 0;
    float be = B + sl * (maxt - t);
    float lo = fminf(B / t, be / maxt);
    return 2.9f * lo >= 1.01f * res;
}

/* The same rule for scene O (rm_render_direct.h
 * shadow_settled_O): sceneSDF >= min(sponge box - 0.33/6, plane - 0.83/6,
 * sphere - 1.33/6, Chebyshev bound of the cube - 1.33/6) (each sminCubic
 * lowers a min by at most k/6; output_shader.frag:38-48 nests sphere and cube
 * (k 0.5), then the plane (k 0.5), then the sponge (k 0.33)); each term is
 * convex along the ray (the plane linear), so each has an affine minorant
 * through its value and a subgradient at t, and the bound's ratio to t' is
 * smallest at t or maxt. */
static int settle_piece(float v, float off, float sl, float t, float maxt, float *lo) {
    float g0 = v - off, g1 = v + sl * (maxt - t) - off;
    if (!(g0 >= 0.1f) || !(g1 >= 0.1f)) return 0;
    float r = fminf(g0 / t, g1 / maxt);
    *lo = fminf(*lo, r);
    return 1;
}
static int settle_test_O(const Ctx *C, vec3 p, vec3 rd, float t, float maxt, float res) {
    vec3 q = transformR(C, sub(p, v3(0.0f, 3.0f, 0.0f))), d = transformR(C, rd);
    float ax = fabsf(q.x), ay = fabsf(q.y), az = fabsf(q.z);
    float m = fmaxf(ax, fmaxf(ay, az));
    float s0 = ax == m ? (q.x < 0 ? -d.x : d.x) : ay == m ? (q.y < 0 ? -d.y : d.y) : (q.z < 0 ? -d.z : d.z);
    vec3 e1 = sub(p, v3(3.0f, 2.0f, 3.0f));
    float l1 = length3(e1);
    vec3 e2 = sub(p, v3(-5.0f, 4.0f, 5.0f));
    float bx = fabsf(e2.x), by = fabsf(e2.y), bz = fabsf(e2.z), m2 = fmaxf(bx, fmaxf(by, bz));
    float s2 = bx == m2 ? (e2.x < 0 ? -rd.x : rd.x) : by == m2 ? (e2.y < 0 ? -rd.y : rd.y) : (e2.z < 0 ? -rd.z : rd.z);
    float lo = 1e30f;
    if (!settle_piece(m - 1.0f, 0.33f / 6.0f, s0, t, maxt, &lo)) return 0;
    if (!settle_piece(l1 - 1.0f, 1.33f / 6.0f, dot3(e1, rd) / l1, t, maxt, &lo)) return 0;
    if (!settle_piece(m2 - 1.0f, 1.33f / 6.0f, s2, t, maxt, &lo)) return 0;
    if (!settle_piece(p.y, 0.83f / 6.0f, rd.y, t, maxt, &lo)) return 0;
    return 2.9f * lo >= 1.01f * res;
}

static float softshadow2(const Ctx *C, vec3 ro, vec3 rd, float mint, float maxt, float k) {
    seg_begin(C, PH_SHADOW);
    float res = 1.0f;
    float ph = 1e20f;
    int it = 0;
    SettleRec *S = C->settle;
    int settled = 0, step = 0;
    float res_at = 0.0f;
    if (S) S->marches++;
    for (float t = mint; t < maxt;) {
        if (C->u.shadow_max_steps > 0 && it++ >= C->u.shadow_max_steps) break;
        float h = sceneSDF(C, add(ro, muls(rd, t))).dist;
        if (S) {
            S->steps++;
            if (S->back) S->back_steps++;
            else if (settled) S->after++;
        }
        if (h < 0.001f) {
            if (S && settled) S->violations++;
            return 0.0f;
        }
        float y = h * h / (2.0f * ph);
        float d = sqrtf(h * h - y * y);
        res = gmin(res, k * d / gmax(0.0f, t - y));
        ph = h;
        if (S) {
            if (settled && res != res_at) S->violations++, res_at = res;
            vec3 pt = add(ro, muls(rd, t));
            if (!settled && ++step % S->every == 0 &&
                (C->scene == SCENE_T ? settle_test(C, pt, rd, t, maxt, res) : settle_test_O(C, pt, rd, t, maxt, res)))
                settled = 1, res_at = res, S->settled++;
        }
        t += h * 0.1f + 0.001f;
    }
    return res;
}

/* common.frag:850-866 (_AOSteps = 4, _AOStepSize = 0.2) */
static float ambientOcclusionReal(const Ctx *C, vec3 pos, vec3 normal) {
    seg_begin(C, PH_AO);
    float sum = 0.0f;
    float maxSum = 0.0f;
    for (int i = 0; i < 4; i++) {
        vec3 p = add(pos, muls(muls(normal, (float)(i + 1)), 0.2f));
        sum += 1.0f / powf(2.0f, (float)i) * sceneSDF(C, p).dist;
        maxSum += 1.0f / powf(2.0f, (float)i) * (float)(i + 1) * 0.2f;
    }
    return sum / maxSum;
}

/* common.frag:879-901 */
static SdResult castRayD(const Ctx *C, vec3 ro, vec3 rd) {
    seg_begin(C, PH_MARCH);
    SdResult res;
    memset(&res, 0, sizeof(res));
    float depth = ZNEAR;
    for (int i = 0; i < C->u.max_steps; i++) {
        res = sceneSDF(C, add(ro, muls(rd, depth)));
        if (res.dist < 0.001f * depth) {
            res.dist = depth;
            return res;
        }
        depth += res.dist;
        if (depth >= ZFAR) {
            res.dist = -1.0f;
            return res;
        }
    }
    return res;
}

/* common.frag:903-925 */
static SdResult castRayDI(const Ctx *C, vec3 ro, vec3 rd) {
    seg_begin(C, PH_MARCH);
    SdResult res;
    memset(&res, 0, sizeof(res));
    float depth = ZNEAR;
    for (int i = 0; i < C->u.max_steps; i++) {
        res = sceneSDF(C, add(ro, muls(rd, depth)));
        if (-res.dist < 0.001f * depth) {
            res.dist = depth;
            return res;
        }
        depth -= res.dist;
        if (depth >= ZFAR) {
            res.dist = -1.0f;
            return res;
        }
    }
    return res;
}

/* common.frag:931-954 */
/* refl: the reflection march of getColorReflect (analysis: with C->settle,
 * its steps begun at depth >= 3 are counted; rm_render_direct.h cast_ray_T RS) */
static vec3 castRay(const Ctx *C, vec3 ro, vec3 rd, int refl) {
    seg_begin(C, PH_MARCH);
    float depth = ZNEAR;
    vec3 p = add(ro, muls(rd, depth));
    for (int i = 0; i < C->u.max_steps; i++) {
        if (refl && C->settle && depth >= 3.0f) C->settle->refl_after++;
        float dist = sceneSDF(C, p).dist;
        if (dist < 0.001f) return p;
        depth += dist;
        p = add(ro, muls(rd, depth));
        if (depth >= ZFAR) return add(ro, muls(rd, ZFAR));
    }
    return p;
}

/* common.frag:991-1002 (getColor :983-986 is white).  The reference's
 * `nr = getNormalFast(pr)` (:995) is dead code and is not evaluated. */
static vec3 getColorReflect(const Ctx *C, vec3 p, vec3 n, vec3 rd) {
    vec3 reflect_dir = reflect3(rd, n);
    SettleRec *S = C->settle;
    const uint64_t before = S ? S->refl_after : 0;
    vec3 pr = castRay(C, add(p, muls(reflect_dir, 0.01f)), reflect_dir, 1);
    vec3 c = v3s(1.0f);
    c = muls(c, gclamp(length3(sub(pr, p)) / 3.0f, 0.0f, 1.0f));
    /* the rule: a march that went on past depth 3 ends with the factor 1 */
    if (S && S->refl_after != before && c.x != 1.0f) S->violations++;
    return c;
}

/* common.frag:1032-1042 */
static vec3 applyScattering(vec3 color, vec3 ro, vec3 p, vec3 fog_color, vec3 be, vec3 bi) {
    float d = 1.0f - gclamp(length3(sub(p, ro)) / ZFAR, 0.0f, 1.0f);
    vec3 ext = v3(expf(-d * be.x), expf(-d * be.y), expf(-d * be.z));
    vec3 ins = v3(expf(-d * bi.x), expf(-d * bi.y), expf(-d * bi.z));
    return add(mul(color, sub(v3s(1.0f), ext)), mul(fog_color, ins));
}

/* common.frag:1044-1051 */
static vec3 tonemap(vec3 color) {
    vec3 col = v3(color.x * 2.0f / (1.0f + color.x), color.y * 2.0f / (1.0f + color.y),
                  color.z * 2.0f / (1.0f + color.z));
    col = v3(powf(col.x, 0.4545f), powf(col.y, 0.4545f), powf(col.z, 0.4545f));
    col = v3(powf(col.x, 0.85f), powf(col.y, 0.97f), powf(col.z, 1.0f));
    col = v3(col.x * 0.5f + 0.5f * col.x * col.x * (3.0f - 2.0f * col.x),
             col.y * 0.5f + 0.5f * col.y * col.y * (3.0f - 2.0f * col.y),
             col.z * 0.5f + 0.5f * col.z * col.z * (3.0f - 2.0f * col.z));
    return col;
}

/* common.frag:1067-1070 */
static vec3 contrast(vec3 c) {
    return v3(gsmoothstep(0.15f, 1.1f, c.x), gsmoothstep(0.15f, 1.1f, c.y), gsmoothstep(0.15f, 1.1f, c.z));
}

/* common.frag:1072-1075 (amount = 0.1, the default the callers use) */
static vec3 vignette(vec3 color, vec2 uv) {
    float amount = 0.1f;
    return muls(color, 0.5f + 0.5f * powf(16.0f * uv.x * uv.y * (1.0f - uv.x) * (1.0f - uv.y), amount));
}

/* ------------------------------------------------ scene O (output_shader) */

static const vec3 FOG = {0.34f, 0.435f, 0.57f};

/* output_shader.frag:54-59 */
static float Hash11(float p) {
    vec3 p3 = v3(gfract(p * 443.897f), gfract(p * 443.897f), gfract(p * 443.897f));
    float dd = dot3(p3, add(v3(p3.y, p3.z, p3.x), v3s(19.19f)));
    p3 = add(p3, v3s(dd));
    return gfract((p3.x + p3.y) * p3.z);
}

/* output_shader.frag:61-66 */
static vec3 Hash33(vec3 p3) {
    p3 = v3(gfract(p3.x * 443.897f), gfract(p3.y * 441.423f), gfract(p3.z * 437.195f));
    float dd = dot3(p3, add(v3(p3.y, p3.x, p3.z), v3s(19.19f)));
    p3 = add(p3, v3s(dd));
    /* fract((p3.xxy + p3.yxx) * p3.zyx) */
    return v3(gfract((p3.x + p3.y) * p3.z), gfract((p3.x + p3.x) * p3.y), gfract((p3.y + p3.x) * p3.x));
}

/* output_shader.frag:70-73 */
static vec3 reflectVector(vec3 v, vec3 n) { return sub(v, muls(muls(n, 2.0f), gmin(0.0f, dot3(v, n)))); }

/* output_shader.frag:77-81 */
static vec3 GenerateSampleVector(vec3 norm, float i) {
    vec3 randDir = normalize3(sub(Hash33(add(norm, v3s(i))), v3s(0.5f)));
    return reflectVector(randDir, norm);
}

/* output_shader.frag:85-116 */
static float CalculateThickness(const Ctx *C, vec3 pos, vec3 norm) {
    seg_begin(C, PH_SSS);
    const float SSSSampleDepth = 1.0f;
    const float SSSThicknessSamples = 32.0f;
    const float SSSThicknessSamplesI = 0.03125f;
    float thickness = 0.0f;
    for (float i = 0.0f; i < SSSThicknessSamples; ++i) {
        float sampleLength = Hash11(i) * SSSSampleDepth;
        vec3 sampleDir = GenerateSampleVector(neg(norm), i);
        thickness += sampleLength + sceneSDF(C, add(pos, muls(sampleDir, sampleLength))).dist;
    }
    return gclamp(thickness * SSSThicknessSamplesI, 0.0f, 1.0f);
}

/* output_shader.frag:127-176 (Attenuation :161 is computed but unused) */
static vec3 light(const Ctx *C, const Material *mat, vec3 ro, vec3 rd, vec3 p, vec3 n, vec3 phongN) {
    vec3 lightPos = v3(20.0f, 50.0f, 0.0f);
    vec3 lightDir = normalize3(sub(lightPos, p));
    float occ = ambientOcclusionReal(C, p, n);
    if (C->settle) C->settle->back = dot3(normalize3(sub(lightPos, p)), phongN) < 0.0f;
    float sha = softshadow2(C, p, lightDir, 0.01f, length3(sub(lightPos, p)), 4.0f);
    if (C->settle) C->settle->back = 0;
    float sky = gclamp(0.5f + 0.5f * n.y, 0.0f, 1.0f);
    float ind = gclamp(dot3(n, normalize3(mul(lightDir, v3(-1.0f, 0.0f, -1.0f)))), 0.0f, 1.0f);
    vec3 shading = phongContribForLight(v3(1.64f, 1.27f, 0.99f), mat->specular, mat->shininess, p, ro,
                                        lightPos, v3s(1.0f), phongN);
    shading = mul(shading, v3(powf(sha, 1.0f), powf(sha, 1.2f), powf(sha, 1.5f)));
    shading = add(shading, muls(muls(v3(0.16f, 0.20f, 0.28f), sky), occ));
    shading = add(shading, muls(muls(v3(0.40f, 0.28f, 0.20f), ind), occ));
    float SSSAmbient = 0.3f;
    float SSSDistortion = 0.6f;
    float SSSPower = 1.1f;
    float SSSScale = 0.3f;
    float thickness = CalculateThickness(C, p, n);
    diag_set(C, C->lvl == 0 ? 1 : 4, thickness, sha, occ, ind);
    vec3 toEye = neg(rd);
    vec3 SSSLight = add(lightDir, muls(n, SSSDistortion));
    float SSSDot = powf(gclamp(dot3(toEye, neg(SSSLight)), 0.0f, 1.0f), SSSPower) * SSSScale;
    float SSS = (SSSDot + SSSAmbient) * thickness;
    shading = add(shading, v3s(SSS));
    vec3 color = add(mul(mat->diffuse, shading), mat->emission);
    color = applyScattering(color, ro, p, FOG, v3s(2.0f), v3s(2.0f));
    return color;
}

/* output_shader.frag:178-182 */
static vec3 background(vec3 ro, vec3 rd) {
    return applyScattering(v3s(0.0f), ro, add(ro, muls(rd, ZFAR)), FOG, v3s(2.0f), v3s(2.0f));
}

/* output_shader.frag:218-230 */
static float fresnelReflection(float n2, vec3 normal, vec3 incident, float reflectivity) {
    float r0 = (1.0f - n2) / (1.0f + n2);
    r0 *= r0;
    float x = 1.0f + dot3(normal, incident);
    float r = r0 + (1.0f - r0) * x * x * x * x * x;
    r = (1.0f - reflectivity) * r + reflectivity;
    return r;
}

/* output_shader.frag:246-262 (MAX_REFLECTIONS == 1) */
static vec3 renderReflection(const Ctx *C, vec3 ro, vec3 rd) {
    SdResult sd = castRayD(C, ro, rd);
    if (sd.dist > 0.0f) {
        vec3 p = add(ro, muls(rd, sd.dist));
        vec3 n = getNormalFast(C, p);
        diag_set(C, 3, n.x, n.y, n.z, sd.dist);
        vec3 lc = light(C, &sd.mat, ro, rd, p, n, n);
        diag_set(C, 5, lc.x, lc.y, lc.z, 0.0f);
        return lc;
    }
    diag_set(C, 3, 0.0f, 0.0f, 0.0f, -1.0f);
    vec3 bc = background(ro, rd);
    diag_set(C, 5, bc.x, bc.y, bc.z, 0.0f);
    return bc;
}

/* output_shader.frag:298-343 (MAX_REFRACTIONS 4) */
static vec3 renderRefraction(const Ctx *C, vec3 ro, vec3 rd, vec3 absorption) {
    vec3 color = v3s(0.0f);
    float invert = -1.0f;
    float absorb_dist = 0.0f;
    for (int i = 0; i < 4; i++) {
        SdResult sd;
        if (invert < 0.0f) sd = castRayDI(C, ro, rd);
        else sd = castRayD(C, ro, rd);
        if (invert < 0.0f) absorb_dist += sd.dist;
        if (sd.dist < 0.0f) {
            if (invert > 0.0f) color = add(color, background(ro, rd));
            break;
        }
        vec3 p = add(ro, muls(rd, sd.dist));
        vec3 g = getNormalFast(C, p);
        vec3 n = muls(g, invert);
        vec3 ref = reflect3(rd, n);
        /* light()'s phong recomputes getNormalFast(p) == g (not n) */
        color = add(color, light(C, &sd.mat, ro, ref, p, n, g));
        if (invert > 0.0f) break;
        float ior = invert < 0.0f ? sd.mat.refraction_index : 1.0f / sd.mat.refraction_index;
        vec3 raf = refract3(rd, n, ior);
        int tif = raf.x == 0.0f && raf.y == 0.0f && raf.z == 0.0f;
        rd = tif ? ref : raf;
        ro = add(p, muls(rd, 0.01f / fabsf(dot3(rd, n))));
        invert = tif ? invert : invert * -1.0f;
    }
    return mul(color, v3(expf(-absorption.x * absorb_dist), expf(-absorption.y * absorb_dist),
                         expf(-absorption.z * absorb_dist)));
}

/* output_shader.frag:348-385 */
static vec3 render_O(const Ctx *C, vec3 ro, vec3 rd) {
    SdResult sd = castRayD(C, ro, rd);
    if (sd.dist > 0.0f) {
        vec3 p = add(ro, muls(rd, sd.dist));
        vec3 n = getNormalFast(C, p);
        diag_set(C, 0, n.x, n.y, n.z, sd.dist);
        vec3 color = light(C, &sd.mat, ro, rd, p, n, n);
        float reflect_factor = fresnelReflection(sd.mat.refraction_index, n, rd,
                                                 sd.mat.transparency > 0.0f ? 0.0f : sd.mat.reflectivity);
        float refract_factor = 1.0f - reflect_factor;
        diag_set(C, 2, color.x, color.y, color.z, reflect_factor);
        ((Ctx *)C)->lvl = 1;
        if (sd.mat.reflectivity > 0.0f) {
            vec3 reflected_rd = reflect3(rd, n);
            vec3 rc = renderReflection(C, add(p, muls(reflected_rd, 0.001f)), reflected_rd);
            color = add(color, muls(muls(rc, reflect_factor), sd.mat.reflectivity));
        }
        if (sd.mat.transparency > 0.0f) {
            vec3 refracted_rd = refract3(rd, n, 1.0f / sd.mat.refraction_index);
            vec3 rc = renderRefraction(C, add(p, muls(refracted_rd, 0.001f)), refracted_rd, sd.mat.absorption);
            color = add(color, muls(muls(rc, refract_factor), sd.mat.transparency));
        }
        diag_set(C, 6, color.x, color.y, color.z, 0.0f);
        return color;
    }
    return background(ro, rd);
}

/* ---------------------------------------------------- scene T (template) */

/* template.frag:45-76 */
static vec3 render_T(const Ctx *C, vec3 ro, vec3 rd) {
    vec3 p = castRay(C, ro, rd, 0);
    vec3 n = getNormalFast(C, p);
    vec3 c = getColorReflect(C, p, n, rd);
    vec3 lightPos = v3(20.0f, 50.0f, 0.0f);
    vec3 lightDir = normalize3(sub(lightPos, p));
    float occ = ambientOcclusionReal(C, p, n);
    if (C->settle) C->settle->back = dot3(normalize3(sub(lightPos, p)), n) < 0.0f;
    float sha = softshadow2(C, p, lightDir, 0.01f, length3(sub(lightPos, p)), 4.0f);
    if (C->settle) C->settle->back = 0;
    float sky = gclamp(0.5f + 0.5f * n.y, 0.0f, 1.0f);
    float ind = gclamp(dot3(n, normalize3(mul(lightDir, v3(-1.0f, 0.0f, -1.0f)))), 0.0f, 1.0f);
    float fre = powf(gclamp(1.0f + dot3(n, rd), 0.0f, 1.0f), 2.0f);
    vec3 shading = phongContribForLight(v3(1.64f, 1.27f, 0.99f), v3(1.0f, 1.0f, 0.0f), 1280.0f, p, ro, lightPos,
                                        v3s(1.0f), n);
    shading = mul(shading, v3(powf(sha, 1.0f), powf(sha, 1.2f), powf(sha, 1.5f)));
    shading = add(shading, muls(muls(v3(0.16f, 0.20f, 0.28f), sky), occ));
    shading = add(shading, muls(muls(v3(0.40f, 0.28f, 0.20f), ind), occ));
    shading = add(shading, muls(muls(v3s(1.0f), fre), occ));
    c = mul(c, shading);
    c = applyScattering(c, ro, p, FOG, v3s(2.0f), v3s(2.0f));
    return c;
}

/* ------------------------------------------- scene S0 (BASELINE config 1) */

/* castRayD + tetrahedral normal + 0.1-ambient lambert from the scene light;
 * background() on a miss.  Defined in DESIGN.md (not a reference scene). */
static vec3 render_S0(const Ctx *C, vec3 ro, vec3 rd) {
    SdResult sd = castRayD(C, ro, rd);
    if (sd.dist > 0.0f) {
        vec3 p = add(ro, muls(rd, sd.dist));
        vec3 n = getNormalFast(C, p);
        vec3 lightDir = normalize3(sub(v3(20.0f, 50.0f, 0.0f), p));
        return muls(sd.mat.diffuse, 0.1f + lambert(lightDir, n));
    }
    return background(ro, rd);
}

/* ------------------------------------------------------------ main() */

/* output_shader.frag:388-420 / template.frag:78-99, at pixel (col,row) of a
 * W x H target: gl_TexCoord = ((col+.5)/W, (row+.5)/H) (row 0 first in
 * memory). */
static void shade_pixel(const Ctx *C, int W, int H, int col, int row, float *out4) {
    vec2 tc = {((float)col + 0.5f + C->u.jit_x) / (float)W, ((float)row + 0.5f + C->u.jit_y) / (float)H};
    vec2 uv = {(tc.x - 0.5f) * C->u.res_x / C->u.res_y, (tc.y - 0.5f) * C->u.res_y / C->u.res_y};
    vec3 ro = v3(C->u.pos_x, C->u.pos_y, C->u.pos_z);
    vec3 rd = normalize3(v3(uv.x, -uv.y, -1.0f));
    /* rd.yz *= rot(-u_mouse.y); rd.xz *= rot(u_mouse.x)   (common.frag:1088-1092) */
    float a = -C->u.mouse_y;
    float s = glsl_sin(a), c = glsl_cos(a);
    float y = rd.y * c + rd.z * -s;
    float z = rd.y * s + rd.z * c;
    rd.y = y; rd.z = z;
    a = C->u.mouse_x;
    s = glsl_sin(a); c = glsl_cos(a);
    float x = rd.x * c + rd.z * -s;
    z = rd.x * s + rd.z * c;
    rd.x = x; rd.z = z;
    vec3 col3;
    switch (C->scene) {
    case SCENE_S0: col3 = render_S0(C, ro, rd); break;
    case SCENE_T: col3 = render_T(C, ro, rd); break;
    default: col3 = render_O(C, ro, rd); break;
    }
    col3 = tonemap(col3);
    col3 = contrast(col3);
    col3 = vignette(col3, tc);
    out4[0] = col3.x; out4[1] = col3.y; out4[2] = col3.z; out4[3] = 1.0f;
}

static void init_ctx(Ctx *C, int scene, const oracle_uniforms *u) {
    memset(C, 0, sizeof(*C));
    C->scene = scene;
    C->u = *u;
    /* transformR(p - vec3(0,3,0), vec3(180, u_time * 2, 0)) (output_shader.frag:42,
     * template.frag:41): rotationY(-rot.y), rotationX(-rot.x), rotationZ(-rot.z) */
    float rot_x = 180.0f, rot_y = u->time * 2.0f, rot_z = 0.0f;
    float ay = radians(-rot_y), ax = radians(-rot_x), az = radians(-rot_z);
    C->ry_c = glsl_cos(ay); C->ry_s = glsl_sin(ay);
    C->rx_c = glsl_cos(ax); C->rx_s = glsl_sin(ax);
    C->rz_c = glsl_cos(az); C->rz_s = glsl_sin(az);
}

/* ---------------------------------------------------------- exported API */

/* Render rows [row0, row0+nrows) of a W x H frame into out (nrows*W*4 f32,
 * row-major RGBA).  evals (optional, nrows*W u32) gets the per-pixel count of
 * sceneSDF calls.  Rows are distributed dynamically over OpenMP threads. */
int oracle_render(int scene, const oracle_uniforms *u, int W, int H, int row0, int nrows, float *out,
                  uint32_t *evals) {
    if (!u || !out || W <= 0 || H <= 0 || row0 < 0 || nrows < 0 || row0 + nrows > H) return 1;
    if (scene < SCENE_S0 || scene > SCENE_OG) return 2;
#pragma omp parallel for schedule(dynamic, 1)
    for (int r = 0; r < nrows; r++) {
        Ctx C;
        uint64_t cnt = 0;
        init_ctx(&C, scene, u);
        C.evals = &cnt;
        for (int x = 0; x < W; x++) {
            uint64_t before = cnt;
            shade_pixel(&C, W, H, x, row0 + r, out + ((size_t)r * W + x) * 4);
            if (evals) evals[(size_t)r * W + x] = (uint32_t)(cnt - before);
        }
    }
    return 0;
}

/* Render an explicit list of rows (used for strided CPU-baseline samples). */
int oracle_render_rows(int scene, const oracle_uniforms *u, int W, int H, const int32_t *rows, int nrows,
                       float *out, uint32_t *evals) {
    if (!u || !out || !rows || W <= 0 || H <= 0 || nrows < 0) return 1;
    if (scene < SCENE_S0 || scene > SCENE_OG) return 2;
    for (int i = 0; i < nrows; i++)
        if (rows[i] < 0 || rows[i] >= H) return 1;
#pragma omp parallel for schedule(dynamic, 1)
    for (int r = 0; r < nrows; r++) {
        Ctx C;
        uint64_t cnt = 0;
        init_ctx(&C, scene, u);
        C.evals = &cnt;
        for (int x = 0; x < W; x++) {
            uint64_t before = cnt;
            shade_pixel(&C, W, H, x, rows[r], out + ((size_t)r * W + x) * 4);
            if (evals) evals[(size_t)r * W + x] = (uint32_t)(cnt - before);
        }
    }
    return 0;
}

/* Render an explicit list of pixels (x, y) = (xy[2i], xy[2i+1]) of a W x H
 * frame: out n*4 f32, evals (optional) n u32.  Full-size parity samples that
 * are not whole rows (column-strided blocks). */
int oracle_render_pixels(int scene, const oracle_uniforms *u, int W, int H, const int32_t *xy, int n, float *out,
                         uint32_t *evals) {
    if (!u || !out || !xy || W <= 0 || H <= 0 || n < 0) return 1;
    if (scene < SCENE_S0 || scene > SCENE_OG) return 2;
    for (int i = 0; i < n; i++)
        if (xy[2 * i] < 0 || xy[2 * i] >= W || xy[2 * i + 1] < 0 || xy[2 * i + 1] >= H) return 1;
#pragma omp parallel for schedule(dynamic, 64)
    for (int i = 0; i < n; i++) {
        Ctx C;
        uint64_t cnt = 0;
        init_ctx(&C, scene, u);
        C.evals = &cnt;
        shade_pixel(&C, W, H, xy[2 * i], xy[2 * i + 1], out + (size_t)i * 4);
        if (evals) evals[i] = (uint32_t)cnt;
    }
    return 0;
}

/* Soft-shadow settle analysis (analysis aid) over rows [row0, row0+nrows),
 * the rule tested on every `every`-th step of a march (the kernels' period):
 * out[7] = marches, steps, steps after the settle point, settled marches,
 * violations (res changed or occluded after settling; a scene-T reflection
 * march past depth 3 whose clamp factor is not 1), scene T's reflection-march
 * steps begun at depth >= 3 (the kernels' reflection stop), the shadow-march
 * steps of points facing away from the light (phong's dotLN < 0: the shadow
 * factor multiplies 0; the kernels skip these marches).  Settle steps are
 * counted for the other marches only. */
int oracle_shadow_settle(int scene, const oracle_uniforms *u, int W, int H, int row0, int nrows, int every,
                         uint64_t *out) {
    if (!u || !out || W <= 0 || H <= 0 || row0 < 0 || nrows < 0 || row0 + nrows > H || every < 1) return 1;
    uint64_t acc[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma omp parallel for schedule(dynamic, 1)
    for (int r = 0; r < nrows; r++) {
        Ctx C;
        uint64_t cnt = 0;
        SettleRec S = {0, 0, 0, 0, 0, every, 0, 0, 0};
        float px[4];
        init_ctx(&C, scene, u);
        C.evals = &cnt;
        C.settle = &S;
        for (int x = 0; x < W; x++) shade_pixel(&C, W, H, x, row0 + r, px);
#pragma omp critical
        {
            acc[0] += S.marches; acc[1] += S.steps; acc[2] += S.after; acc[3] += S.settled; acc[4] += S.violations;
            acc[5] += S.refl_after;
            acc[6] += S.back_steps;
        }
    }
    for (int i = 0; i < 7; i++) out[i] = acc[i];
    return 0;
}

/* Per-pixel sceneSDF segments (analysis aid): seg = nrows*W*MAX_SEG*2 u16,
 * nseg = nrows*W u8. */
int oracle_render_segments(int scene, const oracle_uniforms *u, int W, int H, int row0, int nrows, uint16_t *seg,
                           uint8_t *nseg) {
    if (!u || !seg || !nseg || W <= 0 || H <= 0 || row0 < 0 || nrows < 0 || row0 + nrows > H) return 1;
#pragma omp parallel for schedule(dynamic, 1)
    for (int r = 0; r < nrows; r++) {
        Ctx C;
        uint64_t cnt = 0;
        SegRec rec;
        float px[4];
        init_ctx(&C, scene, u);
        C.evals = &cnt;
        C.rec = &rec;
        for (int x = 0; x < W; x++) {
            size_t i = (size_t)r * W + x;
            memset(&rec, 0, sizeof(rec));
            rec.out = seg + i * MAX_SEG * 2;
            memset(rec.out, 0, MAX_SEG * 2 * sizeof(uint16_t));
            shade_pixel(&C, W, H, x, row0 + r, px);
            nseg[i] = (uint8_t)rec.nseg;
        }
    }
    return 0;
}

/* Scene-O diagnostic channels (N_DIAG vec4 per pixel, -9 = unset) of rows
 * [row0, row0+nrows), plus the image (out, may be NULL) -- test aid. */
int oracle_render_diag(int scene, const oracle_uniforms *u, int W, int H, int row0, int nrows, float *diag,
                       float *out) {
    if (!u || !diag || W <= 0 || H <= 0 || row0 < 0 || nrows < 0 || row0 + nrows > H) return 1;
    if (scene != SCENE_O && scene != SCENE_OG) return 2;
#pragma omp parallel for schedule(dynamic, 1)
    for (int r = 0; r < nrows; r++) {
        Ctx C;
        uint64_t cnt = 0;
        float px[4];
        init_ctx(&C, scene, u);
        C.evals = &cnt;
        for (int x = 0; x < W; x++) {
            size_t i = (size_t)r * W + x;
            C.diag = diag + i * 4 * N_DIAG;
            C.lvl = 0;
            for (int k = 0; k < 4 * N_DIAG; k++) C.diag[k] = -9.0f;
            shade_pixel(&C, W, H, x, row0 + r, out ? out + i * 4 : px);
        }
    }
    return 0;
}

/* Scene distance at explicit points (n x 3 in, n out) — KAT entry. */
int oracle_scene_dist(int scene, const oracle_uniforms *u, const float *pts, int n, float *out) {
    Ctx C;
    uint64_t cnt = 0;
    init_ctx(&C, scene, u);
    C.evals = &cnt;
    for (int i = 0; i < n; i++) out[i] = sceneSDF(&C, v3(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2])).dist;
    return 0;
}

/* Normal at explicit points — KAT entry. */
int oracle_normal(int scene, const oracle_uniforms *u, const float *pts, int n, float *out) {
    Ctx C;
    uint64_t cnt = 0;
    init_ctx(&C, scene, u);
    C.evals = &cnt;
    for (int i = 0; i < n; i++) {
        vec3 g = getNormalFast(&C, v3(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]));
        out[3 * i] = g.x; out[3 * i + 1] = g.y; out[3 * i + 2] = g.z;
    }
    return 0;
}

/* OpenMP threads a render uses (reported as the CPU baseline's core count). */
int oracle_num_threads(void) { return omp_get_max_threads(); }

/* Built-in KATs: name -> f(x, y, z) */
float oracle_glsl_mod(float x, float y) { return gmod(x, y); }
float oracle_glsl_smoothstep(float a, float b, float x) { return gsmoothstep(a, b, x); }
float oracle_sdbox(float px, float py, float pz, float bx, float by, float bz) { return sdBox(v3(px, py, pz), v3(bx, by, bz)); }
float oracle_sphere(float px, float py, float pz, float sx, float sy, float sz, float sw) { return sphere(sx, sy, sz, sw, v3(px, py, pz)); }
float oracle_cube(float px, float py, float pz, float sx, float sy, float sz, float sw) { return cube(sx, sy, sz, sw, v3(px, py, pz)); }
float oracle_menger(float px, float py, float pz) { return mengersponge_x(v3(px, py, pz)); }
float oracle_smin_cubic(float a, float b, float k) {
    SdResult ra, rb;
    memset(&ra, 0, sizeof(ra)); memset(&rb, 0, sizeof(rb));
    ra.dist = a; rb.dist = b;
    return sminCubic(&ra, &rb, k).dist;
}
float oracle_hash11(float p) { return Hash11(p); }

/* ------------------------------------------------ post.frag FXAA pass */

/* The FXAA pass (post.frag:16-61, main :135-144) as the reference runs it on
 * its RGBA8 render target: texture() with the sampler state SFML leaves on an
 * sf::RenderTexture (no setSmooth: GL_NEAREST; not repeated: CLAMP_TO_EDGE),
 * u_resolution = (W, H) (main.cpp:58), unorm8 -> float c/255 on fetch and
 * float -> unorm8 round-to-nearest on store.  Images are row 0 first, as the
 * ray-march output. */
typedef struct { float r, g, b, a; } rgba;
#ifndef UNORM_K
#define UNORM_K (1.0f / 255.0f)
#endif

static rgba tex_nearest(const uint32_t *img, int W, int H, vec2 uv) {
    int x = (int)floorf(uv.x * (float)W);
    int y = (int)floorf(uv.y * (float)H);
    x = x < 0 ? 0 : (x >= W ? W - 1 : x);
    y = y < 0 ? 0 : (y >= H ? H - 1 : y);
    uint32_t v = img[(size_t)y * W + x];
    const float k = UNORM_K;
    rgba c = {(float)(v & 255u) * k, (float)((v >> 8) & 255u) * k, (float)((v >> 16) & 255u) * k,
              (float)(v >> 24) * k};
    return c;
}

static vec3 rgb_of(rgba c) { return v3(c.r, c.g, c.b); }
static vec2 v2(float x, float y) { vec2 r = {x, y}; return r; }

/* post.frag:16-61 */
static rgba fxaa(const uint32_t *tex, int W, int H, vec2 fragCoord, vec2 resolution) {
    const float FXAA_REDUCE_MIN = 1.0f / 128.0f, FXAA_REDUCE_MUL = 1.0f / 8.0f, FXAA_SPAN_MAX = 8.0f;
    vec2 iv = v2(1.0f / resolution.x, 1.0f / resolution.y);
    vec3 rgbNW = rgb_of(tex_nearest(tex, W, H, v2(fragCoord.x + -1.0f * iv.x, fragCoord.y + -1.0f * iv.y)));
    vec3 rgbNE = rgb_of(tex_nearest(tex, W, H, v2(fragCoord.x + 1.0f * iv.x, fragCoord.y + -1.0f * iv.y)));
    vec3 rgbSW = rgb_of(tex_nearest(tex, W, H, v2(fragCoord.x + -1.0f * iv.x, fragCoord.y + 1.0f * iv.y)));
    vec3 rgbSE = rgb_of(tex_nearest(tex, W, H, v2(fragCoord.x + 1.0f * iv.x, fragCoord.y + 1.0f * iv.y)));
    rgba texColor = tex_nearest(tex, W, H, fragCoord);
    vec3 rgbM = rgb_of(texColor);
    vec3 luma = v3(0.299f, 0.587f, 0.114f);
    float lumaNW = dot3(rgbNW, luma), lumaNE = dot3(rgbNE, luma), lumaSW = dot3(rgbSW, luma);
    float lumaSE = dot3(rgbSE, luma), lumaM = dot3(rgbM, luma);
    float lumaMin = gmin(lumaM, gmin(gmin(lumaNW, lumaNE), gmin(lumaSW, lumaSE)));
    float lumaMax = gmax(lumaM, gmax(gmax(lumaNW, lumaNE), gmax(lumaSW, lumaSE)));
    vec2 dir = v2(-((lumaNW + lumaNE) - (lumaSW + lumaSE)), ((lumaNW + lumaSW) - (lumaNE + lumaSE)));
    float dirReduce = gmax((lumaNW + lumaNE + lumaSW + lumaSE) * (0.25f * FXAA_REDUCE_MUL), FXAA_REDUCE_MIN);
    float rcpDirMin = 1.0f / (gmin(fabsf(dir.x), fabsf(dir.y)) + dirReduce);
    dir = v2(gmin(FXAA_SPAN_MAX, gmax(-FXAA_SPAN_MAX, dir.x * rcpDirMin)) * iv.x,
             gmin(FXAA_SPAN_MAX, gmax(-FXAA_SPAN_MAX, dir.y * rcpDirMin)) * iv.y);
    const float k1 = 1.0f / 3.0f - 0.5f, k2 = 2.0f / 3.0f - 0.5f;
    vec3 s1 = rgb_of(tex_nearest(tex, W, H, v2(fragCoord.x + dir.x * k1, fragCoord.y + dir.y * k1)));
    vec3 s2 = rgb_of(tex_nearest(tex, W, H, v2(fragCoord.x + dir.x * k2, fragCoord.y + dir.y * k2)));
    vec3 rgbA = muls(add(s1, s2), 0.5f);
    vec3 s3 = rgb_of(tex_nearest(tex, W, H, v2(fragCoord.x + dir.x * -0.5f, fragCoord.y + dir.y * -0.5f)));
    vec3 s4 = rgb_of(tex_nearest(tex, W, H, v2(fragCoord.x + dir.x * 0.5f, fragCoord.y + dir.y * 0.5f)));
    vec3 rgbB = add(muls(rgbA, 0.5f), muls(add(s3, s4), 0.25f));
    float lumaB = dot3(rgbB, luma);
    rgba color;
    vec3 c = (lumaB < lumaMin || lumaB > lumaMax) ? rgbA : rgbB;
    color.r = c.x; color.g = c.y; color.b = c.z; color.a = texColor.a;
    return color;
}

static uint32_t unorm8(float c) {
    c = c < 0.0f ? 0.0f : (c > 1.0f ? 1.0f : c);
    if (c != c) c = 0.0f;
    return (uint32_t)lrintf(c * 255.0f);
}

/* post.frag:135-144: uv = (tc.x, 1 - tc.y); out = fxaa(u_main_tex, uv, res).
 * out: RGBA8 words (may be NULL); out_f32: the float gl_FragColor (may be NULL). */
int oracle_fxaa(int W, int H, const uint32_t *in, uint32_t *out, float *out_f32) {
    if (!in || W <= 0 || H <= 0) return 1;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            vec2 tc = v2(((float)x + 0.5f) / (float)W, ((float)y + 0.5f) / (float)H);
            rgba c = fxaa(in, W, H, v2(tc.x, 1.0f - tc.y), v2((float)W, (float)H));
            size_t i = (size_t)y * W + x;
            if (out) out[i] = unorm8(c.r) | (unorm8(c.g) << 8) | (unorm8(c.b) << 16) | (unorm8(c.a) << 24);
            if (out_f32) { out_f32[4 * i] = c.r; out_f32[4 * i + 1] = c.g; out_f32[4 * i + 2] = c.b; out_f32[4 * i + 3] = c.a; }
        }
    return 0;
}

/* ---------------------------------------------------------------- bloom
 * shaders/post/bloom.frag:14-43 over postTexture as PostBloom::apply
 * (source/post_bloom.cpp:9-13) samples it after setSmooth(true) +
 * generateMipmap() (main.cpp:212-214): MIN LINEAR_MIPMAP_LINEAR, MAG LINEAR,
 * CLAMP_TO_EDGE.  Mip level k+1 (max(1, w>>1) x max(1, h>>1)) is the bilinear
 * resample of level k at its texel centres in the 0..255 domain, rounded to
 * nearest-even: SwiftShader's glGenerateMipmap bit for bit on the even-sized
 * goldens (tests/test_bloom.py). */

/* level k (w x h) -> level k+1 */
int oracle_mip_down(int w, int h, const uint32_t *in, uint32_t *out) {
    if (!in || !out || w <= 0 || h <= 0) return 1;
    const int w1 = w > 1 ? w >> 1 : 1, h1 = h > 1 ? h >> 1 : 1;
    const float sx = (float)w / (float)w1, sy = (float)h / (float)h1;
    for (int y = 0; y < h1; y++) {
        float v = ((float)y + 0.5f) * sy - 0.5f;
        float fy = floorf(v), b = v - fy;
        int y0 = (int)fy, y1 = y0 + 1;
        y0 = y0 < 0 ? 0 : (y0 >= h ? h - 1 : y0);
        y1 = y1 < 0 ? 0 : (y1 >= h ? h - 1 : y1);
        for (int x = 0; x < w1; x++) {
            float u = ((float)x + 0.5f) * sx - 0.5f;
            float fx = floorf(u), a = u - fx;
            int x0 = (int)fx, x1 = x0 + 1;
            x0 = x0 < 0 ? 0 : (x0 >= w ? w - 1 : x0);
            x1 = x1 < 0 ? 0 : (x1 >= w ? w - 1 : x1);
            uint32_t t00 = in[(size_t)y0 * w + x0], t01 = in[(size_t)y0 * w + x1];
            uint32_t t10 = in[(size_t)y1 * w + x0], t11 = in[(size_t)y1 * w + x1];
            uint32_t r = 0;
            for (int c = 0; c < 32; c += 8) {
                float c00 = (float)((t00 >> c) & 255u), c01 = (float)((t01 >> c) & 255u);
                float c10 = (float)((t10 >> c) & 255u), c11 = (float)((t11 >> c) & 255u);
                float r0 = (1.0f - a) * c00 + a * c01, r1 = (1.0f - a) * c10 + a * c11;
                float s = (1.0f - b) * r0 + b * r1;
                r |= (uint32_t)lrintf(s) << c;
            }
            out[(size_t)y * w1 + x] = r;
        }
    }
    return 0;
}

/* bilinear fetch of a level (w x h) at normalized (u, v), CLAMP_TO_EDGE.
 * The filter is evaluated as the polynomial of its cell, c00 + a Px + b (Py +
 * a Pxy) with Px = c01 - c00, Py = c10 - c00, Pxy = (c11 - c10) - Px, in three
 * fused multiply-adds per channel (GL leaves a filter's arithmetic to the
 * implementation; SwiftShader filters unorm8 in fixed point, and this form
 * stays within 1 LSB of its output, tests/test_bloom.py).  The HIP path
 * (rm_post.hip) tabulates the same four coefficients per cell and evaluates
 * the same three fmaf: bit-identical. */
static vec3 tex_bilinear(const uint32_t *img, int w, int h, float u, float v) {
    float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
    float fx = floorf(x), fy = floorf(y);
    float a = x - fx, b = y - fy;
    int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
    x0 = x0 < 0 ? 0 : (x0 >= w ? w - 1 : x0);
    x1 = x1 < 0 ? 0 : (x1 >= w ? w - 1 : x1);
    y0 = y0 < 0 ? 0 : (y0 >= h ? h - 1 : y0);
    y1 = y1 < 0 ? 0 : (y1 >= h ? h - 1 : y1);
    const uint32_t t00 = img[(size_t)y0 * w + x0], t01 = img[(size_t)y0 * w + x1];
    const uint32_t t10 = img[(size_t)y1 * w + x0], t11 = img[(size_t)y1 * w + x1];
    float o[3];
    for (int c = 0; c < 3; c++) {
        const int s = 8 * c;
        float c00 = (float)((t00 >> s) & 255u) * UNORM_K, c01 = (float)((t01 >> s) & 255u) * UNORM_K;
        float c10 = (float)((t10 >> s) & 255u) * UNORM_K, c11 = (float)((t11 >> s) & 255u) * UNORM_K;
        const float px = c01 - c00, py = c10 - c00, pxy = (c11 - c10) - px;
        o[c] = fmaf(b, fmaf(a, pxy, py), fmaf(a, px, c00));
    }
    return v3(o[0], o[1], o[2]);
}

/* bloom.frag:33-43 for lod > 0 as the HIP path sums it (rm_post.hip, "bloom.frag:33-43
 * for lod > 0"): with the 25 taps' bilinear cells fixed, the weighted 5 x 5 sum of a level
 * is one bilinear polynomial P00 + P10 s' + P01 t' + P11 s' t' of the pixel's texel-space
 * position (s' = s - cx_2, t' = t - cy_2).  The pixel columns (rows) fall into runs of equal
 * cell tuples; each (column run, row run) pair's polynomial is summed in double with the
 * level's blend weight folded in, then rounded to float.  The same function of the same
 * texels as the per-tap sum, rounded differently (~1e-6); tests/test_bloom.py pins it to
 * SwiftShader.  An axis: n pixels of an N-pixel image over a level of lw texels. */
typedef struct {
    int n, N, lw, is_y;
    float off[5]; /* bloom.frag's offset of tap i: u (i iaspect) scale, v j scale */
} bloom_axis;

static float bloom_coord(const bloom_axis *A, int c) {
    const float t = ((float)c + 0.5f) / (float)A->N;
    return (A->is_y ? 1.0f - t : t) * (float)A->lw - 0.5f;
}

static int bloom_cell(const bloom_axis *A, float coord, int i) {
    const double d = (double)A->off[i] * (double)A->lw;
    const double x = floor((double)coord + d);
    return x < -1.0 ? -1 : (x > (double)(A->lw - 1) ? A->lw - 1 : (int)x);
}

/* per pixel (sub[c], run[c]); per run its five cells; returns the number of runs */
static int bloom_runs(const bloom_axis *A, float *sub, int *run, int *tup) {
    int prev = -1, r = -1;
    for (int c = 0; c < A->n; c++) {
        const float coord = bloom_coord(A, c);
        int cell[5], k = 0;
        for (int i = 0; i < 5; i++) {
            cell[i] = bloom_cell(A, coord, i);
            k += cell[i] + 1;
        }
        if (k != prev) {
            r++;
            for (int i = 0; i < 5; i++) tup[r * 5 + i] = cell[i];
        }
        prev = k;
        sub[c] = coord - (float)cell[2];
        run[c] = r;
    }
    return r + 1;
}

static const float BLOOM_G[3][3] = {{41.0f / 273.0f, 26.0f / 273.0f, 7.0f / 273.0f},
                                    {26.0f / 273.0f, 16.0f / 273.0f, 4.0f / 273.0f},
                                    {7.0f / 273.0f, 4.0f / 273.0f, 1.0f / 273.0f}};

/* the polynomial of one run pair: out[12] = P00 rgb, P10 rgb, P01 rgb, P11 rgb, times lam */
static void bloom_poly(const uint32_t *L, const bloom_axis *X, const bloom_axis *Y, const int *cx, const int *cy,
                       double lam, float *out) {
    const int w = X->lw, h = Y->lw;
    double e[5], f[5], P[12] = {0};
    for (int i = 0; i < 5; i++) {
        e[i] = ((double)cx[2] + (double)X->off[i] * (double)w) - (double)cx[i];
        f[i] = ((double)cy[2] + (double)Y->off[i] * (double)h) - (double)cy[i];
    }
    for (int j = 0; j < 5; j++) { /* tap row j summed alone (in i order), then the rows in j order */
        double R[12] = {0};
        const int y0 = cy[j] < 0 ? 0 : (cy[j] > h - 1 ? h - 1 : cy[j]);
        const int y1 = cy[j] + 1 < 0 ? 0 : (cy[j] + 1 > h - 1 ? h - 1 : cy[j] + 1);
        for (int i = 0; i < 5; i++) {
            const int x0 = cx[i] < 0 ? 0 : (cx[i] > w - 1 ? w - 1 : cx[i]);
            const int x1 = cx[i] + 1 < 0 ? 0 : (cx[i] + 1 > w - 1 ? w - 1 : cx[i] + 1);
            const uint32_t t00 = L[(size_t)y0 * w + x0], t01 = L[(size_t)y0 * w + x1];
            const uint32_t t10 = L[(size_t)y1 * w + x0], t11 = L[(size_t)y1 * w + x1];
            const double g = (double)BLOOM_G[abs(i - 2)][abs(j - 2)];
            for (int c = 0; c < 3; c++) {
                const int s = 8 * c;
                /* texel units (0..255): 1/255 goes with the blend weight */
                const double c00 = (double)((t00 >> s) & 255u), c01 = (double)((t01 >> s) & 255u);
                const double c10 = (double)((t10 >> s) & 255u), c11 = (double)((t11 >> s) & 255u);
                const double px = c01 - c00, py = c10 - c00, pxy = (c11 - c10) - px;
                R[c] += g * (((c00 + e[i] * px) + f[j] * py) + (e[i] * f[j]) * pxy);
                R[3 + c] += g * (px + f[j] * pxy);
                R[6 + c] += g * (py + e[i] * pxy);
                R[9 + c] += g * pxy;
            }
        }
        for (int q = 0; q < 12; q++) P[q] += R[q];
    }
    const double scale = lam * (1.0 / 255.0);
    for (int q = 0; q < 12; q++) out[q] = (float)(P[q] * scale);
}

/* the two levels' run tables of one image (lod > 0) */
typedef struct {
    float *sub[4];
    int *run[4], *tup[4], nruns[4];
    float *tab[2];
} bloom_runs_t;

/* The levels bloom.frag reads: textureLod at lod = log2(0.05 * u_resolution.y)
 * (bloom.frag:22, u_resolution = the image size, post_bloom.cpp:6) blends
 * levels d1 = floor(lod) and d2 = d1 + 1, both clamped to the last level q
 * (GL ES 3.0 3.8.10.4).  Returns 1 + d2, the number of levels used. */
int oracle_bloom_levels(int W, int H, float *lod, int *d1, int *d2) {
    int q = 0;
    for (int m = W > H ? W : H; m > 1; m >>= 1) q++;
    const float l = log2f(0.05f * (float)H);
    int a = 0, b = 0;
    if (l > 0.0f) {
        a = (int)floorf(l);
        a = a > q ? q : a;
        b = a + 1 > q ? q : a + 1;
    }
    if (lod) *lod = l;
    if (d1) *d1 = a;
    if (d2) *d2 = b;
    return b + 1;
}

/* bloom.frag:33-43 at output pixel (x, y); levels[k] is lw[k] x lh[k]; B = the run
 * tables when lod > 0 */
static uint32_t bloom_pixel(const uint32_t *const *levels, const int *lw, const int *lh, int W, int H, int x, int y,
                            float lod, const bloom_runs_t *B) {
    const float tcx = ((float)x + 0.5f) / (float)W, tcy = ((float)y + 0.5f) / (float)H;
    const float u = tcx, v = 1.0f - tcy; /* bloom.frag:36 */
    vec3 color = tex_bilinear(levels[0], lw[0], lh[0], u, v);
    const float scale = 0.05f, iaspect = (float)H / (float)W;
    vec3 bl = v3(0.0f, 0.0f, 0.0f);
    if (lod <= 0.0f) {
        for (int j = -2; j <= 2; j++) /* bloom.frag:24-26 */
            for (int i = -2; i <= 2; i++) {
                const float uu = u + ((float)i * iaspect) * scale, vv = v + (float)j * scale;
                const float g = BLOOM_G[abs(i)][abs(j)];
                const vec3 s = tex_bilinear(levels[0], lw[0], lh[0], uu, vv);
                bl = v3(fmaf(g, s.x, bl.x), fmaf(g, s.y, bl.y), fmaf(g, s.z, bl.z));
            }
    } else {
        float val[2][3];
        for (int l = 0; l < 2; l++) {
            const float sx = B->sub[2 * l][x], sy = B->sub[2 * l + 1][y];
            const float *q = B->tab[l] + ((size_t)B->run[2 * l + 1][y] * B->nruns[2 * l] + B->run[2 * l][x]) * 12;
            for (int c = 0; c < 3; c++) val[l][c] = fmaf(fmaf(q[9 + c], sx, q[6 + c]), sy, fmaf(q[3 + c], sx, q[c]));
        }
        bl = v3(val[0][0] + val[1][0], val[0][1] + val[1][1], val[0][2] + val[1][2]);
    }
    color = v3(color.x + gmax(bl.x - 0.3f, 0.0f), color.y + gmax(bl.y - 0.3f, 0.0f),
               color.z + gmax(bl.z - 0.3f, 0.0f)); /* bloom.frag:28,41 (intensity 1) */
    return unorm8(color.x) | (unorm8(color.y) << 8) | (unorm8(color.z) << 16) | (255u << 24);
}

/* mips: optional buffer receiving levels 1..d2 packed one after the other
 * (the HIP path's layout); NULL = internal scratch */
int oracle_bloom(int W, int H, const uint32_t *in, uint32_t *out, uint32_t *mips) {
    if (!in || !out || W <= 0 || H <= 0) return 1;
    float lod;
    int d1, d2;
    const int nl = oracle_bloom_levels(W, H, &lod, &d1, &d2);
    const uint32_t *levels[40];
    int lw[40], lh[40];
    size_t total = 0;
    lw[0] = W;
    lh[0] = H;
    for (int k = 1; k < nl; k++) {
        lw[k] = lw[k - 1] > 1 ? lw[k - 1] >> 1 : 1;
        lh[k] = lh[k - 1] > 1 ? lh[k - 1] >> 1 : 1;
        total += (size_t)lw[k] * lh[k];
    }
    uint32_t *buf = mips ? mips : (uint32_t *)malloc((total ? total : 1) * sizeof(uint32_t));
    if (!buf) return 2;
    levels[0] = in;
    size_t off = 0;
    for (int k = 1; k < nl; k++) {
        oracle_mip_down(lw[k - 1], lh[k - 1], levels[k - 1], buf + off);
        levels[k] = buf + off;
        off += (size_t)lw[k] * lh[k];
    }
    bloom_runs_t B;
    memset(&B, 0, sizeof(B));
    int bad = 0;
    if (lod > 0.0f) {
        const float fr = lod - floorf(lod), iaspect = (float)H / (float)W, scale = 0.05f;
        bloom_axis ax[4];
        for (int a = 0; a < 4; a++) {
            const int lvl = a < 2 ? d1 : d2;
            ax[a].is_y = a & 1;
            ax[a].n = ax[a].N = ax[a].is_y ? H : W;
            ax[a].lw = ax[a].is_y ? lh[lvl] : lw[lvl];
            for (int i = 0; i < 5; i++)
                ax[a].off[i] = ax[a].is_y ? (float)(i - 2) * scale : ((float)(i - 2) * iaspect) * scale;
            B.sub[a] = (float *)malloc(sizeof(float) * ax[a].n);
            B.run[a] = (int *)malloc(sizeof(int) * ax[a].n);
            B.tup[a] = (int *)malloc(sizeof(int) * 5 * (size_t)ax[a].n);
            if (!B.sub[a] || !B.run[a] || !B.tup[a]) bad = 1;
            else B.nruns[a] = bloom_runs(&ax[a], B.sub[a], B.run[a], B.tup[a]);
        }
        for (int l = 0; l < 2 && !bad; l++) {
            const int nx = B.nruns[2 * l], ny = B.nruns[2 * l + 1];
            const double lam = l == 0 ? (double)(1.0f - fr) : (double)fr;
            B.tab[l] = (float *)malloc(sizeof(float) * 12 * (size_t)nx * ny);
            if (!B.tab[l]) {
                bad = 1;
                break;
            }
#pragma omp parallel for schedule(static)
            for (int ry = 0; ry < ny; ry++)
                for (int rx = 0; rx < nx; rx++)
                    bloom_poly(levels[l == 0 ? d1 : d2], &ax[2 * l], &ax[2 * l + 1], B.tup[2 * l] + rx * 5,
                               B.tup[2 * l + 1] + ry * 5, lam, B.tab[l] + ((size_t)ry * nx + rx) * 12);
        }
    }
    if (!bad) {
#pragma omp parallel for schedule(static)
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) out[(size_t)y * W + x] = bloom_pixel(levels, lw, lh, W, H, x, y, lod, &B);
    }
    for (int a = 0; a < 4; a++) {
        free(B.sub[a]);
        free(B.run[a]);
        free(B.tup[a]);
    }
    free(B.tab[0]);
    free(B.tab[1]);
    if (!mips) free(buf);
    return bad ? 2 : 0;
}
