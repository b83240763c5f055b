// rm_device.h -- gfx950 device code for the SDF sphere-tracing pass.
//
// Scene distance functions, materials and shading terms of the reference's
// fragment pass (cahekp/Raymarching common.frag + output_shader.frag +
// template.frag), restructured for CDNA4:
//   * per-frame constants (camera rotations, transformR's rotation, the 32
//     Hash11 sample lengths of CalculateThickness) are computed once on the
//     host and arrive in the kernel-argument segment (SGPRs), instead of being
//     rebuilt per sceneSDF call (the reference builds three mat4 per call,
//     common.frag:434-441);
//   * marching loops evaluate the distance-only scene; the 16-float Material
//     of scene O (common.frag:20-35) is evaluated once, at the point where a
//     march stops, which is the point whose SdResult castRayD returns
//     (common.frag:879-901);
//   * phongContribForLight's getNormalFast(p) (common.frag:733) is the normal
//     the caller already holds (same p, pure function) and is reused.
// All arithmetic is IEEE f32 (GLSL float).
#pragma once
#ifdef __HIPCC_RTC__  // compiled by hiprtc (scene plugins, rm_plugin.h)
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#else
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

namespace rm {

// S0/T/O/OG are compiled in; SCENE_PLUGIN is a scene whose sceneSDF comes
// from a HIP source file compiled at rm_load_scene time (rm_plugin.h)
enum SceneId : int { SCENE_S0 = 0, SCENE_T = 1, SCENE_O = 2, SCENE_OG = 3, SCENE_PLUGIN = 4 };

constexpr float ZNEAR = 0.02f;   // common.frag:13
constexpr float ZFAR = 50.0f;    // common.frag:14
constexpr float PI_REF = 3.1416f;  // common.frag:1108

// Per-frame constants. Passed by value as a kernel argument.
struct FrameConst {
    float res_x, res_y;            // u_resolution
    float pos_x, pos_y, pos_z;     // u_pos
    float cam1_c, cam1_s;          // rot(-u_mouse.y): cos, sin
    float cam2_c, cam2_s;          // rot(u_mouse.x)
    float ry_c, ry_s, rx_c, rx_s;  // transformR(.., vec3(180, 2*u_time, 0)): rotationY(-2t), rotationX(-180);
                                   // rotationZ(-0) is the exact identity and is skipped
    int W, H;                      // target size (gl_TexCoord = ((x+.5)/W, (y+.5)/H))
    int cycle, offset, run;        // frame row y is rendered iff (y mod cycle) - offset lies in [0, run): row
                                   // bands dealt round robin (band, nshards, shard) are run = band, cycle =
                                   // band * nshards, offset = band * shard; weighted parts own longer runs
    int nrows;                     // packed rows rendered by this launch
    int row0;                      // first packed row of the shard this launch renders
    int max_steps;                 // MAX_MARCHING_STEPS (common.frag:15), run-time
    int shadow_max_steps;          // step cap; unbounded (INT_MAX), as softshadow2 (common.frag:814), unless set
    float time;                    // u_time
    float mouse_x, mouse_y;        // u_mouse
    float hash11[32];              // Hash11(i), i = 0..31 (output_shader.frag:54-59,102)
    float sss_floor[2][32];        // CalculateThickness at a floor point whose probes are all plane-only and
                                   // whose normal is (0, 1, 0) / (0, 1 - 2^-24, 0): (sampleDir * Hash11(i)).y
    uint32_t* evals_map;           // instrumented launches: sceneSDF calls per pixel (packed rows), or null
    const uint32_t* tile_order;    // workgroup i renders tile tile_order[i] (a permutation), or null: tile i
    uint32_t* tile_cost;           // if set: each one-wave tile's duration in shader clocks (adaptive order)
    int lat_tiles;                 // with tile_order: the first lat_tiles workgroups (the costliest tiles) render
                                   // with the latency-optimized Menger folds (scene T, render_tile)
    int accumulate;                // rm_render_accumulate*: out holds u_sample (this pixel of the previous frame)
                                   // and receives mix(u_sample, colour, sample_part)
    float sample_part;             // u_sample_part
    float jit_x, jit_y;            // with accumulate: sub-pixel offset of the fragment, fract(u_seed1) - 0.5
    uint32_t* persist;             // KERNEL_PERSIST: {next dispatch ordinal, waves done}, zero between launches
    uint32_t run_magic;            // floor(j / run) = umulhi(j, run_magic) for every packed row j, or 0: divide
    uint32_t gx_magic;             // floor(t / tiles_x) = umulhi(t, gx_magic) for every tile t, or 0: divide
};

// Division by a per-launch divisor d (host: div_magic): with m = floor(2^32 / d)
// + 1 = (2^32 + e) / d, e in [1, d], a m / 2^32 = a / d + a e / (d 2^32), which
// stays below the next integer while a e < 2^32; the host sets m only when
// every dividend a of the launch has a d < 2^32 (and d >= 2): one v_mul_hi_u32
// instead of the ~12 VALU of an integer division by a run-time value.
__host__ __device__ inline uint32_t div_magic(uint32_t d, uint64_t a_end) {
    return d >= 2 && a_end * (uint64_t)d < (1ull << 32) ? (uint32_t)((1ull << 32) / d + 1) : 0u;
}
__device__ __forceinline__ int div_by(int a, uint32_t m, int d) {
    return m ? (int)__umulhi((uint32_t)a, m) : a / d;
}

// Buckets of the adaptive dispatch order (rm_capi.cpp, rm_kernels.hip): 256
// logarithmic buckets of a tile's duration, 8 per octave of shader clocks
// (float exponent and 3 mantissa bits), bucket 0 = costliest.
constexpr int kSchedBuckets = 256;
__device__ __forceinline__ int sched_bucket(uint32_t cost) {
    const int b = (int)(__float_as_uint((float)cost + 64.0f) >> 20) - ((127 + 6) << 3);
    return kSchedBuckets - 1 - (b < 0 ? 0 : b > kSchedBuckets - 1 ? kSchedBuckets - 1 : b);
}

// A scene plugin's sceneSDF, bound in the plugin's translation unit
// (rm_plugin.h) by specializing this for SCENE_PLUGIN: dist(p), mat(p), flop.
template <int SC>
struct PluginScene;

// ------------------------------------------------------------- vec3 helpers
struct V3 {
    float x, y, z;
    V3() = default;
    __host__ __device__ constexpr V3(float x_, float y_, float z_) : x(x_), y(y_), z(z_) {}
    __host__ __device__ constexpr explicit V3(float s) : x(s), y(s), z(s) {}
};
__host__ __device__ constexpr V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__host__ __device__ constexpr V3 v3s(float s) { return V3{s, s, s}; }
__host__ __device__ constexpr V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__host__ __device__ constexpr V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__host__ __device__ constexpr V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__host__ __device__ constexpr V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__host__ __device__ constexpr V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float length(V3 a) { return sqrtf(dot(a, a)); }
__device__ __forceinline__ V3 normalize(V3 a) { return a * (1.0f / sqrtf(dot(a, a))); }
// GLSL min/max/clamp by their spec definitions (min(x,y) = y < x ? y : x,
// max(x,y) = x < y ? y : x), which differ from fminf/fmaxf only when x is NaN.
// Shading code uses these (a NaN colour, e.g. pow() of a negative colour in
// the glass test scene, must propagate as in the GLSL); the distance functions
// use fminf/fmaxf, whose operands are never NaN for finite sample points.
__device__ __forceinline__ float gmin(float x, float y) { return y < x ? y : x; }
__device__ __forceinline__ float gmax(float x, float y) { return x < y ? y : x; }
__device__ __forceinline__ float clamp01(float x) { return gmin(gmax(x, 0.0f), 1.0f); }
// GLSL mix as the implementation that renders the golden fixtures evaluates it:
// x + (y - x) a (the spec writes x (1 - a) + y a; bit-exact on 4096 triples,
// tools/ss_probe.py)
__device__ __forceinline__ float gmix(float x, float y, float a) { return x + (y - x) * a; }
__device__ __forceinline__ V3 mix3(V3 x, V3 y, float a) {
    return v3(gmix(x.x, y.x, a), gmix(x.y, y.y, a), gmix(x.z, y.z, a));
}
__device__ __forceinline__ float fract(float x) { return x - floorf(x); }
__device__ __forceinline__ float smoothstep(float e0, float e1, float x) {
    float t = clamp01((x - e0) / (e1 - e0));
    return t * t * (3.0f - 2.0f * t);
}
// reflect(I,N) = I - 2*dot(N,I)*N
__device__ __forceinline__ V3 reflect(V3 I, V3 N) { return I - N * (2.0f * dot(N, I)); }
__device__ __forceinline__ V3 refract(V3 I, V3 N, float eta) {
    float d = dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return v3s(0.0f);
    return I * eta - N * (eta * d + sqrtf(k));
}

// GLSL sin()/cos().  GLSL leaves their precision to the implementation; these
// restate the implementation that renders the golden fixtures (SwiftShader
// 4.1, tests/golden/make_goldens.py): y = x/2pi - round(x/2pi), cos/sin of
// pi*y by two minimax polynomials, the angle doubled twice and renormalized;
// cos(x) = sin(x + 1.57079632).  Bit-exact against it on 8000 arguments
// (tools/ss_probe.py).  Used for the per-frame rotations (camera rot() and
// transformR, computed on the host) and floorMat: a ulp of the sponge rotation
// moves the distances getNormalFast differentiates, and the normal feeds the
// Hash33 of CalculateThickness.  No contraction.
__host__ __device__ inline float glsl_sin(float x) {
#pragma clang fp contract(off)
    float y = x * 1.59154943e-1f;
    y = y - __builtin_rintf(y);
    const float y2 = y * y;
    const float c1 = y2 * (y2 * (y2 * -0.0204391631f + 0.2536086171f) + -1.2336977925f) + 1.0f;
    const float s1 = y * (y2 * (y2 * (y2 * -0.0046075748f + 0.0796819754f) + -0.645963615f) + 1.5707963235f);
    const float c2 = c1 * c1 - s1 * s1;
    const float s2 = 2.0f * s1 * c1;
    return 2.0f * s2 * c2 * (1.0f / (s2 * s2 + c2 * c2));
}
__host__ __device__ inline float glsl_cos(float x) { return glsl_sin(x + 1.57079632f); }

// ------------------------------------------------------------------ SDFs

// Work tally of the instrumented (COUNT) kernels: sceneSDF calls (ray-steps)
// and the FLOP they needed, per term of SURVEY.md 8(d)'s tally (add, sub,
// mul, min, max, cmp, floor = 1, FMA = 2, sqrt not counted).  Terms that an
// exact early exit skips are not counted; the timed kernels never read it.
struct Tally {
    uint32_t evals = 0;
    uint32_t flop = 0;
    uint32_t skipped = 0;  // of evals: steps the timed kernels leave out (exact early exits)
};
constexpr uint32_t FL_SPHERE = 9;      // sphere(): sub 3, dot 5, sub 1 (+ sqrt)
constexpr uint32_t FL_TRANSFORM = 18;  // p - (0,3,0): 3; transformR's 3x3 rotation: 15
constexpr uint32_t FL_LINRAY = 6;      // o + d t in sponge space: 3 FMA
constexpr uint32_t FL_BOX = 17;        // sdBox(p, vec3(1))
constexpr uint32_t FL_FOLD = 40;       // one mengersponge iteration (common.frag:663-676)
constexpr uint32_t FL_CUBE = 21;       // cube()
constexpr uint32_t FL_SMIN = 12;       // sminCubic, distance part
constexpr uint32_t FL_BOUNDS = 16;     // scene O's two Chebyshev bounds and their test

// x / b for a constant b, correctly rounded in all but rare cases: one
// Markstein refinement of x * RN(1/b) (3 VALU ops; the reference's divisions
// are GLSL "/" with <= 2.5 ulp).  Used on the parity-critical scene-O path.
__device__ __forceinline__ float div_const(float x, float b, float rb) {
    float q = x * rb;
    float r = fmaf(-b, q, x);
    return fmaf(r, rb, q);
}

// mengersponge(p).x (common.frag:654-679) with sdBox(p, vec3(1)) (:595-600).
// Per fold, with xh = x*s/2 (exact: x*s*0.5 == x*(s/2)):
//   mod(x*s, 2) - 1 == 2*(xh - floor(xh)) - 1   (bit-identical, one rounding)
//   min(max(rx,ry), max(ry,rz), max(rz,rx)) == med3(rx, ry, rz)
// EXACT keeps the reference's roundings (separate 1 - 3|a|, division by s);
// the fast form fuses them (fma) and divides by s through a reciprocal.
//
// sdBox(p, vec3(1)) = min(mc, length(max(di, 0))) with mc = max(di)
// (common.frag:595-600) is exactly mc: if mc <= 0 the length is 0 >= mc;
// otherwise the rounded sum of squares is >= RN(mc*mc) and a correctly rounded
// sqrt of RN(mc*mc) is mc, so the length is >= mc.  No sqrt.
// max(|x| - 1, |y| - 1, |z| - 1) == max(|x|, |y|, |z|) - 1 exactly (rounding
// is monotonic): one v_max3 with abs modifiers and one subtraction.
__device__ __forceinline__ float sponge_box(V3 p) {
    return fmaxf(fabsf(p.x), fmaxf(fabsf(p.y), fabsf(p.z))) - 1.0f;
}
// The three folds, starting from the box term d; the result is >= d.
// Fold m yields c = (med3(r) - 1)/s with med3(r) <= 2, so c <= 1/s: once
// d >= 1/s the remaining folds cannot raise d (the `if (c > d)` of
// common.frag:671 never fires) and the result is exactly d.  Lanes that are
// not `active` never ask for a fold.  Far from the sponge (most march and
// shadow steps) whole waves skip the folds.  The exit test is wave-uniform:
// a wave computes fold m if any of its lanes needs it, and
// lanes past their exit point compute a fold that leaves d unchanged.  The
// same VALU as a per-lane branch, without the two exec-mask SALU per test
// (v_cmp to vcc + s_cbranch_vccz), and SALU issue is a co-bottleneck
// (DESIGN.md 2.2).  The FLOP tally counts the folds a lane needs, whatever NB
// and the wave's other lanes make it compute.
// NB: how many of the three folds keep their exit test.  A fold computed past
// its exit point leaves d unchanged, so any NB gives the same distance: 3 (the
// default) executes the fewest instructions, 1 the fewest branches and exec-mask
// updates, which is what bounds the latency of a lone long wave (the tail of a
// launch: render_tile's latency tiles).
template <bool EXACT, int NB = 3>
__device__ __forceinline__ float sponge_folds(V3 p, float d, uint32_t& fl, bool active = true) {
    constexpr float SH[3] = {0.5f, 1.5f, 4.5f};                      // s/2 before s *= 3
    constexpr float S3[3] = {3.0f, 9.0f, 27.0f};                     // s after s *= 3
    constexpr float INV[3] = {1.0f / 3.0f, 1.0f / 9.0f, 1.0f / 27.0f};
    bool need = active;  // this lane's d can still change (fold m's test passed)
#pragma unroll
    for (int m = 0; m < 3; m++) {
        need = active && d < INV[m];  // (d only grows: implies the earlier tests)
        if (m < NB) {
            if (__builtin_amdgcn_ballot_w64(need) == 0) return d;
        }
        if (need) fl += FL_FOLD;
        float rx, ry, rz;
        if constexpr (EXACT) {
            float hx = p.x * SH[m], hy = p.y * SH[m], hz = p.z * SH[m];
            float ax = fmaf(2.0f, hx - floorf(hx), -1.0f);
            float ay = fmaf(2.0f, hy - floorf(hy), -1.0f);
            float az = fmaf(2.0f, hz - floorf(hz), -1.0f);
            rx = fabsf(1.0f - 3.0f * fabsf(ax));
            ry = fabsf(1.0f - 3.0f * fabsf(ay));
            rz = fabsf(1.0f - 3.0f * fabsf(az));
        } else {
            // |a| = |2 fract(x s/2) - 1| = 2 |g|, g = y - rint(y), y = x s/2 - 1/2:
            // the distance from x s/2 to the nearest k + 1/2 (ties give 1/2 both
            // ways).  4 VALU per axis (fma, rndne, sub, fma) instead of 5.
            float yx = fmaf(p.x, SH[m], -0.5f), yy = fmaf(p.y, SH[m], -0.5f), yz = fmaf(p.z, SH[m], -0.5f);
            float gx = yx - __builtin_rintf(yx), gy = yy - __builtin_rintf(yy), gz = yz - __builtin_rintf(yz);
            rx = fabsf(fmaf(-6.0f, fabsf(gx), 1.0f));
            ry = fabsf(fmaf(-6.0f, fabsf(gy), 1.0f));
            rz = fabsf(fmaf(-6.0f, fabsf(gz), 1.0f));
        }
        float med = __builtin_amdgcn_fmed3f(rx, ry, rz);
        float c = EXACT ? div_const(med - 1.0f, S3[m], INV[m]) : fmaf(med, INV[m], -INV[m]);
        // if (c > d) d = c;  as one max: c and d are NaN together or not at all
        // (C4 share -2 %, C2 at P1 -2.5 % against compare + select).  IEEE
        // maximum (v_maximum3_f32) rather than maxNum: fmaxf's operands get a
        // canonicalizing v_max(d, d) each fold, maximum's need none.
        d = __builtin_elementwise_maximum(c, d);
    }
    return d;
}
template <bool EXACT, int NB = 3>
__device__ __forceinline__ float menger(V3 p, uint32_t& fl, bool active = true) {
    return sponge_folds<EXACT, NB>(p, sponge_box(p), fl, active);
}

// transformR(p - vec3(0,3,0), vec3(180, 2t, 0)): row vector times rotationY
// then rotationX (common.frag:434-441); rotation Z is the identity.
template <bool EXACT>
__device__ __forceinline__ V3 sponge_rot(const FrameConst& F, float x, float y, float z) {
    if constexpr (EXACT) {
        float x1 = x * F.ry_c + z * F.ry_s;
        float z1 = x * -F.ry_s + z * F.ry_c;
        float y2 = y * F.rx_c + z1 * -F.rx_s;
        float z2 = y * F.rx_s + z1 * F.rx_c;
        return v3(x1, y2, z2);
    } else {
        float x1 = fmaf(x, F.ry_c, z * F.ry_s);
        float z1 = fmaf(z, F.ry_c, -(x * F.ry_s));
        float y2 = fmaf(y, F.rx_c, -(z1 * F.rx_s));
        float z2 = fmaf(z1, F.rx_c, y * F.rx_s);
        return v3(x1, y2, z2);
    }
}
template <bool EXACT>
__device__ __forceinline__ V3 sponge_space(const FrameConst& F, V3 p) {
    return sponge_rot<EXACT>(F, p.x, p.y - 3.0f, p.z);
}

// A ray in sponge space: the transform is affine, so ro + rd t maps to
// o + d t (scene T's marches step there; only roundings differ).
struct LinRay {
    V3 o, d;
};
__device__ __forceinline__ LinRay sponge_ray(const FrameConst& F, V3 ro, V3 rd) {
    return LinRay{sponge_space<false>(F, ro), sponge_rot<false>(F, rd.x, rd.y, rd.z)};
}
__device__ __forceinline__ V3 at(const LinRay& r, float t) {
    return v3(fmaf(r.d.x, t, r.o.x), fmaf(r.d.y, t, r.o.y), fmaf(r.d.z, t, r.o.z));
}
// scene T's sceneSDF at depth t of a sponge-space ray: one ray-step on the
// active lanes (inactive lanes compute a value nobody reads, without forcing
// folds on the wave)
template <int NB = 3>
__device__ __forceinline__ float menger_at(const LinRay& r, float t, Tally& n, bool active = true) {
    if (active) {
        n.evals++;
        n.flop += FL_LINRAY + FL_BOX;
    }
    return menger<false, NB>(at(r, t), n.flop, active);
}

// sminCubic distance part (common.frag:72-80), k = vec2(k), k > 1e-4.
// The probe form (!EXACT: AO, soft shadow, thickness, whose results are smooth
// in the distance; m unused) is s = x^3 / (6 k^2) in three operations and the
// closer distance as one IEEE minimum (the same value as aCloser ? a : b for
// non-NaN distances): 7 VALU instead of 12 without contraction.
// The exact form's closer distance is one IEEE minimum too, instead of
// compare + select (+ a hazard s_nop): C5 frame 9.89 ->
// 9.59 ms, frames identical (profiles/r03/scene_O_micro_ab.jsonl)
template <bool EXACT>
__device__ __forceinline__ float smin_cubic_d(float a, float b, float k, float& m) {
    if constexpr (!EXACT) {
        const float x = fmaxf(k - fabsf(a - b), 0.0f);
        m = 0.0f;
        return fmaf(-(x * x), x * (1.0f / (6.0f * k * k)), __builtin_elementwise_minimum(a, b));
    }
    float x = fmaxf(k - fabsf(a - b), 0.0f);
    float h = EXACT ? div_const(x, k, 1.0f / k) : x * (1.0f / k);
    m = h * h * h * 0.5f;
    float s = m * k * (1.0f / 3.0f);
    return __builtin_elementwise_minimum(a, b) - s;
}

// FUSE_O: scene O's probe form (its sphere and cube distances, !EXACT) fuses
// the sum of squares (as its probe points, rm_render_direct.h); every other caller
// (scene S0's sphere) keeps the unfused form
template <bool EXACT, bool FUSE_O = false>
__device__ __forceinline__ float len3(float x, float y, float z) {
    if constexpr (!EXACT && FUSE_O) return __builtin_amdgcn_sqrtf(fmaf(z, z, fmaf(y, y, x * x)));
    float l2 = x * x + y * y + z * z;
    return EXACT ? sqrtf(l2) : __builtin_amdgcn_sqrtf(l2);
}

// cube(vec4(c, r), p) (common.frag:589-593), scene O's
template <bool EXACT>
__device__ __forceinline__ float cube(V3 p, V3 c, float r) {
    float qx = fabsf(p.x - c.x) - r, qy = fabsf(p.y - c.y) - r, qz = fabsf(p.z - c.z) - r;
    return len3<EXACT, true>(fmaxf(qx, 0.0f), fmaxf(qy, 0.0f), fmaxf(qz, 0.0f)) + fminf(fmaxf(qx, fmaxf(qy, qz)), 0.0f);
}

// scene O's sceneSDF distance (output_shader.frag:38-48) at world point p with
// q = its sponge-space image (given by the caller: sponge_space(p), or the
// sponge-space ray of a march)
//
// slack = min(lb - 0.0834 - (d3 + 0.51), mc - (d3 + 0.34)): where it is >= 0
// both skips below fire and the result is the plane's p.y bit for bit.  Each
// term is 1-Lipschitz in the Chebyshev norm of a displacement (lb in world
// space, mc in sponge space, a rotation: <= the Euclidean norm) plus the
// displacement's |y| (d3; t2 <= d3 for the sponge test), so at p + u the
// result is still p'.y while |u|_2 + |u_y| <= slack.  The skips have 0.01 of
// margin over what exactness needs; rounding of the extrapolation is ~1e-5.
// Callers use it to replace whole spans of rays and whole probe sets of a
// shading point by the plane (PlaneSpan, rm_render_direct.h).
template <bool EXACT>
__device__ __forceinline__ float scene_dist_O(V3 p, V3 q, Tally& n, float& slack) {
    n.evals++;
    const float d3 = p.y;
    float m;
    // Lower bounds of the sphere and the cube (Chebyshev <= Euclidean
    // distance, exactly also after rounding), and sminCubic lowers the min
    // by at most k/6: if even the bound of t1 is past the floor by more than
    // the blend width, t2 = sminCubic(t1, plane) is exactly the plane.
    const float lbs = fminf(fmaxf(fabsf(p.x - 3.0f), fmaxf(fabsf(p.y - 2.0f), fabsf(p.z - 3.0f))),
                            fmaxf(fabsf(p.x + 5.0f), fmaxf(fabsf(p.y - 4.0f), fabsf(p.z - 5.0f)))) - 1.0834f;
    n.flop += FL_BOUNDS + FL_BOX + 1;
    const float mc = sponge_box(q);
    slack = fminf(lbs - (d3 + 0.51f), mc - (d3 + 0.34f));
    // The sponge d0 >= its box term mc.  If mc - t2 exceeds the blend width
    // k = 0.33 (with a margin far above rounding), sminCubic's h is 0 and the
    // result is exactly t2: the sponge's folds are not needed.
    if (lbs >= d3 + 0.51f) {  // t2 = the plane
        if (mc >= d3 + 0.34f) return d3;
        const float d0 = sponge_folds<EXACT>(q, mc, n.flop);
        n.flop += FL_SMIN;
        return smin_cubic_d<EXACT>(d0, d3, 0.33f, m);
    }
    // Conversely t2 >= A = min(lb - k/6, plane) - k/6 (each sminCubic lowers
    // a min by at most 0.5/6): where the sponge is below A by more than its
    // blend width, the result is exactly d0 and the sphere, the cube and their
    // two blends are not needed (near the sponge, where the folds cost most).
    const float A = fminf(lbs, d3) - 0.0834f;
    float d0 = mc;
    const bool folded = mc + 0.34f <= A;
    if (folded) {
        d0 = sponge_folds<EXACT>(q, mc, n.flop);
        if (d0 + 0.34f <= A) return d0;
    }
    n.flop += FL_SPHERE + FL_CUBE + 2 * FL_SMIN;
    const float d1 = len3<EXACT, true>(p.x - 3.0f, p.y - 2.0f, p.z - 3.0f) - 1.0f;
    const float d2 = cube<EXACT>(p, v3(-5.0f, 4.0f, 5.0f), 1.0f);
    const float t1 = smin_cubic_d<EXACT>(d1, d2, 0.5f, m);
    const float t2 = smin_cubic_d<EXACT>(t1, d3, 0.5f, m);
    if (!folded) {
        if (mc >= t2 + 0.34f) return t2;
        d0 = sponge_folds<EXACT>(q, mc, n.flop);
    }
    n.flop += FL_SMIN;
    return smin_cubic_d<EXACT>(d0, t2, 0.33f, m);
}
template <bool EXACT>
__device__ __forceinline__ float scene_dist_O(V3 p, V3 q, Tally& n) {
    float slack;
    return scene_dist_O<EXACT>(p, q, n, slack);
}


// Scene distances ("one ray-step" = one call).  EXACT keeps the GLSL's
// roundings (scene O's marches and normals, whose results feed the normal
// hash); the fast form serves every other call.
template <int SC, bool EXACT, int NB = 3>
__device__ __forceinline__ float scene_dist(const FrameConst& F, V3 p, Tally& n) {
    if constexpr (SC == SCENE_S0) {
        n.evals++;
        n.flop += FL_SPHERE;
        return len3<EXACT>(p.x, p.y - 1.0f, p.z + 3.0f) - 1.0f;  // sphere(vec4(0,1,-3,1), p)
    } else if constexpr (SC == SCENE_T) {
        n.evals++;
        n.flop += FL_TRANSFORM + FL_BOX;
        return menger<EXACT, NB>(sponge_space<EXACT>(F, p), n.flop);  // template.frag:41 (repaired)
    } else if constexpr (SC == SCENE_PLUGIN) {
        n.evals++;
        n.flop += PluginScene<SC>::flop;
        if constexpr (EXACT) return PluginScene<SC>::dist(p);
        else return PluginScene<SC>::dist_probe(p);
    } else {  // output_shader.frag:38-48
        n.flop += FL_TRANSFORM;
        return scene_dist_O<EXACT>(p, sponge_space<EXACT>(F, p), n);
    }
}

// ------------------------------------------------------------- materials

// struct Material (common.frag:20-35); the constructor takes the GLSL
// constructor's arguments in order
struct Mat {
    V3 diffuse, specular;
    float shininess, reflectivity, transparency;
    V3 absorption;
    float refraction_index;
    V3 emission;
    Mat() = default;
    __host__ __device__ constexpr Mat(V3 d, V3 s, float sh, float refl, float tr, V3 ab, float ior_, V3 em)
        : diffuse(d), specular(s), shininess(sh), reflectivity(refl), transparency(tr), absorption(ab), refraction_index(ior_),
          emission(em) {}
};


__device__ __forceinline__ Mat mat_make(V3 d, V3 s, float sh, float refl, float tr, V3 ab, float ior, V3 em) {
    Mat m;
    m.diffuse = d; m.specular = s; m.shininess = sh; m.reflectivity = refl; m.transparency = tr;
    m.absorption = ab; m.refraction_index = ior; m.emission = em;
    return m;
}
__device__ __forceinline__ Mat mat_red() {  // output_shader.frag:12
    return mat_make(v3(0.2f, 0.02f, 0.02f), v3(0.04f, 0.02f, 0.02f), 32.0f, 0.0f, 0.0f, v3s(0.0f), 1.0f, v3s(0.0f));
}
__device__ __forceinline__ Mat mat_blue(bool glass) {  // output_shader.frag:14 (glass: test scene OG)
    return mat_make(v3(0.02f, 0.02f, 0.2f), v3(0.02f, 0.02f, 0.04f), 32.0f, 0.0f, glass ? 0.9f : 0.0f,
                    v3(2.0f, 2.0f, 0.75f) * 0.2f, 1.52f, v3(0.0f, 0.0f, 100.0f));
}
__device__ __forceinline__ Mat mat_mirror() {  // output_shader.frag:15
    return mat_make(v3s(0.1f), v3s(0.09f), 64.0f, 0.25f, 0.0f, v3s(0.0f), 1.0f, v3s(0.0f));
}
// output_shader.frag:16-28
// (colour only: the blur width and the divisions by it in the hardware
// forms; smoothstep is 150-Lipschitz here, so 1-ulp changes of its
// argument move the colour by ~1e-5 at most)
__device__ __forceinline__ Mat floor_mat(V3 pos) {
    const float l2 = dot(pos, pos);
    const float scale = fmaxf(10.0f, __builtin_amdgcn_exp2f(0.65f * __builtin_amdgcn_logf(l2)));  // |pos|^1.3
    const float is = __builtin_amdgcn_rcpf(scale);
    float tx = smoothstep(-0.005f, 0.005f, glsl_sin(pos.x * PI_REF) * is);
    float ty = smoothstep(-0.005f, 0.005f, glsl_sin(pos.z * PI_REF) * is);
    float tile = fminf(fmaxf(tx, ty), fmaxf(1.0f - tx, 1.0f - ty));
    V3 color = mix3(v3s(0.3f), v3s(0.025f), tile);
    return mat_make(color, v3s(0.03f), 128.0f, 0.0f, 0.0f, v3s(0.0f), 1.0f, v3s(0.0f));
}
// blendMaterial with ALLOW_MATERIAL_BLENDING (common.frag:37-53)
__device__ __forceinline__ Mat blend(const Mat& a, const Mat& b, float k) {
    return mat_make(mix3(a.diffuse, b.diffuse, k), mix3(a.specular, b.specular, k), gmix(a.shininess, b.shininess, k),
                    gmix(a.reflectivity, b.reflectivity, k), gmix(a.transparency, b.transparency, k),
                    mix3(a.absorption, b.absorption, k), gmix(a.refraction_index, b.refraction_index, k), mix3(a.emission, b.emission, k));
}
__device__ __forceinline__ Mat smin_mat(float a, const Mat& ma, float b, const Mat& mb, float m) {
    return blend(ma, mb, a < b ? m : 1.0f - m);
}

// The material half of sceneSDF at p (evaluated once where a march stops).
template <int SC>
__device__ __forceinline__ Mat scene_mat(const FrameConst& F, V3 p) {
    if constexpr (SC == SCENE_O || SC == SCENE_OG) {
        constexpr bool glass = SC == SCENE_OG;
        uint32_t fl = 0;  // (the material evaluation is not a ray-step)
        float d0 = menger<true>(sponge_space<true>(F, p), fl);
        float d1 = len3<true>(p.x - 3.0f, p.y - 2.0f, p.z - 3.0f) - 1.0f;
        float d2 = cube<true>(p, v3(-5.0f, 4.0f, 5.0f), 1.0f);
        float d3 = p.y;
        float m1, m2, m3;
        float t1 = smin_cubic_d<true>(d1, d2, 0.5f, m1);
        Mat b = mat_blue(glass);
        Mat mt1 = smin_mat(d1, b, d2, b, m1);
        float t2 = smin_cubic_d<true>(t1, d3, 0.5f, m2);
        Mat mt2 = smin_mat(t1, mt1, d3, floor_mat(p), m2);
        (void)smin_cubic_d<true>(d0, t2, 0.33f, m3);
        return smin_mat(d0, mat_mirror(), t2, mt2, m3);
    } else if constexpr (SC == SCENE_PLUGIN) {
        return PluginScene<SC>::mat(p);
    } else {
        (void)F; (void)p;
        return mat_red();
    }
}

// ---------------------------------------------------------- post-colour

// common.frag:1044-1051
template <bool FAST>
__device__ __forceinline__ float gpow(float x, float y) {
    if constexpr (FAST) return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
    else return powf(x, y);
}
// FAST (scenes S0/T): the colour path's division and exp as
// the hardware reciprocal and exp2 (1 ulp; the colour is smooth in them):
// arcp division had compiled to a frexp/ldexp-scaled reciprocal, 8 VALU each
template <bool FAST>
__device__ __forceinline__ float tonemap1(float c, float e2) {
    float col = FAST ? (c * 2.0f) * __builtin_amdgcn_rcpf(1.0f + c) : c * 2.0f / (1.0f + c);
    if constexpr (FAST) {  // pow(pow(x, .4545), e2) = exp2(.4545 e2 log2 x): one log2, one exp2
        col = __builtin_amdgcn_exp2f((0.4545f * e2) * __builtin_amdgcn_logf(col));
    } else {
        col = gpow<FAST>(col, 0.4545f);
        col = gpow<FAST>(col, e2);
    }
    return col * 0.5f + 0.5f * col * col * (3.0f - 2.0f * col);
}
// vignette(.., 0.1)'s factor (common.frag:1072): computed before the render, so
// one value instead of the two texture coordinates stays live through it
template <bool FAST>
__device__ __forceinline__ float vignette(float tcx, float tcy) {
    return 0.5f + 0.5f * gpow<FAST>(16.0f * tcx * tcy * (1.0f - tcx) * (1.0f - tcy), 0.1f);
}
// tonemap -> contrast (common.frag:1067) -> vignette (v = vignette(texcoord))
template <bool FAST>
__device__ __forceinline__ V3 post_colour(V3 c, float v) {
    V3 t = v3(tonemap1<FAST>(c.x, 0.85f), tonemap1<FAST>(c.y, 0.97f), tonemap1<FAST>(c.z, 1.0f));
    t = v3(smoothstep(0.15f, 1.1f, t.x), smoothstep(0.15f, 1.1f, t.y), smoothstep(0.15f, 1.1f, t.z));
    return t * v;
}

// common.frag:1032-1042 with be = bi = vec3(2) and the fog colour of the scenes
template <bool FAST = false>
__device__ __forceinline__ V3 apply_scattering(V3 color, V3 ro, V3 p) {
    float d = 1.0f - clamp01(length(p - ro) / ZFAR);
    float e = FAST ? __builtin_amdgcn_exp2f(d * -2.8853900817779268f) : expf(-d * 2.0f);  // 2 log2(e)
    return color * (1.0f - e) + v3(0.34f, 0.435f, 0.57f) * e;
}
// output_shader.frag:178-182
// (the sky's fog in the colour-only fast form, as every scene's colour path, rm_render_direct.h)
__device__ __forceinline__ V3 background(V3 ro, V3 rd) {
    return apply_scattering<true>(v3s(0.0f), ro, ro + rd * ZFAR);
}

// RGBA8 unorm of the reference's RenderTexture: clamp, round to nearest
// (NaN -> 0), R in the low byte
__device__ __forceinline__ uint32_t to_unorm8(float c) {
    c = fminf(fmaxf(c, 0.0f), 1.0f);  // NaN -> 0
    return (uint32_t)__float2int_rn(c * 255.0f);
}
__device__ __forceinline__ uint32_t pack_rgba8(float r, float g, float b, float a) {
    return to_unorm8(r) | (to_unorm8(g) << 8) | (to_unorm8(b) << 16) | (to_unorm8(a) << 24);
}

// ------------------------------------------------------------ hashing

// output_shader.frag:61-66
__device__ __forceinline__ V3 hash33(V3 p3) {
    p3 = v3(fract(p3.x * 443.897f), fract(p3.y * 441.423f), fract(p3.z * 437.195f));
    float dd = dot(p3, v3(p3.y + 19.19f, p3.x + 19.19f, p3.z + 19.19f));
    p3 = p3 + v3s(dd);
    return v3(fract((p3.x + p3.y) * p3.z), fract((p3.x + p3.x) * p3.y), fract((p3.y + p3.x) * p3.x));
}

}  // namespace rm
