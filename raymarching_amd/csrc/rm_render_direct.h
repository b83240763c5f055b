// rm_render_direct.h -- per-pixel render pipelines, one lane = one pixel.
//
// Straight control flow per lane (march, normal, probes, shadow march, ...).
// Lanes of a wave diverge only in loop trip counts; at 4096^2 the 8x8-pixel
// waves are coherent enough that 94 % of lane-steps are useful for scene T
// (tools/wave_sim.py on the oracle's per-pixel step traces), so a
// wave-compacted state machine would not pay for its phase switching.
#pragma once
#include "rm_device.h"
#include "rm_wire_tile.h"

namespace rm {

// Scenes S0 and T use GLSL-precision hardware ops (v_rcp/v_sqrt/v_rsq and
// pow = exp2(y*log2 x), as GPU GLSL compilers emit them); scene O keeps the
// libm-accurate forms because its normal hash amplifies ulp differences.
template <int SC>
struct FastMath {
    static constexpr bool value = SC == SCENE_T || SC == SCENE_S0;
};
template <int SC>
__device__ __forceinline__ float mdiv(float a, float b) {
    if constexpr (FastMath<SC>::value) return a * __builtin_amdgcn_rcpf(b);
    else return a / b;
}
template <int SC>
__device__ __forceinline__ float msqrt(float x) {
    if constexpr (FastMath<SC>::value) return __builtin_amdgcn_sqrtf(x);
    else return sqrtf(x);
}
template <int SC>
__device__ __forceinline__ float mpow(float x, float y) {
    if constexpr (FastMath<SC>::value) return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
    else return powf(x, y);
}
// Colour-only arithmetic (Phong's normalizations and pow, the shadow factor's
// pow, the SSS term's pow, fog, tonemap, vignette): scenes O/OG and plugins
// use the hardware exp2/log2/rsq/rcp forms there too (1-2 ulp).
// Nothing that positions a ray or feeds the thickness hash changes (marches,
// normals, the light direction and distance, the floor pattern keep their
// exact forms), so ray-step counts are untouched and pixels move by ~1e-6.
template <int SC>
struct FastColour {
    static constexpr bool value = true;  // (every scene: FastMath<SC> or the colour-only forms)
};
template <int SC>
__device__ __forceinline__ float cpow(float x, float y) {
    if constexpr (FastColour<SC>::value) return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
    else return powf(x, y);
}
template <int SC>
__device__ __forceinline__ V3 cnormalize(V3 a) {
    if constexpr (FastColour<SC>::value) return a * __builtin_amdgcn_rsqf(dot(a, a));
    else return normalize(a);
}
// the scene distance for marches and normals (exact for scene O), and for
// the AO / shadow / thickness probes, whose results are smooth in the distance
template <int SC, int NB = 3>
__device__ __forceinline__ float dist_march(const FrameConst& F, V3 p, Tally& cnt) {
    return scene_dist<SC, !FastMath<SC>::value, NB>(F, p, cnt);
}
template <int SC, int NB = 3>
__device__ __forceinline__ float dist_probe(const FrameConst& F, V3 p, Tally& cnt) {
    return scene_dist<SC, false, NB>(F, p, cnt);
}
template <int SC>
__device__ __forceinline__ V3 mnormalize(V3 a) {
    if constexpr (FastMath<SC>::value) return a * __builtin_amdgcn_rsqf(dot(a, a));
    else return normalize(a);
}

// Scene O's floor-plane spans (scene_dist_O's slack, rm_device.h).  Along a
// ray with a unit direction d the plane-only result holds for a parameter span
// slack / (1 + |d.y|) (1.01: directions up to 1 % off unit length); the probes
// of a shading point (normal 0.0018, AO <= 0.8, thickness < 1 away) are all
// plane-only when the slack there is >= 2.05.
template <int SC>
constexpr bool kPlaneSpans = SC == SCENE_O || SC == SCENE_OG;
__device__ __forceinline__ float plane_rate(V3 d) {  // (v_rcp: 1 ulp is far inside the margin)
    return __builtin_amdgcn_rcpf(1.01f + fabsf(d.y));
}
template <int SC>
__device__ __forceinline__ bool plane_probes(const FrameConst& F, V3 p) {
    if constexpr (kPlaneSpans<SC>) {
        Tally scratch;  // (not a ray-step of the reference)
        float slack;
        (void)scene_dist_O<false>(p, sponge_space<false>(F, p), scratch, slack);
        return slack >= 2.05f;
    } else {
        (void)F; (void)p;
        return false;
    }
}
// a probe's distance: EXACT = the march form (normals), else the probe form
template <int SC, bool EXACT, int NB = 3>
__device__ __forceinline__ float dist_at(const FrameConst& F, V3 p, Tally& cnt, bool plane) {
    if constexpr (kPlaneSpans<SC>) {
        if (plane) {
            cnt.evals++;
            return p.y;
        }
    }
    if constexpr (EXACT) return dist_march<SC, NB>(F, p, cnt);
    else return dist_probe<SC, NB>(F, p, cnt);
}

// common.frag:697-708 (tetrahedral gradient, h = 0.001)
template <int SC, int NB = 3>
__device__ __forceinline__ V3 normal_fast(const FrameConst& F, V3 p, Tally& cnt, bool plane = false) {
    const float h = 0.001f;
    float d0 = dist_at<SC, true, NB>(F, p + v3(h, -h, -h), cnt, plane);
    float d1 = dist_at<SC, true, NB>(F, p + v3(-h, -h, h), cnt, plane);
    float d2 = dist_at<SC, true, NB>(F, p + v3(-h, h, -h), cnt, plane);
    float d3 = dist_at<SC, true, NB>(F, p + v3(h, h, h), cnt, plane);
    V3 g = v3(d0, -d0, -d0) + v3(-d1, -d1, d1);
    g = g + v3(-d2, d2, -d2);
    g = g + v3(d3, d3, d3);
    return mnormalize<SC>(g);
}

// common.frag:879-901. Returns dist (depth on hit, -1 on miss, last SDF value
// on step exhaustion) and the point whose SdResult is returned.  One exit
// test per step; at a hit depth is left as it was, so the hit flag and depth
// give the three outcomes after the loop.
template <int SC, bool INSIDE>
__device__ __forceinline__ float cast_ray_d(const FrameConst& F, V3 ro, V3 rd, V3& last_q, Tally& cnt) {
    float depth = ZNEAR;
    float res = 0.0f;
    bool hit = false;
    if constexpr (kPlaneSpans<SC>) {
        // depth < t_plane: sceneSDF is the floor plane, (ro + rd depth).y
        const float ia = plane_rate(rd);
        float t_plane = 0.0f, last = 0.0f;
        for (int i = 0; i < F.max_steps; i++) {
            if (depth < t_plane) {
                res = ro.y + rd.y * depth;
                cnt.evals++;
                cnt.flop += 2;
            } else {
                V3 q = ro + rd * depth;
                float slack;
                cnt.flop += FL_TRANSFORM;
                res = scene_dist_O<true>(q, sponge_space<true>(F, q), cnt, slack);
                t_plane = depth + slack * ia;
            }
            last = depth;
            if (INSIDE) {
                hit = -res < 0.001f * depth;
                depth = hit ? depth : depth - res;
            } else {
                hit = res < 0.001f * depth;
                depth = hit ? depth : depth + res;
            }
            if (hit | (depth >= ZFAR)) break;
        }
        last_q = ro + rd * last;  // the point of the last step (ro without steps)
        return hit ? depth : depth >= ZFAR ? -1.0f : res;
    }
    last_q = ro;
    for (int i = 0; i < F.max_steps; i++) {
        V3 q = ro + rd * depth;
        res = dist_march<SC>(F, q, cnt);
        last_q = q;
        if (INSIDE) {  // castRayDI, common.frag:903-925
            hit = -res < 0.001f * depth;
            depth = hit ? depth : depth - res;
        } else {
            hit = res < 0.001f * depth;
            depth = hit ? depth : depth + res;
        }
        if (hit | (depth >= ZFAR)) break;
    }
    return hit ? depth : depth >= ZFAR ? -1.0f : res;
}

// The soft-shadow loops compute P = 2h for the next step before the exit
// test and pin it there (an empty asm): left free, the compiler sinks the add
// into a "continue" block of its own, which costs 4 SALU and 2 branches per
// step (C4 share 0.131 -> 0.119 ms, C2 P1 0.204 -> 0.188, scene O 4096^2
// 2.97 -> 2.92; profiles/r02/shadow_p_pin_ab.jsonl).
// Scene O's settle rule (soft_shadow2_T_loop states it for
// the sponge alone).  sceneSDF >= min(d0 - 0.33/6, d3 - 0.83/6, d1 - 1.33/6,
// d2 - 1.33/6) (each sminCubic lowers a min by at most k/6; output_shader.frag:
// 38-48 nests sphere d1 and cube d2, then the plane d3, then the sponge d0),
// with d0 >= the sponge's box term and d2 >= the cube's Chebyshev term.  Each
// of the four terms is convex along the ray (the plane linear), so it has an
// affine minorant through its value and a subgradient at t; their minimum
// minus the offsets, g, bounds every later h'.  If g >= 0.1 on [t, maxt]
// (checked at both ends: affine) every later step is unoccluded and, sceneSDF
// being 3-Lipschitz, h' / (2 ph) <= 0.665, so every later candidate is
// >= 4 * 0.7469 g(t') / t'; each g_i / t' is monotonic, so the minimum is at t
// or maxt: when 2.9 min(g(t) / t, g(maxt) / maxt) >= 1.01 res no later step
// changes res.  res^2 = 16 num / den (squared, as the loop keeps it).
// oracle settle_test_O restates the rule and checks it on every step of the
// reference's marches.
__device__ __forceinline__ bool shadow_settled_O(const LinRay& w, const LinRay& s, float t, float maxt, float num,
                                                 float den) {
    const float L = maxt - t;
    const V3 p = at(w, t), q = at(s, t);
    // sponge: box term in sponge space, slope along the sponge-space ray
    const float qx = fabsf(q.x), qy = fabsf(q.y), qm = fmaxf(qx, fmaxf(qy, fabsf(q.z)));
    const float sx = q.x < 0.0f ? -s.d.x : s.d.x, sy = q.y < 0.0f ? -s.d.y : s.d.y, sz = q.z < 0.0f ? -s.d.z : s.d.z;
    const float s0 = qx == qm ? sx : qy == qm ? sy : sz;
    const float a0 = qm - (1.0f + 0.33f / 6.0f);
    // sphere (3,2,3) r 1: |e| - 1, slope e.d / |e|
    const V3 e1 = p - v3(3.0f, 2.0f, 3.0f);
    const float l1 = __builtin_amdgcn_sqrtf(dot(e1, e1));
    const float a1 = l1 - (1.0f + 1.33f / 6.0f), s1 = dot(e1, w.d) * __builtin_amdgcn_rcpf(l1);
    // cube (-5,4,5) r 1: Chebyshev term
    const V3 e2 = p - v3(-5.0f, 4.0f, 5.0f);
    const float bx = fabsf(e2.x), by = fabsf(e2.y), bm = fmaxf(bx, fmaxf(by, fabsf(e2.z)));
    const float cx = e2.x < 0.0f ? -w.d.x : w.d.x, cy = e2.y < 0.0f ? -w.d.y : w.d.y, cz = e2.z < 0.0f ? -w.d.z : w.d.z;
    const float s2 = bx == bm ? cx : by == bm ? cy : cz;
    const float a2 = bm - (1.0f + 1.33f / 6.0f);
    const float a3 = p.y - 0.83f / 6.0f;  // plane
    const float g0 = fminf(fminf(a0, a1), fminf(a2, a3));
    const float g1 = fminf(fminf(fmaf(s0, L, a0), fmaf(s1, L, a1)), fminf(fmaf(s2, L, a2), fmaf(w.d.y, L, a3)));
    constexpr float K = (2.9f / 1.01f) * (2.9f / 1.01f) / 16.0f;
    const float m = __builtin_elementwise_minimum(
        __builtin_elementwise_minimum(__builtin_elementwise_minimum(g0, g1) - 0.1f, K * g0 * g0 * den - num * t * t),
        K * g1 * g1 * den - num * maxt * maxt);
    return m >= 0.0f;
}

// A settled lane leaves at the test, and the uniform step cap is a branch of
// its own: the exit test does not materialize four booleans per step (C5
// frame 10.22 -> 10.03 ms; profiles/r03/scene_O_micro_ab.jsonl)
constexpr int kSettleOEvery = 8;  // steps between settle tests (a power of 2)

// common.frag:810-831, k = 4, for scenes O/OG: the probes step along the
// world ray and its sponge-space image, and the candidate is kept squared as
// in soft_shadow2_T below (the shadow factor is smooth in its roundings).
// SM as soft_shadow2_T_loop (0 none, 1 timed kernels: settle exit, 2
// instrumented kernels: every step taken, those after the settle point counted
// in cnt.skipped); O/OG only.  The settle test (~45 VALU) runs on every
// kSettleOEvery-th step: C5 frame 11.25 -> 10.51 ms with 8, 10.79 with 4
// (profiles/r03/scene_O_settle_ab.jsonl).
template <int SC, int SM = 0, bool CAP = true>
__device__ __forceinline__ float soft_shadow2_loop(const FrameConst& F, V3 ro, V3 rd, float mint, float maxt,
                                                   Tally& cnt) {
    constexpr bool kSettle = kPlaneSpans<SC> && SM != 0;
    const LinRay w{ro, rd}, s = sponge_ray(F, ro, rd);
    float num = 1.0f / 16.0f, den = 1.0f, P = 0.0f, h = 1.0f;  // res = 1, k = 4
    float t = mint;
    const float ia = plane_rate(rd);
    float t_plane = 0.0f;  // t < t_plane: sceneSDF is the floor plane (O/OG)
    bool was_settled = false;  // SM == 2
    for (int it = 1; it == 1 ? t < maxt : true; it++) {
        if constexpr (SM == 2) cnt.skipped += was_settled ? 1u : 0u;
        if constexpr (SC == SCENE_PLUGIN) {
            h = dist_probe<SC>(F, at(w, t), cnt);
        } else if (t < t_plane) {
            h = fmaf(w.d.y, t, w.o.y);  // at(w, t).y
            cnt.evals++;
            cnt.flop += 2;
        } else {
            float slack;
            cnt.flop += FL_LINRAY;
            h = scene_dist_O<false>(at(w, t), at(s, t), cnt, slack);
            t_plane = t + slack * ia;
        }
        float h2 = h * h;
        float Q = it == 1 ? 1.0f : fmaf(P, P, -h2);
        float D = it == 1 ? t : fmaf(t, P, -h2);
        float cn = h2 * Q, cd = D * fabsf(D);  // D <= 0: cd <= 0 fails the test (cn, den >= 0)
        bool upd = (Q >= 0.0f) & (cn * den < num * cd);
        num = upd ? cn : num;
        den = upd ? cd : den;
        bool settled = false;
        if constexpr (kSettle) {  // every kSettleOEvery-th step (h >= 0.1 is implied by the rule; h >= ph: moving away)
            if ((it & (kSettleOEvery - 1)) == 0 && __builtin_amdgcn_ballot_w64((h >= 0.1f) & (h + h >= P)) != 0)
                settled = (h >= 0.1f) & shadow_settled_O(w, s, t, maxt, num, den);
            // (a settled lane leaves here: its result needs neither P nor t)
            if constexpr (SM == 1) {
                if (settled) break;
            }
        }
        P = h + h;
        asm volatile("" : "+v"(P));  // keep P's add in the step (not in a continue block of its own)
        t += h * 0.1f + 0.001f;  // the reference's roundings: the step count is part of parity
        if constexpr (SM == 2) {
            was_settled |= settled;
            settled = false;
        }
        if ((h < 0.001f) | !(t < maxt)) break;
        if (CAP && it >= F.shadow_max_steps) break;  // (wave-uniform)
    }
    return h < 0.001f ? 0.0f : sqrtf(16.0f * num / den);
}
// The reference's uncapped march (the default) runs as a loop copy without
// the step-cap test, as scene T's (soft_shadow2_T).  Round 3
// measured no gain while the kernel spilled; without spills: C5 frame
// 8.524 -> 8.510 ms, C5 share 1.082 -> 1.077, O 4096^2 2.219 -> 2.212, frames
// identical (profiles/r05/ab_O_uncapped.jsonl)
template <int SC, int SM = 0>
__device__ __forceinline__ float soft_shadow2(const FrameConst& F, V3 ro, V3 rd, float mint, float maxt,
                                              Tally& cnt) {
    if (F.shadow_max_steps == __INT_MAX__) return soft_shadow2_loop<SC, SM, false>(F, ro, rd, mint, maxt, cnt);
    return soft_shadow2_loop<SC, SM, true>(F, ro, rd, mint, maxt, cnt);
}

// softShadow2 for scene T (fast math), stepping in sponge space and free of
// divisions and square roots.  With P = 2 ph the reference's y = h^2/P gives
//   k sqrt(h^2 - y^2) / (t - y) = k h sqrt(P^2 - h^2) / (t P - h^2),
// and res^2 / k^2 is kept as num/den, candidates h^2 Q / D^2 compared by
// cross-products (branch-free selects; D |D| for D^2 makes t - y <= 0 fail the
// comparison without a test of its own).  Candidates with t - y <= 0 (k d / 0:
// inf or NaN) or h^2 < y^2 (sqrt NaN) never lower res, as GLSL
// min(res, x) = x < res ? x : res.  On the first step ph = 1e20 makes y
// vanish: the candidate is k h / t (Q = 1, D = t below).  The occlusion result
// is recovered after the loop from the last h (a lane leaves through
// t >= maxt only with h >= 0.001).
//
// SETTLE (the timed kernels): a lane leaves the march as soon
// as no later step can change its result.  Every later step t' has h' >= B(t')
// (the sponge's box term, a lower bound of mengersponge), and B along the
// sponge-space ray, max_i |o_i + d_i t'| - 1, is convex: B(t') >= g(t') =
// B(t) + s (t' - t) with s = d_i sign(q_i) on an axis attaining the max.  If
// B(t) >= 0.1 and s >= 0, every later h' >= 0.1 (no occlusion) and the
// previous h >= 0.1, so with mengersponge 3-Lipschitz and the step 0.1 ph +
// 0.001, h' / (2 ph) <= 0.665 and every later candidate
// k h' sqrt(1 - (h'/2ph)^2) / (t' - y) is >= 4 * 0.7469 g(t') / t'.  g / t'
// is monotonic, so its minimum over [t, maxt] is at an endpoint: when
// 2.9 min(B / t, g(maxt) / maxt) >= 1.01 res no later candidate lowers res
// (margins far above the roundings), and the result is res now.  The test
// runs when some lane of the wave has B >= 0.1 and h >= ph (a march moving
// away from the sponge).  tools: oracle_shadow_settle checks the rule on every
// step of the reference's marches (no change of res after it, ever) and
// measures 43-55 % of scene T's shadow steps after it.  The instrumented
// kernels (COUNT) keep every step: their ray-step counts and maps are the
// reference's.
// SM: 0 no settle test, 1 leave the march when settled (timed kernels), 2 run
// the test and count the steps after it in cnt.skipped (instrumented kernels:
// every reference step is still taken and counted)
// A settled lane leaves at the test, as in scene O's loop (C3 0.575 -> 0.568
// ms, C2 P1 0.192 -> 0.181); the test runs on every step.
// The settle gate is the AND of the two compares' own masks (s_and_b64) instead of a ballot of their combined i1, which the
// backend materialized as a 0/1 VGPR and a v_cmp_ne per step: 2 VALU fewer per
// shadow step, C3 0.4603-0.4626 -> 0.4527-0.4549 ms (profiles/r05/ab_settle_T.log)
template <bool CAP, int NB, int SM = 0>
__device__ __forceinline__ float soft_shadow2_T_loop(const FrameConst& F, const LinRay& s, float mint, float maxt,
                                                     Tally& cnt) {
    float num = 1.0f / 16.0f, den = 1.0f, P = 0.0f, h = 1.0f;  // res = 1, k = 4
    float t = mint;
    bool was_settled = false;  // SM == 2
    // one exit test per step (occluded, t >= maxt, settled, or the optional
    // step cap); t grows by >= 0.001 per continuing step, NaN leaves
    for (int it = 1; it == 1 ? t < maxt : true; it++) {
        const V3 q = at(s, t);
        const float box = sponge_box(q);
        cnt.evals++;
        cnt.flop += FL_LINRAY + FL_BOX;
        if constexpr (SM == 2) cnt.skipped += was_settled ? 1u : 0u;
        h = sponge_folds<false, NB>(q, box, cnt.flop);
        float h2 = h * h;
        float Q = it == 1 ? 1.0f : fmaf(P, P, -h2);
        float D = it == 1 ? t : fmaf(t, P, -h2);
        float cn = h2 * Q, cd = D * fabsf(D);  // D <= 0: cd <= 0 fails the test (cn, den >= 0)
        bool upd = (Q >= 0.0f) & (cn * den < num * cd);
        num = upd ? cn : num;
        den = upd ? cd : den;
        bool settled = false;
        if constexpr (SM != 0) {
            const bool any = (__builtin_amdgcn_ballot_w64(box >= 0.1f) & __builtin_amdgcn_ballot_w64(h + h >= P)) != 0;
            if (any) {
                const float ax = fabsf(q.x), ay = fabsf(q.y), m = box + 1.0f;
                const float sx = q.x < 0.0f ? -s.d.x : s.d.x, sy = q.y < 0.0f ? -s.d.y : s.d.y;
                const float sz = q.z < 0.0f ? -s.d.z : s.d.z;
                const float sl = ax == m ? sx : ay == m ? sy : sz;
                const float be = fmaf(sl, maxt - t, box);
                constexpr float K = (2.9f / 1.01f) * (2.9f / 1.01f) / 16.0f;  // res^2 = 16 num / den
                settled = (box >= 0.1f) & (h + h >= P) & (sl >= 0.0f) & (K * box * box * den >= num * t * t) &
                          (K * be * be * den >= num * maxt * maxt);
            }
        }
        if constexpr (SM == 1) {
            if (settled) break;  // (the result needs neither P nor t)
        }
        P = h + h;
        asm volatile("" : "+v"(P));  // keep P's add in the step (not in a continue block of its own)
        t = fmaf(h, 0.1f, t + 0.001f);
        if constexpr (SM == 2) {
            was_settled |= settled;
            settled = false;
        }
        if ((h < 0.001f) | !(t < maxt)) break;
        if (CAP && it >= F.shadow_max_steps) break;
    }
    return h < 0.001f ? 0.0f : __builtin_amdgcn_sqrtf(16.0f * num * __builtin_amdgcn_rcpf(den));
}
// The uncapped loop (the reference's, and the default) carries no step
// counter: a uniform counter test merged into the lanes' exit mask costs 5
// SALU per step, and SALU issue is a co-bottleneck of the kernel.
// (Scene O's soft_shadow2 has the same split since round 5.)
template <int NB = 3, int SETTLE = 0>
__device__ __forceinline__ float soft_shadow2_T(const FrameConst& F, const LinRay& s, float mint, float maxt,
                                                Tally& cnt) {
    if (F.shadow_max_steps == __INT_MAX__) return soft_shadow2_T_loop<false, NB, SETTLE>(F, s, mint, maxt, cnt);
    return soft_shadow2_T_loop<true, NB, SETTLE>(F, s, mint, maxt, cnt);
}

// castRay (common.frag:931-954) for scene T in sponge space; returns the
// depth of the point the reference returns (ZFAR on escape).  depth < ZFAR
// holds at a hit and after step exhaustion, so the escape value is set once,
// after the loop.
// RS, the reflection march of getColorReflect (common.frag:991-1002): its
// point only enters the colour as clamp(length(pr - p) / 3, 0, 1), and depth
// never decreases along the march, so once depth >= 3 (|pr - p| = 0.01 + depth
// within 1e-5) that factor is 1 whatever the march does next.  RS = 1 (timed
// kernels) leaves the march there; RS = 2 (instrumented) takes every step and
// counts those after it in cnt.skipped.
template <int NB = 3, int RS = 0>
__device__ __forceinline__ float cast_ray_T(const FrameConst& F, const LinRay& s, Tally& cnt) {
    constexpr float kStop = RS == 1 ? 3.0f : ZFAR;
    float depth = ZNEAR;
    for (int i = 0; i < F.max_steps; i++) {
        if constexpr (RS == 2) cnt.skipped += depth >= 3.0f ? 1u : 0u;
        float dist = menger_at<NB>(s, depth, cnt);
        bool hit = dist < 0.001f;
        depth = hit ? depth : depth + dist;
        if (hit | (depth >= kStop)) break;  // one exit test per step
    }
    return depth >= ZFAR ? ZFAR : depth;
}

// common.frag:850-866.  Scene O rolls the probe loop: the unrolled loop's
// interleaved probes spilled 18 VGPRs of the 8-wave kernel to scratch, rolled
// 4 (same frames, C5 frame 9.46 -> 9.43 ms; scene T's rolled loop measured
// 3 % slower, profiles/r03/rolled_probes_ab.jsonl)
// Scenes O/OG form the probe points of AO and thickness, and
// the sphere / cube lengths of the probe-form distance, with fused
// multiply-adds (these results are smooth in their roundings; the exact march
// and normal paths, and the thickness hash of the normal, keep the GLSL's)
template <int SC>
constexpr bool kProbeFma = kPlaneSpans<SC>;
__device__ __forceinline__ V3 fma3(V3 a, float s, V3 b) {  // a s + b, one rounding per component
    return v3(fmaf(a.x, s, b.x), fmaf(a.y, s, b.y), fmaf(a.z, s, b.z));
}
__device__ __forceinline__ float dot_fma(V3 a, V3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }

// Scene T's four AO probes step along the normal's
// sponge-space image (q0 + (R n) 0.2 (i + 1), one FMA per axis) instead of
// transforming each probe point (the AO factor is smooth in the roundings;
// step counts do not depend on it)
template <int SC, int NB = 3>
__device__ __forceinline__ float ao_real(const FrameConst& F, V3 pos, V3 n, Tally& cnt, bool plane = false) {
    float sum = 0.0f;
    if constexpr (SC == SCENE_T) {
        const LinRay r = sponge_ray(F, pos, n);
#pragma unroll
        for (int i = 0; i < 4; i++) sum += (1.0f / (float)(1 << i)) * menger_at<NB>(r, (float)(i + 1) * 0.2f, cnt);
        float maxSum = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; i++) maxSum += (1.0f / (float)(1 << i)) * (float)(i + 1) * 0.2f;
        return sum / maxSum;
    }
    auto probe = [&](int i) {
        V3 p = kProbeFma<SC> ? fma3(n, (float)(i + 1) * 0.2f, pos) : pos + (n * (float)(i + 1)) * 0.2f;
        sum += (1.0f / (float)(1 << i)) * dist_at<SC, false, NB>(F, p, cnt, plane);
    };
    if constexpr (kPlaneSpans<SC>) {
#pragma unroll 1
        for (int i = 0; i < 4; i++) probe(i);
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) probe(i);
    }
    // maxSum = sum_i 2^-i (i+1) 0.2, accumulated in f32 as the reference does
    float maxSum = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; i++) maxSum += (1.0f / (float)(1 << i)) * (float)(i + 1) * 0.2f;
    return sum / maxSum;
}

// common.frag:730-754 (N = the caller's normal; L = normalize(lightPos - p),
// the caller's light direction, the same value)
template <int SC>
__device__ __forceinline__ V3 phong(V3 k_d, V3 k_s, float alpha, V3 L, V3 p, V3 eye, V3 N) {
    V3 V = cnormalize<SC>(eye - p);
    V3 R = cnormalize<SC>(reflect(-L, N));
    float dotLN = dot(L, N);
    float dotRV = dot(R, V);
    if (dotLN < 0.0f) return v3s(0.0f);
    if (dotRV < 0.0f) return k_d * dotLN;
    return k_d * dotLN + k_s * cpow<SC>(dotRV, alpha);
}

// Soft shadows of points facing away from the light: phong returns 0 when
// dot(L, N) < 0 (common.frag:738-745), and the shadow factor only multiplies
// phong's term (template.frag:58,66; output_shader.frag:133,148),
// by shadow_pow(sha), finite for any sha in [0, 1]: the product
// is 0 whatever the march returns.  SM 1 (timed kernels) skips the march
// (sha = 1), SM 2 (instrumented) takes it and counts its steps in
// cnt.skipped, SM 0 takes it.  dotLN is phong's own dot(L, N): the same
// value, so the same decision.  Scene T at P0: 54 % of the shadow-march steps
// (oracle shadow_settle back_steps), scene O 0-6 % (its floor faces the light).
template <int SM, typename March>
__device__ __forceinline__ float shadow_if_lit(float dotLN, Tally& cnt, March march) {
    const bool lit = !(dotLN < 0.0f);
    if constexpr (SM == 1) {
        return lit ? march() : 1.0f;
    } else {
        const uint32_t e0 = cnt.evals, s0 = cnt.skipped;
        const float sha = march();
        if constexpr (SM == 2) {
            if (!lit) cnt.skipped = s0 + (cnt.evals - e0);
        }
        (void)e0; (void)s0; (void)lit;
        return sha;
    }
}

template <int SC>
__device__ __forceinline__ V3 shadow_pow(float sha) {
    if constexpr (FastColour<SC>::value) {  // pow(x, 1) = x; one log2 shared by the other two
        const float l = __builtin_amdgcn_logf(sha);
        return v3(sha, __builtin_amdgcn_exp2f(1.2f * l), __builtin_amdgcn_exp2f(1.5f * l));
    }
    return v3(mpow<SC>(sha, 1.0f), mpow<SC>(sha, 1.2f), mpow<SC>(sha, 1.5f));
}

// output_shader.frag:85-116
template <int SC>
__device__ __forceinline__ float thickness(const FrameConst& F, V3 pos, V3 norm, Tally& cnt, bool plane) {
    if constexpr (kPlaneSpans<SC>) {
        // A floor point whose probes are all plane-only: every sample is
        // pos.y + (sampleDir * sampleLength).y, and the sample directions depend
        // on the normal alone, which the floor's tetrahedral gradient makes
        // exactly (0, 1, 0) or (0, 1 - 2^-24, 0): per-frame tables (the host
        // evaluates GenerateSampleVector in GLSL float semantics).
        const bool n1 = norm.y == 1.0f;
        if (plane && norm.x == 0.0f && norm.z == 0.0f && (n1 || norm.y == 0x1.fffffep-1f)) {
            float th = 0.0f;
            for (int i = 0; i < 32; i++) th += F.hash11[i] + (pos.y + (n1 ? F.sss_floor[0][i] : F.sss_floor[1][i]));
            cnt.evals += 32;
            return clamp01(th * 0.03125f);
        }
    }
    float th = 0.0f;
    V3 nn = -norm;
    for (int i = 0; i < 32; i++) {
        float fi = (float)i;
        float sl = F.hash11[i];
        // the sample direction is not amplified (unlike the hash of the normal),
        // so it is normalized with v_rsq (~1 ulp) instead of a correctly
        // rounded sqrt and division: -22 VALU per sample, 32 samples
        const V3 hd = hash33(nn + v3s(fi)) - v3s(0.5f);
        if constexpr (kProbeFma<SC>) {
            const V3 rnd = hd * __builtin_amdgcn_rsqf(dot_fma(hd, hd));
            const V3 dir = fma3(nn * -2.0f, fminf(0.0f, dot_fma(rnd, nn)), rnd);  // reflectVector (:70-73)
            th += sl + dist_at<SC, false>(F, fma3(dir, sl, pos), cnt, plane);
            continue;
        }
        V3 rnd = hd * __builtin_amdgcn_rsqf(dot(hd, hd));
        V3 dir = rnd - (nn * 2.0f) * fminf(0.0f, dot(rnd, nn));  // reflectVector (:70-73)
        th += sl + dist_at<SC, false>(F, pos + dir * sl, cnt, plane);
    }
    return clamp01(th * 0.03125f);
}

// output_shader.frag:127-176.  The material of the hit (the SdResult at mq)
// is evaluated after the AO / shadow / thickness loops and returned in mat: it
// is not live across them (16 floats fewer in registers during the loops).
template <int SC, int SETTLE = 0>
__device__ __forceinline__ V3 light_O(const FrameConst& F, V3 mq, V3 ro, V3 rd, V3 p, V3 n, V3 phongN, bool plane,
                                     Mat& mat, Tally& cnt) {
    const V3 lightPos = v3(20.0f, 50.0f, 0.0f);
    V3 Ld = lightPos - p;
    V3 lightDir = normalize(Ld);
    float occ = ao_real<SC>(F, p, n, cnt, plane);
    float sha = shadow_if_lit<SETTLE>(dot(lightDir, phongN), cnt, [&] {
        return soft_shadow2<SC, SETTLE>(F, p, lightDir, 0.01f, length(Ld), cnt);
    });
    float th = thickness<SC>(F, p, n, cnt, plane);
    mat = scene_mat<SC>(F, mq);
    float sky = clamp01(0.5f + 0.5f * n.y);
    float ind = clamp01(dot(n, cnormalize<SC>(lightDir * v3(-1.0f, 0.0f, -1.0f))));
    V3 shading =
        phong<SC>(v3(1.64f, 1.27f, 0.99f), mat.specular, mat.shininess, lightDir, p, ro, phongN) * shadow_pow<SC>(sha);
    shading = shading + v3(0.16f, 0.20f, 0.28f) * sky * occ;
    shading = shading + v3(0.40f, 0.28f, 0.20f) * ind * occ;
    V3 sssl = lightDir + n * 0.6f;
    float sssdot = cpow<SC>(clamp01(dot(-rd, -sssl)), 1.1f) * 0.3f;
    shading = shading + v3s((sssdot + 0.3f) * th);
    V3 color = mat.diffuse * shading + mat.emission;
    return apply_scattering<FastColour<SC>::value>(color, ro, p);
}

// output_shader.frag:218-230
__device__ __forceinline__ float fresnel(float n2, V3 normal, V3 incident, float reflectivity) {
    float r0 = (1.0f - n2) * __builtin_amdgcn_rcpf(1.0f + n2);  // (colour only: the hardware reciprocal)
    r0 *= r0;
    float x = 1.0f + dot(normal, incident);
    float r = r0 + (1.0f - r0) * x * x * x * x * x;
    return (1.0f - reflectivity) * r + reflectivity;
}

// output_shader.frag:246-262
template <int SC, int SETTLE = 0>
__device__ __forceinline__ V3 render_reflection(const FrameConst& F, V3 ro, V3 rd, Tally& cnt) {
    V3 q;
    float dist = cast_ray_d<SC, false>(F, ro, rd, q, cnt);
    if (dist > 0.0f) {
        Mat m;
        V3 p = ro + rd * dist;
        const bool pl = plane_probes<SC>(F, p);
        V3 n = normal_fast<SC>(F, p, cnt, pl);
        return light_O<SC, SETTLE>(F, q, ro, rd, p, n, n, pl, m, cnt);
    }
    return background(ro, rd);
}

// output_shader.frag:298-343 (MAX_REFRACTIONS 4); live only in test scene OG
template <int SC, int SETTLE = 0>
__device__ __forceinline__ V3 render_refraction(const FrameConst& F, V3 ro, V3 rd, V3 absorption, Tally& cnt) {
    V3 color = v3s(0.0f);
    float invert = -1.0f;
    float absorb = 0.0f;
    for (int i = 0; i < 4; i++) {
        V3 q;
        float dist = invert < 0.0f ? cast_ray_d<SC, true>(F, ro, rd, q, cnt) : cast_ray_d<SC, false>(F, ro, rd, q, cnt);
        if (invert < 0.0f) absorb += dist;
        if (dist < 0.0f) {
            if (invert > 0.0f) color = color + background(ro, rd);
            break;
        }
        Mat m;
        V3 p = ro + rd * dist;
        const bool pl = plane_probes<SC>(F, p);
        V3 g = normal_fast<SC>(F, p, cnt, pl);
        V3 n = g * invert;
        V3 ref = reflect(rd, n);
        color = color + light_O<SC, SETTLE>(F, q, ro, ref, p, n, g, pl, m, cnt);
        if (invert > 0.0f) break;
        float ior = invert < 0.0f ? m.refraction_index : 1.0f / m.refraction_index;
        V3 raf = refract(rd, n, ior);
        bool tif = raf.x == 0.0f && raf.y == 0.0f && raf.z == 0.0f;
        rd = tif ? ref : raf;
        ro = p + rd * (0.01f / fabsf(dot(rd, n)));
        invert = tif ? invert : -invert;
    }
    if constexpr (FastColour<SC>::value) {
        constexpr float kLog2e = 1.4426950408889634f;
        return color * v3(__builtin_amdgcn_exp2f(-absorption.x * absorb * kLog2e),
                          __builtin_amdgcn_exp2f(-absorption.y * absorb * kLog2e),
                          __builtin_amdgcn_exp2f(-absorption.z * absorb * kLog2e));
    }
    return color * v3(expf(-absorption.x * absorb), expf(-absorption.y * absorb), expf(-absorption.z * absorb));
}

// output_shader.frag:348-385 (SETTLE: soft_shadow2's SM)
template <int SC, int SETTLE = 0>
__device__ __forceinline__ V3 render_O(const FrameConst& F, V3 ro, V3 rd, Tally& cnt) {
    V3 q;
    float dist = cast_ray_d<SC, false>(F, ro, rd, q, cnt);
    if (!(dist > 0.0f)) return background(ro, rd);
    Mat m;
    V3 p = ro + rd * dist;
    const bool pl = plane_probes<SC>(F, p);
    V3 n = normal_fast<SC>(F, p, cnt, pl);
    V3 color = light_O<SC, SETTLE>(F, q, ro, rd, p, n, n, pl, m, cnt);
    float rf = fresnel(m.refraction_index, n, rd, m.transparency > 0.0f ? 0.0f : m.reflectivity);
    if (m.reflectivity > 0.0f) {
        V3 r = reflect(rd, n);
        color = color + (render_reflection<SC, SETTLE>(F, p + r * 0.001f, r, cnt) * rf) * m.reflectivity;
    }
    if constexpr (SC == SCENE_OG || SC == SCENE_PLUGIN) {  // (scene O has no transparent material)
        if (m.transparency > 0.0f) {
            V3 r = refract(rd, n, 1.0f / m.refraction_index);
            color = color + (render_refraction<SC, SETTLE>(F, p + r * 0.001f, r, m.absorption, cnt) * (1.0f - rf)) *
                                m.transparency;
        }
    }
    return color;
}

// template.frag:45-76 (scene T); NB: sponge_folds; SETTLE: soft_shadow2_T_loop;
// RSTOP: cast_ray_T's RS for the reflection march
template <int NB = 3, int SETTLE = 0, int RSTOP = 0>
__device__ __forceinline__ V3 render_T(const FrameConst& F, V3 ro, V3 rd, Tally& cnt) {
    constexpr int SC = SCENE_T;
    V3 p = ro + rd * cast_ray_T<NB>(F, sponge_ray(F, ro, rd), cnt);
    V3 n = normal_fast<SC, NB>(F, p, cnt);
    // getColorReflect (common.frag:991-1002); its dead nr normal is skipped
    V3 rdir = reflect(rd, n);
    V3 ror = p + rdir * 0.01f;
    V3 pr = ror + rdir * cast_ray_T<NB, RSTOP>(F, sponge_ray(F, ror, rdir), cnt);
    float c = clamp01(length(pr - p) * (1.0f / 3.0f));
    const V3 lightPos = v3(20.0f, 50.0f, 0.0f);
    V3 Ld = lightPos - p;
    float ld2 = dot(Ld, Ld);
    V3 lightDir = Ld * __builtin_amdgcn_rsqf(ld2);
    float occ = ao_real<SC, NB>(F, p, n, cnt);
    float sha = shadow_if_lit<RSTOP>(dot(lightDir, n), cnt, [&] {
        return soft_shadow2_T<NB, SETTLE>(F, sponge_ray(F, p, lightDir), 0.01f, __builtin_amdgcn_sqrtf(ld2), cnt);
    });
    float sky = clamp01(0.5f + 0.5f * n.y);
    float ind = clamp01(dot(n, mnormalize<SC>(lightDir * v3(-1.0f, 0.0f, -1.0f))));
    float fre = clamp01(1.0f + dot(n, rd));
    fre = fre * fre;  // pow(x, 2.0)
    V3 shading =
        phong<SC>(v3(1.64f, 1.27f, 0.99f), v3(1.0f, 1.0f, 0.0f), 1280.0f, lightDir, p, ro, n) * shadow_pow<SC>(sha);
    shading = shading + v3(0.16f, 0.20f, 0.28f) * sky * occ;
    shading = shading + v3(0.40f, 0.28f, 0.20f) * ind * occ;
    shading = shading + v3s(fre * occ);
    return apply_scattering<true>(v3s(c) * shading, ro, p);
}

// BASELINE config-1 scene S0: castRayD + normal + lambert
__device__ __forceinline__ V3 render_S0(const FrameConst& F, V3 ro, V3 rd, Tally& cnt) {
    constexpr int SC = SCENE_S0;
    V3 q;
    float dist = cast_ray_d<SC, false>(F, ro, rd, q, cnt);
    if (dist > 0.0f) {
        V3 p = ro + rd * dist;
        V3 n = normal_fast<SC>(F, p, cnt);
        V3 lightDir = mnormalize<SC>(v3(20.0f, 50.0f, 0.0f) - p);
        return v3(0.2f, 0.02f, 0.02f) * (0.1f + clamp01(dot(n, lightDir)));
    }
    return background(ro, rd);
}

// Camera (output_shader.frag:388-404): gl_TexCoord at the pixel centre.
// FAST (scenes S0/T): the divisions by the per-frame W, H and u_resolution.y
// as v_rcp + mul, spelled out: left to -freciprocal-math, the compiler hoisted
// a correctly rounded 1/W out of the persistent kernel's tile loop but not out
// of the one-tile kernels, and their frames differed in a pixel.
template <bool FAST>
__device__ __forceinline__ void camera_ray(const FrameConst& F, int x, int y, float& tcx, float& tcy, V3& ro, V3& rd) {
    if constexpr (FAST) {
        tcx = ((float)x + 0.5f + F.jit_x) * __builtin_amdgcn_rcpf((float)F.W);
        tcy = ((float)y + 0.5f + F.jit_y) * __builtin_amdgcn_rcpf((float)F.H);
    } else {
        tcx = ((float)x + 0.5f + F.jit_x) / (float)F.W;  // (jitter 0 outside rm_render_accumulate*)
        tcy = ((float)y + 0.5f + F.jit_y) / (float)F.H;
    }
    const float ux = FAST ? (tcx - 0.5f) * F.res_x * __builtin_amdgcn_rcpf(F.res_y) : (tcx - 0.5f) * F.res_x / F.res_y;
    const float uy = FAST ? (tcy - 0.5f) * F.res_y * __builtin_amdgcn_rcpf(F.res_y) : (tcy - 0.5f) * F.res_y / F.res_y;
    ro = v3(F.pos_x, F.pos_y, F.pos_z);
    rd = normalize(v3(ux, -uy, -1.0f));
    // rd.yz *= rot(-u_mouse.y); rd.xz *= rot(u_mouse.x)  (row vector x mat2(c,-s,s,c))
    float y1 = rd.y * F.cam1_c + rd.z * -F.cam1_s;
    float z1 = rd.y * F.cam1_s + rd.z * F.cam1_c;
    float x2 = rd.x * F.cam2_c + z1 * -F.cam2_s;
    float z2 = rd.x * F.cam2_s + z1 * F.cam2_c;
    rd = v3(x2, y1, z2);
}

// The pixel store of a render launch.  With F.accumulate (progressive
// accumulation, rm_render_accumulate*: the ping-pong u_sample plumbing of
// main.cpp:192-207 and common.frag:8-11, read by the pass) the target holds
// u_sample, this pixel of the previous frame, and receives
// mix(u_sample, colour, u_sample_part) (GLSL mix as the fixture renderer
// evaluates it, x + (y - x) a, no contraction); RGBA8 targets are read as GL
// reads unorm8 texels, b * RN(1/255) (within 1 ulp of b / 255).  A part >= 1
// (the first frame of a still camera) stores the colour: the target needs no
// clearing.
template <typename OUT>
__device__ __forceinline__ void store_pixel(const FrameConst& F, OUT* __restrict__ out, size_t i, V3 c) {
#pragma clang fp contract(off)
    if (F.accumulate && F.sample_part < 1.0f) {
        V3 prev;
        if constexpr (sizeof(OUT) == 4) {
            const uint32_t w = out[i];
            const float k = 1.0f / 255.0f;
            prev = v3((float)(w & 255u) * k, (float)((w >> 8) & 255u) * k, (float)((w >> 16) & 255u) * k);
        } else {
            const float4 v = out[i];
            prev = v3(v.x, v.y, v.z);
        }
        const float a = F.sample_part;
        c = v3(prev.x + (c.x - prev.x) * a, prev.y + (c.y - prev.y) * a, prev.z + (c.z - prev.z) * a);
    }
    if constexpr (sizeof(OUT) == 4) out[i] = pack_rgba8(c.x, c.y, c.z, 1.0f);
    else out[i] = make_float4(c.x, c.y, c.z, 1.0f);
}

// local packed row j of this shard -> frame row y
__device__ __forceinline__ int shard_row(const FrameConst& F, int j) {
    int c = div_by(j, F.run_magic, F.run), r = j - c * F.run;
    return c * F.cycle + F.offset + r;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// SETTLE: the timed kernels' exact early exits (1), which the instrumented
// (COUNT) kernels do not take but count (2): their ray-step counts and maps
// stay the reference's, rm_stats.skipped the steps the timed kernels leave out
template <int SC, int NB = 3, int SETTLE = 0, int RSTOP = 0>
__device__ __forceinline__ V3 render_pixel(const FrameConst& F, V3 ro, V3 rd, Tally& cnt) {
    if constexpr (SC == SCENE_S0) return render_S0(F, ro, rd, cnt);
    else if constexpr (SC == SCENE_T) return render_T<NB, SETTLE, RSTOP>(F, ro, rd, cnt);
    else return render_O<SC, SETTLE>(F, ro, rd, cnt);  // O, OG and plugins: output_shader.frag's render()
}

// sceneSDF(p) of the scene at n points (rm_scene_eval): the distance in the
// reference's arithmetic (the EXACT form), and, when mat is set, the 16 floats
// of struct Material (common.frag:20-35) in declaration order.
template <int SC>
__device__ __forceinline__ void scene_eval_one(const FrameConst& F, const float* pts, long long n, float* dist,
                                               float* mat) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const V3 p = v3(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
    Tally t;
    dist[i] = scene_dist<SC, true>(F, p, t);
    if (mat) {
        const Mat m = scene_mat<SC>(F, p);
        const float v[16] = {m.diffuse.x,    m.diffuse.y,    m.diffuse.z,    m.specular.x,    m.specular.y,  m.specular.z,
                             m.shininess,    m.reflectivity, m.transparency, m.absorption.x,  m.absorption.y,
                             m.absorption.z, m.refraction_index,          m.emission.x,   m.emission.y,    m.emission.z};
        for (int k = 0; k < 16; k++) mat[16 * i + k] = v[k];
    }
}

// Workgroup shapes (KernelKind): KERNEL_TILE16 = 16x16 pixels as 2x2 waves
// of 8x8; KERNEL_TILE8 = one 8x8-pixel wave per workgroup (the dispatcher
// then refills CUs at wave granularity, which shortens the tail of small or
// uneven launches); KERNEL_TILE16X4 = one 16x4-pixel wave.
// KERNEL_PERSIST = 8x8-pixel one-wave tiles pulled by persistent waves from an
// atomic tile counter (SURVEY.md 7.5's refill at tile granularity, rm_params.kernel 4).
enum KernelKind : int { KERNEL_TILE16 = 0, KERNEL_TILE8 = 1, KERNEL_TILE16X4 = 2, KERNEL_PERSIST = 3 };
template <int K> struct Tiling;
template <> struct Tiling<KERNEL_TILE16> { static constexpr int TW = 16, TH = 16, WPB = 4, LW = 8; };
template <> struct Tiling<KERNEL_TILE8> { static constexpr int TW = 8, TH = 8, WPB = 1, LW = 8; };
template <> struct Tiling<KERNEL_TILE16X4> { static constexpr int TW = 16, TH = 4, WPB = 1, LW = 16; };
template <> struct Tiling<KERNEL_PERSIST> : Tiling<KERNEL_TILE8> {};

// The body of a render launch: one lane per pixel of the workgroup's tile.
// OUT = float4 (gl_FragColor) or uint32_t (RGBA8, packed in the epilogue, so
// the displayed frame costs 4 B/px of HBM instead of 16 + 20 for a pack
// pass).  COUNT: instrumented build, ray-steps and FLOP summed per wave into
// evals[0..2] (ray-steps, FLOP, ray-steps the timed kernels skip).
// (bx, by): the tile's position in dispatch order on a gx-wide tile grid
// (blockIdx for the hardware-dispatched kernels).
template <int SC, bool COUNT, int K, typename OUT>
__device__ __forceinline__ void render_tile_at(const FrameConst& F, OUT* __restrict__ out,
                                               unsigned long long* __restrict__ evals, int bx, int by, int gx) {
    using T = Tiling<K>;
    const uint64_t t_start = T::WPB == 1 && F.tile_cost ? clock64() : 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // scene T: the first lat_tiles workgroups of an ordered launch are its
    // costliest tiles, whose lone waves end the launch; they render with one
    // fold exit test instead of three (fewer branches, more VALU: C4 share and
    // C2 tails -16..19 %, a whole C3 frame +5 % if every tile did)
    const bool lat = T::WPB == 1 && SC == SCENE_T && F.tile_order && by * gx + bx < F.lat_tiles;
    if (F.tile_order) {  // dispatch order != tile order (costliest tiles first, rm_set_tile_order)
        const uint32_t t = F.tile_order[by * gx + bx];
        by = div_by((int)t, F.gx_magic, gx);
        bx = (int)t - by * gx;
    }
    const int x = bx * T::TW + (w & 1) * 8 + (lane % T::LW);
    const int j = by * T::TH + (w >> 1) * 8 + (lane / T::LW);
    // OUT = WireTile (rm_render_cycle_rows_wire): the wave's 8x8 tile is not
    // stored as pixels but encoded for the compressed wire from registers
    // (rm_wire_tile.h) into the workspace, tile by * gx + bx of the part
    constexpr bool kWire = IsWireTile<OUT>::value;
    static_assert(!kWire || (T::WPB == 1 && T::TW == 8 && T::TH == 8), "the wire codes one 8x8 wave tile");
    uint32_t wire_px = 0;  // (kWire: this lane's RGBA8 word, 0 outside the part)
    Tally cnt;
    if (x < F.W && j < F.nrows) {
        const int y = shard_row(F, F.row0 + j);
        float tcx, tcy;
        V3 ro, rd;
        camera_ray<FastMath<SC>::value>(F, x, y, tcx, tcy, ro, rd);
        const float vig = vignette<FastColour<SC>::value>(tcx, tcy);
        V3 c;
        if constexpr (SC == SCENE_T) {
            // (no settle exit in the latency tiles: their long grazing shadow marches
            // settle late or never, and the test lengthens the lone waves that end
            // the launch: C4 share +16 %, C2 P1 +12 % with it)
            if (lat) c = render_pixel<SC, 1, 0, COUNT ? 2 : 1>(F, ro, rd, cnt);
            else c = render_pixel<SC, 3, COUNT ? 2 : 1, COUNT ? 2 : 1>(F, ro, rd, cnt);
        } else {
            (void)lat;
            c = render_pixel<SC, 3, kPlaneSpans<SC> ? (COUNT ? 2 : 1) : 0>(F, ro, rd, cnt);
        }
        c = post_colour<FastColour<SC>::value>(c, vig);
        if constexpr (kWire) wire_px = pack_rgba8(c.x, c.y, c.z, 1.0f);
        else store_pixel(F, out, (size_t)j * F.W + x, c);
    }
    if constexpr (kWire)
        wire_encode_tile(wire_px, reinterpret_cast<WireTile*>(out), (long long)gx * ((F.nrows + 7) / 8),
                         (long long)by * gx + bx);
    if (T::WPB == 1 && F.tile_cost && lane == 0) {  // this tile's duration: the next launch's dispatch order
        const uint64_t dt = clock64() - t_start;
        F.tile_cost[by * gx + bx] = dt > 0xffffffffull ? 0xffffffffu : (uint32_t)dt;
    }
    if constexpr (COUNT) {
        if (F.evals_map && x < F.W && j < F.nrows) F.evals_map[(size_t)j * F.W + x] = cnt.evals;
        uint32_t se = wave_sum_u32(cnt.evals), sf = wave_sum_u32(cnt.flop), ss = wave_sum_u32(cnt.skipped);
        if (lane == 0) {
            atomicAdd(&evals[0], (unsigned long long)se);
            atomicAdd(&evals[1], (unsigned long long)sf);
            if (ss) atomicAdd(&evals[2], (unsigned long long)ss);
        }
    }
}

template <int SC, bool COUNT, int K, typename OUT>
__device__ __forceinline__ void render_tile(const FrameConst& F, OUT* __restrict__ out,
                                            unsigned long long* __restrict__ evals) {
    render_tile_at<SC, COUNT, K, OUT>(F, out, evals, blockIdx.x, blockIdx.y, gridDim.x);
}

// Persistent waves (KERNEL_PERSIST): the dispatch ordinals k of the launch's
// tiles are dealt to the 8 XCDs (k = x + 8 j on XCD x = blockIdx.x % 8, the
// dispatcher's round robin), each XCD's waves pulling j from a counter of
// their own (F.persist[kPersistStride * x]: device-scope atomics on one address
// from all XCDs serialize), the next j fetched before the current tile renders
// (the atomic's latency hides behind the tile).  Tile k renders as the
// hardware-dispatched kernel renders workgroup k (same tile order, latency
// tiles, tile durations), so pixels are identical.  The last wave to leave
// (counter 8 counts them) resets the counters for the next launch that uses
// them; no wave waits for another.
constexpr int kPersistStride = 32;  // uint32 words between counters (128 B lines)
constexpr int kPersistWords = 9 * kPersistStride;
template <int SC, bool COUNT, typename OUT>
__device__ __forceinline__ void render_persistent(const FrameConst& F, OUT* __restrict__ out,
                                                  unsigned long long* __restrict__ evals, int gx, int ntiles) {
    const int xcd = blockIdx.x & 7;
    uint32_t* ctr = F.persist + kPersistStride * xcd;
    const int nj = (ntiles - xcd + 7) >> 3;  // ordinals xcd, xcd + 8, ... below ntiles
    auto ticket = [&]() {
        int j = 0;
        if (threadIdx.x == 0) j = (int)atomicAdd(ctr, 1u);
        return __builtin_amdgcn_readfirstlane(j);
    };
    for (int j = ticket(); j < nj;) {
        const int jn = ticket();
        const int k = xcd + 8 * j;
        const int ky = div_by((int)k, F.gx_magic, gx);
        render_tile_at<SC, COUNT, KERNEL_PERSIST, OUT>(F, out, evals, (int)k - ky * gx, ky, gx);
        j = jn;
    }
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(F.persist + 8 * kPersistStride, 1u) == gridDim.x - 1)
            for (int x = 0; x < 9; x++) atomicExch(F.persist + kPersistStride * x, 0u);
    }
}

}  // namespace rm
