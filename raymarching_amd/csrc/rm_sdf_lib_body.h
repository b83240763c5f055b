// rm_sdf_lib_body.h -- the body of the scene library (rm_sdf_lib.h), included
// twice there: in rm::glsl with the GLSL's roundings (RM_LIB_PROBE 0: the
// marches, normals and rm_scene_eval of a plugin) and in rm::glsl::probe with
// the hardware square root and reciprocals and FMA contraction (RM_LIB_PROBE
// 1: the AO, soft-shadow and thickness probes, whose results are smooth in
// the roundings, as the built-in scenes' probe forms).  Each instance has its
// own vec2 / vec4 / mat4 / SdResult types, so argument-dependent lookup never
// sees the other instance's functions; vec3 (rm::V3) and Material (rm::Mat)
// are shared.  No include guard: rm_sdf_lib.h includes it once per instance.

using vec3 = V3;
using Material = Mat;

struct vec2 {
    float x, y;
    vec2() = default;
    __host__ __device__ constexpr vec2(float x_, float y_) : x(x_), y(y_) {}
    __host__ __device__ constexpr explicit vec2(float s) : x(s), y(s) {}
};
struct vec4 {
    float x, y, z, w;
    vec4() = default;
    __host__ __device__ constexpr vec4(float x_, float y_, float z_, float w_) : x(x_), y(y_), z(z_), w(w_) {}
    __host__ __device__ constexpr explicit vec4(float s) : x(s), y(s), z(s), w(s) {}
    __host__ __device__ constexpr vec4(vec3 v, float w_) : x(v.x), y(v.y), z(v.z), w(w_) {}
    __host__ __device__ constexpr vec4(float x_, vec3 v) : x(x_), y(v.x), z(v.y), w(v.z) {}
    __host__ __device__ constexpr vec4(vec2 a, vec2 b) : x(a.x), y(a.y), z(b.x), w(b.y) {}
};

// swizzle reads: component i of a vector, and e.xz / e.xyz / e.xyzw as the
// source translation spells them
__host__ __device__ constexpr float comp(vec2 v, int i) { return i == 0 ? v.x : v.y; }
__host__ __device__ constexpr float comp(vec3 v, int i) { return i == 0 ? v.x : i == 1 ? v.y : v.z; }
__host__ __device__ constexpr float comp(vec4 v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
template <int A, int B, class V>
__host__ __device__ constexpr vec2 swz2(V v) { return vec2(comp(v, A), comp(v, B)); }
template <int A, int B, int C, class V>
__host__ __device__ constexpr vec3 swz3(V v) { return vec3(comp(v, A), comp(v, B), comp(v, C)); }
template <int A, int B, int C, int D, class V>
__host__ __device__ constexpr vec4 swz4(V v) { return vec4(comp(v, A), comp(v, B), comp(v, C), comp(v, D)); }
__host__ __device__ constexpr vec3 xyz(vec4 v) { return vec3(v.x, v.y, v.z); }
__host__ __device__ constexpr vec2 xy(vec3 v) { return vec2(v.x, v.y); }
__host__ __device__ constexpr vec2 xz(vec3 v) { return vec2(v.x, v.z); }
__host__ __device__ constexpr vec2 yz(vec3 v) { return vec2(v.y, v.z); }

#define RM_V2_OP(op)                                                                                           \
    __host__ __device__ constexpr vec2 operator op(vec2 a, vec2 b) { return vec2(a.x op b.x, a.y op b.y); }   \
    __host__ __device__ constexpr vec2 operator op(vec2 a, float s) { return vec2(a.x op s, a.y op s); }      \
    __host__ __device__ constexpr vec2 operator op(float s, vec2 a) { return vec2(s op a.x, s op a.y); }
RM_V2_OP(+)
RM_V2_OP(-)
RM_V2_OP(*)
RM_V2_OP(/)
#undef RM_V2_OP
__host__ __device__ constexpr vec2 operator-(vec2 a) { return vec2(-a.x, -a.y); }
#define RM_V4_OP(op)                                                                                           \
    __host__ __device__ constexpr vec4 operator op(vec4 a, vec4 b) {                                          \
        return vec4(a.x op b.x, a.y op b.y, a.z op b.z, a.w op b.w);                                          \
    }                                                                                                          \
    __host__ __device__ constexpr vec4 operator op(vec4 a, float s) {                                         \
        return vec4(a.x op s, a.y op s, a.z op s, a.w op s);                                                  \
    }
RM_V4_OP(+)
RM_V4_OP(-)
RM_V4_OP(*)
RM_V4_OP(/)
#undef RM_V4_OP
__device__ __forceinline__ vec2& operator+=(vec2& a, vec2 b) { return a = a + b; }
__device__ __forceinline__ vec2& operator*=(vec2& a, float s) { return a = a * s; }

// GLSL 1.30 built-ins (min/max/clamp by their spec definitions, mod = x - y floor(x/y))
__device__ __forceinline__ float abs(float x) { return fabsf(x); }
__device__ __forceinline__ float sign(float x) { return x > 0.0f ? 1.0f : x < 0.0f ? -1.0f : 0.0f; }
// min / max as single instructions (v_minimum3_f32 / v_maximum3_f32): equal to
// the GLSL 1.30 definitions (y < x ? y : x, x < y ? y : x) for every non-NaN
// operand pair up to the sign of a zero result; a NaN operand gives NaN (the
// definitions return x).  The compare + select pair of the definitions was
// ~15 % of a plugin's march step.
__device__ __forceinline__ float min(float x, float y) { return __builtin_elementwise_minimum(x, y); }
__device__ __forceinline__ float max(float x, float y) { return __builtin_elementwise_maximum(x, y); }
// x / k for a divisor that is a constant once the scene is inlined: one
// Markstein correction of x * RN(1/k) (rm_device.h div_const), the correctly
// rounded quotient (checked exhaustively over two binades of x for the
// library's divisors), 3 VALU instead of the ~12 of the IEEE division.
// A power-of-two divisor (k = 0.5 in the smooth minima of most scenes) is one
// multiplication by its exact reciprocal in both instances: x * (1/k) is then
// the exact quotient rounded once, the IEEE division's bits.
__device__ __forceinline__ constexpr bool pow2_normal(float k) {
    return k > 0.0f && (__builtin_bit_cast(unsigned, k) & 0x7FFFFFu) == 0u &&
           (__builtin_bit_cast(unsigned, k) >> 23) > 1u && (__builtin_bit_cast(unsigned, k) >> 23) < 254u;
}
__device__ __forceinline__ float div_k(float x, float k) {
    if (RM_LIB_PROBE) return __builtin_constant_p(k) ? x * (1.0f / k) : x * __builtin_amdgcn_rcpf(k);
    if (__builtin_constant_p(k) && pow2_normal(k)) return x * (1.0f / k);
    return __builtin_constant_p(k) ? div_const(x, k, 1.0f / k) : x / k;
}
__device__ __forceinline__ float clamp(float x, float lo, float hi) { return min(max(x, lo), hi); }
__device__ __forceinline__ float mix(float x, float y, float a) { return x + (y - x) * a; }  // rm_device.h gmix
__device__ __forceinline__ float mod(float x, float y) { return x - y * floorf(x / y); }
__device__ __forceinline__ float fract(float x) { return x - floorf(x); }
__device__ __forceinline__ float step(float e, float x) { return x < e ? 0.0f : 1.0f; }
__device__ __forceinline__ float smoothstep(float e0, float e1, float x) {
    float t = clamp((x - e0) / (e1 - e0), 0.0f, 1.0f);
    return t * t * (3.0f - 2.0f * t);
}
__device__ __forceinline__ float radians(float d) { return d * 0.017453292519943295f; }
__device__ __forceinline__ float degrees(float r) { return r * 57.29577951308232f; }
// (the probe instance: the hardware exp2 / log2, 1-2 ulp; GLSL allows 3 ulp
// for exp2/log2 and derives pow from them)
__device__ __forceinline__ float pow(float x, float y) {
    return RM_LIB_PROBE ? __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x)) : powf(x, y);
}
__device__ __forceinline__ float exp(float x) {
    return RM_LIB_PROBE ? __builtin_amdgcn_exp2f(x * 1.4426950408889634f) : expf(x);
}
__device__ __forceinline__ float exp2(float x) { return RM_LIB_PROBE ? __builtin_amdgcn_exp2f(x) : exp2f(x); }
__device__ __forceinline__ float log(float x) {
    return RM_LIB_PROBE ? __builtin_amdgcn_logf(x) * 0.6931471805599453f : logf(x);
}
__device__ __forceinline__ float log2(float x) { return RM_LIB_PROBE ? __builtin_amdgcn_logf(x) : log2f(x); }
__device__ __forceinline__ float sqrt(float x) { return RM_LIB_PROBE ? __builtin_amdgcn_sqrtf(x) : sqrtf(x); }
__device__ __forceinline__ float inversesqrt(float x) { return 1.0f / sqrtf(x); }
// sin/cos as the implementation that renders the golden fixtures (rm_device.h glsl_sin)
__device__ __forceinline__ float sin(float x) { return glsl_sin(x); }
__device__ __forceinline__ float cos(float x) { return glsl_cos(x); }
__device__ __forceinline__ float tan(float x) { return tanf(x); }
__device__ __forceinline__ float asin(float x) { return asinf(x); }
__device__ __forceinline__ float acos(float x) { return acosf(x); }
__device__ __forceinline__ float atan(float y, float x) { return atan2f(y, x); }
__device__ __forceinline__ float atan(float y_over_x) { return atanf(y_over_x); }
__device__ __forceinline__ float floor(float x) { return floorf(x); }
__device__ __forceinline__ float ceil(float x) { return ceilf(x); }
__device__ __forceinline__ float length(float x) { return fabsf(x); }

#define RM_V3_FN1(fn) \
    __device__ __forceinline__ vec3 fn(vec3 a) { return vec3(fn(a.x), fn(a.y), fn(a.z)); }
#define RM_V2_FN1(fn) \
    __device__ __forceinline__ vec2 fn(vec2 a) { return vec2(fn(a.x), fn(a.y)); }
RM_V3_FN1(abs)
RM_V3_FN1(sign)
RM_V3_FN1(fract)
RM_V3_FN1(floor)
RM_V3_FN1(sin)
RM_V3_FN1(cos)
RM_V3_FN1(exp)
RM_V3_FN1(sqrt)
RM_V2_FN1(abs)
RM_V2_FN1(sign)
RM_V2_FN1(fract)
RM_V2_FN1(floor)
RM_V2_FN1(sin)
RM_V2_FN1(cos)
#undef RM_V3_FN1
#undef RM_V2_FN1
__device__ __forceinline__ vec4 abs(vec4 a) { return vec4(abs(a.x), abs(a.y), abs(a.z), abs(a.w)); }
__device__ __forceinline__ vec3 min(vec3 a, vec3 b) { return vec3(min(a.x, b.x), min(a.y, b.y), min(a.z, b.z)); }
__device__ __forceinline__ vec3 max(vec3 a, vec3 b) { return vec3(max(a.x, b.x), max(a.y, b.y), max(a.z, b.z)); }
__device__ __forceinline__ vec3 min(vec3 a, float s) { return vec3(min(a.x, s), min(a.y, s), min(a.z, s)); }
__device__ __forceinline__ vec3 max(vec3 a, float s) { return vec3(max(a.x, s), max(a.y, s), max(a.z, s)); }
__device__ __forceinline__ vec2 min(vec2 a, vec2 b) { return vec2(min(a.x, b.x), min(a.y, b.y)); }
__device__ __forceinline__ vec2 max(vec2 a, vec2 b) { return vec2(max(a.x, b.x), max(a.y, b.y)); }
__device__ __forceinline__ vec2 max(vec2 a, float s) { return vec2(max(a.x, s), max(a.y, s)); }
__device__ __forceinline__ vec2 min(vec2 a, float s) { return vec2(min(a.x, s), min(a.y, s)); }
__device__ __forceinline__ vec4 min(vec4 a, vec4 b) {
    return vec4(min(a.x, b.x), min(a.y, b.y), min(a.z, b.z), min(a.w, b.w));
}
__device__ __forceinline__ vec3 clamp(vec3 x, float lo, float hi) { return min(max(x, lo), hi); }
__device__ __forceinline__ vec3 mix(vec3 x, vec3 y, float a) {
    return vec3(mix(x.x, y.x, a), mix(x.y, y.y, a), mix(x.z, y.z, a));
}
__device__ __forceinline__ vec3 mix(vec3 x, vec3 y, vec3 a) {
    return vec3(mix(x.x, y.x, a.x), mix(x.y, y.y, a.y), mix(x.z, y.z, a.z));
}
__device__ __forceinline__ vec3 pow(vec3 x, vec3 y) { return vec3(pow(x.x, y.x), pow(x.y, y.y), pow(x.z, y.z)); }
__device__ __forceinline__ vec3 mod(vec3 x, float y) { return vec3(mod(x.x, y), mod(x.y, y), mod(x.z, y)); }
__device__ __forceinline__ vec2 mod(vec2 x, vec2 y) { return vec2(mod(x.x, y.x), mod(x.y, y.y)); }
__device__ __forceinline__ vec2 smoothstep(float e0, float e1, vec2 x) {
    return vec2(smoothstep(e0, e1, x.x), smoothstep(e0, e1, x.y));
}
__device__ __forceinline__ vec3 smoothstep(float e0, float e1, vec3 x) {
    return vec3(smoothstep(e0, e1, x.x), smoothstep(e0, e1, x.y), smoothstep(e0, e1, x.z));
}
__device__ __forceinline__ float dot(vec2 a, vec2 b) { return a.x * b.x + a.y * b.y; }
__device__ __forceinline__ float dot(vec4 a, vec4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
__device__ __forceinline__ float length(vec2 a) { return sqrt(dot(a, a)); }
// |a| of a vec3 in the library's shapes (rm::length, or the hardware square root in the probe instance)
// (the probe form's sum of squares as explicit FMAs: rm_device.h's dot of the
// shared vec3 lies outside this instance's contraction pragma)
__device__ __forceinline__ float len3_(vec3 a) {
    return RM_LIB_PROBE ? __builtin_amdgcn_sqrtf(fmaf(a.z, a.z, fmaf(a.y, a.y, a.x * a.x))) : length(a);
}
__device__ __forceinline__ float distance(vec3 a, vec3 b) { return length(a - b); }
__device__ __forceinline__ vec2 normalize(vec2 a) { return a * (1.0f / length(a)); }
// dot, length, normalize, reflect and refract of vec3 are rm_device.h's (found
// through the argument type)
__device__ __forceinline__ vec3 cross(vec3 a, vec3 b) {
    return vec3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
// dot, length, normalize, reflect and refract of vec3 are rm_device.h's
// (found through the argument type)

// mat4 of four columns, as GLSL's mat4(vec4 c0, c1, c2, c3); the library
// multiplies row vectors: (v * M)[i] = dot(v, column i)
struct mat4 {
    vec4 c0, c1, c2, c3;
    mat4() = default;
    __host__ __device__ constexpr mat4(vec4 a, vec4 b, vec4 c, vec4 d) : c0(a), c1(b), c2(c), c3(d) {}
};
__device__ __forceinline__ vec4 operator*(vec4 v, const mat4& m) {
    return vec4(dot(v, m.c0), dot(v, m.c1), dot(v, m.c2), dot(v, m.c3));
}

// ----------------------------------------------------------- materials

// common.frag:57-61
struct SdResult {
    float dist;
    Material mat;
    SdResult() = default;
    __host__ __device__ constexpr SdResult(float d, const Material& m) : dist(d), mat(m) {}
};

// common.frag:37-53 (ALLOW_MATERIAL_BLENDING, as output_shader.frag:9 defines;
// RM_NO_MATERIAL_BLENDING selects the #else branch)
__device__ __forceinline__ Material blendMaterial(const Material& a, const Material& b, float k) {
#ifndef RM_NO_MATERIAL_BLENDING
    return Material(mix(a.diffuse, b.diffuse, k), mix(a.specular, b.specular, k), mix(a.shininess, b.shininess, k),
                    mix(a.reflectivity, b.reflectivity, k), mix(a.transparency, b.transparency, k),
                    mix(a.absorption, b.absorption, k), mix(a.refraction_index, b.refraction_index, k), mix(a.emission, b.emission, k));
#else
    return k < 0.5f ? a : b;
#endif
}

// ---------------------------------------------------------- operations

// common.frag:66-69
__device__ __forceinline__ SdResult sdUnion(const SdResult& a, const SdResult& b) { return a.dist < b.dist ? a : b; }

// common.frag:72-85: k.x blends the shape, k.y the material
__device__ __forceinline__ SdResult sminCubic(const SdResult& a, const SdResult& b, vec2 k) {
    k = max(k, 0.0001f);
    const vec2 x = max(k - fabsf(a.dist - b.dist), 0.0f);
    vec2 h = vec2(div_k(x.x, k.x), div_k(x.y, k.y));
    vec2 m = h * h * h * 0.5f;
    vec2 s = m * k * (1.0f / 3.0f);
    SdResult res;
    bool aCloser = a.dist < b.dist;
    res.dist = (aCloser ? a.dist : b.dist) - s.x;
    float blendCoeff = aCloser ? m.y : 1.0f - m.y;
    res.mat = blendMaterial(a.mat, b.mat, blendCoeff);
    return res;
}
// common.frag:87-89
__device__ __forceinline__ SdResult sminCubic(const SdResult& a, const SdResult& b, float k) {
    return sminCubic(a, b, vec2(k));
}

// common.frag:93-124
__device__ __forceinline__ float opUnion(float d1, float d2) { return min(d1, d2); }
__device__ __forceinline__ float opSubtraction(float d1, float d2) { return max(-d1, d2); }
__device__ __forceinline__ float opIntersection(float d1, float d2) { return max(d1, d2); }
__device__ __forceinline__ float opSmoothUnion(float d1, float d2, float k) {
    float h = clamp(0.5f + div_k(0.5f * (d2 - d1), k), 0.0f, 1.0f);
    return mix(d2, d1, h) - k * h * (1.0f - h);
}
__device__ __forceinline__ float opSmoothSubtraction(float d1, float d2, float k) {
    float h = clamp(0.5f - div_k(0.5f * (d2 + d1), k), 0.0f, 1.0f);
    return mix(d2, -d1, h) + k * h * (1.0f - h);
}
__device__ __forceinline__ float opSmoothIntersection(float d1, float d2, float k) {
    float h = clamp(0.5f - div_k(0.5f * (d2 - d1), k), 0.0f, 1.0f);
    return mix(d2, d1, h) + k * h * (1.0f - h);
}
// common.frag:128-131
__device__ __forceinline__ float sdf_blend(float d1, float d2, float a) { return a * d1 + (1.0f - a) * d2; }
// common.frag:135-139
__device__ __forceinline__ float smin(float a, float b, float k) {
    float h = clamp(0.5f + div_k(0.5f * (b - a), k), 0.0f, 1.0f);
    return mix(b, a, h) - k * h * (1.0f - h);
}
// common.frag:142-146
__device__ __forceinline__ float smin_exp(float a, float b, float k = 32.0f) {
    float res = exp(-k * a) + exp(-k * b);
    return div_k(-log(max(0.0001f, res)), k);
}
// common.frag:148-151
__device__ __forceinline__ float rounding(float d, float h = 0.1f) { return d - h; }

// ----------------------------------------------- transformations (fast)

// common.frag:155-158
__device__ __forceinline__ void translatePoint(vec3& p, vec3 offset) { p = p - offset; }
// common.frag:163-165 (for p.xz etc. pass a vec2 and write it back)
__device__ __forceinline__ void rotatePoint(vec2& p, float a) { p = cos(a) * p + sin(a) * vec2(p.y, -p.x); }
// common.frag:167-183
__device__ __forceinline__ vec3 rotatePointX(vec3 p, float a) {
    vec2 q = cos(a) * vec2(p.y, p.z) + sin(a) * vec2(p.z, -p.y);
    return vec3(p.x, q.x, q.y);
}
__device__ __forceinline__ vec3 rotatePointY(vec3 p, float a) {
    vec2 q = cos(a) * vec2(p.x, p.z) + sin(a) * vec2(p.z, -p.x);
    return vec3(q.x, p.y, q.y);
}
__device__ __forceinline__ vec3 rotatePointZ(vec3 p, float a) {
    vec2 q = cos(a) * vec2(p.x, p.y) + sin(a) * vec2(p.y, -p.x);
    return vec3(q.x, q.y, p.z);
}

// common.frag:185-186
#define scaleSDF(func, samplePoint, scaleFactor) (func((samplePoint) / (scaleFactor)) * (scaleFactor))
#define scaleSDF3(func, samplePoint, s_x, s_y, s_z) \
    (func((samplePoint) / ::rm::glsl::vec3(s_x, s_y, s_z)) * ::rm::glsl::min(s_x, ::rm::glsl::min(s_y, s_z)))

// ---------------------------------------------- transformations (mat4)

// common.frag:190-227 (angles in degrees)
__device__ __forceinline__ mat4 rotationX(float angle_deg) {
    float a = radians(angle_deg), c = cos(a), s = sin(a);
    return mat4(vec4(1, 0, 0, 0), vec4(0, c, -s, 0), vec4(0, s, c, 0), vec4(0, 0, 0, 1));
}
__device__ __forceinline__ mat4 rotationY(float angle_deg) {
    float a = radians(angle_deg), c = cos(a), s = sin(a);
    return mat4(vec4(c, 0, s, 0), vec4(0, 1, 0, 0), vec4(-s, 0, c, 0), vec4(0, 0, 0, 1));
}
__device__ __forceinline__ mat4 rotationZ(float angle_deg) {
    float a = radians(angle_deg), c = cos(a), s = sin(a);
    return mat4(vec4(c, -s, 0, 0), vec4(s, c, 0, 0), vec4(0, 0, 1, 0), vec4(0, 0, 0, 1));
}
// the `t` and `s` matrices of transform() (common.frag:250-264)
__device__ __forceinline__ mat4 translation_inv(vec3 pos) {
    return mat4(vec4(1, 0, 0, -pos.x), vec4(0, 1, 0, -pos.y), vec4(0, 0, 1, -pos.z), vec4(0, 0, 0, 1));
}
__device__ __forceinline__ mat4 scale_inv(vec3 scale) {
    return mat4(vec4(1.0f / scale.x, 0, 0, 0), vec4(0, 1.0f / scale.y, 0, 0), vec4(0, 0, 1.0f / scale.z, 0),
                vec4(0, 0, 0, 1));
}

// Row vectors times the structured matrices above, rounded as the full
// vec4 * mat4 product rounds them: a product with an exact 0 or 1 entry is an
// exact zero or the operand itself, and adding an exact zero leaves a sum
// unchanged for finite operands (up to the sign of a zero result), so only the
// other terms are formed, in the dot product's order.  (IEEE semantics keep
// the compiler from dropping x * 0 itself: it is NaN for an infinite x.)
struct Rot {
    float c, s;
};
__device__ __forceinline__ Rot rot_of(float angle_deg) {  // cos / sin as rotationX/Y/Z form them
    float a = radians(angle_deg);
    return Rot{cos(a), sin(a)};
}
// The probe instance drops a rotation whose sine is a compile-time zero (an
// angle of 0 in the scene source: the cosine is then 1, the product the
// identity); the exact instance keeps the GLSL's products (x * 0 is not
// foldable in IEEE arithmetic).
__device__ __forceinline__ bool rot_is_identity(Rot r) {
    return RM_LIB_PROBE && __builtin_constant_p(r.s) && __builtin_constant_p(r.c) && r.s == 0.0f && r.c == 1.0f;
}
__device__ __forceinline__ vec4 mul_rx(vec4 v, Rot r) {  // v * rotationX
    if (rot_is_identity(r)) return v;
    return vec4(v.x, v.y * r.c + v.z * -r.s, v.y * r.s + v.z * r.c, v.w);
}
__device__ __forceinline__ vec4 mul_ry(vec4 v, Rot r) {  // v * rotationY
    if (rot_is_identity(r)) return v;
    return vec4(v.x * r.c + v.z * r.s, v.y, v.x * -r.s + v.z * r.c, v.w);
}
__device__ __forceinline__ vec4 mul_rz(vec4 v, Rot r) {  // v * rotationZ
    if (rot_is_identity(r)) return v;
    return vec4(v.x * r.c + v.y * -r.s, v.x * r.s + v.y * r.c, v.z, v.w);
}
__device__ __forceinline__ vec4 mul_t(vec4 v, vec3 pos) {  // v * translation_inv(pos)
    return vec4(v.x + v.w * -pos.x, v.y + v.w * -pos.y, v.z + v.w * -pos.z, v.w);
}
__device__ __forceinline__ vec4 mul_s(vec4 v, vec3 scale) {  // v * scale_inv(scale)
    return vec4(v.x * (1.0f / scale.x), v.y * (1.0f / scale.y), v.z * (1.0f / scale.z), v.w);
}
__device__ __forceinline__ vec4 mul_yxz(vec4 v, vec3 rot) {  // v * r_y * r_x * r_z
    return mul_rz(mul_rx(mul_ry(v, rot_of(-rot.y)), rot_of(-rot.x)), rot_of(-rot.z));
}

// common.frag:248-267
__device__ __forceinline__ vec3 transform(vec3 sp, vec3 pos, vec3 rot, vec3 scale) {
    return xyz(mul_s(mul_yxz(mul_t(vec4(sp, 1.0f), pos), rot), scale));
}
// common.frag:269-282
__device__ __forceinline__ vec3 transformTR(vec3 sp, vec3 pos, vec3 rot) {
    return xyz(mul_yxz(mul_t(vec4(sp, 1.0f), pos), rot));
}
// common.frag:284-321
__device__ __forceinline__ vec3 transformTRX(vec3 sp, vec3 pos, float rot_x) {
    return xyz(mul_rx(mul_t(vec4(sp, 1.0f), pos), rot_of(-rot_x)));
}
__device__ __forceinline__ vec3 transformTRY(vec3 sp, vec3 pos, float rot_y) {
    return xyz(mul_ry(mul_t(vec4(sp, 1.0f), pos), rot_of(-rot_y)));
}
__device__ __forceinline__ vec3 transformTRZ(vec3 sp, vec3 pos, float rot_z) {
    return xyz(mul_rz(mul_t(vec4(sp, 1.0f), pos), rot_of(-rot_z)));
}
// common.frag:323-378
__device__ __forceinline__ vec3 transformTRXS(vec3 sp, vec3 pos, float rot_x, vec3 scale) {
    return xyz(mul_s(mul_rx(mul_t(vec4(sp, 1.0f), pos), rot_of(-rot_x)), scale));
}
__device__ __forceinline__ vec3 transformTRYS(vec3 sp, vec3 pos, float rot_y, vec3 scale) {
    return xyz(mul_s(mul_ry(mul_t(vec4(sp, 1.0f), pos), rot_of(-rot_y)), scale));
}
__device__ __forceinline__ vec3 transformTRZS(vec3 sp, vec3 pos, float rot_z, vec3 scale) {
    return xyz(mul_s(mul_rz(mul_t(vec4(sp, 1.0f), pos), rot_of(-rot_z)), scale));
}
// common.frag:380-432
__device__ __forceinline__ vec3 transformTRS1(vec3 sp, vec3 pos, vec3 rot, float scale) {
    return xyz(mul_yxz(mul_t(vec4(sp, 1.0f), pos), rot)) / scale;
}
__device__ __forceinline__ vec3 transformTRXS1(vec3 sp, vec3 pos, float rot_x, float scale) {
    return xyz(mul_rx(mul_t(vec4(sp, 1.0f), pos), rot_of(-rot_x))) / scale;
}
__device__ __forceinline__ vec3 transformTRYS1(vec3 sp, vec3 pos, float rot_y, float scale) {
    return xyz(mul_ry(mul_t(vec4(sp, 1.0f), pos), rot_of(-rot_y))) / scale;
}
__device__ __forceinline__ vec3 transformTRZS1(vec3 sp, vec3 pos, float rot_z, float scale) {
    return xyz(mul_rz(mul_t(vec4(sp, 1.0f), pos), rot_of(-rot_z))) / scale;
}
// common.frag:434-462
__device__ __forceinline__ vec3 transformR(vec3 sp, vec3 rot) { return xyz(mul_yxz(vec4(sp, 1.0f), rot)); }
__device__ __forceinline__ vec3 transformRX(vec3 sp, float rot_x) { return xyz(mul_rx(vec4(sp, 1.0f), rot_of(-rot_x))); }
__device__ __forceinline__ vec3 transformRY(vec3 sp, float rot_y) { return xyz(mul_ry(vec4(sp, 1.0f), rot_of(-rot_y))); }
__device__ __forceinline__ vec3 transformRZ(vec3 sp, float rot_z) { return xyz(mul_rz(vec4(sp, 1.0f), rot_of(-rot_z))); }
// common.frag:464-501
__device__ __forceinline__ vec3 transformRXS(vec3 sp, float rot_x, vec3 scale) {
    return xyz(mul_s(mul_rx(vec4(sp, 1.0f), rot_of(-rot_x)), scale));
}
__device__ __forceinline__ vec3 transformRYS(vec3 sp, float rot_y, vec3 scale) {
    return xyz(mul_s(mul_ry(vec4(sp, 1.0f), rot_of(-rot_y)), scale));
}
__device__ __forceinline__ vec3 transformRZS(vec3 sp, float rot_z, vec3 scale) {
    return xyz(mul_s(mul_rz(vec4(sp, 1.0f), rot_of(-rot_z)), scale));
}
// common.frag:503-531
__device__ __forceinline__ vec3 transformRS1(vec3 sp, vec3 rot, float scale) {
    return xyz(mul_yxz(vec4(sp, 1.0f), rot)) / scale;
}
__device__ __forceinline__ vec3 transformRXS1(vec3 sp, float rot_x, float scale) {
    return xyz(mul_rx(vec4(sp, 1.0f), rot_of(-rot_x))) / scale;
}
__device__ __forceinline__ vec3 transformRYS1(vec3 sp, float rot_y, float scale) {
    return xyz(mul_ry(vec4(sp, 1.0f), rot_of(-rot_y))) / scale;
}
__device__ __forceinline__ vec3 transformRZS1(vec3 sp, float rot_z, float scale) {
    return xyz(mul_rz(vec4(sp, 1.0f), rot_of(-rot_z))) / scale;
}

// --------------------------------------------------- domain operations

// common.frag:538-543
__device__ __forceinline__ float pMod1(float& p, float size) {
    float halfsize = size * 0.5f;
    float c = floor((p + halfsize) / size);
    p = mod(p + halfsize, size) - halfsize;
    return c;
}
// common.frag:546-550
__device__ __forceinline__ vec2 pMod2(vec2& p, vec2 size) {
    vec2 c = floor((p + size * 0.5f) / size);
    p = mod(p + size * 0.5f, size) - size * 0.5f;
    return c;
}
// common.frag:553-557
__device__ __forceinline__ float pMirror(float& p, float dist) {
    float s = (p < 0.0f) ? -1.0f : 1.0f;
    p = fabsf(p) - dist;
    return s;
}
// common.frag:560-566
__device__ __forceinline__ float pReflect(vec3& p, vec3 planeNormal, float offset) {
    float t = dot(p, planeNormal) + offset;
    if (t < 0.0f) p = p - (2.0f * t) * planeNormal;
    return (t < 0.0f) ? -1.0f : 1.0f;
}

// -------------------------------------------------------------- shapes

// common.frag:572-617
__device__ __forceinline__ float plane(vec3 p) { return p.y; }
__device__ __forceinline__ float sdPlane(vec3 p, vec4 n) { return dot(p, xyz(n)) + n.w; }
__device__ __forceinline__ float sphere(vec4 s, vec3 p) { return len3_(p - xyz(s)) - s.w; }
__device__ __forceinline__ float cube(vec4 s, vec3 p) {
    vec3 q = abs(p - xyz(s)) - s.w;
    return len3_(max(q, 0.0f)) + min(max(q.x, max(q.y, q.z)), 0.0f);
}
// = mc exactly: if mc <= 0 every max(di, 0) is 0 and min(mc, 0) = mc;
// otherwise the rounded sum of squares is >= RN(mc^2), whose correctly rounded
// square root is mc, so the length is >= mc (a plugin's sqrt is correctly
// rounded, rm_plugin_host.cpp).  No length, no sqrt.
__device__ __forceinline__ float sdBox(vec3 p, vec3 b) {
    vec3 di = abs(p) - b;
    return max(di.x, max(di.y, di.z));
}
__device__ __forceinline__ float cylinder(vec3 p, float r) { return length(xy(p)) - r; }
__device__ __forceinline__ float cone(vec3 p, vec2 c) {  // c must be normalized
    float q = length(xy(p));
    return dot(c, vec2(q, p.z));
}
__device__ __forceinline__ float torus(vec3 p, vec2 t) {
    vec2 q = vec2(length(xy(p)) - t.x, p.z);
    return length(q) - t.y;
}

// common.frag:622-651
__device__ __forceinline__ float mandelbulb(vec3 p, vec4& resColor) {
    vec3 w = p;
    float m = dot(w, w);
    vec4 trap = vec4(abs(w), m);
    float dz = 1.0f;
    for (int i = 0; i < 4; i++) {
        dz = 8.0f * pow(m, 3.5f) * dz + 1.0f;
        float r = len3_(w);
        float b = 8.0f * acos(w.y / r);
        float a = 8.0f * atan(w.x, w.z);
        w = p + pow(r, 8.0f) * vec3(sin(b) * sin(a), cos(b), sin(b) * cos(a));
        trap = min(trap, vec4(abs(w), m));
        m = dot(w, w);
        if (m > 256.0f) break;
    }
    resColor = vec4(m, trap.y, trap.z, trap.w);
    return 0.25f * log(m) * sqrt(m) / dz;
}

// common.frag:654-679 (res = (d, 0.2 da db dc, (1 + m) / 4) of the last fold that won)
__device__ __forceinline__ vec3 mengersponge(vec3 p) {
    float d = sdBox(p, vec3(1.0f));
    vec3 res = vec3(d, 1.0f, 0.0f);
    float s = 1.0f;
    for (int m = 0; m < 3; m++) {
        // fold m yields c = (min(da, db, dc) - 1) / s <= 1/s (r <= 2), so once
        // d >= RN(1/s) no later fold can win `c > d`: an exact early exit
        // (rm_device.h sponge_folds), which skips the folds far from the sponge
        // (wave-uniform, as rm_device.h sponge_folds: a fold runs while any lane
        // needs it, and leaves d and res unchanged on the lanes past their exit;
        // a per-lane break was if-converted, every fold computed on every call)
        if (__builtin_amdgcn_ballot_w64(d < 1.0f / (s * 3.0f)) == 0) break;
        // r = abs(1 - 3 abs(mod(p s, 2) - 1)) as rm_device.h sponge_folds forms it
        // (round 5: 29 -> ~17 VALU per fold in the probe instance).  With
        // h = x (s/2) (exact: s/2 is a power of 3 over 2 and x s / 2 = RN(x s) / 2),
        // the exact instance's mod(x s, 2) - 1 is fma(2, h - floor(h), -1), the
        // same bits as the GLSL's x s - 2 floor(x s / 2) - 1 (one rounding);
        // the probe instance uses |mod(x s, 2) - 1| = 2 |g|, g = y - rint(y),
        // y = x s/2 - 1/2 (the distance to the nearest k + 1/2), one fma less
        // and no floor.  min(max(rx, ry), max(ry, rz), max(rz, rx)) is their
        // median (v_med3).
        const float sh = s * 0.5f;
        vec3 r;
        if (RM_LIB_PROBE) {
            const float yx = fmaf(p.x, sh, -0.5f), yy = fmaf(p.y, sh, -0.5f), yz = fmaf(p.z, sh, -0.5f);
            r = vec3(fabsf(fmaf(-6.0f, fabsf(yx - __builtin_rintf(yx)), 1.0f)),
                     fabsf(fmaf(-6.0f, fabsf(yy - __builtin_rintf(yy)), 1.0f)),
                     fabsf(fmaf(-6.0f, fabsf(yz - __builtin_rintf(yz)), 1.0f)));
        } else {
            const float hx = p.x * sh, hy = p.y * sh, hz = p.z * sh;
            r = vec3(fabsf(1.0f - 3.0f * fabsf(fmaf(2.0f, hx - floorf(hx), -1.0f))),
                     fabsf(1.0f - 3.0f * fabsf(fmaf(2.0f, hy - floorf(hy), -1.0f))),
                     fabsf(1.0f - 3.0f * fabsf(fmaf(2.0f, hz - floorf(hz), -1.0f))));
        }
        s *= 3.0f;
        float da = max(r.x, r.y);
        float db = max(r.y, r.z);
        float dc = max(r.z, r.x);
        float c = div_k(__builtin_amdgcn_fmed3f(r.x, r.y, r.z) - 1.0f, s);
        if (c > d) {
            d = c;
            res = vec3(d, 0.2f * da * db * dc, (1.0f + (float)m) / 4.0f);
        }
    }
    return res;
}

constexpr float PI = 3.1416f;  // common.frag:1108

