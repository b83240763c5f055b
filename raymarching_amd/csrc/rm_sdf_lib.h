// rm_sdf_lib.h -- the reference's scene-authoring library for HIP scene plugins.
//
// A scene plugin (rm_plugin.h) is a source file that defines
//     SdResult sceneSDF(vec3 p)
// as output_shader.frag:38-48 / template.frag:39-43 do, with the functions of
// common.frag:37-679 under their GLSL names and argument meanings: materials
// (Material, blendMaterial), SdResult operations (sdUnion, sminCubic),
// distance operators (op*, smin, smin_exp, sdf_blend, rounding), point
// transformations (translatePoint, rotatePoint*, rotationX/Y/Z, transform*,
// the scaleSDF macros), domain repetition (pMod1/2, pMirror, pReflect) and
// shapes (plane, sdPlane, sphere, cube, sdBox, cylinder, cone, torus,
// mandelbulb, mengersponge), plus the GLSL built-ins they use (vec2/vec3/vec4,
// mat4 as four columns, min/max/clamp/mix/mod/fract/smoothstep/... with the
// GLSL 1.30 definitions).  The source translation of rm_plugin_host.cpp maps
// the GLSL spellings the C++ cannot take: float literals, file-scope `const`,
// `in`/`out`/`inout` parameters and swizzle reads (`s.xyz` -> swz3<0,1,2>(s)).
//
// Every function follows the GLSL expression order (a plugin's translation
// unit is compiled without FMA contraction and with correctly rounded '/' and
// sqrt, like scene O), so values match the reference GLSL to the precision of
// the transcendental functions; tests/test_plugins.py pins each one against
// SwiftShader runs of common.frag itself (tests/golden/LIB_kat.npz).
#pragma once
#include "rm_device.h"

namespace rm {

// vec3 arithmetic the GLSL scenes use (rm_device.h holds + - * and unary -)
__host__ __device__ constexpr V3 operator*(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
__host__ __device__ constexpr V3 operator/(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
__host__ __device__ constexpr V3 operator/(V3 a, V3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
__host__ __device__ constexpr V3 operator/(float s, V3 a) { return v3(s / a.x, s / a.y, s / a.z); }
__host__ __device__ constexpr V3 operator+(V3 a, float s) { return v3(a.x + s, a.y + s, a.z + s); }
__host__ __device__ constexpr V3 operator+(float s, V3 a) { return v3(s + a.x, s + a.y, s + a.z); }
__host__ __device__ constexpr V3 operator-(V3 a, float s) { return v3(a.x - s, a.y - s, a.z - s); }
__host__ __device__ constexpr V3 operator-(float s, V3 a) { return v3(s - a.x, s - a.y, s - a.z); }
__device__ __forceinline__ V3& operator+=(V3& a, V3 b) { return a = a + b; }
__device__ __forceinline__ V3& operator-=(V3& a, V3 b) { return a = a - b; }
__device__ __forceinline__ V3& operator*=(V3& a, V3 b) { return a = a * b; }
__device__ __forceinline__ V3& operator*=(V3& a, float s) { return a = a * s; }
__device__ __forceinline__ V3& operator/=(V3& a, float s) { return a = a / s; }

namespace glsl {
#define RM_LIB_PROBE 0
#include "rm_sdf_lib_body.h"
#undef RM_LIB_PROBE
namespace probe {
#pragma clang fp contract(fast)
#define RM_LIB_PROBE 1
#include "rm_sdf_lib_body.h"
#undef RM_LIB_PROBE
#pragma clang fp contract(off)
}  // namespace probe
}  // namespace glsl
}  // namespace rm
