// rm_post_common.h -- what the post passes (rm_fxaa.hip: FXAA, post.frag;
// rm_post.hip: bloom, bloom.frag) share: the texel fetch and unpacking of an
// RGBA8 frame in GL's unorm8 semantics, luma, and the RGBA8 store's rounding.
// Both translation units are built without FMA contraction and with
// correctly rounded division, so their float paths are bit-identical to
// oracle/rm_oracle.c.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rm_launch.h"

namespace rm {

struct RGB { float r, g, b; };

__device__ __forceinline__ float gmin_(float x, float y) { return y < x ? y : x; }
__device__ __forceinline__ float gmax_(float x, float y) { return x < y ? y : x; }

// NEAREST + CLAMP_TO_EDGE fetch.  Each clamp is one v_med3_i32, and the load
// takes a 32-bit byte offset from the uniform base (the saddr form, no 64-bit
// address math; rm_fxaa rejects frames of 2^30 texels or more).
__device__ __forceinline__ int clamp_med3(int v, int hi) {
    int r;
    asm("v_med3_i32 %0, %1, 0, %2" : "=v"(r) : "v"(v), "v"(hi));
    return r;
}
__device__ __forceinline__ uint32_t texel(const uint32_t* __restrict__ img, int W, int H, float u, float v) {
    const int x = clamp_med3((int)floorf(u * (float)W), W - 1);
    const int y = clamp_med3((int)floorf(v * (float)H), H - 1);
    const uint32_t off = (uint32_t)(y * W + x) * 4u;
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(img) + off);
}

__device__ __forceinline__ RGB rgb(uint32_t t) {
    const float k = 1.0f / 255.0f;
    return RGB{(float)(t & 255u) * k, (float)((t >> 8) & 255u) * k, (float)((t >> 16) & 255u) * k};
}

__device__ __forceinline__ float luma(RGB c) { return c.r * 0.299f + c.g * 0.587f + c.b * 0.114f; }

__device__ __forceinline__ uint32_t unorm8(float c) {
    c = c < 0.0f ? 0.0f : (c > 1.0f ? 1.0f : c);
    if (c != c) c = 0.0f;
    return (uint32_t)__float2int_rn(c * 255.0f);
}

// unorm8 of a finite colour: clamp as one v_med3, round to nearest
__device__ __forceinline__ uint32_t unorm8_finite(float c) {
    return (uint32_t)__float2int_rn(__builtin_amdgcn_fmed3f(c, 0.0f, 1.0f) * 255.0f);
}

}  // namespace rm
