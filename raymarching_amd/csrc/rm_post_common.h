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

// One texel of the next mip level by an exact halving (even level sizes): the
// bilinear resample of glGenerateMipmap at sx = sy = 2 has u = 2x + 0.5, a = b
// = 0.5 exactly and every float operation exact, so the texel is the mean of
// its 2x2 texels rounded half to even, per channel: (s + 1 + ((s >> 2) & 1))
// >> 2 for the 4-texel sum s (s = 4q + r: r < 2 -> q, r > 2 -> q + 1, r = 2 ->
// the even one of q, q + 1).  Two channels per 32-bit add (16-bit fields, sums
// <= 1020).  Used by bloom's mip pyramid (rm_post.hip) and by FXAA's level-3
// epilogue (rm_fxaa.hip, rm_post_chain).
__device__ __forceinline__ uint32_t mip_mean4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const uint32_t m = 0x00FF00FFu, one = 0x00010001u;
    const uint32_t lo = (a & m) + (b & m) + (c & m) + (d & m);
    const uint32_t hi = ((a >> 8) & m) + ((b >> 8) & m) + ((c >> 8) & m) + ((d >> 8) & m);
    return (((lo + one + ((lo >> 2) & one)) >> 2) & m) | ((((hi + one + ((hi >> 2) & one)) >> 2) & m) << 8);
}

}  // namespace rm
