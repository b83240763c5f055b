// rm_post.hip -- the FXAA post pass of the reference (post.frag:16-61, main
// :135-144) as a gfx950 stencil kernel over the RGBA8 frame the ray-march
// pass produced (it consumes the hot path's
// framebuffer directly).
//
// The reference samples u_main_tex with texture() on an sf::RenderTexture
// that was never setSmooth()ed or setRepeated(): GL_NEAREST, CLAMP_TO_EDGE;
// unorm8 texels become c * (1/255) floats and gl_FragColor is stored to an
// RGBA8 target with round-to-nearest.  post.frag flips the frame vertically
// (uv = (tc.x, 1 - tc.y)); that is part of the pass and is kept.
//
// Built without FMA contraction and with correctly rounded division (like
// rm_kernels_o.hip) so the float path is bit-identical to the restatement in
// oracle/rm_oracle.c; the nearest-texel choices then agree exactly too.
// One thread per output pixel, 16x16-pixel workgroups (neighbour texels are
// re-read from L1/L2; 4 B in + 4 B out of HBM per pixel).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rm_launch.h"

namespace rm {

struct RGB { float r, g, b; };

__device__ __forceinline__ float gmin_(float x, float y) { return y < x ? y : x; }
__device__ __forceinline__ float gmax_(float x, float y) { return x < y ? y : x; }

__device__ __forceinline__ uint32_t texel(const uint32_t* __restrict__ img, int W, int H, float u, float v) {
    int x = (int)floorf(u * (float)W);
    int y = (int)floorf(v * (float)H);
    x = x < 0 ? 0 : (x >= W ? W - 1 : x);
    y = y < 0 ? 0 : (y >= H ? H - 1 : y);
    return img[(size_t)y * W + x];
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

__global__ __launch_bounds__(256) void rm_fxaa_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       int W, int H) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    const float FXAA_REDUCE_MIN = 1.0f / 128.0f, FXAA_REDUCE_MUL = 1.0f / 8.0f, FXAA_SPAN_MAX = 8.0f;
    // post.frag:138: uv = vec2(gl_TexCoord.x, 1 - gl_TexCoord.y)
    const float fx = ((float)x + 0.5f) / (float)W;
    const float fy = 1.0f - ((float)y + 0.5f) / (float)H;
    const float ivx = 1.0f / (float)W, ivy = 1.0f / (float)H;  // inverseVP = 1 / u_resolution
    RGB rgbNW = rgb(texel(in, W, H, fx + -1.0f * ivx, fy + -1.0f * ivy));
    RGB rgbNE = rgb(texel(in, W, H, fx + 1.0f * ivx, fy + -1.0f * ivy));
    RGB rgbSW = rgb(texel(in, W, H, fx + -1.0f * ivx, fy + 1.0f * ivy));
    RGB rgbSE = rgb(texel(in, W, H, fx + 1.0f * ivx, fy + 1.0f * ivy));
    const uint32_t tM = texel(in, W, H, fx, fy);
    RGB rgbM = rgb(tM);
    float lNW = luma(rgbNW), lNE = luma(rgbNE), lSW = luma(rgbSW), lSE = luma(rgbSE), lM = luma(rgbM);
    float lMin = gmin_(lM, gmin_(gmin_(lNW, lNE), gmin_(lSW, lSE)));
    float lMax = gmax_(lM, gmax_(gmax_(lNW, lNE), gmax_(lSW, lSE)));
    float dx = -((lNW + lNE) - (lSW + lSE));
    float dy = ((lNW + lSW) - (lNE + lSE));
    float dirReduce = gmax_((lNW + lNE + lSW + lSE) * (0.25f * FXAA_REDUCE_MUL), FXAA_REDUCE_MIN);
    float rcpDirMin = 1.0f / (gmin_(fabsf(dx), fabsf(dy)) + dirReduce);
    dx = gmin_(FXAA_SPAN_MAX, gmax_(-FXAA_SPAN_MAX, dx * rcpDirMin)) * ivx;
    dy = gmin_(FXAA_SPAN_MAX, gmax_(-FXAA_SPAN_MAX, dy * rcpDirMin)) * ivy;
    const float k1 = 1.0f / 3.0f - 0.5f, k2 = 2.0f / 3.0f - 0.5f;
    RGB s1 = rgb(texel(in, W, H, fx + dx * k1, fy + dy * k1));
    RGB s2 = rgb(texel(in, W, H, fx + dx * k2, fy + dy * k2));
    RGB a = RGB{(s1.r + s2.r) * 0.5f, (s1.g + s2.g) * 0.5f, (s1.b + s2.b) * 0.5f};
    RGB s3 = rgb(texel(in, W, H, fx + dx * -0.5f, fy + dy * -0.5f));
    RGB s4 = rgb(texel(in, W, H, fx + dx * 0.5f, fy + dy * 0.5f));
    RGB b = RGB{a.r * 0.5f + (s3.r + s4.r) * 0.25f, a.g * 0.5f + (s3.g + s4.g) * 0.25f,
                a.b * 0.5f + (s3.b + s4.b) * 0.25f};
    float lB = luma(b);
    RGB c = (lB < lMin || lB > lMax) ? a : b;
    float alpha = (float)(tM >> 24) * (1.0f / 255.0f);
    out[(size_t)y * W + x] = unorm8(c.r) | (unorm8(c.g) << 8) | (unorm8(c.b) << 16) | (unorm8(alpha) << 24);
}

hipError_t launch_fxaa(const uint32_t* in, uint32_t* out, int W, int H, hipStream_t s) {
    if (W <= 0 || H <= 0) return hipSuccess;
    dim3 grid((W + 15) / 16, (H + 15) / 16);
    hipLaunchKernelGGL(rm_fxaa_kernel, grid, dim3(256), 0, s, in, out, W, H);
    return hipGetLastError();
}

}  // namespace rm
