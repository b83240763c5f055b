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

// ------------------------------------------------------------------ bloom
//
// shaders/post/bloom.frag:14-43 over the mip chain of main.cpp:212-214
// (postTexture.setSmooth(true); generateMipmap(): MIN LINEAR_MIPMAP_LINEAR,
// MAG LINEAR, CLAMP_TO_EDGE).  Only the levels bloom.frag reads are built:
// textureLod at lod = log2(0.05 H) blends levels floor(lod) and floor(lod)+1.
// A level is the bilinear resample of the one above at its texel centres in
// the 0..255 domain, rounded to nearest even (SwiftShader's glGenerateMipmap,
// bit for bit on even sizes; tests/test_bloom.py).  Same float operations,
// in the same order, as oracle/rm_oracle.c (no contraction in this TU).

__device__ __forceinline__ int clampi(int v, int hi) { return v < 0 ? 0 : (v > hi ? hi : v); }

__global__ __launch_bounds__(256) void rm_mip_down_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                          int w, int h, int w1, int h1, float sx, float sy) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= w1 || y >= h1) return;
    const float v = ((float)y + 0.5f) * sy - 0.5f, u = ((float)x + 0.5f) * sx - 0.5f;
    const float fy = floorf(v), fx = floorf(u), b = v - fy, a = u - fx;
    const int y0 = clampi((int)fy, h - 1), y1 = clampi((int)fy + 1, h - 1);
    const int x0 = clampi((int)fx, w - 1), x1 = clampi((int)fx + 1, w - 1);
    const uint32_t t00 = in[(size_t)y0 * w + x0], t01 = in[(size_t)y0 * w + x1];
    const uint32_t t10 = in[(size_t)y1 * w + x0], t11 = in[(size_t)y1 * w + x1];
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < 32; c += 8) {
        const float c00 = (float)((t00 >> c) & 255u), c01 = (float)((t01 >> c) & 255u);
        const float c10 = (float)((t10 >> c) & 255u), c11 = (float)((t11 >> c) & 255u);
        const float r0 = (1.0f - a) * c00 + a * c01, r1 = (1.0f - a) * c10 + a * c11;
        r |= (uint32_t)__float2int_rn((1.0f - b) * r0 + b * r1) << c;
    }
    out[(size_t)y * w1 + x] = r;
}

struct Level {
    const uint32_t* p;
    int w, h;
};

// bilinear fetch at normalized (u, v), CLAMP_TO_EDGE, unorm8 -> c * (1/255)
__device__ __forceinline__ RGB tex_bilinear(Level L, float u, float v) {
    const float x = u * (float)L.w - 0.5f, y = v * (float)L.h - 0.5f;
    const float fx = floorf(x), fy = floorf(y), a = x - fx, b = y - fy;
    const int x0 = clampi((int)fx, L.w - 1), x1 = clampi((int)fx + 1, L.w - 1);
    const int y0 = clampi((int)fy, L.h - 1), y1 = clampi((int)fy + 1, L.h - 1);
    const uint32_t t00 = L.p[(size_t)y0 * L.w + x0], t01 = L.p[(size_t)y0 * L.w + x1];
    const uint32_t t10 = L.p[(size_t)y1 * L.w + x0], t11 = L.p[(size_t)y1 * L.w + x1];
    float o[3];
    const float k = 1.0f / 255.0f;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const int s = 8 * c;
        const float c00 = (float)((t00 >> s) & 255u) * k, c01 = (float)((t01 >> s) & 255u) * k;
        const float c10 = (float)((t10 >> s) & 255u) * k, c11 = (float)((t11 >> s) & 255u) * k;
        const float r0 = (1.0f - a) * c00 + a * c01, r1 = (1.0f - a) * c10 + a * c11;
        o[c] = (1.0f - b) * r0 + b * r1;
    }
    return RGB{o[0], o[1], o[2]};
}

// bloom.frag:33-43, one lane per output pixel, 16x16-pixel workgroups
__global__ __launch_bounds__(256) void rm_bloom_kernel(Level L0, Level L1, Level L2, uint32_t* __restrict__ out,
                                                       int W, int H, float lod, float fr) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    const float G[3][3] = {{41.0f / 273.0f, 26.0f / 273.0f, 7.0f / 273.0f},
                           {26.0f / 273.0f, 16.0f / 273.0f, 4.0f / 273.0f},
                           {7.0f / 273.0f, 4.0f / 273.0f, 1.0f / 273.0f}};
    const float u = ((float)x + 0.5f) / (float)W, v = 1.0f - ((float)y + 0.5f) / (float)H;  // bloom.frag:36
    RGB color = tex_bilinear(L0, u, v);
    const float scale = 0.05f, iaspect = (float)H / (float)W;
    RGB bl{0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int j = -2; j <= 2; j++)
#pragma unroll
        for (int i = -2; i <= 2; i++) {
            const float uu = u + ((float)i * iaspect) * scale, vv = v + (float)j * scale;
            RGB s;
            if (lod <= 0.0f) {
                s = tex_bilinear(L0, uu, vv);  // magnification: the base level
            } else {
                const RGB s1 = tex_bilinear(L1, uu, vv), s2 = tex_bilinear(L2, uu, vv);
                s = RGB{(1.0f - fr) * s1.r + fr * s2.r, (1.0f - fr) * s1.g + fr * s2.g, (1.0f - fr) * s1.b + fr * s2.b};
            }
            const float g = G[i < 0 ? -i : i][j < 0 ? -j : j];
            bl = RGB{bl.r + g * s.r, bl.g + g * s.g, bl.b + g * s.b};
        }
    color = RGB{color.r + gmax_(bl.r - 0.3f, 0.0f), color.g + gmax_(bl.g - 0.3f, 0.0f),
                color.b + gmax_(bl.b - 0.3f, 0.0f)};
    out[(size_t)y * W + x] = unorm8(color.r) | (unorm8(color.g) << 8) | (unorm8(color.b) << 16) | (255u << 24);
}

BloomPlan bloom_plan(int W, int H) {
    BloomPlan p{};
    int q = 0;
    for (int m = W > H ? W : H; m > 1; m >>= 1) q++;
    p.lod = log2f(0.05f * (float)H);  // bloom.frag:22 (u_resolution = the image, post_bloom.cpp:6)
    if (p.lod > 0.0f) {
        p.d1 = (int)floorf(p.lod);
        p.d1 = p.d1 > q ? q : p.d1;
        p.d2 = p.d1 + 1 > q ? q : p.d1 + 1;
    }
    p.fr = p.lod - floorf(p.lod);
    int w = W, h = H;
    p.w[0] = W;
    p.h[0] = H;
    for (int k = 1; k <= p.d2; k++) {
        w = w > 1 ? w >> 1 : 1;
        h = h > 1 ? h >> 1 : 1;
        p.w[k] = w;
        p.h[k] = h;
        p.offset[k] = p.texels;
        p.texels += (size_t)w * h;
    }
    return p;
}

hipError_t launch_bloom(const uint32_t* in, uint32_t* out, uint32_t* mips, const BloomPlan& p, hipStream_t s) {
    const int W = p.w[0], H = p.h[0];
    if (W <= 0 || H <= 0) return hipSuccess;
    const uint32_t* lv[40] = {in};
    for (int k = 1; k <= p.d2; k++) {
        uint32_t* dst = mips + p.offset[k];
        const int w = p.w[k - 1], h = p.h[k - 1], w1 = p.w[k], h1 = p.h[k];
        hipLaunchKernelGGL(rm_mip_down_kernel, dim3((w1 + 15) / 16, (h1 + 15) / 16), dim3(256), 0, s, lv[k - 1], dst,
                           w, h, w1, h1, (float)w / (float)w1, (float)h / (float)h1);
        lv[k] = dst;
    }
    const Level L0{in, W, H}, L1{lv[p.d1], p.w[p.d1], p.h[p.d1]}, L2{lv[p.d2], p.w[p.d2], p.h[p.d2]};
    hipLaunchKernelGGL(rm_bloom_kernel, dim3((W + 15) / 16, (H + 15) / 16), dim3(256), 0, s, L0, L1, L2, out, W, H,
                       p.lod, p.fr);
    return hipGetLastError();
}

}  // namespace rm
