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
// Four pixels per lane, 64x16-pixel workgroups (neighbour texels are re-read
// from L1/L2; 4 B in + 4 B out of HBM per pixel).
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

__device__ __forceinline__ uint32_t fxaa_px(const uint32_t* __restrict__ in, int W, int H, int x, int y) {
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
    return unorm8(c.r) | (unorm8(c.g) << 8) | (unorm8(c.b) << 16) | (unorm8(alpha) << 24);
}

// One lane per 4 pixels (rows y, y+4, y+8, y+12 of a 64x16-pixel workgroup
// tile): the kernel is latency-bound (two dependent rounds of L2 taps per
// pixel), so each lane keeps four pixels' taps in flight at once.
constexpr int FXAA_TX = 64, FXAA_TY = 16, FXAA_PX = 4;
__global__ __launch_bounds__(256) void rm_fxaa_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       int W, int H) {
    const int x = blockIdx.x * FXAA_TX + (threadIdx.x & 63);
    const int y0 = blockIdx.y * FXAA_TY + (threadIdx.x >> 6);
    if (x >= W) return;
    uint32_t r[FXAA_PX];
#pragma unroll
    for (int k = 0; k < FXAA_PX; k++) {
        const int y = y0 + 4 * k;
        r[k] = fxaa_px(in, W, H, x, y < H ? y : H - 1);  // straight-line: the four pixels' taps overlap
    }
#pragma unroll
    for (int k = 0; k < FXAA_PX; k++) {
        const int y = y0 + 4 * k;
        if (y < H) out[(size_t)y * W + x] = r[k];
    }
}

hipError_t launch_fxaa(const uint32_t* in, uint32_t* out, int W, int H, hipStream_t s) {
    if (W <= 0 || H <= 0) return hipSuccess;
    dim3 grid((W + FXAA_TX - 1) / FXAA_TX, (H + FXAA_TY - 1) / FXAA_TY);
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

// bloom.frag:33-43, one lane per output pixel, 16x16-pixel workgroups.  The
// general form: any lod, the levels read as RGBA8 words.  Used when lod <= 0
// (magnification: every tap reads the base level).
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

// The two minified levels bloom.frag reads, unpacked once to c * (1/255)
// floats (the same product tex_bilinear forms per tap): RGB + pad.
__global__ __launch_bounds__(256) void rm_level_f4_kernel(const uint32_t* __restrict__ a, int na,
                                                          const uint32_t* __restrict__ b, int nb,
                                                          float4* __restrict__ out) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= na + nb) return;
    const uint32_t w = t < na ? a[t] : b[t - na];
    const float k = 1.0f / 255.0f;
    out[t] = make_float4((float)(w & 255u) * k, (float)((w >> 8) & 255u) * k, (float)((w >> 16) & 255u) * k, 0.0f);
}

struct LevelF {
    const float4* __restrict__ p;
    int w, h;
};

// One bilinear axis of a tap: weight and the two clamped texel indices.
struct Axis {
    float f;
    int i0, i1;
    bool uni;    // i0, i1 the same on every active lane of the wave
    int so0, so1;  // when uni: i0, i1 times the axis' byte stride (wave-uniform)
};

__device__ __forceinline__ Axis axis(float t, int n, int stride) {
    const float x = t * (float)n - 0.5f, fx = floorf(x);
    Axis A;
    A.f = x - fx;
    A.i0 = clampi((int)fx, n - 1);
    A.i1 = clampi((int)fx + 1, n - 1);
    const int f0 = __builtin_amdgcn_readfirstlane(A.i0), f1 = __builtin_amdgcn_readfirstlane(A.i1);
    A.uni = __builtin_amdgcn_ballot_w64(A.i0 == f0 && A.i1 == f1) == __builtin_amdgcn_read_exec();
    A.so0 = f0 * stride;
    A.so1 = f1 * stride;
    return A;
}

__device__ __forceinline__ RGB lerp2(float4 t00, float4 t01, float4 t10, float4 t11, float a, float b) {
    const float ia = 1.0f - a, ib = 1.0f - b;
    const float r0 = ia * t00.x + a * t01.x, r1 = ia * t10.x + a * t11.x;
    const float g0 = ia * t00.y + a * t01.y, g1 = ia * t10.y + a * t11.y;
    const float b0 = ia * t00.z + a * t01.z, b1 = ia * t10.z + a * t11.z;
    return RGB{ib * r0 + b * r1, ib * g0 + b * g1, ib * b0 + b * b1};
}

// tex_bilinear over an unpacked level.  When both axes pick the same texels on
// every lane (a wave is an 8x8-pixel tile; at 4096^2 a level texel spans 128+
// pixels) the four texels are fetched once per wave through the scalar cache
// into SGPRs; otherwise per lane.  Same floats, same operations either way.
// Four float4 texels at wave-uniform byte offsets through the scalar cache
// (read-only: the level was written by the previous launch on the stream).
__device__ __forceinline__ void sload4(const float4* base, int o00, int o01, int o10, int o11, float4& t00, float4& t01,
                                       float4& t10, float4& t11) {
    asm volatile(
        "s_load_dwordx4 %0, %4, %5\n\t"
        "s_load_dwordx4 %1, %4, %6\n\t"
        "s_load_dwordx4 %2, %4, %7\n\t"
        "s_load_dwordx4 %3, %4, %8\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(t00), "=&s"(t01), "=&s"(t10), "=&s"(t11)
        : "s"(base), "s"(o00), "s"(o01), "s"(o10), "s"(o11)
        : "memory");
}

// Both levels' quads of one tap: eight loads in flight, one wait.
__device__ __forceinline__ void sload8(const float4* a, int a00, int a01, int a10, int a11, const float4* b, int b00,
                                       int b01, int b10, int b11, float4 (&t)[8]) {
    asm volatile(
        "s_load_dwordx4 %0, %8, %9\n\t"
        "s_load_dwordx4 %1, %8, %10\n\t"
        "s_load_dwordx4 %2, %8, %11\n\t"
        "s_load_dwordx4 %3, %8, %12\n\t"
        "s_load_dwordx4 %4, %13, %14\n\t"
        "s_load_dwordx4 %5, %13, %15\n\t"
        "s_load_dwordx4 %6, %13, %16\n\t"
        "s_load_dwordx4 %7, %13, %17\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(t[0]), "=&s"(t[1]), "=&s"(t[2]), "=&s"(t[3]), "=&s"(t[4]), "=&s"(t[5]), "=&s"(t[6]), "=&s"(t[7])
        : "s"(a), "s"(a00), "s"(a01), "s"(a10), "s"(a11), "s"(b), "s"(b00), "s"(b01), "s"(b10), "s"(b11)
        : "memory");
}

// Waterfall over the distinct texel quads of a tap that the wave's lanes need:
// the first remaining lane's quad is fetched into SGPRs, the lanes that share
// it interpolate and leave.
__device__ __forceinline__ RGB tap_waterfall(const LevelF& L, const Axis& X, const Axis& Y) {
    RGB r;
    for (;;) {
        const int x0 = __builtin_amdgcn_readfirstlane(X.i0), x1 = __builtin_amdgcn_readfirstlane(X.i1);
        const int y0 = __builtin_amdgcn_readfirstlane(Y.i0), y1 = __builtin_amdgcn_readfirstlane(Y.i1);
        if (X.i0 == x0 && X.i1 == x1 && Y.i0 == y0 && Y.i1 == y1) {
            const int r0 = y0 * L.w, r1 = y1 * L.w;
            float4 t00, t01, t10, t11;
            sload4(L.p, __builtin_amdgcn_readfirstlane((r0 + x0) * 16), __builtin_amdgcn_readfirstlane((r0 + x1) * 16),
                   __builtin_amdgcn_readfirstlane((r1 + x0) * 16), __builtin_amdgcn_readfirstlane((r1 + x1) * 16),
                   t00, t01, t10, t11);
            r = lerp2(t00, t01, t10, t11, X.f, Y.f);
            break;
        }
    }
    return r;
}

// One tap of bloom.frag:26 over levels A (d1) and B (d2), before the level
// mix.  A wave is an 8x8-pixel tile and a level texel spans 2^d1 >= 0.025 H
// pixels, so at frame sizes the wave's lanes nearly always share one texel
// quad per level: both quads are fetched once into SGPRs and every lane
// interpolates.  Otherwise the waterfall.  Same floats, same operations.
__device__ __forceinline__ void tap2(const LevelF& A, const LevelF& B, const Axis& xa, const Axis& ya, const Axis& xb,
                                     const Axis& yb, RGB& s1, RGB& s2) {
    if (xa.uni && ya.uni && xb.uni && yb.uni) {
        float4 t[8];
        sload8(A.p, ya.so0 + xa.so0, ya.so0 + xa.so1, ya.so1 + xa.so0, ya.so1 + xa.so1, B.p, yb.so0 + xb.so0,
               yb.so0 + xb.so1, yb.so1 + xb.so0, yb.so1 + xb.so1, t);
        s1 = lerp2(t[0], t[1], t[2], t[3], xa.f, ya.f);
        s2 = lerp2(t[4], t[5], t[6], t[7], xb.f, yb.f);
    } else {
        s1 = tap_waterfall(A, xa, ya);
        s2 = tap_waterfall(B, xb, yb);
    }
}

// bloom.frag:33-43 for lod > 0 (minification: levels d1, d2 blended by fr).
// One wave per 8x8-pixel tile, 2x2 waves per workgroup.  The tap coordinates
// depend on x or y alone, so the 10 column and 10 row axes are formed once per
// lane (the general kernel forms them per tap: same values).
// 5 waves per SIMD (<= 96 VGPRs, a 32-byte spill): hides more scalar-load latency than 4 (-4 %)
#ifndef RM_BLOOM_WAVES
#define RM_BLOOM_WAVES 5
#endif
__global__ __launch_bounds__(256, RM_BLOOM_WAVES) void rm_bloom_min_kernel(Level L0, LevelF A, LevelF B, uint32_t* __restrict__ out,
                                                           int W, int H, float fr) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wv & 1) * 8 + (lane & 7), y = blockIdx.y * 16 + (wv >> 1) * 8 + (lane >> 3);
    if (x >= W || y >= H) return;
    const float G[3][3] = {{41.0f / 273.0f, 26.0f / 273.0f, 7.0f / 273.0f},
                           {26.0f / 273.0f, 16.0f / 273.0f, 4.0f / 273.0f},
                           {7.0f / 273.0f, 4.0f / 273.0f, 1.0f / 273.0f}};
    const float u = ((float)x + 0.5f) / (float)W, v = 1.0f - ((float)y + 0.5f) / (float)H;  // bloom.frag:36
    RGB color = tex_bilinear(L0, u, v);
    const float scale = 0.05f, iaspect = (float)H / (float)W;
    Axis xa[5], xb[5];
#pragma unroll
    for (int i = -2; i <= 2; i++) {
        const float uu = u + ((float)i * iaspect) * scale;
        xa[i + 2] = axis(uu, A.w, 16);
        xb[i + 2] = axis(uu, B.w, 16);
    }
    RGB bl{0.0f, 0.0f, 0.0f};
#pragma unroll 1
    for (int j = -2; j <= 2; j++) {  // rolled: keeps the tap addresses of one row live, not all 50
        const float vv = v + (float)j * scale;
        const Axis ya = axis(vv, A.h, 16 * A.w), yb = axis(vv, B.h, 16 * B.w);
        const int aj = j < 0 ? -j : j;
#pragma unroll
        for (int i = -2; i <= 2; i++) {
            RGB s1, s2;
            tap2(A, B, xa[i + 2], ya, xb[i + 2], yb, s1, s2);
            const RGB s{(1.0f - fr) * s1.r + fr * s2.r, (1.0f - fr) * s1.g + fr * s2.g, (1.0f - fr) * s1.b + fr * s2.b};
            const float g = G[i < 0 ? -i : i][aj];
            bl = RGB{bl.r + g * s.r, bl.g + g * s.g, bl.b + g * s.b};
        }
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
    if (p.lod > 0.0f) {  // levels d1, d2 unpacked to float4, 16-byte aligned
        p.f4_offset = (p.texels + 3) & ~(size_t)3;
        p.texels = p.f4_offset + 4 * ((size_t)p.w[p.d1] * p.h[p.d1] + (size_t)p.w[p.d2] * p.h[p.d2]);
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
    const Level L0{in, W, H};
    if (p.lod <= 0.0f) {
        hipLaunchKernelGGL(rm_bloom_kernel, dim3((W + 15) / 16, (H + 15) / 16), dim3(256), 0, s, L0, L0, L0, out, W, H,
                           p.lod, p.fr);
        return hipGetLastError();
    }
    const int na = p.w[p.d1] * p.h[p.d1], nb = p.w[p.d2] * p.h[p.d2];
    float4* f4 = reinterpret_cast<float4*>(mips + p.f4_offset);
    hipLaunchKernelGGL(rm_level_f4_kernel, dim3((na + nb + 255) / 256), dim3(256), 0, s, lv[p.d1], na, lv[p.d2], nb,
                       f4);
    const LevelF A{f4, p.w[p.d1], p.h[p.d1]}, B{f4 + na, p.w[p.d2], p.h[p.d2]};
    hipLaunchKernelGGL(rm_bloom_min_kernel, dim3((W + 15) / 16, (H + 15) / 16), dim3(256), 0, s, L0, A, B, out, W, H,
                       p.fr);
    return hipGetLastError();
}

}  // namespace rm
