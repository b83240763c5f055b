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

// The LDS-staged form (the default).  A workgroup renders a 64x32-pixel tile
// from the texels it can reach, staged once in LDS with their luma:
//  * the five +-1 / centre taps land on integer texels.  With fx = (x+.5)/W and
//    ivx = 1/W correctly rounded, (fx - ivx) W = x - 0.5 up to three
//    roundings of relative size 2^-24, i.e. within 3 * 2^-24 * (x + 1.5) <
//    0.5 for W <= 2^20, so floor gives x - 1 (x, x + 1 likewise; rows: 1 -
//    (y+.5)/H flips to H - 1 - y, +-1).  Their texel and luma are LDS reads:
//    no float address math, and each texel's luma is formed once per tile
//    instead of once per tap (same operations, same order: the same bits);
//  * the four span taps keep post.frag's float addressing exactly (fx + dx k,
//    NEAREST).  dx, dy are clamped to +-8 texels and |k| <= 0.5, so u W lies
//    within x + 0.5 +- 4 (+ roundings far below 0.5 for W <= 2^20) and the
//    texel within x +- 4: inside the block (halo 5).  The block holds the
//    CLAMP_TO_EDGE texel of every position, so the unclamped index minus the
//    block origin addresses it (clamped into the block, which only guards
//    memory: the bound above keeps it inside);
//  * lumas of unorm8 texels are never NaN, so GLSL min/max are v_min3/v_max3
//    and the span clamp one v_med3.
// Frames wider or taller than 2^20 use rm_fxaa_kernel.
#ifndef RM_FXAA_TY
#define RM_FXAA_TY 32
#endif
// RM_FXAA_ADDR: span taps addressed without the guard clamps (0.0782 ->
// 0.0742 ms at 4096^2, same frame; profiles/r05/fxaa_ab.log)
#ifndef RM_FXAA_ADDR
#define RM_FXAA_ADDR 1
#endif
#ifndef RM_FXAA_RCP_NR
#define RM_FXAA_RCP_NR 1
#endif
#ifndef RM_FXAA_F4
#define RM_FXAA_F4 0
#endif
constexpr int FXL_TX = 64, FXL_TY = RM_FXAA_TY, FXL_HALO = 5, FXL_W = FXL_TX + 2 * FXL_HALO, FXL_H = FXL_TY + 2 * FXL_HALO;
constexpr int FXL_MAX_DIM = 1 << 20;
static_assert((FXL_TY & (FXL_TY - 1)) == 0 && FXL_TY <= 64, "fy_lane: one lane per tile row");
__device__ __forceinline__ int clamp_to(int v, int hi) {  // v_med3_i32(v, 0, hi)
    int r;
    asm("v_med3_i32 %0, %1, 0, %2" : "=v"(r) : "v"(v), "v"(hi));
    return r;
}
__device__ __forceinline__ int floor_i32(float v) {  // (int)floorf(v) for |v| < 2^31: one v_cvt_flr_i32_f32
    int r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(v));
    return r;
}
// unorm8 of a finite colour: clamp as one v_med3, round to nearest
__device__ __forceinline__ uint32_t unorm8_finite(float c) {
    return (uint32_t)__float2int_rn(__builtin_amdgcn_fmed3f(c, 0.0f, 1.0f) * 255.0f);
}
__global__ __launch_bounds__(256) void rm_fxaa_lds_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                          int W, int H) {
#if RM_FXAA_F4
    // RM_FXAA_F4: each staged texel as the floats GL reads (r, g, b) and its
    // luma, plus its alpha byte: a span tap is one 16-byte LDS read instead of
    // a 4-byte read and six unpacking VALU, and a texel is unpacked once per
    // tile instead of once per tap
    __shared__ float4 sf4[FXL_H * FXL_W];
    __shared__ uint8_t salpha[FXL_H * FXL_W];
#else
    __shared__ uint32_t stex[FXL_H * FXL_W];
    __shared__ float slum[FXL_H * FXL_W];
#endif
    const int x0 = blockIdx.x * FXL_TX, y0 = blockIdx.y * FXL_TY;
    // output rows y0 .. y0 + TY - 1 read texel rows H-1-y (+-1, span): the block
    // [tx0, tx0 + FXL_W) x [ty0, ty0 + FXL_H), each texel clamped to the frame
    const int tx0 = x0 - FXL_HALO, ty0 = H - (y0 + FXL_TY) - FXL_HALO;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // staging: wave wv loads block rows wv, wv + 4, ...; lane -> column lane and
    // lane + 64 (the last FXL_W - 64 columns); every load in flight before the
    // first LDS store
    constexpr int NR = (FXL_H + 3) / 4;
    const int gx0 = clamp_med3(tx0 + lane, W - 1), gx1 = clamp_med3(tx0 + 64 + (lane < FXL_W - 64 ? lane : 0), W - 1);
    uint32_t t0[NR], t1[NR];
#pragma unroll
    for (int k = 0; k < NR; k++) {
        const int r = wv + 4 * k;
        const int gy = clamp_med3(ty0 + (r < FXL_H ? r : FXL_H - 1), H - 1);
        const char* row = reinterpret_cast<const char*>(in) + (uint32_t)(gy * W) * 4u;
        t0[k] = *reinterpret_cast<const uint32_t*>(row + (uint32_t)gx0 * 4u);
        t1[k] = *reinterpret_cast<const uint32_t*>(row + (uint32_t)gx1 * 4u);
    }
#pragma unroll
    for (int k = 0; k < NR; k++) {
        const int r = wv + 4 * k;
        if (r < FXL_H) {
#if RM_FXAA_F4
            const RGB c0 = rgb(t0[k]);
            sf4[r * FXL_W + lane] = make_float4(c0.r, c0.g, c0.b, luma(c0));
            salpha[r * FXL_W + lane] = (uint8_t)(t0[k] >> 24);
            if (lane < FXL_W - 64) {
                const RGB c1 = rgb(t1[k]);
                sf4[r * FXL_W + 64 + lane] = make_float4(c1.r, c1.g, c1.b, luma(c1));
                salpha[r * FXL_W + 64 + lane] = (uint8_t)(t1[k] >> 24);
            }
#else
            stex[r * FXL_W + lane] = t0[k];
            slum[r * FXL_W + lane] = luma(rgb(t0[k]));
            if (lane < FXL_W - 64) {
                stex[r * FXL_W + 64 + lane] = t1[k];
                slum[r * FXL_W + 64 + lane] = luma(rgb(t1[k]));
            }
#endif
        }
    }
    __syncthreads();
    const float FXAA_REDUCE_MIN = 1.0f / 128.0f, FXAA_REDUCE_MUL = 1.0f / 8.0f, FXAA_SPAN_MAX = 8.0f;
    const float ivx = 1.0f / (float)W, ivy = 1.0f / (float)H;  // inverseVP = 1 / u_resolution
    const float k1 = 1.0f / 3.0f - 0.5f, k2 = 2.0f / 3.0f - 0.5f;
    const int x = x0 + lane;
    const float fx = ((float)x + 0.5f) / (float)W;  // post.frag:140: uv = (tc.x, 1 - tc.y)
    // a span tap: post.frag's float address (NEAREST), then the staged texel
    // (block row * FXL_W as a 24-bit multiply: the row is clamped into the block)
#if RM_FXAA_F4
    const int blk0 = -(ty0 * FXL_W + tx0);  // (the bound above keeps every span texel inside the block)
    auto span_tap = [&](float u, float v) -> RGB {
        const float4 t = sf4[__mul24(floor_i32(v * (float)H), FXL_W) + floor_i32(u * (float)W) + blk0];
        return RGB{t.x, t.y, t.z};
    };
#elif RM_FXAA_ADDR
    // (the bound above keeps every span texel inside the block, so no clamp:
    // the block index is one signed 24-bit multiply-add of the texel
    // coordinates and a wave-uniform offset; an LDS read outside the
    // workgroup's allocation returns 0 on this hardware in any case)
    const int blk4 = -4 * (ty0 * FXL_W + tx0);  // (byte offsets)
    auto span_tap = [&](float u, float v) -> RGB {
        // byte offset 4 gx + (296 gy + blk4): v_mad_i32_i24 + v_lshl_add_u32 (left
        // to itself the compiler forms mul + shift + add3)
        const int row = __mul24(floor_i32(v * (float)H), 4 * FXL_W) + blk4;
        int a;
        asm("v_lshl_add_u32 %0, %1, 2, %2" : "=v"(a) : "v"(floor_i32(u * (float)W)), "v"(row));
        return rgb(*reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(stex) + a));
    };
#else
    auto span_tap = [&](float u, float v) -> RGB {
        const int gx = clamp_to(floor_i32(u * (float)W) - tx0, FXL_W - 1);
        const int gy = clamp_to(floor_i32(v * (float)H) - ty0, FXL_H - 1);
        return rgb(stex[__umul24(gy, FXL_W) + gx]);
    };
#endif
    // fy of row y0 + l in lane l (rows past the frame: the clamped row), one
    // correctly rounded division per tile instead of one per row; a row reads
    // its lane's value as a wave-uniform scalar
    const float fy_lane = 1.0f - ((float)min(y0 + (lane & (FXL_TY - 1)), H - 1) + 0.5f) / (float)H;
    // one pixel of row y0 + ly (its value; rows past the frame are computed on a
    // clamped row and not stored)
    auto pixel = [&](int ly) -> uint32_t {
        const int y = min(y0 + ly, H - 1);
        const int m = (FXL_TY - 1 - (y - y0) + FXL_HALO) * FXL_W + (lane + FXL_HALO);
#if RM_FXAA_F4
        const float lNW = sf4[m - FXL_W - 1].w, lNE = sf4[m - FXL_W + 1].w, lSW = sf4[m + FXL_W - 1].w;
        const float lSE = sf4[m + FXL_W + 1].w, lM = sf4[m].w;
        const uint32_t tM = (uint32_t)salpha[m] << 24;
#else
        const float lNW = slum[m - FXL_W - 1], lNE = slum[m - FXL_W + 1], lSW = slum[m + FXL_W - 1];
        const float lSE = slum[m + FXL_W + 1], lM = slum[m];
        const uint32_t tM = stex[m];
#endif
        const float fy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fy_lane), ly));
        const float lMin = fminf(lM, fminf(fminf(lNW, lNE), fminf(lSW, lSE)));
        const float lMax = fmaxf(lM, fmaxf(fmaxf(lNW, lNE), fmaxf(lSW, lSE)));
        float dx = -((lNW + lNE) - (lSW + lSE));
        float dy = ((lNW + lSW) - (lNE + lSE));
        float dirReduce = fmaxf((lNW + lNE + lSW + lSE) * (0.25f * FXAA_REDUCE_MUL), FXAA_REDUCE_MIN);
#if RM_FXAA_RCP_NR
        // 1/x correctly rounded as one Newton step from v_rcp_f32: x lies in
        // [1/128, 2.125] (dirReduce in [1/128, 1/8], |dx|, |dy| <= 2 for lumas
        // in [0, 1]), and over every float of [2^-8, 4) the step equals the IEEE
        // quotient bit for bit on gfx950 (tools/rcp_exhaustive.hip: 83,886,080
        // floats, 0 mismatches; profiles/r05/rcp_exhaustive.json): 3 VALU
        // instead of the 12 of the div_scale / div_fmas / div_fixup expansion
        const float dmin = fminf(fabsf(dx), fabsf(dy)) + dirReduce;
        const float r0 = __builtin_amdgcn_rcpf(dmin);
        float rcpDirMin = fmaf(fmaf(-dmin, r0, 1.0f), r0, r0);
#else
        float rcpDirMin = 1.0f / (fminf(fabsf(dx), fabsf(dy)) + dirReduce);
#endif
        dx = __builtin_amdgcn_fmed3f(dx * rcpDirMin, -FXAA_SPAN_MAX, FXAA_SPAN_MAX) * ivx;
        dy = __builtin_amdgcn_fmed3f(dy * rcpDirMin, -FXAA_SPAN_MAX, FXAA_SPAN_MAX) * ivy;
        RGB s1 = span_tap(fx + dx * k1, fy + dy * k1);
        RGB s2 = span_tap(fx + dx * k2, fy + dy * k2);
        RGB a = RGB{(s1.r + s2.r) * 0.5f, (s1.g + s2.g) * 0.5f, (s1.b + s2.b) * 0.5f};
        RGB s3 = span_tap(fx + dx * -0.5f, fy + dy * -0.5f);
        RGB s4 = span_tap(fx + dx * 0.5f, fy + dy * 0.5f);
        RGB b = RGB{a.r * 0.5f + (s3.r + s4.r) * 0.25f, a.g * 0.5f + (s3.g + s4.g) * 0.25f,
                    a.b * 0.5f + (s3.b + s4.b) * 0.25f};
        float lB = luma(b);
        RGB c = (lB < lMin || lB > lMax) ? a : b;
        // (the colour is finite: unorm8 inputs, a correctly rounded, positive rcpDirMin;
        // alpha stays the texel's own byte: (b / 255) * 255 rounds back to b)
        return unorm8_finite(c.r) | (unorm8_finite(c.g) << 8) | (unorm8_finite(c.b) << 16) | (tM & 0xff000000u);
    };
    // two rows at a time: their dependent chains (LDS taps -> division -> span
    // taps) interleave
    for (int ly = wv; ly < FXL_TY; ly += 8) {
        const uint32_t v0 = pixel(ly), v1 = pixel(ly + 4);
        if (x < W && y0 + ly < H) out[(size_t)(y0 + ly) * W + x] = v0;
        if (x < W && y0 + ly + 4 < H) out[(size_t)(y0 + ly + 4) * W + x] = v1;
    }
}

#ifndef RM_FXAA_LDS
#define RM_FXAA_LDS 1
#endif
hipError_t launch_fxaa(const uint32_t* in, uint32_t* out, int W, int H, hipStream_t s) {
    if (W <= 0 || H <= 0) return hipSuccess;
    if (RM_FXAA_LDS && W <= FXL_MAX_DIM && H <= FXL_MAX_DIM) {
        dim3 grid((W + FXL_TX - 1) / FXL_TX, (H + FXL_TY - 1) / FXL_TY);
        hipLaunchKernelGGL(rm_fxaa_lds_kernel, grid, dim3(256), 0, s, in, out, W, H);
        return hipGetLastError();
    }
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

// The bilinear filter as the polynomial of its cell (oracle tex_bilinear):
// c00 + a Px + b (Py + a Pxy), Px = c01 - c00, Py = c10 - c00,
// Pxy = (c11 - c10) - Px, three fused multiply-adds per channel.
__device__ __forceinline__ float cell_poly(float c00, float px, float py, float pxy, float a, float b) {
    return fmaf(b, fmaf(a, pxy, py), fmaf(a, px, c00));
}

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
        const float px = c01 - c00, py = c10 - c00, pxy = (c11 - c10) - px;
        o[c] = cell_poly(c00, px, py, pxy, a, b);
    }
    return RGB{o[0], o[1], o[2]};
}

__constant__ const float kGauss[3][3] = {{41.0f / 273.0f, 26.0f / 273.0f, 7.0f / 273.0f},
                                         {26.0f / 273.0f, 16.0f / 273.0f, 4.0f / 273.0f},
                                         {7.0f / 273.0f, 4.0f / 273.0f, 1.0f / 273.0f}};

// bloom.frag:33-43, one lane per output pixel, 16x16-pixel workgroups.  The
// general form: any lod, the levels read as RGBA8 words.  Used when lod <= 0
// (magnification: every tap reads the base level).
__global__ __launch_bounds__(256) void rm_bloom_kernel(Level L0, uint32_t* __restrict__ out, int W, int H) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    const float u = ((float)x + 0.5f) / (float)W, v = 1.0f - ((float)y + 0.5f) / (float)H;  // bloom.frag:36
    RGB color = tex_bilinear(L0, u, v);
    const float scale = 0.05f, iaspect = (float)H / (float)W;
    RGB bl{0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int j = -2; j <= 2; j++)
#pragma unroll
        for (int i = -2; i <= 2; i++) {
            const float uu = u + ((float)i * iaspect) * scale, vv = v + (float)j * scale;
            const RGB s = tex_bilinear(L0, uu, vv);
            const float g = kGauss[i < 0 ? -i : i][j < 0 ? -j : j];
            bl = RGB{fmaf(g, s.r, bl.r), fmaf(g, s.g, bl.g), fmaf(g, s.b, bl.b)};
        }
    color = RGB{color.r + gmax_(bl.r - 0.3f, 0.0f), color.g + gmax_(bl.g - 0.3f, 0.0f),
                color.b + gmax_(bl.b - 0.3f, 0.0f)};
    out[(size_t)y * W + x] = unorm8(color.r) | (unorm8(color.g) << 8) | (unorm8(color.b) << 16) | (255u << 24);
}

// The cells of the two minified levels bloom.frag reads (lod > 0): for a
// level of w x h texels, cell (cx, cy), cx in [-1, w-1], cy in [-1, h-1],
// holds the filter polynomial of texels (clamp(cx), clamp(cx+1)) x (clamp(cy),
// clamp(cy+1)) per channel: c00 rgb, Px rgb, Py rgb, Pxy rgb (12 floats,
// 48 B; the same float operations tex_bilinear forms per tap).
constexpr int kCellFloats = 12;
__global__ __launch_bounds__(256) void rm_bloom_cells_kernel(const uint32_t* __restrict__ a, int wa, int ha,
                                                             const uint32_t* __restrict__ b, int wb, int hb,
                                                             float* __restrict__ cells) {
    const int na = (wa + 1) * (ha + 1), nb = (wb + 1) * (hb + 1);
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= na + nb) return;
    const bool first = t < na;
    const uint32_t* L = first ? a : b;
    const int w = first ? wa : wb, h = first ? ha : hb, k = first ? t : t - na;
    const int cx = k % (w + 1) - 1, cy = k / (w + 1) - 1;
    const int x0 = clampi(cx, w - 1), x1 = clampi(cx + 1, w - 1), y0 = clampi(cy, h - 1), y1 = clampi(cy + 1, h - 1);
    const uint32_t t00 = L[y0 * w + x0], t01 = L[y0 * w + x1], t10 = L[y1 * w + x0], t11 = L[y1 * w + x1];
    const float kk = 1.0f / 255.0f;
    float o[kCellFloats];
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const int s = 8 * c;
        const float c00 = (float)((t00 >> s) & 255u) * kk, c01 = (float)((t01 >> s) & 255u) * kk;
        const float c10 = (float)((t10 >> s) & 255u) * kk, c11 = (float)((t11 >> s) & 255u) * kk;
        o[c] = c00;
        o[3 + c] = c01 - c00;
        o[6 + c] = c10 - c00;
        o[9 + c] = (c11 - c10) - o[3 + c];
    }
    float4* dst = reinterpret_cast<float4*>(cells + (size_t)t * kCellFloats);
    dst[0] = make_float4(o[0], o[1], o[2], o[3]);
    dst[1] = make_float4(o[4], o[5], o[6], o[7]);
    dst[2] = make_float4(o[8], o[9], o[10], o[11]);
}

struct Cells {
    const float* __restrict__ p;
    int w, h;  // the level's texels; (w + 1) x (h + 1) cells
};

// One bilinear axis of a tap: weight and cell index (0 .. n: cx + 1).
struct CAxis {
    float f;
    int c;
};
__device__ __forceinline__ CAxis caxis(float t, int n) {
    const float x = t * (float)n - 0.5f, fx = floorf(x);
    CAxis A;
    A.f = x - fx;
    A.c = (int)fminf(fmaxf(fx, -1.0f), (float)(n - 1)) + 1;
    return A;
}
__device__ __forceinline__ bool wave_uniform(int v, int& first) {
    first = __builtin_amdgcn_readfirstlane(v);
    return __builtin_amdgcn_ballot_w64(v == first) == __builtin_amdgcn_read_exec();
}

typedef float f8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
// Both levels' cells of one tap at wave-uniform byte offsets through the
// scalar cache (read-only: written by the previous launch on the stream).
__device__ __forceinline__ void sload_cells(const float* a, int oa, const float* b, int ob, f8v& a8, f4v& a4, f8v& b8,
                                            f4v& b4) {
    asm volatile(
        "s_load_dwordx8 %0, %4, %5\n\t"
        "s_load_dwordx4 %1, %4, %5 offset:32\n\t"
        "s_load_dwordx8 %2, %6, %7\n\t"
        "s_load_dwordx4 %3, %6, %7 offset:32\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(a8), "=&s"(a4), "=&s"(b8), "=&s"(b4)
        : "s"(a), "s"(oa), "s"(b), "s"(ob)
        : "memory");
}

// One tap of a level, accumulated: acc += g (c00 + a Px + b Py + a b Pxy) as
// four multiply-adds per channel, acc += c00 g, Px (g a), Py (g b), Pxy (g a b)
// in that order (oracle bloom_tap_acc): each reads one cell coefficient, so
// the wave-uniform cells stay SGPR operands (one SGPR per VALU instruction).
__device__ __forceinline__ void cell_acc(const f8v& c8, const f4v& c4, float a, float b, float g, RGB& acc) {
    const float ga = g * a, gb = g * b, gab = ga * b;
    acc.r = fmaf(c4[1], gab, fmaf(c8[6], gb, fmaf(c8[3], ga, fmaf(c8[0], g, acc.r))));
    acc.g = fmaf(c4[2], gab, fmaf(c8[7], gb, fmaf(c8[4], ga, fmaf(c8[1], g, acc.g))));
    acc.b = fmaf(c4[3], gab, fmaf(c4[0], gb, fmaf(c8[5], ga, fmaf(c8[2], g, acc.b))));
}
__device__ __forceinline__ void vload_cell(const float* base, int cell, f8v& c8, f4v& c4) {
    const float4* q = reinterpret_cast<const float4*>(base + (size_t)cell * kCellFloats);
    const float4 q0 = q[0], q1 = q[1], q2 = q[2];
    c8 = f8v{q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    c4 = f4v{q2.x, q2.y, q2.z, q2.w};
}

// bloom.frag:33-43 for lod > 0 (minification: levels d1, d2 blended by fr).
// One wave per 8x8-pixel tile, 2x2 waves per workgroup.  A tap's value is
// its cell's polynomial; a level texel spans 2^d1 >= 0.025 H pixels, so the
// lanes of a wave mostly share a tap's cell on both levels: the two cells are
// then read once per wave into SGPRs (otherwise per lane).  The Gaussian sums
// of the two levels are blended once at the end (oracle bloom_pixel).
// Round 5 (0.488 -> 0.444 ms at 4096^2, bit-identical; profiles/r05/bloom_ab.log):
//  * the row's three Gaussian weights chosen by scalar selects (no load per
//    tap) and copied to VGPRs once per row (the c00 g term's operand), and the
//    products g b shared by the symmetric taps of a row (g[i] = g[4-i]);
//  * a row whose ten cells (5 taps x 2 levels) are all wave-uniform -- most
//    rows -- runs without a branch per tap, so the compiler schedules its
//    scalar loads ahead of the arithmetic; other rows branch per tap as before;
//  * the wave-uniform cells read by compiler-scheduled scalar loads from the
//    constant address space instead of an asm block that waited on each tap.
typedef const __attribute__((address_space(4))) float* cfloat_p;
__device__ __forceinline__ void sload_cell(const float* base, int off_bytes, f8v& c8, f4v& c4) {
    cfloat_p p = (cfloat_p)(const void*)base;
    const int o = __builtin_amdgcn_readfirstlane(off_bytes) >> 2;
    c8 = f8v{p[o], p[o + 1], p[o + 2], p[o + 3], p[o + 4], p[o + 5], p[o + 6], p[o + 7]};
    c4 = f4v{p[o + 8], p[o + 9], p[o + 10], p[o + 11]};
}
__global__ __launch_bounds__(256) void rm_bloom_min_kernel(Level L0, Cells A, Cells B, uint32_t* __restrict__ out,
                                                           int W, int H, float fr) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wv & 1) * 8 + (lane & 7), y = blockIdx.y * 16 + (wv >> 1) * 8 + (lane >> 3);
    if (x >= W || y >= H) return;
    const float u = ((float)x + 0.5f) / (float)W, v = 1.0f - ((float)y + 0.5f) / (float)H;  // bloom.frag:36
    RGB color = tex_bilinear(L0, u, v);
    const float scale = 0.05f, iaspect = (float)H / (float)W;
    CAxis xa[5], xb[5];
    int sxa[5], sxb[5];
    bool ux[5], allx = true;
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const float uu = u + ((float)(i - 2) * iaspect) * scale;
        xa[i] = caxis(uu, A.w);
        xb[i] = caxis(uu, B.w);
        const bool ua = wave_uniform(xa[i].c, sxa[i]), ub = wave_uniform(xb[i].c, sxb[i]);
        ux[i] = ua && ub;
        allx = allx && ux[i];
        sxa[i] *= kCellFloats * 4;
        sxb[i] *= kCellFloats * 4;
    }
    RGB ba{0.0f, 0.0f, 0.0f}, bb{0.0f, 0.0f, 0.0f};
#pragma unroll 1
    for (int j = 0; j < 5; j++) {  // (rolled: one row's cells and weights live at a time)
        const float vv = v + (float)(j - 2) * scale;
        const CAxis ya = caxis(vv, A.h), yb = caxis(vv, B.h);
        int sya, syb;
        const bool uya = wave_uniform(ya.c, sya), uyb = wave_uniform(yb.c, syb);
        const bool uy = uya && uyb;
        sya *= (A.w + 1) * kCellFloats * 4;
        syb *= (B.w + 1) * kCellFloats * 4;
        // kGauss[|i - 2|][|j - 2|] of this row (scalar selects)
        const int jr = j < 2 ? 2 - j : j - 2;
        const float g0 = jr == 0 ? 41.0f / 273.0f : jr == 1 ? 26.0f / 273.0f : 7.0f / 273.0f;
        const float g1 = jr == 0 ? 26.0f / 273.0f : jr == 1 ? 16.0f / 273.0f : 4.0f / 273.0f;
        const float g2 = jr == 0 ? 7.0f / 273.0f : jr == 1 ? 4.0f / 273.0f : 1.0f / 273.0f;
        const float gi[5] = {g2, g1, g0, g1, g2};
        if (uy && allx) {
#pragma unroll
            for (int i = 0; i < 5; i++) {
                f8v a8, b8;
                f4v a4, b4;
                sload_cell(A.p, sya + sxa[i], a8, a4);
                sload_cell(B.p, syb + sxb[i], b8, b4);
                cell_acc(a8, a4, xa[i].f, ya.f, gi[i], ba);
                cell_acc(b8, b4, xb[i].f, yb.f, gi[i], bb);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 5; i++) {
                f8v a8, b8;
                f4v a4, b4;
                if (uy & ux[i]) {  // (as rm_bloom_min_kernel: SGPR operands stay SGPRs)
                    sload_cells(A.p, sya + sxa[i], B.p, syb + sxb[i], a8, a4, b8, b4);
                    cell_acc(a8, a4, xa[i].f, ya.f, gi[i], ba);
                    cell_acc(b8, b4, xb[i].f, yb.f, gi[i], bb);
                } else {
                    vload_cell(A.p, ya.c * (A.w + 1) + xa[i].c, a8, a4);
                    vload_cell(B.p, yb.c * (B.w + 1) + xb[i].c, b8, b4);
                    cell_acc(a8, a4, xa[i].f, ya.f, gi[i], ba);
                    cell_acc(b8, b4, xb[i].f, yb.f, gi[i], bb);
                }
            }
        }
    }
    const float ifr = 1.0f - fr;
    const RGB bl{ifr * ba.r + fr * bb.r, ifr * ba.g + fr * bb.g, ifr * ba.b + fr * bb.b};
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
    if (p.lod > 0.0f) {  // the cells of levels d1, d2 (rm_bloom_cells_kernel), 16-byte aligned
        p.cell_offset = (p.texels + 3) & ~(size_t)3;
        p.texels = p.cell_offset + (size_t)kCellFloats * ((size_t)(p.w[p.d1] + 1) * (p.h[p.d1] + 1) +
                                                          (size_t)(p.w[p.d2] + 1) * (p.h[p.d2] + 1));
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
        hipLaunchKernelGGL(rm_bloom_kernel, dim3((W + 15) / 16, (H + 15) / 16), dim3(256), 0, s, L0, out, W, H);
        return hipGetLastError();
    }
    const int wa = p.w[p.d1], ha = p.h[p.d1], wb = p.w[p.d2], hb = p.h[p.d2];
    const int nc = (wa + 1) * (ha + 1) + (wb + 1) * (hb + 1);
    float* cells = reinterpret_cast<float*>(mips + p.cell_offset);
    hipLaunchKernelGGL(rm_bloom_cells_kernel, dim3((nc + 255) / 256), dim3(256), 0, s, lv[p.d1], wa, ha, lv[p.d2], wb,
                       hb, cells);
    const Cells A{cells, wa, ha}, B{cells + (size_t)kCellFloats * (wa + 1) * (ha + 1), wb, hb};
    hipLaunchKernelGGL(rm_bloom_min_kernel, dim3((W + 15) / 16, (H + 15) / 16), dim3(256), 0, s, L0, A, B, out, W, H,
                       p.fr);
    return hipGetLastError();
}

}  // namespace rm
