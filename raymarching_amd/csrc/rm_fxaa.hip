// rm_fxaa.hip -- the FXAA post pass of the reference (post.frag:16-61, main
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
//
// Rows whose span is short output their centre texel without the span taps
// (RM_FXAA_FLAT, proof at the test): 0.069-0.072 -> 0.052-0.053 ms on the C3
// frame, same bits (profiles/r05/fxaa_flat/); with 8x8-pixel blocks per wave
// pass (RM_FXAA_BW) instead of rows, 0.046-0.047 (profiles/r05/fxaa_blocks/).
// Its own translation unit (split from rm_post.hip in round 5) so that it can
// be scheduled with LLVM's max-ilp strategy, which shortens the latency-bound
// FXAA kernel (0.0721-0.0729 -> 0.0697-0.0706 ms) but slows bloom's
// (profiles/r05/post_ilp_ab.log).
#include "rm_post_common.h"

namespace rm {

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
#ifndef RM_FXAA_ROWS
#define RM_FXAA_ROWS 2  // rows per pass of a wave (2 or 4)
#endif
#ifndef RM_FXAA_LINEAR
#define RM_FXAA_LINEAR 0
#endif
#ifndef RM_FXAA_GTAP
#define RM_FXAA_GTAP 0
#endif
#ifndef RM_FXAA_FLAT
#define RM_FXAA_FLAT 1  // short-span rows output their centre texel (below)
#endif
#ifndef RM_FXAA_BW
#define RM_FXAA_BW 8  // a wave pass covers BW x (64 / BW) pixels: 8x8 blocks (64: one row)
#endif
// RM_FXAA_HALO: the span texels lie within +-4 of the pixel (above), so a
// halo of 4 holds them all; RM_FXAA_TRIM: lumas only for the texels the +-1
// taps read, (TX + 2) x (TY + 2), not the whole block; RM_FXAA_NW: waves per
// workgroup (LDS per workgroup and the 32-waves-per-CU cap set the occupancy)
#ifndef RM_FXAA_HALO
#define RM_FXAA_HALO 4
#endif
#ifndef RM_FXAA_TRIM
#define RM_FXAA_TRIM 0
#endif
#ifndef RM_FXAA_NW
#define RM_FXAA_NW 4
#endif
constexpr int FXL_TX = 64, FXL_TY = RM_FXAA_TY, FXL_HALO = RM_FXAA_HALO, FXL_W = FXL_TX + 2 * FXL_HALO,
              FXL_H = FXL_TY + 2 * FXL_HALO;
constexpr int FXL_NW = RM_FXAA_NW, FXL_NT = 64 * FXL_NW;
#if RM_FXAA_TRIM
constexpr int SL_W = FXL_TX + 2, SL_H = FXL_TY + 2, SL_O = FXL_HALO - 1;  // luma region: block (SL_O, SL_O) on
static_assert(!RM_FXAA_LINEAR && !RM_FXAA_F4 && !RM_FXAA_GTAP, "RM_FXAA_TRIM: column staging only");
#else
constexpr int SL_W = FXL_W, SL_H = FXL_H, SL_O = 0;
#endif
constexpr int FXL_MAX_DIM = 1 << 20;
static_assert(FXL_HALO >= 4 && FXL_W - 64 <= 64, "span texels within +-4; two staging columns per lane");
static_assert((FXL_TY & (FXL_TY - 1)) == 0 && FXL_TY <= 64, "fy_lane: one lane per tile row");
static_assert(FXL_TY % (RM_FXAA_ROWS * FXL_NW) == 0, "whole passes of RM_FXAA_ROWS rows per wave");
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
__global__ __launch_bounds__(FXL_NT) void rm_fxaa_lds_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                          int W, int H) {
#if RM_FXAA_F4
    // RM_FXAA_F4: each staged texel as the floats GL reads (r, g, b) and its
    // luma, plus its alpha byte: a span tap is one 16-byte LDS read instead of
    // a 4-byte read and six unpacking VALU, and a texel is unpacked once per
    // tile instead of once per tap
    __shared__ float4 sf4[FXL_H * FXL_W];
    __shared__ uint8_t salpha[FXL_H * FXL_W];
#else
#if !RM_FXAA_GTAP
    __shared__ uint32_t stex[FXL_H * FXL_W];
#endif
    __shared__ float slum[SL_H * SL_W];
#endif
    const int x0 = blockIdx.x * FXL_TX, y0 = blockIdx.y * FXL_TY;
    // output rows y0 .. y0 + TY - 1 read texel rows H-1-y (+-1, span): the block
    // [tx0, tx0 + FXL_W) x [ty0, ty0 + FXL_H), each texel clamped to the frame
    const int tx0 = x0 - FXL_HALO, ty0 = H - (y0 + FXL_TY) - FXL_HALO;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // staging: wave wv loads block rows wv, wv + 4, ...; lane -> column lane and
    // lane + 64 (the last FXL_W - 64 columns); every load in flight before the
    // first LDS store
#if RM_FXAA_LINEAR && !RM_FXAA_F4
    // RM_FXAA_LINEAR: the block's texels in row-major order, 256 per pass (13
    // passes for 74 x 42), so every lane's load and luma is a staged texel
    // (the column layout above loads 22 words per lane and forms the lumas of
    // the last ten columns in full-wave instructions for ten lanes)
    {
        constexpr int NT = FXL_H * FXL_W, NP = (NT + FXL_NT - 1) / FXL_NT;
        uint32_t tt[NP];
#pragma unroll
        for (int k = 0; k < NP; k++) {
            const int idx = min((int)threadIdx.x + FXL_NT * k, NT - 1);
            const int r = idx / FXL_W, c = idx - r * FXL_W;  // (constant divisor: a multiply-high)
            const int gy = clamp_med3(ty0 + r, H - 1), gx = clamp_med3(tx0 + c, W - 1);
            const uint32_t off = __umul24((uint32_t)gy, (uint32_t)W) + (uint32_t)gx;  // (W, H <= 2^20)
            tt[k] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(in) + off * 4u);
        }
#pragma unroll
        for (int k = 0; k < NP; k++) {
            const int idx = (int)threadIdx.x + FXL_NT * k;
            if (k < NP - 1 || idx < NT) {
                stex[idx] = tt[k];
                slum[idx] = luma(rgb(tt[k]));
            }
        }
    }
#else
    constexpr int NR = (FXL_H + FXL_NW - 1) / FXL_NW;
    const int gx0 = clamp_med3(tx0 + lane, W - 1), gx1 = clamp_med3(tx0 + 64 + (lane < FXL_W - 64 ? lane : 0), W - 1);
    uint32_t t0[NR], t1[NR];
#pragma unroll
    for (int k = 0; k < NR; k++) {
        const int r = wv + FXL_NW * k;
        const int gy = clamp_med3(ty0 + (r < FXL_H ? r : FXL_H - 1), H - 1);
        // one 32-bit byte offset from the kernel-argument base per load (the
        // saddr form: no 64-bit address add; frames < 2^30 texels)
        const uint32_t rowoff = __umul24((uint32_t)gy, (uint32_t)W);  // (W, H <= 2^20: 24-bit operands)
        t0[k] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(in) + (rowoff + (uint32_t)gx0) * 4u);
        t1[k] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(in) + (rowoff + (uint32_t)gx1) * 4u);
    }
#pragma unroll
    for (int k = 0; k < NR; k++) {
        const int r = wv + FXL_NW * k;
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
#if !RM_FXAA_GTAP
            stex[r * FXL_W + lane] = t0[k];
            if (lane < FXL_W - 64) stex[r * FXL_W + 64 + lane] = t1[k];
#endif
            const int lr = r - SL_O;  // (wave-uniform)
            if (lr >= 0 && lr < SL_H) {
                if (lane >= SL_O) slum[lr * SL_W + lane - SL_O] = luma(rgb(t0[k]));
                if (lane < FXL_W - 64 && 64 + lane - SL_O < SL_W) slum[lr * SL_W + 64 + lane - SL_O] = luma(rgb(t1[k]));
            }
#endif
        }
    }
#endif
    __syncthreads();
    const float FXAA_REDUCE_MIN = 1.0f / 128.0f, FXAA_REDUCE_MUL = 1.0f / 8.0f, FXAA_SPAN_MAX = 8.0f;
    const float ivx = 1.0f / (float)W, ivy = 1.0f / (float)H;  // inverseVP = 1 / u_resolution
    const float k1 = 1.0f / 3.0f - 0.5f, k2 = 2.0f / 3.0f - 0.5f;
    constexpr int BW = RM_FXAA_BW, BH = 64 / BW, NBX = FXL_TX / BW;
    static_assert(BW * BH == 64 && FXL_TX % BW == 0 && FXL_TY % BH == 0, "RM_FXAA_BW: blocks tile the tile");
    const int xl = x0 + lane;
    const float fx_lane = ((float)xl + 0.5f) / (float)W;  // post.frag:140: uv = (tc.x, 1 - tc.y)
    // a span tap: post.frag's float address (NEAREST), then the staged texel
    // (block row * FXL_W as a 24-bit multiply: the row is clamped into the block)
#if RM_FXAA_GTAP
    // RM_FXAA_GTAP: the span taps read the frame (L1/L2: the block was just
    // loaded), NEAREST + CLAMP_TO_EDGE as texel() forms it; LDS holds only the
    // lumas (12 KB a workgroup: eight waves per SIMD instead of six)
    auto span_tap = [&](float u, float v) -> RGB { return rgb(texel(in, W, H, u, v)); };
#elif RM_FXAA_F4
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
    // pixel block b of the tile: lane -> column col, row ly (BW = 64: row b)
    auto px_col = [&](int b) { return (b % NBX) * BW + (BW == 64 ? lane : (lane & (BW - 1))); };
    auto px_row = [&](int b) { return (b / NBX) * BH + (BW == 64 ? 0 : lane / BW); };
    auto pixel = [&](int blk) -> uint32_t {
        const int col = px_col(blk), ly = px_row(blk);
        const int y = min(y0 + ly, H - 1);
        const int rr = FXL_TY - 1 - (y - y0);  // block row of the pixel's texel, less the halo
        const int m = (rr + FXL_HALO) * FXL_W + (col + FXL_HALO);
        const int ml = (rr + FXL_HALO - SL_O) * SL_W + (col + FXL_HALO - SL_O);
#if RM_FXAA_F4
        const float lNW = sf4[m - FXL_W - 1].w, lNE = sf4[m - FXL_W + 1].w, lSW = sf4[m + FXL_W - 1].w;
        const float lSE = sf4[m + FXL_W + 1].w, lM = sf4[m].w;
        const uint32_t tM = (uint32_t)salpha[m] << 24;
#else
        const float lNW = slum[ml - SL_W - 1], lNE = slum[ml - SL_W + 1], lSW = slum[ml + SL_W - 1];
        const float lSE = slum[ml + SL_W + 1], lM = slum[ml];
#if RM_FXAA_GTAP
        const uint32_t tM = in[(size_t)(H - 1 - y) * W + min(x0 + col, W - 1)];  // (the centre texel, stex[m])
#else
        const uint32_t tM = stex[m];
#endif
#endif
        float fx, fy;
        if constexpr (BW == 64) {
            fx = fx_lane;
            fy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fy_lane), ly));
        } else {  // (lane col's fx and lane ly's fy, one ds_bpermute each)
            fx = __int_as_float(__builtin_amdgcn_ds_bpermute(col * 4, __float_as_int(fx_lane)));
            fy = __int_as_float(__builtin_amdgcn_ds_bpermute(ly * 4, __float_as_int(fy_lane)));
        }
        // (lumas are never NaN or -0: IEEE minimum/maximum, v_minimum3/v_maximum3,
        // equal GLSL min/max here without minNum's canonicalizing v_max per operand)
        const float lMin = __builtin_elementwise_minimum(
            lM, __builtin_elementwise_minimum(__builtin_elementwise_minimum(lNW, lNE),
                                              __builtin_elementwise_minimum(lSW, lSE)));
        const float lMax = __builtin_elementwise_maximum(
            lM, __builtin_elementwise_maximum(__builtin_elementwise_maximum(lNW, lNE),
                                              __builtin_elementwise_maximum(lSW, lSE)));
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
        const float dxs = __builtin_amdgcn_fmed3f(dx * rcpDirMin, -FXAA_SPAN_MAX, FXAA_SPAN_MAX);
        const float dys = __builtin_amdgcn_fmed3f(dy * rcpDirMin, -FXAA_SPAN_MAX, FXAA_SPAN_MAX);
#if RM_FXAA_FLAT
        // A short span: with |dxs|, |dys| <= 0.5 texel every span tap (|k| <=
        // 0.5) lies within 0.25 texel of the pixel centre x + 0.5 (row: H - y -
        // 0.5), and the roundings of its float address stay below 0.19 texel for
        // W, H <= 2^20 (the bound above), so all four taps read the centre texel
        // tM.  Then a = (s + s) * 0.5 = s and b = s * 0.5 + (s + s) * 0.25 = s
        // exactly, luma(b) = lM lies in [lMin, lMax], c = s, and unorm8 of
        // byte / 255 is the byte again for all 256 bytes: the output is tM.
        // Taken when the wave's whole row (or block, RM_FXAA_BW) is short-span.
        if (__builtin_amdgcn_ballot_w64(fmaxf(fabsf(dxs), fabsf(dys)) > 0.5f) == 0) return tM;
#endif
        dx = dxs * ivx;
        dy = dys * ivy;
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
    // RM_FXAA_ROWS rows at a time: their dependent chains (LDS taps -> division
    // -> span taps) interleave
#if RM_FXAA_ROWS == 4
    constexpr int N = FXL_NW;
    static_assert(BW == 64, "RM_FXAA_ROWS = 4: row passes");
    const int x = xl;
    for (int ly = wv; ly < FXL_TY; ly += 4 * N) {
        const uint32_t v0 = pixel(ly), v1 = pixel(ly + N), v2 = pixel(ly + 2 * N), v3 = pixel(ly + 3 * N);
        if (x < W && y0 + ly < H) out[(size_t)(y0 + ly) * W + x] = v0;
        if (x < W && y0 + ly + N < H) out[(size_t)(y0 + ly + N) * W + x] = v1;
        if (x < W && y0 + ly + 2 * N < H) out[(size_t)(y0 + ly + 2 * N) * W + x] = v2;
        if (x < W && y0 + ly + 3 * N < H) out[(size_t)(y0 + ly + 3 * N) * W + x] = v3;
    }
#else
    constexpr int NB = (FXL_TX / BW) * (FXL_TY / BH);  // pixel blocks (rows when BW = 64) per tile
    for (int b = wv; b < NB; b += 2 * FXL_NW) {
        const uint32_t v0 = pixel(b), v1 = pixel(b + FXL_NW);
        const int xa = x0 + px_col(b), ya = y0 + px_row(b), xb = x0 + px_col(b + FXL_NW), yb = y0 + px_row(b + FXL_NW);
        if (xa < W && ya < H) out[(size_t)ya * W + xa] = v0;
        if (xb < W && yb < H) out[(size_t)yb * W + xb] = v1;
    }
#endif
}

#ifndef RM_FXAA_LDS
#define RM_FXAA_LDS 1
#endif
hipError_t launch_fxaa(const uint32_t* in, uint32_t* out, int W, int H, hipStream_t s) {
    if (W <= 0 || H <= 0) return hipSuccess;
    if (RM_FXAA_LDS && W <= FXL_MAX_DIM && H <= FXL_MAX_DIM) {
        dim3 grid((W + FXL_TX - 1) / FXL_TX, (H + FXL_TY - 1) / FXL_TY);
        hipLaunchKernelGGL(rm_fxaa_lds_kernel, grid, dim3(FXL_NT), 0, s, in, out, W, H);
        return hipGetLastError();
    }
    dim3 grid((W + FXAA_TX - 1) / FXAA_TX, (H + FXAA_TY - 1) / FXAA_TY);
    hipLaunchKernelGGL(rm_fxaa_kernel, grid, dim3(256), 0, s, in, out, W, H);
    return hipGetLastError();
}

}  // namespace rm
