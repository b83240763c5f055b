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
// Blocks whose span is short output their centre texel without the span taps
// (proof at the test): 0.069-0.072 -> 0.052-0.053 ms on the C3 frame, same
// bits (profiles/r05/fxaa_flat/); with 8x8-pixel blocks per wave pass instead
// of rows, 0.046-0.047 (profiles/r05/fxaa_blocks/); a halo of 4 (its rows are
// then 72 words, 8 banks apart: a block's 8 x 8 reads hit 64 distinct banks)
// 0.041 -> 0.039 (round 6, profiles/r06/fxaa_halo4_ab.log).
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
// The span texels lie within +-4 of the pixel (above), so a halo of 4 holds
// them all.  A workgroup is FXL_NW waves (LDS per workgroup and the
// 32-waves-per-CU cap set the occupancy); a wave pass covers two 8x8-pixel
// blocks.
constexpr int FXL_TX = 64, FXL_TY = 32, FXL_HALO = 4, FXL_W = FXL_TX + 2 * FXL_HALO, FXL_H = FXL_TY + 2 * FXL_HALO;
constexpr int FXL_NW = 4, FXL_NT = 64 * FXL_NW;
constexpr int FXL_MAX_DIM = 1 << 20;
static_assert(FXL_HALO >= 4 && FXL_W - 64 <= 64, "span texels within +-4; two staging columns per lane");
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
__global__ __launch_bounds__(FXL_NT) void rm_fxaa_lds_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                          int W, int H) {
    __shared__ uint32_t stex[FXL_H * FXL_W];
    __shared__ float slum[FXL_H * FXL_W];
    const int x0 = blockIdx.x * FXL_TX, y0 = blockIdx.y * FXL_TY;
    // output rows y0 .. y0 + TY - 1 read texel rows H-1-y (+-1, span): the block
    // [tx0, tx0 + FXL_W) x [ty0, ty0 + FXL_H), each texel clamped to the frame
    const int tx0 = x0 - FXL_HALO, ty0 = H - (y0 + FXL_TY) - FXL_HALO;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // staging: wave wv loads block rows wv, wv + 4, ...; lane -> column lane and
    // lane + 64 (the last FXL_W - 64 columns); every load in flight before the
    // first LDS store
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
            stex[r * FXL_W + lane] = t0[k];
            slum[r * FXL_W + lane] = luma(rgb(t0[k]));
            if (lane < FXL_W - 64) {
                stex[r * FXL_W + 64 + lane] = t1[k];
                slum[r * FXL_W + 64 + lane] = luma(rgb(t1[k]));
            }
        }
    }
    __syncthreads();
    const float FXAA_REDUCE_MIN = 1.0f / 128.0f, FXAA_REDUCE_MUL = 1.0f / 8.0f, FXAA_SPAN_MAX = 8.0f;
    const float ivx = 1.0f / (float)W, ivy = 1.0f / (float)H;  // inverseVP = 1 / u_resolution
    const float k1 = 1.0f / 3.0f - 0.5f, k2 = 2.0f / 3.0f - 0.5f;
    constexpr int NBX = FXL_TX / 8;  // 8x8-pixel blocks across the tile
    const int xl = x0 + lane;
    const float fx_lane = ((float)xl + 0.5f) / (float)W;  // post.frag:140: uv = (tc.x, 1 - tc.y)
    // a span tap: post.frag's float address (NEAREST), then the staged texel
    // (block row * FXL_W as a 24-bit multiply: the row is clamped into the block)
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
    // fy of row y0 + l in lane l (rows past the frame: the clamped row), one
    // correctly rounded division per tile instead of one per row; a row reads
    // its lane's value as a wave-uniform scalar
    const float fy_lane = 1.0f - ((float)min(y0 + (lane & (FXL_TY - 1)), H - 1) + 0.5f) / (float)H;
    // one pixel of row y0 + ly (its value; rows past the frame are computed on a
    // clamped row and not stored)
    // pixel block b of the tile: lane -> column col, row ly
    auto px_col = [&](int b) { return (b % NBX) * 8 + (lane & 7); };
    auto px_row = [&](int b) { return (b / NBX) * 8 + (lane >> 3); };
    auto pixel = [&](int blk) -> uint32_t {
        const int col = px_col(blk), ly = px_row(blk);
        const int y = min(y0 + ly, H - 1);
        const int rr = FXL_TY - 1 - (y - y0);  // block row of the pixel's texel, less the halo
        const int m = (rr + FXL_HALO) * FXL_W + (col + FXL_HALO);
        const float lNW = slum[m - FXL_W - 1], lNE = slum[m - FXL_W + 1], lSW = slum[m + FXL_W - 1];
        const float lSE = slum[m + FXL_W + 1], lM = slum[m];
        const uint32_t tM = stex[m];
        // (lane col's fx and lane ly's fy, one ds_bpermute each)
        const float fx = __int_as_float(__builtin_amdgcn_ds_bpermute(col * 4, __float_as_int(fx_lane)));
        const float fy = __int_as_float(__builtin_amdgcn_ds_bpermute(ly * 4, __float_as_int(fy_lane)));
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
        // 1/x correctly rounded as one Newton step from v_rcp_f32: x lies in
        // [1/128, 2.125] (dirReduce in [1/128, 1/8], |dx|, |dy| <= 2 for lumas
        // in [0, 1]), and over every float of [2^-8, 4) the step equals the IEEE
        // quotient bit for bit on gfx950 (tools/rcp_exhaustive.hip: 83,886,080
        // floats, 0 mismatches; profiles/r05/rcp_exhaustive.json): 3 VALU
        // instead of the 12 of the div_scale / div_fmas / div_fixup expansion
        const float dmin = fminf(fabsf(dx), fabsf(dy)) + dirReduce;
        const float r0 = __builtin_amdgcn_rcpf(dmin);
        float rcpDirMin = fmaf(fmaf(-dmin, r0, 1.0f), r0, r0);
        const float dxs = __builtin_amdgcn_fmed3f(dx * rcpDirMin, -FXAA_SPAN_MAX, FXAA_SPAN_MAX);
        const float dys = __builtin_amdgcn_fmed3f(dy * rcpDirMin, -FXAA_SPAN_MAX, FXAA_SPAN_MAX);
        // A short span: with |dxs|, |dys| <= 0.5 texel every span tap (|k| <=
        // 0.5) lies within 0.25 texel of the pixel centre x + 0.5 (row: H - y -
        // 0.5), and the roundings of its float address stay below 0.19 texel for
        // W, H <= 2^20 (the bound above), so all four taps read the centre texel
        // tM.  Then a = (s + s) * 0.5 = s and b = s * 0.5 + (s + s) * 0.25 = s
        // exactly, luma(b) = lM lies in [lMin, lMax], c = s, and unorm8 of
        // byte / 255 is the byte again for all 256 bytes: the output is tM.
        // Taken when the wave's whole block is short-span.
        if (__builtin_amdgcn_ballot_w64(fmaxf(fabsf(dxs), fabsf(dys)) > 0.5f) == 0) return tM;
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
    // two blocks at a time: their dependent chains (LDS taps -> division -> span
    // taps) interleave
    constexpr int NB = NBX * (FXL_TY / 8);  // pixel blocks per tile
    for (int b = wv; b < NB; b += 2 * FXL_NW) {
        const uint32_t v0 = pixel(b), v1 = pixel(b + FXL_NW);
        const int xa = x0 + px_col(b), ya = y0 + px_row(b), xb = x0 + px_col(b + FXL_NW), yb = y0 + px_row(b + FXL_NW);
        if (xa < W && ya < H) out[(size_t)ya * W + xa] = v0;
        if (xb < W && yb < H) out[(size_t)yb * W + xb] = v1;
    }
}

hipError_t launch_fxaa(const uint32_t* in, uint32_t* out, int W, int H, hipStream_t s) {
    if (W <= 0 || H <= 0) return hipSuccess;
    if (W <= FXL_MAX_DIM && H <= FXL_MAX_DIM) {
        dim3 grid((W + FXL_TX - 1) / FXL_TX, (H + FXL_TY - 1) / FXL_TY);
        hipLaunchKernelGGL(rm_fxaa_lds_kernel, grid, dim3(FXL_NT), 0, s, in, out, W, H);
        return hipGetLastError();
    }
    dim3 grid((W + FXAA_TX - 1) / FXAA_TX, (H + FXAA_TY - 1) / FXAA_TY);
    hipLaunchKernelGGL(rm_fxaa_kernel, grid, dim3(256), 0, s, in, out, W, H);
    return hipGetLastError();
}

}  // namespace rm
