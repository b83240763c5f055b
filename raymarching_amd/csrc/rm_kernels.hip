// rm_kernels.hip -- gfx950 kernels of the ray-march pass and their launchers.
//
// The render kernels live in rm_kernels_impl.h, instantiated per scene in
// rm_kernels_t.hip / rm_kernels_o.hip; this file holds the scene dispatch and
// the small frame kernels:
//   rm_deinterleave              root-side permute of gathered row bands.
//   rm_pack_rgba8                float4 -> RGBA8 (the reference target format).
//   rm_pack_rgb8 / rm_deinterleave_rgb8   the 3 B/px wire of row-sharded RGBA8
//                                frames (alpha is 1 by construction).
// COUNT=true is the instrumented build used to count sceneSDF calls
// (ray-steps); timing runs use COUNT=false.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rm_device.h"
#include "rm_launch.h"

namespace rm {

// gathered: nshards blocks of rows_per_shard packed rows (W elements each);
// out: the W x H frame.  One thread per element (float4 or RGBA8 word).
// Frame rows blockIdx.y, blockIdx.y + gridDim.y, ...: the shard / packed-row
// arithmetic is wave-uniform (scalar), once per row.
template <typename E>
__global__ __launch_bounds__(256) void rm_deinterleave(const E* __restrict__ gathered, E* __restrict__ out, int W,
                                                         int H, int band, int nshards, int rows_per_shard) {
    for (int y = blockIdx.y; y < H; y += gridDim.y) {
        const int gb = y / band, r = y - gb * band;
        const int shard = gb % nshards, lb = gb / nshards;
        const E* src = gathered + ((size_t)shard * rows_per_shard + lb * band + r) * W;
        E* dst = out + (size_t)y * W;
        for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < W; x += gridDim.x * blockDim.x) dst[x] = src[x];
    }
}

__global__ __launch_bounds__(256) void rm_pack_rgba8(const float4* __restrict__ in, uint32_t* __restrict__ out,
                                                       size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = in[i];
        out[i] = pack_rgba8(v.x, v.y, v.z, v.w);
    }
}

// RGBA8 words -> 3-byte RGB.  The pass writes gl_FragColor = vec4(col, 1.0)
// (output_shader.frag:419, template.frag:98), so alpha carries no information
// on the wire; the root restores it as 255.  vec: in 16-byte and out 4-byte
// aligned, then 4 pixels per lane (one 16-byte load, three 4-byte stores).
__global__ __launch_bounds__(256) void rm_pack_rgb8(const uint32_t* __restrict__ in, uint8_t* __restrict__ out,
                                                      size_t n, int vec) {
    const size_t stride = (size_t)gridDim.x * blockDim.x, t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t ng = vec ? n / 4 : 0;
    for (size_t g = t0; g < ng; g += stride) {
        const uint4 v = reinterpret_cast<const uint4*>(in)[g];
        uint32_t* o = reinterpret_cast<uint32_t*>(out) + 3 * g;
        o[0] = (v.x & 0xFFFFFFu) | (v.y << 24);
        o[1] = ((v.y >> 8) & 0xFFFFu) | (v.z << 16);
        o[2] = ((v.z >> 16) & 0xFFu) | (v.w << 8);
    }
    for (size_t i = 4 * ng + t0; i < n; i += stride) {
        const uint32_t w = in[i];
        out[3 * i] = (uint8_t)w;
        out[3 * i + 1] = (uint8_t)(w >> 8);
        out[3 * i + 2] = (uint8_t)(w >> 16);
    }
}

// gathered: nshards blocks of rows_per_shard packed rows of 3*W bytes; out:
// the W x H RGBA8 frame (alpha 255).  One workgroup row per frame row
// (blockIdx.y = y: the shard / packed-row arithmetic is wave-uniform, scalar,
// once per row); vec (W % 4 == 0, aligned buffers): one lane per 4 pixels
// (three 4-byte loads, one 16-byte store).
__global__ __launch_bounds__(256) void rm_deinterleave_rgb8(const uint8_t* __restrict__ gathered,
                                                              uint32_t* __restrict__ out, int W, int H, int band,
                                                              int nshards, int rows_per_shard, int vec) {
    const int per_row = vec ? W / 4 : W;
    for (int y = blockIdx.y; y < H; y += gridDim.y) {
    const int gb = y / band, r = y - gb * band;
    const int shard = gb % nshards, lb = gb / nshards;
    const uint8_t* src = gathered + ((size_t)shard * rows_per_shard + lb * band + r) * 3 * (size_t)W;
    uint32_t* dst = out + (size_t)y * W;
    for (int xg = blockIdx.x * blockDim.x + threadIdx.x; xg < per_row; xg += gridDim.x * blockDim.x) {
        if (vec) {
            const uint32_t* s = reinterpret_cast<const uint32_t*>(src) + 3 * xg;
            const uint32_t w0 = s[0], w1 = s[1], w2 = s[2];
            reinterpret_cast<uint4*>(dst)[xg] =
                make_uint4((w0 & 0xFFFFFFu) | 0xFF000000u, (w0 >> 24) | ((w1 & 0xFFFFu) << 8) | 0xFF000000u,
                           (w1 >> 16) | ((w2 & 0xFFu) << 16) | 0xFF000000u, (w2 >> 8) | 0xFF000000u);
        } else {
            const uint8_t* q = src + 3 * (size_t)xg;
            dst[xg] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | 0xFF000000u;
        }
    }
    }
}

// Frame rows of cyclic parts (rm_deinterleave_cycle_rgb8): part p owns the rows
// y with (y mod cycle) - off[p] in [0, run[p]); its packed rows start at byte
// base[p] of `gathered` (3 * W bytes each).  The parts partition [0, cycle).
__global__ __launch_bounds__(256) void rm_deinterleave_cycle_rgb8(const uint8_t* __restrict__ gathered,
                                                                    uint32_t* __restrict__ out, int W, int H,
                                                                    int cycle, CycleParts parts, int vec) {
    const int per_row = vec ? W / 4 : W;
    for (int y = blockIdx.y; y < H; y += gridDim.y) {
        const int c = y / cycle, m = y - c * cycle;
        int p = 0;
        while (p + 1 < parts.n && parts.off[p + 1] <= m) p++;  // (wave-uniform)
        const uint8_t* src = gathered + parts.base[p] + ((size_t)c * parts.run[p] + (m - parts.off[p])) * 3 * (size_t)W;
        uint32_t* dst = out + (size_t)y * W;
        for (int xg = blockIdx.x * blockDim.x + threadIdx.x; xg < per_row; xg += gridDim.x * blockDim.x) {
            if (vec) {
                const uint32_t* s = reinterpret_cast<const uint32_t*>(src) + 3 * xg;
                const uint32_t w0 = s[0], w1 = s[1], w2 = s[2];
                reinterpret_cast<uint4*>(dst)[xg] =
                    make_uint4((w0 & 0xFFFFFFu) | 0xFF000000u, (w0 >> 24) | ((w1 & 0xFFFFu) << 8) | 0xFF000000u,
                               (w1 >> 16) | ((w2 & 0xFFu) << 16) | 0xFF000000u, (w2 >> 8) | 0xFF000000u);
            } else {
                const uint8_t* q = src + 3 * (size_t)xg;
                dst[xg] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | 0xFF000000u;
            }
        }
    }
}

// ------------------------------------------------ adaptive dispatch order
// Next launch's tile order from this launch's tile durations (rm_params.
// schedule): a counting sort, costliest first, over the sched_bucket buckets
// (rm_device.h) of the durations the render kernel wrote.  Within a bucket
// the order is arbitrary; the result is a permutation.  Two kernels:
// rm_sched_hist counts tiles per bucket (per-block LDS histograms, one global
// add per non-empty bucket and block: a global add per tile from the render
// epilogue instead measured 3x slower frames, 256 hot addresses);
// rm_sched_scatter places each block's 1024 tiles at bucket offset (exclusive
// scan of the histogram) + the block's reservation in the bucket (cursor) +
// the tile's rank in the block, and clears the other parity's histogram and
// cursors (`next`) for the following sort (no memset on the stream).  The
// context runs both on the frame's stream right after the measuring launch.
// The sort key of tile i: its duration, or with a dilation radius r > 0 the
// longest duration among the tiles within r of it on the gx-wide tile grid
// (an order that stays right while the costly regions move a few tiles
// between the launch that measured them and the launches that use the order).
__device__ __forceinline__ uint32_t tile_key(const uint32_t* __restrict__ cost, int i, int n, int gx, int r) {
    if (r <= 0) return cost[i];
    const int x = i % gx, y = i / gx;
    uint32_t m = 0;
    for (int yy = max(0, y - r); yy <= y + r; yy++)
        for (int xx = max(0, x - r); xx <= min(gx - 1, x + r); xx++) {
            const int j = yy * gx + xx;
            if (j < n) m = max(m, cost[j]);
        }
    return m;
}

// tile_key for a compile-time radius: every load in flight at once (the
// run-time loop waited on each of its 25 loads in turn: 17 us per sort)
template <int R>
__device__ __forceinline__ uint32_t tile_key_r(const uint32_t* __restrict__ cost, int i, int n, int gx) {
    const int x = i % gx, y = i / gx;
    uint32_t m = 0;
#pragma unroll
    for (int dy = -R; dy <= R; dy++)
#pragma unroll
        for (int dx = -R; dx <= R; dx++) {
            const int yy = y + dy, xx = x + dx, j = yy * gx + xx;
            const bool in = yy >= 0 && xx >= 0 && xx < gx && j < n;
            const uint32_t v = cost[in ? j : i];
            m = max(m, v);
        }
    return m;
}

// one tile per thread: its bucket (kept for the scatter: the dilated key reads
// (2r + 1)^2 durations, formed once) and the block's histogram
__global__ __launch_bounds__(256) void rm_sched_hist(const uint32_t* __restrict__ cost, int n, int gx, int r,
                                                      uint32_t* __restrict__ hist, uint8_t* __restrict__ bucket) {
    __shared__ uint32_t h[kSchedBuckets];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        const int b = sched_bucket(r == 2 ? tile_key_r<2>(cost, i, n, gx) : tile_key(cost, i, n, gx, r));
        bucket[i] = (uint8_t)b;
        atomicAdd(&h[b], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(256) void rm_sched_scatter(const uint8_t* __restrict__ bucket, int n,
                                                         const uint32_t* __restrict__ hist, uint32_t* __restrict__ cursor,
                                                         uint32_t* __restrict__ order, uint32_t* __restrict__ next) {
    __shared__ uint32_t base[kSchedBuckets], cnt[kSchedBuckets];
    const int t = threadIdx.x;
    if (blockIdx.x == 0) next[t] = next[kSchedBuckets + t] = 0;
    base[t] = hist[t];
    cnt[t] = 0;
    __syncthreads();
    for (int o = 1; o < kSchedBuckets; o <<= 1) {  // inclusive scan (Hillis-Steele)
        const uint32_t v = t >= o ? base[t - o] : 0;
        __syncthreads();
        base[t] += v;
        __syncthreads();
    }
    const uint32_t excl = base[t] - hist[t];
    __syncthreads();
    base[t] = excl;
    int b[4];
    uint32_t rank[4];
    const int i0 = blockIdx.x * 1024 + t;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = i0 + 256 * k;
        b[k] = i < n ? (int)bucket[i] : -1;
        rank[k] = b[k] >= 0 ? atomicAdd(&cnt[b[k]], 1u) : 0;
    }
    __syncthreads();
    if (cnt[t]) base[t] += atomicAdd(&cursor[t], cnt[t]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (b[k] >= 0) order[base[b[k]] + rank[k]] = (uint32_t)(i0 + 256 * k);
}

hipError_t launch_tile_order(const uint32_t* cost, int n, int gx, int radius, uint32_t* order, uint32_t* hist,
                             uint32_t* next, uint8_t* bucket, hipStream_t s) {
    if (n <= 0 || gx <= 0) return hipSuccess;
    hipLaunchKernelGGL(rm_sched_hist, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, cost, n, gx, radius, hist,
                       bucket);
    hipLaunchKernelGGL(rm_sched_scatter, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, s, bucket, n, hist,
                       hist + kSchedBuckets, order, next);
    return hipGetLastError();
}

// ------------------------------------------------------------- launchers

#define RM_SCENE_LAUNCHER(name) \
    hipError_t name(const FrameConst& F, void* out, bool rgba8, unsigned long long* evals, int kernel, hipStream_t s);
RM_SCENE_LAUNCHER(launch_scene_s0)
RM_SCENE_LAUNCHER(launch_scene_t)
RM_SCENE_LAUNCHER(launch_scene_o)
RM_SCENE_LAUNCHER(launch_scene_og)

hipError_t launch_render(int scene, const FrameConst& F, void* out, bool rgba8, unsigned long long* evals, int kernel,
                         hipStream_t s) {
    if (F.W <= 0 || F.nrows <= 0) return hipSuccess;
    switch (scene) {
    case SCENE_S0: return launch_scene_s0(F, out, rgba8, evals, kernel, s);
    case SCENE_T: return launch_scene_t(F, out, rgba8, evals, kernel, s);
    case SCENE_O: return launch_scene_o(F, out, rgba8, evals, kernel, s);
    case SCENE_OG: return launch_scene_og(F, out, rgba8, evals, kernel, s);
    default: return hipErrorInvalidValue;
    }
}

#define RM_WIRE_LAUNCHER(name) \
    hipError_t name(const FrameConst& F, WireTile* slots, unsigned long long* evals, hipStream_t s);
RM_WIRE_LAUNCHER(launch_wire_s0)
RM_WIRE_LAUNCHER(launch_wire_t)
RM_WIRE_LAUNCHER(launch_wire_o)
RM_WIRE_LAUNCHER(launch_wire_og)

hipError_t launch_render_wire(int scene, const FrameConst& F, WireTile* slots, unsigned long long* evals,
                              hipStream_t s) {
    if (F.W <= 0 || F.nrows <= 0) return hipSuccess;
    switch (scene) {
    case SCENE_S0: return launch_wire_s0(F, slots, evals, s);
    case SCENE_T: return launch_wire_t(F, slots, evals, s);
    case SCENE_O: return launch_wire_o(F, slots, evals, s);
    case SCENE_OG: return launch_wire_og(F, slots, evals, s);
    default: return hipErrorInvalidValue;
    }
}

#define RM_EVAL_LAUNCHER(name) \
    hipError_t name(const FrameConst& F, const float* pts, long long n, float* dist, float* mat, hipStream_t s);
RM_EVAL_LAUNCHER(launch_eval_s0)
RM_EVAL_LAUNCHER(launch_eval_t)
RM_EVAL_LAUNCHER(launch_eval_o)
RM_EVAL_LAUNCHER(launch_eval_og)

hipError_t launch_scene_eval(int scene, const FrameConst& F, const float* pts, long long n, float* dist, float* mat,
                             hipStream_t s) {
    switch (scene) {
    case SCENE_S0: return launch_eval_s0(F, pts, n, dist, mat, s);
    case SCENE_T: return launch_eval_t(F, pts, n, dist, mat, s);
    case SCENE_O: return launch_eval_o(F, pts, n, dist, mat, s);
    case SCENE_OG: return launch_eval_og(F, pts, n, dist, mat, s);
    default: return hipErrorInvalidValue;
    }
}

template <typename E>
static hipError_t deinterleave_t(const E* gathered, E* out, int W, int H, int band, int nshards, int rows_per_shard,
                                 hipStream_t s) {
    if (W <= 0 || H <= 0) return hipSuccess;
    const unsigned bx = (unsigned)std::min((W + 255) / 256, 64);
    hipLaunchKernelGGL(rm_deinterleave<E>, dim3(bx, (unsigned)std::min(H, 65535)), dim3(256), 0, s, gathered, out, W, H,
                       band, nshards, rows_per_shard);
    return hipGetLastError();
}

hipError_t launch_deinterleave(const float4* gathered, float4* out, int W, int H, int band, int nshards,
                               int rows_per_shard, hipStream_t s) {
    return deinterleave_t(gathered, out, W, H, band, nshards, rows_per_shard, s);
}

hipError_t launch_deinterleave_u32(const uint32_t* gathered, uint32_t* out, int W, int H, int band, int nshards,
                                   int rows_per_shard, hipStream_t s) {
    return deinterleave_t(gathered, out, W, H, band, nshards, rows_per_shard, s);
}

hipError_t launch_pack_rgba8(const float4* in, uint32_t* out, size_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    unsigned blocks = (unsigned)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
    hipLaunchKernelGGL(rm_pack_rgba8, dim3(blocks), dim3(256), 0, s, in, out, n);
    return hipGetLastError();
}

hipError_t launch_pack_rgb8(const uint32_t* in, uint8_t* out, size_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    const int vec = ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 4 == 0);
    const size_t work = vec ? (n + 3) / 4 : n;
    unsigned blocks = (unsigned)((work + 255) / 256 < 8192 ? (work + 255) / 256 : 8192);
    hipLaunchKernelGGL(rm_pack_rgb8, dim3(blocks), dim3(256), 0, s, in, out, n, vec);
    return hipGetLastError();
}

hipError_t launch_deinterleave_cycle_rgb8(const uint8_t* gathered, uint32_t* out, int W, int H, int cycle,
                                          const CycleParts& parts, hipStream_t s) {
    if (W <= 0 || H <= 0) return hipSuccess;
    int vec = (W % 4 == 0) && ((uintptr_t)gathered % 4 == 0) && ((uintptr_t)out % 16 == 0);
    for (int p = 0; p < parts.n; p++) vec = vec && parts.base[p] % 4 == 0;
    const int per_row = vec ? W / 4 : W;
    const unsigned bx = (unsigned)std::min((per_row + 255) / 256, 64);
    hipLaunchKernelGGL(rm_deinterleave_cycle_rgb8, dim3(bx, (unsigned)std::min(H, 65535)), dim3(256), 0, s, gathered,
                       out, W, H, cycle, parts, vec);
    return hipGetLastError();
}

hipError_t launch_deinterleave_rgb8(const uint8_t* gathered, uint32_t* out, int W, int H, int band, int nshards,
                                    int rows_per_shard, hipStream_t s) {
    const size_t n = (size_t)W * H;
    if (!n) return hipSuccess;
    const int vec = (W % 4 == 0) && ((uintptr_t)gathered % 4 == 0) && ((uintptr_t)out % 16 == 0);
    const int per_row = vec ? W / 4 : W;
    const unsigned bx = (unsigned)std::min((per_row + 255) / 256, 64);
    hipLaunchKernelGGL(rm_deinterleave_rgb8, dim3(bx, (unsigned)std::min(H, 65535)), dim3(256), 0, s, gathered, out,
                       W, H, band, nshards, rows_per_shard, vec);
    return hipGetLastError();
}

}  // namespace rm
