// rm_kernels.hip -- gfx950 kernels of the ray-march pass and their launchers.
//
// The render kernels live in rm_kernels_impl.h, instantiated per scene in
// rm_kernels_t.hip / rm_kernels_o.hip; this file holds the scene dispatch and
// the small frame kernels:
//   rm_deinterleave              root-side permute of gathered row bands.
//   rm_pack_rgba8                float4 -> RGBA8 (the reference target format).
// COUNT=true is the instrumented build used to count sceneSDF calls
// (ray-steps); timing runs use COUNT=false.
#include <hip/hip_runtime.h>

#include "rm_device.h"
#include "rm_launch.h"

namespace rm {

// gathered: nshards blocks of rows_per_shard packed rows (W elements each);
// out: the W x H frame.  One thread per element (float4 or RGBA8 word).
template <typename E>
__global__ __launch_bounds__(256) void rm_deinterleave(const E* __restrict__ gathered, E* __restrict__ out, int W,
                                                         int H, int band, int nshards, int rows_per_shard) {
    const size_t n = (size_t)W * H;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        int y = (int)(i / W), x = (int)(i - (size_t)y * W);
        int gb = y / band, r = y - gb * band;
        int shard = gb % nshards, lb = gb / nshards;
        int j = lb * band + r;
        out[i] = gathered[((size_t)shard * rows_per_shard + j) * W + x];
    }
}

__global__ __launch_bounds__(256) void rm_pack_rgba8(const float4* __restrict__ in, uint32_t* __restrict__ out,
                                                       size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = in[i];
        out[i] = pack_rgba8(v.x, v.y, v.z, v.w);
    }
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
    size_t n = (size_t)W * H;
    if (!n) return hipSuccess;
    unsigned blocks = (unsigned)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
    hipLaunchKernelGGL(rm_deinterleave<E>, dim3(blocks), dim3(256), 0, s, gathered, out, W, H, band, nshards,
                       rows_per_shard);
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

}  // namespace rm
