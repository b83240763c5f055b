// rm_kernels_impl.h -- the per-pixel render kernel template and its launcher,
// instantiated per scene in rm_kernels_t.hip (S0, T) and rm_kernels_o.hip
// (O, OG; compiled without FMA contraction, see DESIGN.md "Parity policy").
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rm_device.h"
#include "rm_launch.h"
#include "rm_render_direct.h"

namespace rm {

// Minimum waves per SIMD the register allocator must allow.  Scene O asks
// for 8 (64 VGPRs): its kernel needs ~82, and the few spills to scratch cost
// less than occupancy 5 does (C5 frame 12.29 -> 11.56 ms,
// profiles/r02/scene_O_occupancy_ab.jsonl); S0/T fit 8 waves unasked; the
// glass test scene OG would spill ~80 VGPRs and keeps its allocation.
template <int SC>
constexpr int kWavesPerEU = SC == SCENE_O ? 8 : 1;
template <int SC, bool COUNT, int K, typename OUT>
__global__ __launch_bounds__(64 * Tiling<K>::WPB) __attribute__((amdgpu_waves_per_eu(kWavesPerEU<SC>)))
void rm_render_direct(FrameConst F, OUT* __restrict__ out, unsigned long long* __restrict__ evals) {
    render_tile<SC, COUNT, K, OUT>(F, out, evals);
}

template <int SC, bool COUNT, typename OUT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kWavesPerEU<SC>)))
void rm_render_persist(FrameConst F, OUT* __restrict__ out, unsigned long long* __restrict__ evals, int gx,
                       int ntiles) {
    render_persistent<SC, COUNT, OUT>(F, out, evals, gx, ntiles);
}

template <int SC>
__global__ __launch_bounds__(256) void rm_scene_eval(FrameConst F, const float* __restrict__ pts, long long n,
                                                     float* __restrict__ dist, float* __restrict__ mat) {
    scene_eval_one<SC>(F, pts, n, dist, mat);
}

template <int SC>
hipError_t launch_eval(const FrameConst& F, const float* pts, long long n, float* dist, float* mat, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL((rm_scene_eval<SC>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, F, pts, n, dist, mat);
    return hipGetLastError();
}

template <int SC, int K, typename OUT>
hipError_t launch_direct(const FrameConst& F, OUT* out, unsigned long long* evals, hipStream_t s) {
    using T = Tiling<K>;
    dim3 grid((F.W + T::TW - 1) / T::TW, (F.nrows + T::TH - 1) / T::TH), block(64 * T::WPB);
    FrameConst G = F;
    G.gx_magic = div_magic(grid.x, (uint64_t)grid.x * grid.y);
    if (evals) hipLaunchKernelGGL((rm_render_direct<SC, true, K, OUT>), grid, block, 0, s, G, out, evals);
    else hipLaunchKernelGGL((rm_render_direct<SC, false, K, OUT>), grid, block, 0, s, G, out, evals);
    return hipGetLastError();
}

// As many persistent waves as the device holds at once (the occupancy of the
// kernel on every CU), at most one per tile.
template <int SC, typename OUT>
hipError_t launch_persist(const FrameConst& F, OUT* out, unsigned long long* evals, hipStream_t s) {
    if (!F.persist) return hipErrorInvalidValue;
    const TileGrid g = tile_grid(KERNEL_PERSIST, F.W, F.nrows);
    const int ntiles = g.x * g.y;
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess)
        e = evals ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rm_render_persist<SC, true, OUT>, 64, 0)
                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rm_render_persist<SC, false, OUT>, 64, 0);
    if (e != hipSuccess) return e;
    const int waves = std::max(1, std::min(ntiles, cus * std::max(per_cu, 1)));
    FrameConst G = F;
    G.gx_magic = div_magic(g.x, (uint64_t)ntiles);
    if (evals) hipLaunchKernelGGL((rm_render_persist<SC, true, OUT>), dim3(waves), dim3(64), 0, s, G, out, evals, g.x, ntiles);
    else hipLaunchKernelGGL((rm_render_persist<SC, false, OUT>), dim3(waves), dim3(64), 0, s, G, out, evals, g.x, ntiles);
    return hipGetLastError();
}

template <int SC, typename OUT>
hipError_t launch_tiling(const FrameConst& F, OUT* out, unsigned long long* evals, int kernel, hipStream_t s) {
    if (kernel == KERNEL_PERSIST) return launch_persist<SC>(F, out, evals, s);
    if (kernel == KERNEL_TILE16) return launch_direct<SC, KERNEL_TILE16>(F, out, evals, s);
    if (kernel == KERNEL_TILE16X4) return launch_direct<SC, KERNEL_TILE16X4>(F, out, evals, s);
    return launch_direct<SC, KERNEL_TILE8>(F, out, evals, s);
}

// the compressed wire's tile slots (rm_wire_tile.h) instead of pixels: the
// one-wave 8x8 tiling only
template <int SC>
hipError_t launch_scene_wire(const FrameConst& F, WireTile* slots, unsigned long long* evals, hipStream_t s) {
    return launch_direct<SC, KERNEL_TILE8>(F, slots, evals, s);
}

template <int SC>
hipError_t launch_scene(const FrameConst& F, void* out, bool rgba8, unsigned long long* evals, int kernel,
                        hipStream_t s) {
    if (rgba8) return launch_tiling<SC>(F, static_cast<uint32_t*>(out), evals, kernel, s);
    return launch_tiling<SC>(F, static_cast<float4*>(out), evals, kernel, s);
}

}  // namespace rm
