// rm_kernels_impl.h -- the per-pixel render kernel template and its launcher,
// instantiated per scene in rm_kernels_t.hip (S0, T) and rm_kernels_o.hip
// (O, OG; compiled without FMA contraction, see DESIGN.md "Parity policy").
#pragma once
#include <hip/hip_runtime.h>

#include "rm_device.h"
#include "rm_launch.h"
#include "rm_render_direct.h"

namespace rm {

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int SC>
__device__ __forceinline__ V3 render_pixel(const FrameConst& F, V3 ro, V3 rd, Tally& cnt) {
    if constexpr (SC == SCENE_S0) return render_S0(F, ro, rd, cnt);
    else if constexpr (SC == SCENE_T) return render_T(F, ro, rd, cnt);
    else return render_O<SC>(F, ro, rd, cnt);
}

// Workgroup shapes (KernelKind): KERNEL_TILE16 = 16x16 pixels as 2x2 waves
// of 8x8; KERNEL_TILE8 = one 8x8-pixel wave per workgroup (the dispatcher
// then refills CUs at wave granularity, which shortens the tail of small or
// uneven launches); KERNEL_TILE16X4 = one 16x4-pixel wave.
template <int K> struct Tiling;
template <> struct Tiling<KERNEL_TILE16> { static constexpr int TW = 16, TH = 16, WPB = 4, LW = 8; };
template <> struct Tiling<KERNEL_TILE8> { static constexpr int TW = 8, TH = 8, WPB = 1, LW = 8; };
template <> struct Tiling<KERNEL_TILE16X4> { static constexpr int TW = 16, TH = 4, WPB = 1, LW = 16; };

// OUT = float4 (gl_FragColor) or uint32_t (RGBA8, packed in the epilogue, so
// the displayed frame costs 4 B/px of HBM instead of 16 + 20 for a pack pass)
template <int SC, bool COUNT, int K, typename OUT>
__global__ __launch_bounds__(64 * Tiling<K>::WPB) void rm_render_direct(FrameConst F, OUT* __restrict__ out,
                                                                        unsigned long long* __restrict__ evals) {
    using T = Tiling<K>;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int x = blockIdx.x * T::TW + (w & 1) * 8 + (lane % T::LW);
    const int j = blockIdx.y * T::TH + (w >> 1) * 8 + (lane / T::LW);
    Tally cnt;
    if (x < F.W && j < F.nrows) {
        const int y = shard_row(F, F.row0 + j);
        float tcx, tcy;
        V3 ro, rd;
        camera_ray(F, x, y, tcx, tcy, ro, rd);
        V3 c = render_pixel<SC>(F, ro, rd, cnt);
        c = post_colour<FastMath<SC>::value>(c, tcx, tcy);
        if constexpr (sizeof(OUT) == 4) out[(size_t)j * F.W + x] = pack_rgba8(c.x, c.y, c.z, 1.0f);
        else out[(size_t)j * F.W + x] = make_float4(c.x, c.y, c.z, 1.0f);
    }
    if constexpr (COUNT) {
        uint32_t se = wave_sum_u32(cnt.evals), sf = wave_sum_u32(cnt.flop);
        if (lane == 0) {
            atomicAdd(&evals[0], (unsigned long long)se);
            atomicAdd(&evals[1], (unsigned long long)sf);
        }
    }
}

template <int SC, int K, typename OUT>
hipError_t launch_direct(const FrameConst& F, OUT* out, unsigned long long* evals, hipStream_t s) {
    using T = Tiling<K>;
    dim3 grid((F.W + T::TW - 1) / T::TW, (F.nrows + T::TH - 1) / T::TH), block(64 * T::WPB);
    if (evals) hipLaunchKernelGGL((rm_render_direct<SC, true, K, OUT>), grid, block, 0, s, F, out, evals);
    else hipLaunchKernelGGL((rm_render_direct<SC, false, K, OUT>), grid, block, 0, s, F, out, evals);
    return hipGetLastError();
}

template <int SC, typename OUT>
hipError_t launch_tiling(const FrameConst& F, OUT* out, unsigned long long* evals, int kernel, hipStream_t s) {
    if (kernel == KERNEL_TILE16) return launch_direct<SC, KERNEL_TILE16>(F, out, evals, s);
    if (kernel == KERNEL_TILE16X4) return launch_direct<SC, KERNEL_TILE16X4>(F, out, evals, s);
    return launch_direct<SC, KERNEL_TILE8>(F, out, evals, s);
}

template <int SC>
hipError_t launch_scene(const FrameConst& F, void* out, bool rgba8, unsigned long long* evals, int kernel,
                        hipStream_t s) {
    if (rgba8) return launch_tiling<SC>(F, static_cast<uint32_t*>(out), evals, kernel, s);
    return launch_tiling<SC>(F, static_cast<float4*>(out), evals, kernel, s);
}

}  // namespace rm
