// rm_kernels_impl.h -- the per-pixel render kernel template and its launcher,
// instantiated per scene in rm_kernels_t.hip (S0, T) and rm_kernels_o.hip
// (O, OG; compiled without FMA contraction, see DESIGN.md "Parity policy").
#pragma once
#include <hip/hip_runtime.h>

#include "rm_device.h"
#include "rm_launch.h"
#include "rm_render_direct.h"
#include "rm_render_wave.h"

namespace rm {

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int SC>
__device__ __forceinline__ V3 render_pixel(const FrameConst& F, V3 ro, V3 rd, uint32_t& cnt) {
    if constexpr (SC == SCENE_S0) return render_S0(F, ro, rd, cnt);
    else if constexpr (SC == SCENE_T) return render_T(F, ro, rd, cnt);
    else return render_O<SC>(F, ro, rd, cnt);
}

template <int SC, bool COUNT>
__global__ __launch_bounds__(256) void rm_render_direct(FrameConst F, float4* __restrict__ out,
                                                          unsigned long long* __restrict__ evals) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (w & 1) * 8 + (lane & 7);
    const int j = blockIdx.y * 16 + (w >> 1) * 8 + (lane >> 3);
    uint32_t cnt = 0;
    if (x < F.W && j < F.nrows) {
        const int y = shard_row(F, F.row0 + j);
        float tcx, tcy;
        V3 ro, rd;
        camera_ray(F, x, y, tcx, tcy, ro, rd);
        V3 c = render_pixel<SC>(F, ro, rd, cnt);
        c = post_colour<FastMath<SC>::value>(c, tcx, tcy);
        out[(size_t)j * F.W + x] = make_float4(c.x, c.y, c.z, 1.0f);
    }
    if constexpr (COUNT) {
        uint32_t s = wave_sum_u32(cnt);
        if (lane == 0) atomicAdd(evals, (unsigned long long)s);
    }
}

template <int SC>
hipError_t launch_scene(const FrameConst& F, float4* out, unsigned long long* evals, int kernel,
                               hipStream_t s) {
    if (kernel == KERNEL_WAVE && has_wave_kernel(SC)) return launch_wave<SC>(F, out, evals, s);
    dim3 grid((F.W + 15) / 16, (F.nrows + 15) / 16), block(256);
    if (evals) hipLaunchKernelGGL((rm_render_direct<SC, true>), grid, block, 0, s, F, out, evals);
    else hipLaunchKernelGGL((rm_render_direct<SC, false>), grid, block, 0, s, F, out, evals);
    return hipGetLastError();
}

}  // namespace rm
