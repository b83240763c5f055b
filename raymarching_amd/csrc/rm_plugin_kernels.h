// rm_plugin_kernels.h -- epilogue of a scene plugin's translation unit
// (rm_plugin.h): binds the scene's sceneSDF to the render pipeline and defines
// the plugin's kernels, looked up by name (rm_plugin_host.cpp).  The first
// argument of every kernel is the FrameConst the uniforms are bound from.
#pragma once

template <>
struct rm::PluginScene<rm::SCENE_PLUGIN> {
#ifdef RM_SCENE_FLOP
    static constexpr uint32_t flop = RM_SCENE_FLOP;  // per-ray-step FLOP, when the scene states it
#else
    static constexpr uint32_t flop = 0;
#endif
    __device__ __forceinline__ static float dist(rm::V3 p) { return rm::glsl::sceneSDF(p).dist; }
    // the probe form: the scene compiled against the library's probe instance
    __device__ __forceinline__ static float dist_probe(rm::V3 p) { return rm::glsl::probe::sceneSDF(p).dist; }
    __device__ __forceinline__ static rm::Mat mat(rm::V3 p) { return rm::glsl::sceneSDF(p).mat; }
};

#ifndef RM_PLUGIN_EVAL_ONLY
// output_shader.frag's pass over 8x8-pixel one-wave tiles, as two kernels: the
// timed one (rm_plugin_render) and the instrumented one (rm_plugin_render_count:
// ray-step tallies and step maps).  One kernel serving both paid the
// instrumented pipeline's registers in every timed launch (occupancy 5).  The
// output format is a run-time argument.
namespace rm {
template <bool COUNT>
__device__ __forceinline__ void plugin_render_tile(const FrameConst& F, void* out, int rgba8,
                                                   unsigned long long* evals) {
    const uint64_t t_start = F.tile_cost ? clock64() : 0;
    const int lane = threadIdx.x;
    int bx = blockIdx.x, by = blockIdx.y;
    if (F.tile_order) {  // costliest tiles first (rm_params.schedule, rm_set_tile_order)
        const uint32_t t = F.tile_order[by * gridDim.x + bx];
        by = div_by((int)t, F.gx_magic, (int)gridDim.x);
        bx = (int)t - by * (int)gridDim.x;
    }
    const int x = bx * 8 + (lane & 7), j = by * 8 + (lane >> 3);
    Tally cnt;
    if (x < F.W && j < F.nrows) {
        const int y = shard_row(F, F.row0 + j);
        float tcx, tcy;
        V3 ro, rd;
        camera_ray<false>(F, x, y, tcx, tcy, ro, rd);
        const float vig = vignette<FastColour<SCENE_PLUGIN>::value>(tcx, tcy);
        // the exact skips of scene O's pipeline that hold for any scene (the soft
        // shadows of points facing away from the light): taken
        // by the timed launches, counted by the instrumented ones
        V3 c = render_pixel<SCENE_PLUGIN, 3, COUNT ? 2 : 1>(F, ro, rd, cnt);
        c = post_colour<FastColour<SCENE_PLUGIN>::value>(c, vig);
        const size_t i = (size_t)j * F.W + x;
        if (rgba8) store_pixel(F, static_cast<uint32_t*>(out), i, c);
        else store_pixel(F, static_cast<float4*>(out), i, c);
    }
    if (F.tile_cost && lane == 0) {  // this tile's duration: the next launch's dispatch order
        const uint64_t dt = clock64() - t_start;
        F.tile_cost[by * gridDim.x + bx] = dt > 0xffffffffull ? 0xffffffffu : (uint32_t)dt;
    }
    if constexpr (COUNT) {
        if (F.evals_map && x < F.W && j < F.nrows) F.evals_map[(size_t)j * F.W + x] = cnt.evals;
        uint32_t se = wave_sum_u32(cnt.evals), sf = wave_sum_u32(cnt.flop), ss = wave_sum_u32(cnt.skipped);
        if (lane == 0) {
            atomicAdd(&evals[0], (unsigned long long)se);
            atomicAdd(&evals[1], (unsigned long long)sf);
            if (ss) atomicAdd(&evals[2], (unsigned long long)ss);
        }
    }
}
}  // namespace rm
extern "C" __global__ __launch_bounds__(64) void rm_plugin_render(rm::FrameConst F, void* out, int rgba8,
                                                                  unsigned long long* evals) {
    rm::plugin_render_tile<false>(F, out, rgba8, evals);
}
extern "C" __global__ __launch_bounds__(64) void rm_plugin_render_count(rm::FrameConst F, void* out, int rgba8,
                                                                         unsigned long long* evals) {
    rm::plugin_render_tile<true>(F, out, rgba8, evals);
}
#endif

// sceneSDF(p) at explicit points (rm_scene_eval)
extern "C" __global__ __launch_bounds__(256) void rm_plugin_eval(rm::FrameConst F, const float* pts, long long n,
                                                                 float* dist, float* mat) {
    rm::scene_eval_one<rm::SCENE_PLUGIN>(F, pts, n, dist, mat);
}
