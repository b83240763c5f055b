// rm_plugin.h -- prelude of a scene plugin's translation unit.
//
// rm_load_scene("scene.hip") compiles, with hiprtc for gfx950,
//
//     #include "rm_plugin.h"
//     namespace rm { namespace glsl {            // GLSL names win over HIP's
//     #pragma clang force_cuda_host_device begin // GLSL has no __device__
//     <the preprocessed scene source, GLSL spellings translated>
//     #pragma clang force_cuda_host_device end
//     } }
//     #include "rm_plugin_kernels.h"
//
// The scene source defines `SdResult sceneSDF(vec3 p)` with the library of
// rm_sdf_lib.h, as output_shader.frag:12-48 does with common.frag, and may
// read the pass's uniforms u_resolution, u_pos, u_mouse, u_time
// (common.frag:4-7).  The render pipeline is output_shader.frag's render()
// and main() (rm_render_direct.h render_O), as for the compiled-in scene O.
#pragma once
#include "rm_render_direct.h"
#include "rm_sdf_lib.h"

namespace rm {
namespace glsl {

// The pass's uniforms, copied at the start of every plugin kernel from its
// FrameConst argument into LDS, where any function of the scene can read
// them (the kernel-argument segment is addressable only in the kernel's own
// body, and hiprtc does not inline every call).
struct PluginUniforms {
    float res_x, res_y, pos_x, pos_y, pos_z, mouse_x, mouse_y, time;
};
__shared__ PluginUniforms plugin_lds_uniforms;

__device__ __forceinline__ void plugin_bind_uniforms(const FrameConst& F) {
    if (threadIdx.x == 0)
        plugin_lds_uniforms = PluginUniforms{F.res_x, F.res_y, F.pos_x, F.pos_y, F.pos_z, F.mouse_x, F.mouse_y, F.time};
    __syncthreads();
}
__device__ __forceinline__ const PluginUniforms& plugin_uniforms() { return plugin_lds_uniforms; }

}  // namespace glsl
}  // namespace rm

#define u_resolution (::rm::glsl::vec2(::rm::glsl::plugin_uniforms().res_x, ::rm::glsl::plugin_uniforms().res_y))
#define u_pos                                                                                            \
    (::rm::glsl::vec3(::rm::glsl::plugin_uniforms().pos_x, ::rm::glsl::plugin_uniforms().pos_y,          \
                      ::rm::glsl::plugin_uniforms().pos_z))
#define u_mouse (::rm::glsl::vec2(::rm::glsl::plugin_uniforms().mouse_x, ::rm::glsl::plugin_uniforms().mouse_y))
#define u_time (::rm::glsl::plugin_uniforms().time)
