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

// The pass's uniforms, read where a scene function needs them from the
// kernel's own FrameConst argument: every plugin kernel takes it first, so it
// sits at offset 0 of the kernel-argument segment, and the scene's functions
// are force-inlined into the kernels (rm_plugin_host.cpp), where that segment
// is addressable.  These are constant-address-space loads, invariant, so a
// uniform read inside a march loop -- transformR's sin and cos of u_time --
// is hoisted out of it.  (Round 4 copied the uniforms to LDS; the LDS read of
// u_time stayed inside the loops, whose volatile asm statements LLVM must
// assume to write memory, and the scene-O plugin evaluated two sin and two
// cos, with two IEEE divisions, on every ray-step.)
typedef const __attribute__((address_space(4))) FrameConst* KernargFrame;
__device__ __forceinline__ KernargFrame plugin_frame() {
    return (KernargFrame)__builtin_amdgcn_kernarg_segment_ptr();
}

}  // namespace glsl
}  // namespace rm

#define u_resolution (::rm::glsl::vec2(::rm::glsl::plugin_frame()->res_x, ::rm::glsl::plugin_frame()->res_y))
#define u_pos                                                                                              \
    (::rm::glsl::vec3(::rm::glsl::plugin_frame()->pos_x, ::rm::glsl::plugin_frame()->pos_y,               \
                      ::rm::glsl::plugin_frame()->pos_z))
#define u_mouse (::rm::glsl::vec2(::rm::glsl::plugin_frame()->mouse_x, ::rm::glsl::plugin_frame()->mouse_y))
#define u_time (::rm::glsl::plugin_frame()->time)
