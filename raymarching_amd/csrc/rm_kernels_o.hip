// rm_kernels_o.hip -- render kernels of scene O (output_shader.frag) and its
// glass test variant OG.  Built with -ffp-contract=off: scene O's subsurface
// term hashes the surface normal with fract(x * 443.897) (output_shader.frag:
// 54-81), which turns one-ulp differences of the normal into different sample
// directions; without fused multiply-adds the marching and normals round like
// the GLSL (and the oracle) and the image matches to ~1e-5 mean instead of
// ~4e-4 (DESIGN.md "Parity policy").
#include "rm_kernels_impl.h"

namespace rm {

hipError_t launch_scene_o(const FrameConst& F, void* out, bool rgba8, unsigned long long* evals, int kernel,
                           hipStream_t s) {
    return launch_scene<SCENE_O>(F, out, rgba8, evals, kernel, s);
}
hipError_t launch_scene_og(const FrameConst& F, void* out, bool rgba8, unsigned long long* evals, int kernel,
                           hipStream_t s) {
    return launch_scene<SCENE_OG>(F, out, rgba8, evals, kernel, s);
}

hipError_t launch_eval_o(const FrameConst& F, const float* pts, long long n, float* dist, float* mat,
                          hipStream_t s) {
    return launch_eval<SCENE_O>(F, pts, n, dist, mat, s);
}
hipError_t launch_eval_og(const FrameConst& F, const float* pts, long long n, float* dist, float* mat,
                          hipStream_t s) {
    return launch_eval<SCENE_OG>(F, pts, n, dist, mat, s);
}

hipError_t launch_wire_o(const FrameConst& F, WireTile* slots, unsigned long long* evals, hipStream_t s) {
    return launch_scene_wire<SCENE_O>(F, slots, evals, s);
}
hipError_t launch_wire_og(const FrameConst& F, WireTile* slots, unsigned long long* evals, hipStream_t s) {
    return launch_scene_wire<SCENE_OG>(F, slots, evals, s);
}

}  // namespace rm
