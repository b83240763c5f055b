// rm_kernels_t.hip -- render kernels of scenes S0 and T (FMA contraction on).
#include "rm_kernels_impl.h"

namespace rm {

hipError_t launch_scene_s0(const FrameConst& F, void* out, bool rgba8, unsigned long long* evals, int kernel,
                           hipStream_t s) {
    return launch_scene<SCENE_S0>(F, out, rgba8, evals, kernel, s);
}
hipError_t launch_scene_t(const FrameConst& F, void* out, bool rgba8, unsigned long long* evals, int kernel,
                           hipStream_t s) {
    return launch_scene<SCENE_T>(F, out, rgba8, evals, kernel, s);
}

hipError_t launch_eval_s0(const FrameConst& F, const float* pts, long long n, float* dist, float* mat,
                          hipStream_t s) {
    return launch_eval<SCENE_S0>(F, pts, n, dist, mat, s);
}
hipError_t launch_eval_t(const FrameConst& F, const float* pts, long long n, float* dist, float* mat,
                          hipStream_t s) {
    return launch_eval<SCENE_T>(F, pts, n, dist, mat, s);
}

hipError_t launch_wire_s0(const FrameConst& F, WireTile* slots, unsigned long long* evals, hipStream_t s) {
    return launch_scene_wire<SCENE_S0>(F, slots, evals, s);
}
hipError_t launch_wire_t(const FrameConst& F, WireTile* slots, unsigned long long* evals, hipStream_t s) {
    return launch_scene_wire<SCENE_T>(F, slots, evals, s);
}

}  // namespace rm
