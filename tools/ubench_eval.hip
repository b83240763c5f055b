// ubench_eval.hip -- issue-bound ceiling of the scene-T distance evaluation:
// every lane evaluates the sponge SDF at points along its own ray with a fixed
// step (no divergence, no shading).  Reports evaluations/s and the implied
// cycles per evaluation-wave, to compare with the render kernel's ray-steps/s.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-hip-fp32-correctly-rounded-divide-sqrt \
//        -I raymarching_amd/csrc tools/ubench_eval.hip -o tools/ubench_eval
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "rm_device.h"

using namespace rm;

template <int SC, bool NEAR>
__global__ __launch_bounds__(256) void k(FrameConst F, int steps, float* out) {
    int gid = blockIdx.x * blockDim.x + threadIdx.x;
    // rays through the sponge (NEAR: start inside its bounding box so no fold
    // is skipped) or from far away (the early exit fires)
    float u = (gid & 1023) * (1.0f / 1024.0f) - 0.5f, v = (gid >> 10 & 1023) * (1.0f / 1024.0f) - 0.5f;
    V3 ro = NEAR ? v3(u * 1.8f, 3.0f + v * 1.8f, 1.2f) : v3(u * 40.0f, 3.0f + v * 40.0f, 30.0f);
    V3 rd = v3(0.01f, 0.02f, -1.0f);
    float acc = 0.0f, t = 0.0f;
    for (int i = 0; i < steps; i++) {
        Tally n;
        float d = scene_dist<SC, false>(F, ro + rd * t, n);
        acc += d;
        t += NEAR ? 0.0007f : 0.01f;
    }
    if (acc == 12345.0f) out[gid] = acc;
}

int main() {
    FrameConst F;
    std::memset(&F, 0, sizeof(F));
    F.ry_c = 1.0f; F.ry_s = 0.0f; F.rx_c = -1.0f; F.rx_s = 8.742278e-08f;
    float* d;
    (void)hipMalloc(&d, 1 << 24);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int blocks = 256 * 32, steps = 2048;
    auto run = [&](auto kern, const char* name) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, F, steps, d);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, F, steps, d);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        double evals = (double)blocks * 256 * steps;
        double wave_evals_per_simd = evals / 64 / 1024;
        std::printf("%-28s %8.3f ms  %.3e evals/s  %.0f cycles per wave-eval at 2.4 GHz\n", name, ms,
                    evals / ms * 1e3, ms * 1e-3 * 2.4e9 / wave_evals_per_simd);
    };
    run(k<SCENE_T, true>, "T fast, inside box");
    run(k<SCENE_T, false>, "T fast, far (early exit)");
    run(k<SCENE_O, true>, "O fast, inside box");
    return 0;
}
