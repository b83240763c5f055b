// rm_render_wave.h -- wave-compacted state-machine kernels (placeholder).
#pragma once
#include "rm_device.h"

namespace rm {

constexpr bool has_wave_kernel(int) { return false; }

template <int SC>
hipError_t launch_wave(const FrameConst&, float4*, unsigned long long*, hipStream_t) {
    return hipErrorNotSupported;
}

}  // namespace rm
