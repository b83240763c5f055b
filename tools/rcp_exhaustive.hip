// rcp_exhaustive.hip -- is one Newton step from v_rcp_f32,
//     r = rcp(x); r' = fma(fma(-x, r, 1), r, r),
// the correctly rounded 1/x for every float x in [lo, hi)?  Compared on the
// GPU against the IEEE division of a translation unit built with
// -fhip-fp32-correctly-rounded-divide-sqrt.  Used to replace post.frag's
// rcpDirMin = 1.0 / (...) in rm_fxaa (rm_fxaa.hip) whose argument lies in
// [1/128, 2.125]: prints the mismatch count (and the first mismatches).
// Build: hipcc --offload-arch=gfx950 -O3 -fhip-fp32-correctly-rounded-divide-sqrt \
//        tools/rcp_exhaustive.hip -o tools/rcp_exhaustive
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

__global__ void check(uint32_t lo, uint32_t n, unsigned long long* bad, uint32_t* first) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = __uint_as_float(lo + i);
    const float ref = 1.0f / x;
    const float r = __builtin_amdgcn_rcpf(x);
    const float rn = fmaf(fmaf(-x, r, 1.0f), r, r);
    if (__float_as_uint(rn) != __float_as_uint(ref)) {
        const unsigned long long k = atomicAdd(bad, 1ull);
        if (k < 8) first[k] = lo + i;
    }
}

int main(int argc, char** argv) {
    const float flo = argc > 1 ? std::atof(argv[1]) : 1.0f / 256.0f;
    const float fhi = argc > 2 ? std::atof(argv[2]) : 4.0f;
    uint32_t lo, hi;
    std::memcpy(&lo, &flo, 4);
    std::memcpy(&hi, &fhi, 4);
    const uint32_t n = hi - lo;
    unsigned long long* d_bad;
    uint32_t* d_first;
    if (hipMalloc(&d_bad, 8) != hipSuccess || hipMalloc(&d_first, 32) != hipSuccess) return 2;
    hipMemset(d_bad, 0, 8);
    hipMemset(d_first, 0, 32);
    hipLaunchKernelGGL(check, dim3((n + 255) / 256), dim3(256), 0, 0, lo, n, d_bad, d_first);
    unsigned long long bad = 0;
    uint32_t first[8];
    if (hipMemcpy(&bad, d_bad, 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    hipMemcpy(first, d_first, 32, hipMemcpyDeviceToHost);
    std::printf("{\"lo\": %.9g, \"hi\": %.9g, \"floats\": %u, \"mismatches\": %llu", flo, fhi, n, bad);
    std::printf(", \"first\": [");
    for (unsigned long long k = 0; k < bad && k < 8; k++) {
        float f;
        std::memcpy(&f, &first[k], 4);
        std::printf("%s%.9g", k ? ", " : "", f);
    }
    std::printf("]}\n");
    hipFree(d_bad);
    hipFree(d_first);
    return 0;
}
