// ubench_valu.hip -- VALU issue-rate microbenchmarks on gfx950.
// Measures wave64 instruction throughput of the op classes the ray-march
// evaluation is made of (plain vs packed f32 FMA, floor, med3, sqrt ...),
// with 8 independent chains per lane so latency is hidden.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o /tmp/ubench_valu
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHK(x)                                                                               \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k(float* out, float a, float b) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = threadIdx.x * 1e-3f + j;
    // VGPR operands that the compiler cannot fold into SGPRs
    const float va = a + threadIdx.x * 1e-9f, vb = b + threadIdx.x * 1e-9f;
    const f2 vp = f2{va, va}, vq = f2{vb, vb};
    f2 y[4];
#pragma unroll
    for (int j = 0; j < 4; j++) y[j] = f2{x[2 * j], x[2 * j + 1]};
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if constexpr (OP == 0) x[j] = fmaf(x[j], a, b);                          // v_fma_f32
            if constexpr (OP == 2) x[j] = floorf(x[j] * a);                          // mul + floor
            if constexpr (OP == 3) x[j] = __builtin_amdgcn_fmed3f(x[j], a, b);       // v_med3
            if constexpr (OP == 4) x[j] = __builtin_amdgcn_sqrtf(x[j]);             // v_sqrt
            if constexpr (OP == 5) x[j] = x[j] * a;                                 // v_mul
            if constexpr (OP == 6) x[j] = __builtin_amdgcn_fractf(x[j]);            // v_fract
        }
        if constexpr (OP == 1) {
#pragma unroll
            for (int j = 0; j < 4; j++) y[j] = __builtin_elementwise_fma(y[j], f2{a, a}, f2{b, b});  // v_pk_fma_f32
        }
        if constexpr (OP == 7) {
#pragma unroll
            for (int j = 0; j < 4; j++) y[j] = y[j] + f2{a, b};  // v_pk_add_f32
        }
        if constexpr (OP == 8) {
#pragma unroll
            for (int j = 0; j < 4; j++) y[j] = y[j] * f2{a, b};  // v_pk_mul_f32
        }
        if constexpr (OP == 10) {  // v_fma_f32, all VGPR operands
#pragma unroll
            for (int j = 0; j < 8; j++) x[j] = fmaf(x[j], va, vb);
        }
        if constexpr (OP == 11) {  // v_mul_f32, VGPR operand
#pragma unroll
            for (int j = 0; j < 8; j++) x[j] = x[j] * va;
        }
        if constexpr (OP == 12) {  // v_floor_f32
#pragma unroll
            for (int j = 0; j < 8; j++) x[j] = floorf(x[j]);
        }
        if constexpr (OP == 13) {  // v_add_f32 with an inline constant
#pragma unroll
            for (int j = 0; j < 8; j++) x[j] = x[j] + 1.0f;
        }
        if constexpr (OP == 14) {  // v_pk_fma_f32, VGPR operands
#pragma unroll
            for (int j = 0; j < 4; j++) y[j] = __builtin_elementwise_fma(y[j], vp, vq);
        }
        if constexpr (OP == 15) {  // v_fma_f32 with an inline constant and a VGPR
#pragma unroll
            for (int j = 0; j < 8; j++) x[j] = fmaf(x[j], va, 0.5f);
        }
        if constexpr (OP == 16) {  // v_max3_f32, VGPR operands
#pragma unroll
            for (int j = 0; j < 8; j++) x[j] = fmaxf(x[j], fmaxf(va, vb));
        }
        if constexpr (OP == 9) {  // 2 v_pk_fma_f32 + 4 v_fma_f32 interleaved
#pragma unroll
            for (int j = 0; j < 2; j++) y[j] = __builtin_elementwise_fma(y[j], f2{a, a}, f2{b, b});
#pragma unroll
            for (int j = 0; j < 4; j++) x[j] = fmaf(x[j], a, b);
        }
    }
    float s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s += x[j];
#pragma unroll
    for (int j = 0; j < 4; j++) s += y[j].x + y[j].y;
    if (s == 12345.0f) out[threadIdx.x] = s;
}

template <int OP>
int run(const char* name, int ops_per_iter) {
    float* d;
    CHK(hipMalloc(&d, 1024 * sizeof(float)));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    int blocks = 256 * 8 * 4;  // 8 waves/SIMD worth of 256-thread blocks, x4
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 1e-3f);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 1e-3f);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    double insts = 5.0 * blocks * 4.0 /*waves*/ * ITERS * ops_per_iter;  // wave instructions
    double per_simd_per_ns = insts / 1024.0 / (ms * 1e6);
    std::printf("%-26s %8.3f ms  %7.1f G wave-inst/s  %.3f inst/ns/SIMD  (%.2f cyc/inst at 2.4 GHz)\n", name, ms,
                insts / ms / 1e6, per_simd_per_ns, 2.4 / per_simd_per_ns);
    CHK(hipFree(d));
    return 0;
}

int main() {
    run<0>("v_fma_f32 x8", 8);
    run<1>("v_pk_fma_f32 x4", 4);
    run<7>("v_pk_add_f32 x4", 4);
    run<8>("v_pk_mul_f32 x4", 4);
    run<9>("2 v_pk_fma + 4 v_fma", 6);
    run<0>("v_fma_f32 x8 (again)", 8);
    run<1>("v_pk_fma_f32 x4 (again)", 4);
    run<5>("v_mul_f32 x8", 8);
    run<10>("v_fma_f32 x8 (vgpr ops)", 8);
    run<11>("v_mul_f32 x8 (vgpr op)", 8);
    run<12>("v_floor_f32 x8", 8);
    run<13>("v_add_f32 x8 (inline 1.0)", 8);
    run<14>("v_pk_fma_f32 x4 (vgpr)", 4);
    run<15>("v_fma_f32 x8 (vgpr, inl)", 8);
    run<16>("v_max3_f32 x8 (vgpr)", 8);
    run<2>("v_mul+v_floor x8", 16);
    run<3>("v_med3_f32 x8", 8);
    run<6>("v_fract_f32 x8", 8);
    run<4>("v_sqrt_f32 x8", 8);
    return 0;
}
