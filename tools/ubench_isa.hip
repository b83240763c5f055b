// ubench_isa.hip -- per-instruction VALU issue cost on gfx950 (wave64).
//
// Each kernel runs one instruction form, written as inline asm so that the
// compiler can neither fold nor drop it, over 8 independent chains per lane
// (latency hidden), 8 waves per SIMD.  Printed: SIMD cycles per wave
// instruction at 2.4 GHz, and the same from the waves' own shader-clock ticks
// (s_memtime; clock-independent) with the clock they imply.  The forms are the ones the ray-march evaluation is
// made of: VOP2/VOP3 f32 arithmetic with VGPR, inline-constant, SGPR and
// literal operands, the packed f32 forms, med3/max3/maximum3, floor/rndne/
// fract, compares and selects, conversions, transcendentals.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_isa.hip -o tools/ubench_isa
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#define CHK(x)                                                                               \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

constexpr int ITERS = 2048;

// one instruction on chain register X; V/W: VGPR operands, S: an SGPR operand,
// P/Q: 64-bit VGPR pairs (packed forms use chain pairs)
#define FORMS(F)                                                                   \
    F(0, "v_fma_f32 v,v,v,v", "v_fma_f32 %0, %0, %1, %2")                          \
    F(1, "v_fma_f32 v,v,v,0.5", "v_fma_f32 %0, %0, %1, 0.5")                       \
    F(2, "v_fma_f32 v,v,s,v", "v_fma_f32 %0, %0, %3, %2")                          \
    F(3, "v_fma_f32 v,|v|,v,v", "v_fma_f32 %0, |%0|, %1, %2")                      \
    F(4, "v_mul_f32 v,v,v", "v_mul_f32 %0, %0, %1")                                \
    F(5, "v_mul_f32 v,s,v", "v_mul_f32 %0, %3, %0")                                \
    F(6, "v_mul_f32_e32 v,lit,v", "v_mul_f32_e32 %0, 0x3fc00000, %0")             \
    F(7, "v_fmac_f32_e32 v,lit,v", "v_fmac_f32_e32 %0, 0x3fc00000, %1")           \
    F(8, "v_fmaak_f32 v,v,v,lit", "v_fmaak_f32 %0, %0, %1, 0x3fc00000")            \
    F(9, "v_add_f32 v,v,v", "v_add_f32 %0, %0, %1")                                \
    F(10, "v_sub_f32 v,v,v", "v_sub_f32 %0, %1, %0")                               \
    F(11, "v_max_f32 v,v,v", "v_max_f32 %0, %0, %1")                               \
    F(12, "v_max3_f32 v,v,v,v", "v_max3_f32 %0, %0, %1, %2")                       \
    F(13, "v_med3_f32 v,v,v,v", "v_med3_f32 %0, %0, %1, %2")                       \
    F(14, "v_maximum3_f32 v,v,v,v", "v_maximum3_f32 %0, %0, %1, %2")               \
    F(15, "v_floor_f32 v,v", "v_floor_f32 %0, %0")                                 \
    F(16, "v_rndne_f32 v,v", "v_rndne_f32 %0, %0")                                 \
    F(17, "v_fract_f32 v,v", "v_fract_f32 %0, %0")                                 \
    F(18, "v_cndmask_b32 v,v,v,vcc", "v_cndmask_b32 %0, %0, %1, vcc")              \
    F(19, "v_cmp_lt_f32 vcc,v,v", "v_cmp_lt_f32 vcc, %0, %1")                      \
    F(20, "v_cmp_lt_f32 s[],v,v", "v_cmp_lt_f32 s[40:41], %0, %1")                 \
    F(21, "v_mov_b32 v,v", "v_mov_b32 %0, %1")                                     \
    F(22, "v_add_u32 v,v,v", "v_add_u32 %0, %0, %1")                               \
    F(23, "v_mul_hi_u32 v,v,v", "v_mul_hi_u32 %0, %0, %1")                         \
    F(24, "v_cvt_f32_u32 v,v", "v_cvt_f32_u32 %0, %0")                             \
    F(25, "v_exp_f32 v,v", "v_exp_f32 %0, %0")                                     \
    F(26, "v_rcp_f32 v,v", "v_rcp_f32 %0, %0")                                     \
    F(27, "v_min3_f32 v,v,s,v", "v_min3_f32 %0, %0, %3, %1")                       \
    F(28, "v_fma_f32 v,v,s,s", "v_fma_f32 %0, %0, %3, %3")                         \
    F(29, "v_add_f32 v,v,s", "v_add_f32 %0, %0, %3")                               \
    F(30, "v_fma_f32 v,-v,v,v (neg)", "v_fma_f32 %0, -%0, %1, %2")                 \
    F(31, "v_xor_b32 v,v,v", "v_xor_b32 %0, %0, %1")

#define PACKED(F)                                                                  \
    F(40, "v_pk_fma_f32 p,p,p,p", "v_pk_fma_f32 %0, %0, %1, %2")                   \
    F(41, "v_pk_add_f32 p,p,p", "v_pk_add_f32 %0, %0, %1")                         \
    F(42, "v_pk_mul_f32 p,p,p", "v_pk_mul_f32 %0, %0, %1")                         \
    F(43, "v_pk_fma_f32 p,p,p,p op_sel_hi", "v_pk_fma_f32 %0, %0, %1, %2 op_sel_hi:[1,0,1]")

template <int OP>
struct Form;
#define DEF(N, NAME, ASM)                                                                \
    template <>                                                                          \
    struct Form<N> {                                                                     \
        static constexpr const char* name = NAME;                                        \
        __device__ __forceinline__ static void op(float& x, float v, float w, float s) { \
            asm volatile(ASM : "+v"(x) : "v"(v), "v"(w), "s"(s) : "vcc", "s40", "s41");                     \
        }                                                                                \
    };
FORMS(DEF)
#undef DEF
typedef float f2 __attribute__((ext_vector_type(2)));
#define DEFP(N, NAME, ASM)                                                          \
    template <>                                                                     \
    struct Form<N> {                                                                \
        static constexpr const char* name = NAME;                                   \
        __device__ __forceinline__ static void op(f2& x, f2 v, f2 w, float s) {     \
            (void)s;                                                                \
            asm volatile(ASM : "+v"(x) : "v"(v), "v"(w));                     \
        }                                                                           \
    };
PACKED(DEFP)
#undef DEFP

template <int OP, int OP2>
__global__ __launch_bounds__(256) void k(float* out, float a, float b, unsigned long long* cyc) {
    const unsigned long long t0 = clock64();  // s_memtime: shader clock ticks
    const float v = a + threadIdx.x * 1e-9f, w = b + threadIdx.x * 1e-9f;
    if constexpr (OP >= 40) {
        f2 x[8];
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = f2{threadIdx.x * 1e-3f + j, 0.5f * j};
        const f2 pv{v, w}, pw{w, v};
        for (int i = 0; i < ITERS; i++) {
#pragma unroll
            for (int j = 0; j < 8; j++) Form<OP>::op(x[j], pv, pw, a);
        }
        float s = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) s += x[j].x + x[j].y;
        if (s == 12345.0f) out[threadIdx.x] = s;
        if ((threadIdx.x & 63) == 0) atomicAdd(cyc, clock64() - t0);
    } else {
        float x[8];
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = threadIdx.x * 1e-3f + j;
        for (int i = 0; i < ITERS; i++) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                Form<OP>::op(x[j], v, w, a);
                if constexpr (OP2 >= 0) Form<OP2>::op(x[j], v, w, a);
            }
        }
        float s = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) s += x[j];
        if (s == 12345.0f) out[threadIdx.x] = s;
        if ((threadIdx.x & 63) == 0) atomicAdd(cyc, clock64() - t0);
    }
}

template <int OP, int OP2 = -1>
int run() {
    float* d;
    CHK(hipMalloc(&d, 1024 * sizeof(float)));
    unsigned long long* cyc_dev;
    CHK(hipMalloc(&cyc_dev, sizeof(unsigned long long)));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const int blocks = 256 * 8 * 4;  // 32 waves per SIMD over the launch, 8 resident
    hipLaunchKernelGGL((k<OP, OP2>), dim3(blocks), dim3(256), 0, 0, d, 0.999f, 1e-3f, cyc_dev);
    CHK(hipDeviceSynchronize());
    CHK(hipMemset(cyc_dev, 0, sizeof(unsigned long long)));
    CHK(hipEventRecord(e0));
    for (int r = 0; r < 3; r++) hipLaunchKernelGGL((k<OP, OP2>), dim3(blocks), dim3(256), 0, 0, d, 0.999f, 1e-3f, cyc_dev);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const int per = OP2 >= 0 ? 16 : 8;
    const double insts = 3.0 * blocks * 4.0 * ITERS * per;  // wave instructions
    const double cyc = 2.4 / (insts / 1024.0 / (ms * 1e6));
    // clock-independent: a wave's shader-clock ticks (s_memtime) over its instructions, with 8 waves sharing
    // each SIMD; the launch runs 4 rounds of 8 resident waves per SIMD, so the clock is ~4 wave durations per
    // launch time
    unsigned long long ticks = 0;
    CHK(hipMemcpy(&ticks, cyc_dev, sizeof ticks, hipMemcpyDeviceToHost));
    const double nwaves = 3.0 * blocks * 4.0, wave_ticks = (double)ticks / nwaves;
    const double tick_cyc = wave_ticks / ((double)ITERS * per) / 8.0;
    const double clk_ghz = 4.0 * wave_ticks / (ms / 3.0 * 1e6);
    char name[128];
    if constexpr (OP2 >= 0)
        std::snprintf(name, sizeof name, "%s + %s", Form<OP>::name, Form<OP2>::name);
    else
        std::snprintf(name, sizeof name, "%s", Form<OP>::name);
    std::printf("{\"form\": \"%s\", \"cyc_per_wave_inst\": %.3f, \"tick_cyc_per_wave_inst\": %.3f, "
                "\"clock_ghz_est\": %.3f, \"ms\": %.3f}\n", name, cyc, tick_cyc, clk_ghz, ms);
    CHK(hipFree(d));
    CHK(hipFree(cyc_dev));
    return 0;
}

int main() {
#define RUN(N, NAME, ASM) run<N>();
    FORMS(RUN)
    PACKED(RUN)
#undef RUN
    // mixes: an SGPR-operand form beside a VGPR-only one; floor/rndne beside fma
    run<2, 0>();
    run<2, 1>();
    run<5, 4>();
    run<16, 1>();
    run<15, 1>();
    run<13, 1>();
    run<18, 1>();
    run<26, 1>();
    run<6, 1>();
    run<0, 0>();
    run<1, 1>();
    return 0;
}
