// tools/ubench_issue.hip -- issue cost of single VALU instructions on one MI355X SIMD (diagnostic tool).
//
// Each kernel runs a loop of 16 independent copies of one instruction (inline asm, so the compiler
// cannot fold or reorder them), with W waves per SIMD (grid = 256 CUs x 4 SIMDs x W). The cost per
// wave-instruction on one SIMD is  kernel time * clock / (instructions issued per SIMD).
// Used to price v_rcp_f64 against v_fma_f64 for the cosh tail (aq_libm.h cosh_main_k).
//   hipcc --offload-arch=gfx950 -O3 -o ubench_issue ubench_issue.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                               \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); \
            return 1;                                                          \
        }                                                                      \
    } while (0)

#define R16(OP)                                                                                 \
    asm volatile(OP " %0, %0\n" OP " %1, %1\n" OP " %2, %2\n" OP " %3, %3\n"                     \
                 OP " %4, %4\n" OP " %5, %5\n" OP " %6, %6\n" OP " %7, %7\n"                     \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),        \
                   "+v"(a[6]), "+v"(a[7]));                                                       \
    asm volatile(OP " %0, %0\n" OP " %1, %1\n" OP " %2, %2\n" OP " %3, %3\n"                     \
                 OP " %4, %4\n" OP " %5, %5\n" OP " %6, %6\n" OP " %7, %7\n"                     \
                 : "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]),    \
                   "+v"(a[14]), "+v"(a[15]));

#define R16_3(OP)                                                                               \
    asm volatile(OP " %0, %0, %0, %0\n" OP " %1, %1, %1, %1\n" OP " %2, %2, %2, %2\n"            \
                 OP " %3, %3, %3, %3\n" OP " %4, %4, %4, %4\n" OP " %5, %5, %5, %5\n"            \
                 OP " %6, %6, %6, %6\n" OP " %7, %7, %7, %7\n"                                   \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),        \
                   "+v"(a[6]), "+v"(a[7]));                                                       \
    asm volatile(OP " %0, %0, %0, %0\n" OP " %1, %1, %1, %1\n" OP " %2, %2, %2, %2\n"            \
                 OP " %3, %3, %3, %3\n" OP " %4, %4, %4, %4\n" OP " %5, %5, %5, %5\n"            \
                 OP " %6, %6, %6, %6\n" OP " %7, %7, %7, %7\n"                                   \
                 : "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]),    \
                   "+v"(a[14]), "+v"(a[15]));

#define R16_2(OP)                                                                               \
    asm volatile(OP " %0, %0, %0\n" OP " %1, %1, %1\n" OP " %2, %2, %2\n" OP " %3, %3, %3\n"     \
                 OP " %4, %4, %4\n" OP " %5, %5, %5\n" OP " %6, %6, %6\n" OP " %7, %7, %7\n"     \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),        \
                   "+v"(a[6]), "+v"(a[7]));                                                       \
    asm volatile(OP " %0, %0, %0\n" OP " %1, %1, %1\n" OP " %2, %2, %2\n" OP " %3, %3, %3\n"     \
                 OP " %4, %4, %4\n" OP " %5, %5, %5\n" OP " %6, %6, %6\n" OP " %7, %7, %7\n"     \
                 : "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]),    \
                   "+v"(a[14]), "+v"(a[15]));

// 64-bit shift-add with a constant shift (the round's dt + 1)
#define R16_SH(OP)                                                                              \
    asm volatile(OP " %0, %0, 0, %0\n" OP " %1, %1, 0, %1\n" OP " %2, %2, 0, %2\n" OP " %3, %3, 0, %3\n" \
                 OP " %4, %4, 0, %4\n" OP " %5, %5, 0, %5\n" OP " %6, %6, 0, %6\n" OP " %7, %7, 0, %7\n" \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),        \
                   "+v"(a[6]), "+v"(a[7]));                                                       \
    asm volatile(OP " %0, %0, 0, %0\n" OP " %1, %1, 0, %1\n" OP " %2, %2, 0, %2\n" OP " %3, %3, 0, %3\n" \
                 OP " %4, %4, 0, %4\n" OP " %5, %5, 0, %5\n" OP " %6, %6, 0, %6\n" OP " %7, %7, 0, %7\n" \
                 : "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]),    \
                   "+v"(a[14]), "+v"(a[15]));

// VOPC: compares writing vcc (independent sources, one destination)
#define R16_CMP(OP)                                                                             \
    asm volatile(OP " %0, %1\n" OP " %1, %2\n" OP " %2, %3\n" OP " %3, %4\n"                     \
                 OP " %4, %5\n" OP " %5, %6\n" OP " %6, %7\n" OP " %7, %0\n"                     \
                 OP " %0, %1\n" OP " %1, %2\n" OP " %2, %3\n" OP " %3, %4\n"                     \
                 OP " %4, %5\n" OP " %5, %6\n" OP " %6, %7\n" OP " %7, %0\n"                     \
                 :: "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]),    \
                   "v"(a[7]) : "vcc");

template <int OPID, typename T>
__global__ void __launch_bounds__(256) k_issue(T* out, int iters) {
    T a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = (T)(1.0 + 1e-3 * (threadIdx.x + i));
    for (int it = 0; it < iters; ++it) {
        if constexpr (OPID == 0) { R16_3("v_fma_f64") }
        else if constexpr (OPID == 1) { R16_2("v_mul_f64") }
        else if constexpr (OPID == 2) { R16_2("v_add_f64") }
        else if constexpr (OPID == 3) { R16("v_rcp_f64") }
        else if constexpr (OPID == 4) { R16_2("v_add_u32") }
        else if constexpr (OPID == 5) { R16("v_rcp_f32") }
        else if constexpr (OPID == 6) { R16_2("v_max_f64") }
        else if constexpr (OPID == 7) { R16("v_frexp_mant_f64") }
        else if constexpr (OPID == 9) { R16_3("v_fma_f32") }
        else if constexpr (OPID == 10) { R16("v_mov_b64") }
        else if constexpr (OPID == 11) { R16_3("v_and_or_b32") }
        else if constexpr (OPID == 12) { R16_2("v_mbcnt_lo_u32_b32") }
        else if constexpr (OPID == 13) { R16_3("v_lshl_add_u32") }
        else if constexpr (OPID == 14) { R16_SH("v_lshl_add_u64") }
        else if constexpr (OPID == 15) { R16_CMP("v_cmp_gt_f64_e32 vcc,") }
        else if constexpr (OPID == 16) { R16_2("v_cndmask_b32") }
    }
    T s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OPID, typename T>
int run(const char* name, T* d, int waves_per_simd) {
    const int iters = 4096;
    const int threads = 256;                          // 4 waves per workgroup = one per SIMD
    const int blocks = 256 * waves_per_simd;          // 256 CUs
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    k_issue<OPID, T><<<blocks, threads>>>(d, 16);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    k_issue<OPID, T><<<blocks, threads>>>(d, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    // instructions per SIMD: waves_per_simd * iters * 16
    const double per_simd = (double)waves_per_simd * iters * 16;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const double clk = p.clockRate * 1e3;             // Hz
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cycles_per_wave_instr\": %.3f}\n", name,
           waves_per_simd, ms, ms * 1e-3 * clk / per_simd);
    return 0;
}

int main() {
    double* d;
    CHECK(hipMalloc(&d, sizeof(double) * 256 * 256 * 8));
    float* f = (float*)d;
    for (int w : {1, 2, 3, 4}) {
        run<0>("v_fma_f64", d, w);
        run<1>("v_mul_f64", d, w);
        run<2>("v_add_f64", d, w);
        run<3>("v_rcp_f64", d, w);
        run<7>("v_frexp_mant_f64", d, w);
        run<4, float>("v_add_u32", f, w);
        run<5, float>("v_rcp_f32", f, w);
        run<9, float>("v_fma_f32", f, w);
        run<6, double>("v_max_f64", d, w);
        run<10, double>("v_mov_b64", d, w);
        run<11, float>("v_and_or_b32", f, w);
        run<12, float>("v_mbcnt_lo_u32_b32", f, w);
        run<13, float>("v_lshl_add_u32", f, w);
        run<14, double>("v_lshl_add_u64", d, w);
        run<15, double>("v_cmp_gt_f64", d, w);
        run<16, float>("v_cndmask_b32", f, w);
    }
    CHECK(hipFree(d));
    return 0;
}
