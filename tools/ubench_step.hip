// tools/ubench_step.hip -- the issue-bound ceiling of the hot path's arithmetic (diagnostic tool).
//
// Every lane runs k_stream's per-pair work -- pair_step_halves<F_COSH4> (two midpoints, two glibc
// cosh^4 chains interleaved, the doubled trapezoid areas and both :191 tests) plus the masked area
// accumulation -- on pairs held in REGISTERS: no ring, no LDS pair traffic, no ballots or pushes.
// After each step the lane descends into one child pair (the right one where the left accepted), so
// the work stays data-dependent like the kernel's, and restarts from its seed pair every 24 levels.
// The FP64 instruction stream per pair is the kernel round's 76 (tools/isa_stats.py counts both), so
// this rate bounds what any scheduling of the same arithmetic can reach on the chip; the persistent
// kernel's bench rate divided by it is the share lost to the ring, the compaction and the schedule.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../include -I../ppls_amd/csrc ubench_step.hip
//   prints one JSON line per occupancy: tasks/s and the FP64 roofline fraction at 38 FLOP per task.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "aq_exp_table.h"
#include "aq_libm.h"
#include "aq_device.h"

#pragma clang fp contract(off)

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__);         \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_step(const aq::ExpPair* __restrict__ gtab, double* out, int iters,
                                                double eps2) {
    __shared__ aq::ExpEntry tab[128];
    aq::stage_exp_table(tab, gtab);
    __syncthreads();
    const aq::ExpConsts kk = aq::pinned_exp_consts();
    const unsigned gid = blockIdx.x * BLOCK + threadIdx.x;
    // seed pair: an interval of [0.4, 5] (the exp path of cosh), F at both ends and the midpoint,
    // scaled by 16 as the kernel carries them; halved endpoints
    const double a0 = 0.4 + 4.0 * (double)(gid % 4093) / 4093.0, b0 = a0 + 0.5;
    auto F16 = [&](double x) { return 16.0 * aq::integrand<aq::F_COSH4>(x, tab); };
    const double s_ha = 0.5 * a0, s_hb = 0.5 * b0, s_fa = F16(a0), s_fm = F16(0.5 * (a0 + b0)), s_fb = F16(b0);
    double ha = s_ha, hb = s_hb, fa = s_fa, fm = s_fm, fb = s_fb;
    double acc = 0.0;
    unsigned refined = 0;
    int lev = 0;
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
        aq::Step2 st[2];
        double m, hm;
        aq::pair_step_halves<aq::F_COSH4>(ha, hb, fa, fm, fb, eps2, tab, st, m, hm, kk, 2, 0ull);
        // the kernel's masked accumulation of accepted areas
        if (!st[0].refine) acc += st[0].area2;
        if (!st[1].refine) acc += st[1].area2;
        refined += (unsigned)st[0].refine + (unsigned)st[1].refine;
        // descend: the left child pair, or the right one where the left task accepted
        const bool right = !st[0].refine;
        const double nha = right ? hm : ha, nhb = right ? hb : hm;
        const double nfa = right ? fm : fa, nfm = right ? st[1].fmid : st[0].fmid, nfb = right ? fb : fm;
        if (++lev == 24) {
            lev = 0;
            ha = s_ha; hb = s_hb; fa = s_fa; fm = s_fm; fb = s_fb;
        } else {
            ha = nha; hb = nhb; fa = nfa; fm = nfm; fb = nfb;
        }
    }
    out[gid] = acc + (double)refined;
}

// The same walk with the parent's doubled areas carried in the pair (aq_device.h pair_step_carry):
// what the step costs if the ring held two more doubles per pair.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_step_carry(const aq::ExpPair* __restrict__ gtab, double* out, int iters,
                                                      double eps2) {
    __shared__ aq::ExpEntry tab[128];
    aq::stage_exp_table(tab, gtab);
    __syncthreads();
    const aq::ExpConsts kk = aq::pinned_exp_consts();
    const unsigned gid = blockIdx.x * BLOCK + threadIdx.x;
    const double a0 = 0.4 + 4.0 * (double)(gid % 4093) / 4093.0, b0 = a0 + 0.5;
    auto F16 = [&](double x) { return 16.0 * aq::integrand<aq::F_COSH4>(x, tab); };
    const double s_ha = 0.5 * a0, s_hb = 0.5 * b0, s_fa = F16(a0), s_fm = F16(0.5 * (a0 + b0)), s_fb = F16(b0);
    const double s_m = s_ha + s_hb;
    const double s_l2 = (s_fa + s_fm) * (s_m - a0), s_r2 = (s_fm + s_fb) * (b0 - s_m);
    double ha = s_ha, hb = s_hb, fa = s_fa, fm = s_fm, fb = s_fb, l2 = s_l2, r2 = s_r2;
    double acc = 0.0;
    unsigned refined = 0;
    int lev = 0;
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
        aq::Step2c st[2];
        double m, hm;
        aq::pair_step_carry<aq::F_COSH4>(ha, hb, fa, fm, fb, l2, r2, eps2, tab, st, m, hm, kk, 2, 0ull);
        if (!st[0].refine) acc += st[0].area2;
        if (!st[1].refine) acc += st[1].area2;
        refined += (unsigned)st[0].refine + (unsigned)st[1].refine;
        const bool right = !st[0].refine;
        const double nha = right ? hm : ha, nhb = right ? hb : hm;
        const double nfa = right ? fm : fa, nfm = right ? st[1].fmid : st[0].fmid, nfb = right ? fb : fm;
        const double nl2 = right ? st[1].l2 : st[0].l2, nr2 = right ? st[1].r2 : st[0].r2;
        if (++lev == 24) {
            lev = 0;
            ha = s_ha; hb = s_hb; fa = s_fa; fm = s_fm; fb = s_fb; l2 = s_l2; r2 = s_r2;
        } else {
            ha = nha; hb = nhb; fa = nfa; fm = nfm; fb = nfb; l2 = nl2; r2 = nr2;
        }
    }
    out[gid] = acc + (double)refined;
}

template <int BLOCK>
int run(aq::ExpPair* dtab, double* dout, int cus, int blocks_per_cu, int iters, bool carry = false) {
    const int grid = cus * blocks_per_cu;
    hipFuncAttributes attr;
    auto kern = carry ? &k_step_carry<BLOCK> : &k_step<BLOCK>;
    CHECK(hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(kern)));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const double eps2 = 1e-10 * 32.0;   // the bench's eps on doubled areas of 16 F
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), 0, 0, dtab, dout, 16, eps2);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), 0, 0, dtab, dout, iters, eps2);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    const double tasks = 2.0 * (double)grid * BLOCK * iters;
    const double rate = tasks / (best * 1e-3);
    printf("{\"carry\": %d, \"block\": %d, \"blocks_per_cu\": %d, \"waves_per_simd\": %d, \"vgprs\": %d, \"ms\": %.3f, "
           "\"tasks_per_s\": %.4e, \"frac_fp64_38flop\": %.4f}\n",
           (int)carry, BLOCK, blocks_per_cu, BLOCK * blocks_per_cu / 256, attr.numRegs, best, rate, 38.0 * rate / 78.6e12);
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    aq::ExpPair* dtab;
    double* dout;
    CHECK(hipMalloc(&dtab, sizeof(aq::ExpPair) * 128));
    CHECK(hipMemcpy(dtab, aq_exp_tab_host, sizeof(aq::ExpPair) * 128, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&dout, sizeof(double) * (size_t)cus * 1024 * 8));
    const int it = 4000;
    run<256>(dtab, dout, cus, 1, it);    // 1 wave per SIMD
    run<512>(dtab, dout, cus, 1, it);    // 2
    run<768>(dtab, dout, cus, 1, it);    // 3: the persistent kernel's occupancy
    run<1024>(dtab, dout, cus, 1, it);   // 4
    run<1024>(dtab, dout, cus, 2, it);   // 8
    run<512>(dtab, dout, cus, 1, it, true);    // carried parent areas (pair_step_carry)
    run<768>(dtab, dout, cus, 1, it, true);
    run<1024>(dtab, dout, cus, 1, it, true);
    return 0;
}
