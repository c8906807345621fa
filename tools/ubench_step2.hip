// tools/ubench_step2.hip -- ubench_step.hip with NP sibling pairs per lane (2 NP interleaved cosh
// chains): the issue-bound ceiling of a round that evaluates more independent tasks per lane at
// lower occupancy (diagnostic tool).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../include -I../ppls_amd/csrc ubench_step2.hip
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

// NP pairs per lane: the arithmetic of aq_device.h pair_step_halves, K = 2 NP chains at once
template <int NP>
__device__ __forceinline__ void step_n(const double (&ha)[NP], const double (&hb)[NP], const double (&fa)[NP],
                                       const double (&fm)[NP], const double (&fb)[NP], double eps2,
                                       const aq::ExpEntry* tab, const aq::ExpConsts& kk, double (&fmid)[2 * NP],
                                       double (&area2)[2 * NP], bool (&refine)[2 * NP], double (&hm)[NP]) {
    double m[NP], mid[2 * NP], lr2e[2 * NP], wl[2 * NP], wr[2 * NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        m[p] = ha[p] + hb[p];
        hm[p] = 0.5 * m[p];
        mid[2 * p] = ha[p] + hm[p];
        mid[2 * p + 1] = hm[p] + hb[p];
        lr2e[2 * p] = (fa[p] + fm[p]) * __fma_rn(ha[p], -2.0, m[p]);
        lr2e[2 * p + 1] = (fm[p] + fb[p]) * __fma_rn(hb[p], 2.0, -m[p]);
        wl[2 * p] = __fma_rn(ha[p], -2.0, mid[2 * p]);
        wl[2 * p + 1] = mid[2 * p + 1] - m[p];
        wr[2 * p] = m[p] - mid[2 * p];
        wr[2 * p + 1] = __fma_rn(hb[p], 2.0, -mid[2 * p + 1]);
    }
#pragma unroll
    for (int k = 0; k < 2 * NP; ++k) asm volatile("" : "+v"(lr2e[k]), "+v"(wl[k]), "+v"(wr[k]));
    aq::integrand_k<aq::F_COSH4, 2 * NP, true>(mid, fmid, tab, kk, 2, 0ull);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const double fl[2] = {fa[p], fm[p]}, fr[2] = {fm[p], fb[p]};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int k = 2 * p + c;
            const double l2 = (fl[c] + fmid[k]) * wl[k], r2 = (fmid[k] + fr[c]) * wr[k];
            area2[k] = l2 + r2;
            refine[k] = fabs(area2[k] - lr2e[k]) > eps2;
        }
    }
}

template <int BLOCK, int NP>
__global__ __launch_bounds__(BLOCK) void k_step(const aq::ExpPair* __restrict__ gtab, double* out, int iters,
                                                double eps2) {
    __shared__ aq::ExpEntry tab[128];
    aq::stage_exp_table(tab, gtab);
    __syncthreads();
    const aq::ExpConsts kk = aq::pinned_exp_consts();
    const unsigned gid = blockIdx.x * BLOCK + threadIdx.x;
    auto F16 = [&](double x) { return 16.0 * aq::integrand<aq::F_COSH4>(x, tab); };
    double s_ha[NP], s_hb[NP], s_fa[NP], s_fm[NP], s_fb[NP], ha[NP], hb[NP], fa[NP], fm[NP], fb[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const double a0 = 0.4 + 4.0 * (double)((gid * NP + p) % 4093) / 4093.0, b0 = a0 + 0.5;
        s_ha[p] = ha[p] = 0.5 * a0; s_hb[p] = hb[p] = 0.5 * b0;
        s_fa[p] = fa[p] = F16(a0); s_fm[p] = fm[p] = F16(0.5 * (a0 + b0)); s_fb[p] = fb[p] = F16(b0);
    }
    double acc = 0.0;
    unsigned refined = 0;
    int lev = 0;
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
        double fmid[2 * NP], area2[2 * NP], hm[NP];
        bool refine[2 * NP];
        step_n<NP>(ha, hb, fa, fm, fb, eps2, tab, kk, fmid, area2, refine, hm);
        const bool reset = ++lev == 24;
        if (reset) lev = 0;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            if (!refine[2 * p]) acc += area2[2 * p];
            if (!refine[2 * p + 1]) acc += area2[2 * p + 1];
            refined += (unsigned)refine[2 * p] + (unsigned)refine[2 * p + 1];
            const bool right = !refine[2 * p];
            const double nha = right ? hm[p] : ha[p], nhb = right ? hb[p] : hm[p];
            const double nfa = right ? fm[p] : fa[p], nfm = right ? fmid[2 * p + 1] : fmid[2 * p], nfb = right ? fb[p] : fm[p];
            ha[p] = reset ? s_ha[p] : nha; hb[p] = reset ? s_hb[p] : nhb;
            fa[p] = reset ? s_fa[p] : nfa; fm[p] = reset ? s_fm[p] : nfm; fb[p] = reset ? s_fb[p] : nfb;
        }
    }
    out[gid] = acc + (double)refined;
}

template <int BLOCK, int NP>
int run(aq::ExpPair* dtab, double* dout, int cus, int blocks_per_cu, int iters) {
    const int grid = cus * blocks_per_cu;
    hipFuncAttributes attr;
    CHECK(hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&k_step<BLOCK, NP>)));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const double eps2 = 1e-10 * 32.0;
    hipLaunchKernelGGL((k_step<BLOCK, NP>), dim3(grid), dim3(BLOCK), 0, 0, dtab, dout, 16, eps2);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL((k_step<BLOCK, NP>), dim3(grid), dim3(BLOCK), 0, 0, dtab, dout, iters, eps2);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    const double tasks = 2.0 * NP * (double)grid * BLOCK * iters;
    const double rate = tasks / (best * 1e-3);
    printf("{\"pairs_per_lane\": %d, \"block\": %d, \"blocks_per_cu\": %d, \"waves_per_simd\": %d, \"vgprs\": %d, \"ms\": %.3f, "
           "\"tasks_per_s\": %.4e, \"frac_fp64_38flop\": %.4f}\n",
           NP, BLOCK, blocks_per_cu, BLOCK * blocks_per_cu / 256, attr.numRegs, best, rate, 38.0 * rate / 78.6e12);
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
    run<256, 1>(dtab, dout, cus, 1, it);
    run<512, 1>(dtab, dout, cus, 1, it);
    run<768, 1>(dtab, dout, cus, 1, it);
    run<256, 2>(dtab, dout, cus, 1, it / 2);
    run<512, 2>(dtab, dout, cus, 1, it / 2);
    run<768, 2>(dtab, dout, cus, 1, it / 2);
    run<256, 3>(dtab, dout, cus, 1, it / 3);
    run<512, 3>(dtab, dout, cus, 1, it / 3);
    return 0;
}
