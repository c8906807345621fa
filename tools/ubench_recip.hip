// tools/ubench_recip.hip -- how many Newton steps RN(0.5 / t) needs after v_rcp_f64 (diagnostic tool).
//
// cosh's main path (aq_libm.h) needs the correctly rounded 0.5 / t for t = exp(|x|) in [1.41, 3.6e9].
// half_recip_n<N> is v_rcp_f64, N Newton steps on the reciprocal, then the quotient correction
// q + (0.5 - t*q)*y (N = 3: one second-order step y0 (1 + e + e^2) instead). This tool counts, over
// a few billion t, where each variant differs from the IEEE division the compiler emits for `0.5 / t` (div_scale / rcp / 2 Newton / div_fmas / div_fixup):
//   * pass 0: t = exp_glibc(x), x uniform in the main range [0.5*ln2, 22) (the values the kernel sees)
//   * pass 1: t with random exponent in [0, 31] and random 52-bit mantissa (every bit pattern in range)
// plus the largest relative error of y after N steps (in units of 2^-53). Per-thread counts are written
// with plain vector stores and reduced on the host.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../include -I../ppls_amd/csrc ubench_recip.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "aq_exp_table.h"
#include "aq_libm.h"

#pragma clang fp contract(off)

#define CHECK(x)                                                               \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

struct Counts {
    unsigned long long n, bad0, bad1, bad2, bad3;
    double relerr_y0, relerr_y1;
};

__global__ void k_recip(const aq::ExpPair* __restrict__ gtab, Counts* out, int iters, int pass, uint64_t seed) {
    __shared__ aq::ExpEntry tab[128];
    aq::stage_exp_table(tab, gtab);
    __syncthreads();
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    Counts c = {0, 0, 0, 0, 0, 0.0, 0.0};
    for (int it = 0; it < iters; ++it) {
        const uint64_t z = mix64(seed + (gid * (uint64_t)iters + it) * 0x9E3779B97F4A7C15ull);
        if (pass == 2) {
            // the batched path itself: cosh_main_k on two points (table reciprocal estimate when
            // AQ_TAB_RECIP) against RN(0.5 t + RN(0.5 / t)) with the compiler's IEEE division
            double xs[2], cm[2];
            for (int k = 0; k < 2; ++k) {
                const uint64_t zk = mix64(z + k);
                xs[k] = 0.34657359027997264 + (double)(zk >> 11) * 0x1p-53 * (22.0 - 0.34657359027997264);
            }
            aq::cosh_main_k<2, false>(xs, cm, tab, aq::pinned_exp_consts());
            for (int k = 0; k < 2; ++k) {
                const double tk = aq::exp_glibc(xs[k], tab);
                c.n += 1;
                c.bad3 += (cm[k] != __fma_rn(tk, 0.5, 0.5 / tk));
            }
            continue;
        }
        double t;
        if (pass == 0) {
            const double u = (double)(z >> 11) * 0x1p-53;
            const double x = 0.34657359027997264 + u * (22.0 - 0.34657359027997264);
            t = aq::exp_glibc(x, tab);
        } else {
            const uint64_t e = 1023 + ((z >> 52) & 31);
            t = __longlong_as_double((long long)((e << 52) | (z & 0xfffffffffffffull)));
            if (t < 1.4142135623730951) t += 1.5;
        }
        const double ref = 0.5 / t;
        const double v0 = aq::half_recip_n<0>(t);
        const double v1 = aq::half_recip_n<1>(t);
        const double v2 = aq::half_recip_n<2>(t);
        const double v3 = aq::half_recip_n<3>(t);
        c.n += 1;
        c.bad0 += (v0 != ref);
        c.bad1 += (v1 != ref);
        c.bad2 += (v2 != ref);
        c.bad3 += (v3 != ref);
        // relative error of the reciprocal estimate itself, in ulps of 2^-53: |1 - t*y|
        const double y0 = __builtin_amdgcn_rcp(t);
        const double y1 = __fma_rn(y0, __fma_rn(-t, y0, 1.0), y0);
        c.relerr_y0 = fmax(c.relerr_y0, fabs(__fma_rn(-t, y0, 1.0)) * 0x1p53);
        c.relerr_y1 = fmax(c.relerr_y1, fabs(__fma_rn(-t, y1, 1.0)) * 0x1p53);
    }
    out[gid] = c;
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 16384;
    const int iters = argc > 2 ? atoi(argv[2]) : 256;
    const int threads = 256;
    const size_t nt = (size_t)blocks * threads;
    aq::ExpPair* dtab;
    Counts* dout;
    CHECK(hipMalloc(&dtab, sizeof(aq::ExpPair) * 128));
    CHECK(hipMemcpy(dtab, aq_exp_tab_host, sizeof(aq::ExpPair) * 128, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&dout, nt * sizeof(Counts)));
    std::vector<Counts> h(nt);
    const int reps2 = argc > 3 ? atoi(argv[3]) : 1;   // launches of pass 2 (the batched cosh path)
    for (int pass = 0; pass < 2 + reps2; ++pass) {
        k_recip<<<blocks, threads>>>(dtab, dout, iters, pass < 2 ? pass : 2, 0x1234567ull + pass);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(h.data(), dout, nt * sizeof(Counts), hipMemcpyDeviceToHost));
        Counts s = {0, 0, 0, 0, 0, 0.0, 0.0};
        for (const Counts& c : h) {
            s.n += c.n;
            s.bad0 += c.bad0;
            s.bad1 += c.bad1;
            s.bad2 += c.bad2;
            s.bad3 += c.bad3;
            s.relerr_y0 = std::fmax(s.relerr_y0, c.relerr_y0);
            s.relerr_y1 = std::fmax(s.relerr_y1, c.relerr_y1);
        }
        if (pass >= 2) {
            printf("{\"pass\": 2, \"seed\": %d, \"cosh_main_k_samples\": %llu, \"cosh_main_k_mismatch\": %llu}\n", pass,
                   s.n, s.bad3);
            continue;
        }
        printf("{\"pass\": %d, \"samples\": %llu, \"mismatch_newton0\": %llu, \"mismatch_newton1\": %llu, "
               "\"mismatch_newton2\": %llu, \"mismatch_second_order\": %llu, \"max_relerr_rcp_ulp53\": %.6g, \"max_relerr_newton1_ulp53\": %.6g}\n",
               pass, s.n, s.bad0, s.bad1, s.bad2, s.bad3, s.relerr_y0, s.relerr_y1);
    }
    CHECK(hipFree(dtab));
    CHECK(hipFree(dout));
    return 0;
}
