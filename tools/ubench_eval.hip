// tools/ubench_eval.hip -- throughput floor of the device integrand (diagnostic tool, not product).
//
// Each thread evaluates F at ITER points held in registers (no memory traffic in the loop), with
// ILP independent chains per thread; the sum is stored so nothing is dead-code eliminated.
// Reports F-evals/s for the whole chip at several occupancies: the issue-bound ceiling of the
// hot path's FP64 work, against which the persistent kernel's per-round cost is judged.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../include -I../ppls_amd/csrc ubench_eval.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "aq_exp_table.h"
#include "aq_libm.h"

#pragma clang fp contract(off)

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__);         \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

template <int ILP, int MODE>
__global__ void k_ubench(const aq::ExpPair* __restrict__ gtab, double* out, int iters, double x0, double dx) {
    __shared__ aq::ExpEntry tab[128];
    aq::stage_exp_table(tab, gtab);
    __syncthreads();
    const unsigned gid = blockIdx.x * blockDim.x + threadIdx.x;
    double x[ILP], acc[ILP];
#pragma unroll
    for (int j = 0; j < ILP; ++j) {
        x[j] = x0 + dx * (double)((gid * ILP + j) % 4096);
        acc[j] = 0.0;
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < ILP; ++j) {
            double v;
            if (MODE == 0) v = aq::integrand<aq::F_COSH4>(x[j], tab);
            else if (MODE == 1) v = aq::exp_glibc(x[j], tab);
            else v = 0.5 / x[j];
            acc[j] += v;
            x[j] += 1e-7;
        }
    }
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < ILP; ++j) s += acc[j];
    out[gid] = s;
}

template <int ILP, int MODE>
int run(const char* name, aq::ExpPair* dtab, double* dout, int cus, int block, int blocks_per_cu, int iters) {
    const int grid = cus * blocks_per_cu;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_ubench<ILP, MODE>), dim3(grid), dim3(block), 0, 0, dtab, dout, 4, 0.4, 1e-3);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((k_ubench<ILP, MODE>), dim3(grid), dim3(block), 0, 0, dtab, dout, iters, 0.4, 1e-3);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double evals = (double)grid * block * ILP * iters;
    printf("%-10s ILP=%d block=%4d blocks/CU=%d waves/SIMD=%d : %8.3f ms  %.3e evals/s  %.2f cycles/eval/CU@2.4GHz\n",
           name, ILP, block, blocks_per_cu, block * blocks_per_cu / 256, ms, evals / (ms * 1e-3),
           (ms * 1e-3) * 2.4e9 * cus / evals);
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
    CHECK(hipMalloc(&dout, sizeof(double) * (size_t)cus * 2048 * 4));
    const int it = 2000;
    for (int bpc : {1, 2, 4, 8}) run<1, 0>("F=cosh^4", dtab, dout, cus, 256, bpc, it);
    for (int bpc : {1, 2, 4}) run<2, 0>("F=cosh^4", dtab, dout, cus, 256, bpc, it);
    for (int bpc : {1, 2}) run<4, 0>("F=cosh^4", dtab, dout, cus, 256, bpc, it);
    run<1, 0>("F=cosh^4", dtab, dout, cus, 512, 1, it);
    run<2, 0>("F=cosh^4", dtab, dout, cus, 512, 1, it);
    run<1, 1>("exp", dtab, dout, cus, 256, 8, it);
    run<1, 2>("0.5/x", dtab, dout, cus, 256, 8, it);
    run<1, 2>("0.5/x", dtab, dout, cus, 256, 2, it);
    return 0;
}
