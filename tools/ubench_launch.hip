// tools/ubench_launch.hip -- launch + workgroup-start cost of the persistent kernel's shape (diagnostic).
// Empty kernels with the persistent kernel's geometry (256 x 768 threads, ~152 KiB LDS) and
// smaller shapes; back-to-back launches timed with HIP events, plus per-XCD first-start offsets.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int LDS_DOUBLES>
__global__ void k_empty(unsigned long long* out) {
    __shared__ double s[LDS_DOUBLES > 0 ? LDS_DOUBLES : 1];
    if (LDS_DOUBLES > 0) s[threadIdx.x % (LDS_DOUBLES > 0 ? LDS_DOUBLES : 1)] = threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
        out[blockIdx.x * 2] = __builtin_amdgcn_s_memrealtime();
        out[blockIdx.x * 2 + 1] = xcc + (LDS_DOUBLES > 0 ? (unsigned long long)s[1] * 0 : 0);
    }
}

template <int L>
int run(const char* name, int grid, int block, unsigned long long* d, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k_empty<L>, dim3(grid), dim3(block), 0, 0, d);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_empty<L>, dim3(grid), dim3(block), 0, 0, d);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms; CHECK(hipEventElapsedTime(&ms, a, b));
    // single launch, per-XCD first start
    hipLaunchKernelGGL(k_empty<L>, dim3(grid), dim3(block), 0, 0, d);
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(2 * grid);
    CHECK(hipMemcpy(h.data(), d, 16 * grid, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int i = 0; i < grid; ++i) { t0 = std::min(t0, h[2 * i]); t1 = std::max(t1, h[2 * i]); }
    // one launch alone between two events (how the lone-integral kernel time is taken): median of 50
    std::vector<float> one;
    for (int i = 0; i < 50; ++i) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_empty<L>, dim3(grid), dim3(block), 0, 0, d);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float m1; CHECK(hipEventElapsedTime(&m1, a, b));
        one.push_back(m1 * 1e3f);
    }
    std::sort(one.begin(), one.end());
    printf("%-28s grid=%5d block=%4d LDS=%6d B : %7.2f us/launch (back-to-back), %7.2f us alone (median), WG start spread %.2f us\n",
           name, grid, block, L * 8, ms * 1e3 / reps, one[25], (t1 - t0) / 100.0);
    return 0;
}

int main() {
    unsigned long long* d;
    CHECK(hipMalloc(&d, 16 * 4096));
    run<19400>("k_stream shape (768 thr)", 256, 768, d, 200);
    run<0>("no LDS, 768 thr", 256, 768, d, 200);
    run<17000>("persistent shape", 256, 512, d, 200);
    run<17000>("persistent shape, 256 thr", 256, 256, d, 200);
    run<8000>("64 KiB LDS, 512 thr", 256, 512, d, 200);
    run<0>("no LDS, 512 thr", 256, 512, d, 200);
    run<0>("no LDS, 256 thr", 256, 256, d, 200);
    run<0>("no LDS, 64 thr", 256, 64, d, 200);
    run<0>("no LDS, 1024 thr", 256, 1024, d, 200);
    run<0>("no LDS, 2048x256", 2048, 256, d, 200);
    return 0;
}
