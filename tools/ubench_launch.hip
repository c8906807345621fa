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

// k_stream's resource shape without its work: 168 VGPRs (clobbered), ~100 SGPRs, a ~400-byte kernel
// argument block, 152 KiB of LDS -- whether the wave launch itself depends on them
struct BigArgs {
    unsigned long long* out;
    double pad[48];
};
__global__ __launch_bounds__(768) void k_heavy(BigArgs a) {
    __shared__ double s[19400];
    s[threadIdx.x] = a.pad[threadIdx.x % 48];
    asm volatile("" ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63","v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79","v80","v81","v82","v83","v84","v85","v86","v87","v88","v89","v90","v91","v92","v93","v94","v95","v96","v97","v98","v99","v100","v101","v102","v103","v104","v105","v106","v107","v108","v109","v110","v111","v112","v113","v114","v115","v116","v117","v118","v119","v120","v121","v122","v123","v124","v125","v126","v127","v128","v129","v130","v131","v132","v133","v134","v135","v136","v137","v138","v139","v140","v141","v142","v143","v144","v145","v146","v147","v148","v149","v150","v151","v152","v153","v154","v155","v156","v157","v158","v159","v160","v161","v162","v163","v164","v165","v166","v167");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
        a.out[blockIdx.x * 2] = __builtin_amdgcn_s_memrealtime();
        a.out[blockIdx.x * 2 + 1] = xcc + (unsigned long long)s[1] * 0;
    }
}

int run_heavy(unsigned long long* d) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    BigArgs args{};
    args.out = d;
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k_heavy, dim3(256), dim3(768), 0, 0, args);
    CHECK(hipDeviceSynchronize());
    std::vector<float> one;
    for (int i = 0; i < 50; ++i) {
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_heavy, dim3(256), dim3(768), 0, 0, args);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float m1; CHECK(hipEventElapsedTime(&m1, a, b));
        one.push_back(m1 * 1e3f);
    }
    std::sort(one.begin(), one.end());
    std::vector<unsigned long long> h(2 * 256);
    CHECK(hipMemcpy(h.data(), d, 16 * 256, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int i = 0; i < 256; ++i) { t0 = std::min(t0, h[2 * i]); t1 = std::max(t1, h[2 * i]); }
    printf("%-28s grid=%5d block=%4d LDS=%6d B : %7.2f us alone (median), WG start spread %.2f us (168 VGPRs, 400-B args)\n",
           "k_stream resources", 256, 768, 19400 * 8, one[25], (t1 - t0) / 100.0);
    return 0;
}

int main() {
    unsigned long long* d;
    CHECK(hipMalloc(&d, 16 * 4096));
    run_heavy(d);
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
