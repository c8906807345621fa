// tools/ubench_icache.hip -- cost of cold instruction bytes in a lone launch (diagnostic).
// Kernels with k_stream's launch shape (256 x 768 threads) run a straight-line block of KB kilobytes
// of 8-byte scalar instructions `reps` times. The first pass fetches every line into the
// instruction cache (invalidated at each dispatch); later passes hit. cold(KB) = T(KB, 1) -
// (T(KB, 2) - T(KB, 1)) over KB gives the price of one kilobyte of code executed once per launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define STR2(x) #x
#define STR(x) STR2(x)

template <int KB>
__global__ __launch_bounds__(768) void k_code(unsigned* out, int reps) {
    unsigned x = blockIdx.x;
    for (int r = 0; r < reps; ++r) {
        if constexpr (KB > 0)
            asm volatile(".rept " STR(128) " * %c1\n s_add_u32 %0, %0, 0x9e3779b9\n .endr" : "+s"(x) : "i"(KB));
    }
    if (threadIdx.x == 0) out[blockIdx.x] = x;
}

template <int KB>
int run(unsigned* d, FILE* js) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    float med[3] = {0, 0, 0};
    for (int reps = 1; reps <= 3; ++reps) {
        for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k_code<KB>, dim3(256), dim3(768), 0, 0, d, reps);
        CHECK(hipDeviceSynchronize());
        std::vector<float> one;
        for (int i = 0; i < 41; ++i) {
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k_code<KB>, dim3(256), dim3(768), 0, 0, d, reps);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float m1; CHECK(hipEventElapsedTime(&m1, a, b));
            one.push_back(m1 * 1e3f);
        }
        std::sort(one.begin(), one.end());
        med[reps - 1] = one[20];
    }
    const float hot = med[1] - med[0];
    printf("code %3d KB: alone %7.2f / %7.2f / %7.2f us (1 / 2 / 3 passes) -> hot pass %6.2f us, cold pass %6.2f us\n",
           KB, med[0], med[1], med[2], hot, med[0] - hot);
    fprintf(js, "{\"kb\": %d, \"us_1pass\": %.3f, \"us_2pass\": %.3f, \"us_3pass\": %.3f}\n", KB, med[0], med[1], med[2]);
    return 0;
}

int main(int argc, char** argv) {
    unsigned* d;
    CHECK(hipMalloc(&d, 4 * 4096));
    FILE* js = fopen(argc > 1 ? argv[1] : "/dev/null", "w");
    if (!js) return 1;
    run<0>(d, js);
    run<1>(d, js);
    run<2>(d, js);
    run<4>(d, js);
    run<8>(d, js);
    run<16>(d, js);
    run<32>(d, js);
    fclose(js);
    return 0;
}
