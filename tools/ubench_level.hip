// tools/ubench_level.hip -- what bounds the frontier's widest level step (diagnostic tool).
//
// The level step (ppls_amd/csrc/aquad.hip k_level_step) reads one 32-B record {l, r, F(l), F(r)} per
// task, evaluates F at the midpoint (glibc-exact cosh^4, four chains per lane), appends the refining
// records' two children with ONE atomic per 256-thread block and 1024-record chunk, and writes them.
// This harness runs the same per-record work on a synthetic level of the widest level's size
// (1.65 M records on [0.4, 5], eps set so ~94 % refine, as cosh4 at eps=1e-12's level 23) in four
// forms, to separate the costs:
//   full      -- as the library: block atomic + child stores
//   noatomic  -- each block writes at a fixed offset (blockIdx * 2 * chunk): no atomic
//   nostore   -- the atomic, no child stores
//   neither   -- loads + F + the block's partial row only
// plus a pure copy kernel of the same bytes (the achievable HBM rate for this access pattern).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../include -I../ppls_amd/csrc ubench_level.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

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

struct Rec {
    double l, r, fl, fr;
};
constexpr int T = 256, R = 4, NW = T / 64;

template <bool ATOMIC, bool STORE>
__global__ __launch_bounds__(T) void k_lvl(const Rec* __restrict__ in, unsigned n_in, Rec* __restrict__ out,
                                           unsigned* __restrict__ n_out, double eps, double* parts,
                                           const aq::ExpPair* __restrict__ gtab) {
    __shared__ aq::ExpEntry tab[128];
    __shared__ unsigned s_wc[2][NW], s_base[2];
    aq::stage_exp_table(tab, gtab);
    __syncthreads();
    double hi = 0.0, lo = 0.0;
    const unsigned w = threadIdx.x >> 6;
    const unsigned chunk = T * R;
    unsigned parity = 0;
    for (unsigned base = blockIdx.x * chunk; base < n_in; base += gridDim.x * chunk, parity ^= 1u) {
        Rec rc[R];
        bool active[R];
        double x[R], f[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const unsigned i = base + (unsigned)k * T + threadIdx.x;
            active[k] = i < n_in;
            rc[k] = active[k] ? in[i] : Rec{1.0, 1.0, 0.0, 0.0};
            x[k] = (rc[k].l + rc[k].r) / 2;
        }
        aq::integrand_k<aq::F_COSH4, R>(x, f, tab);
        bool refine[R];
        unsigned long long m[R];
        unsigned c[R + 1];
        c[0] = 0;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const double lrarea = (rc[k].fl + rc[k].fr) * (rc[k].r - rc[k].l) / 2;
            const double larea = (rc[k].fl + f[k]) * (x[k] - rc[k].l) / 2;
            const double rarea = (f[k] + rc[k].fr) * (rc[k].r - x[k]) / 2;
            refine[k] = active[k] && fabs((larea + rarea) - lrarea) > eps;
            if (active[k] && !refine[k]) aq::dd_add(hi, lo, larea + rarea);
            m[k] = __ballot(refine[k]);
            c[k + 1] = c[k] + (unsigned)__popcll(m[k]);
        }
        if (aq::lane_id() == 0) s_wc[parity][w] = c[R];
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned tot = 0;
            for (int v = 0; v < NW; ++v) tot += s_wc[parity][v];
            s_base[parity] = ATOMIC ? (tot ? atomicAdd(n_out, 2u * tot) : 0u) : 2u * base;
        }
        __syncthreads();
        unsigned off = s_base[parity];
        for (unsigned v = 0; v < w; ++v) off += 2u * s_wc[parity][v];
        if (STORE) {
#pragma unroll
            for (int k = 0; k < R; ++k) {
                if (refine[k]) {
                    const unsigned pos = off + 2u * (c[k] + aq::mbcnt(m[k]));
                    out[pos] = Rec{rc[k].l, x[k], rc[k].fl, f[k]};
                    out[pos + 1] = Rec{x[k], rc[k].r, f[k], rc[k].fr};
                }
            }
        }
    }
    if (threadIdx.x == 0) parts[blockIdx.x] = hi + lo;
}

// the same bytes as a plain copy: read n records, write 2 * 0.94 n (coalesced)
__global__ __launch_bounds__(256) void k_copy(const Rec* __restrict__ in, unsigned n_in, Rec* __restrict__ out,
                                              unsigned n_out) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i < n_in) {
        const Rec v = in[i];
        if (2 * i + 1 < n_out) {
            out[2 * i] = v;
            out[2 * i + 1] = v;
        }
    }
}

// The copy at the part's streaming rate: 16 B per lane per access, a grid-stride loop
// over a grid sized for the 256 CUs (4 workgroups of 256 per CU), non-temporal stores -- the same 1:2
// read:write shape (every 16-B piece of the input is written twice, to two output halves)
typedef double d2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_copy4(const d2* __restrict__ in, size_t n16, d2* __restrict__ out) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
        const d2 v = __builtin_nontemporal_load(in + i);
        __builtin_nontemporal_store(v, out + i);
        __builtin_nontemporal_store(v, out + n16 + i);
    }
}

// The HBM baseline shapes: OUTS (1 or 2) 16-B stores per 16-B load, U loads in flight per thread
// before their stores, non-temporal (NT) or default cache policy; a grid-stride loop over n16 pieces.
template <int OUTS, int U, bool NT>
__global__ __launch_bounds__(256) void k_copy_u(const d2* __restrict__ in, size_t n16, d2* __restrict__ out) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t i0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n16; i0 += stride) {
        d2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = i0 + (size_t)u * 256;
            if (i < n16) v[u] = NT ? __builtin_nontemporal_load(in + i) : in[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = i0 + (size_t)u * 256;
            if (i < n16) {
#pragma unroll
                for (int o = 0; o < OUTS; ++o) {
                    if (NT) __builtin_nontemporal_store(v[u], out + (size_t)o * n16 + i);
                    else out[(size_t)o * n16 + i] = v[u];
                }
            }
        }
    }
}

// write-only and read-only passes of the same sizes
__global__ __launch_bounds__(256) void k_write(Rec* __restrict__ out, unsigned n_out) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i < n_out) out[i] = Rec{(double)i, 1.0, 2.0, 3.0};
}
__global__ __launch_bounds__(256) void k_read(const Rec* __restrict__ in, unsigned n_in, double* sink) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x;
    double v = 0.0;
    if (i < n_in) { const Rec r = in[i]; v = r.l + r.r + r.fl + r.fr; }
    if (v == 12345.678) sink[0] = v;   // never true for these records: keeps the loads
}

int main() {
    const unsigned n = 1652276;
    std::vector<Rec> h(n);
    const double w = 4.6 / n;
    auto F = [](double x) { const double c = std::cosh(x); return c * c * c * c; };
    for (unsigned i = 0; i < n; ++i) {
        const double l = 0.4 + i * w, r = l + w;
        h[i] = Rec{l, r, F(l), F(r)};
    }
    // eps: the 6th percentile of |(larea + rarea) - lrarea| over the records (~94 % refine)
    std::vector<double> d(n);
    for (unsigned i = 0; i < n; ++i) {
        const double m = (h[i].l + h[i].r) / 2, fm = F(m);
        d[i] = std::fabs(((h[i].fl + fm) * (m - h[i].l) / 2 + (fm + h[i].fr) * (h[i].r - m) / 2) -
                         (h[i].fl + h[i].fr) * (h[i].r - h[i].l) / 2);
    }
    std::vector<double> ds = d;
    std::nth_element(ds.begin(), ds.begin() + n / 16, ds.end());
    const double eps = ds[n / 16];
    Rec *din, *dout;
    unsigned* dn;
    double* dparts;
    aq::ExpPair* dtab;
    CHECK(hipMalloc(&din, sizeof(Rec) * n));
    CHECK(hipMalloc(&dout, sizeof(Rec) * 2 * (size_t)n + 64 * 1024));
    CHECK(hipMalloc(&dn, 4));
    CHECK(hipMalloc(&dparts, 8 * 8192));
    CHECK(hipMalloc(&dtab, sizeof(aq::ExpPair) * 128));
    CHECK(hipMemcpy(dtab, aq_exp_tab_host, sizeof(aq::ExpPair) * 128, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(din, h.data(), sizeof(Rec) * n, hipMemcpyHostToDevice));
    const unsigned grid = (n + T * R - 1) / (T * R);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    unsigned refined_children = 0;
    auto timeit = [&](const char* name, auto launch) -> int {
        std::vector<float> t;
        for (int rep = 0; rep < 12; ++rep) {
            CHECK(hipMemset(dn, 0, 4));
            CHECK(hipEventRecord(a));
            launch();
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        unsigned nout = 0;
        CHECK(hipMemcpy(&nout, dn, 4, hipMemcpyDeviceToHost));
        if (nout) refined_children = nout;
        const double bytes = 32.0 * n + 32.0 * refined_children;
        printf("{\"variant\": \"%s\", \"records\": %u, \"children\": %u, \"us_median\": %.2f, \"us_min\": %.2f, "
               "\"alg_GBps_median\": %.1f}\n", name, n, refined_children, t[6], t[0], bytes / (t[6] * 1e-6) / 1e9);
        return 0;
    };
    if (timeit("full", [&] { hipLaunchKernelGGL((k_lvl<true, true>), dim3(grid), dim3(T), 0, 0, din, n, dout, dn, eps, dparts, dtab); })) return 1;
    if (timeit("noatomic", [&] { hipLaunchKernelGGL((k_lvl<false, true>), dim3(grid), dim3(T), 0, 0, din, n, dout, dn, eps, dparts, dtab); })) return 1;
    if (timeit("nostore", [&] { hipLaunchKernelGGL((k_lvl<true, false>), dim3(grid), dim3(T), 0, 0, din, n, dout, dn, eps, dparts, dtab); })) return 1;
    if (timeit("neither", [&] { hipLaunchKernelGGL((k_lvl<false, false>), dim3(grid), dim3(T), 0, 0, din, n, dout, dn, eps, dparts, dtab); })) return 1;
    if (timeit("copy", [&] { hipLaunchKernelGGL(k_copy, dim3((n + 255) / 256), dim3(256), 0, 0, din, n, dout, refined_children); })) return 1;
    // the streaming copy at the level's size and at 10x (launch ramp < 10 %): bytes = read + 2 x read
    for (size_t mult : {(size_t)1, (size_t)10}) {
        const size_t n16 = (size_t)n * 2 * mult;   // 16-B pieces of the input (32 B per record)
        d2 *ci, *co;
        CHECK(hipMalloc(&ci, n16 * 16));
        CHECK(hipMalloc(&co, 2 * n16 * 16));
        CHECK(hipMemset(ci, 0, n16 * 16));
        std::vector<float> t;
        for (int rep = 0; rep < 12; ++rep) {
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k_copy4, dim3(1024), dim3(256), 0, 0, ci, n16, co);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms; CHECK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        const double bytes = 3.0 * 16.0 * (double)n16;
        printf("{\"variant\": \"copy16_nt_x%zu\", \"bytes\": %.0f, \"us_median\": %.2f, \"us_min\": %.2f, \"GBps_median\": %.1f}\n",
               mult, bytes, t[6], t[0], bytes / (t[6] * 1e-6) / 1e9);
        CHECK(hipFree(ci));
        CHECK(hipFree(co));
    }
    // the baseline shapes at 10x the level's input (1.06 GB read): 1:1 and 1:2, unroll 1 / 4, both policies
    {
        const size_t n16 = (size_t)n * 2 * 10;
        d2 *ci, *co;
        CHECK(hipMalloc(&ci, n16 * 16));
        CHECK(hipMalloc(&co, 2 * n16 * 16));
        CHECK(hipMemset(ci, 0, n16 * 16));
        CHECK(hipMemset(co, 0, 2 * n16 * 16));
        auto shape = [&](const char* name, int outs, auto launch) -> int {
            std::vector<float> t;
            for (int rep = 0; rep < 12; ++rep) {
                CHECK(hipEventRecord(a));
                launch();
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                float ms; CHECK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms * 1e3f);
            }
            std::sort(t.begin(), t.end());
            const double bytes = (1.0 + outs) * 16.0 * (double)n16;
            printf("{\"variant\": \"%s\", \"bytes\": %.0f, \"us_median\": %.2f, \"us_min\": %.2f, \"GBps_median\": %.1f}\n",
                   name, bytes, t[6], t[0], bytes / (t[6] * 1e-6) / 1e9);
            return 0;
        };
        const int g = 2048;
        if (shape("copy1to1_u1", 1, [&] { hipLaunchKernelGGL((k_copy_u<1, 1, false>), dim3(g), dim3(256), 0, 0, ci, n16, co); })) return 1;
        if (shape("copy1to1_u4", 1, [&] { hipLaunchKernelGGL((k_copy_u<1, 4, false>), dim3(g), dim3(256), 0, 0, ci, n16, co); })) return 1;
        if (shape("copy1to1_u4_nt", 1, [&] { hipLaunchKernelGGL((k_copy_u<1, 4, true>), dim3(g), dim3(256), 0, 0, ci, n16, co); })) return 1;
        if (shape("copy1to2_u1", 2, [&] { hipLaunchKernelGGL((k_copy_u<2, 1, false>), dim3(g), dim3(256), 0, 0, ci, n16, co); })) return 1;
        if (shape("copy1to2_u4", 2, [&] { hipLaunchKernelGGL((k_copy_u<2, 4, false>), dim3(g), dim3(256), 0, 0, ci, n16, co); })) return 1;
        if (shape("copy1to2_u4_nt", 2, [&] { hipLaunchKernelGGL((k_copy_u<2, 4, true>), dim3(g), dim3(256), 0, 0, ci, n16, co); })) return 1;
        CHECK(hipFree(ci));
        CHECK(hipFree(co));
    }
    // (alg_GBps below counts the copy's bytes; the pure passes move only their own)
    {
        std::vector<float> t;
        for (int rep = 0; rep < 12; ++rep) {
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k_write, dim3((refined_children + 255) / 256), dim3(256), 0, 0, dout, refined_children);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms; CHECK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        printf("{\"variant\": \"write_only\", \"bytes\": %.0f, \"us_median\": %.2f, \"GBps\": %.1f}\n",
               32.0 * refined_children, t[6], 32.0 * refined_children / (t[6] * 1e-6) / 1e9);
        t.clear();
        for (int rep = 0; rep < 12; ++rep) {
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k_read, dim3((n + 255) / 256), dim3(256), 0, 0, din, n, dparts);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms; CHECK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        printf("{\"variant\": \"read_only\", \"bytes\": %.0f, \"us_median\": %.2f, \"GBps\": %.1f}\n",
               32.0 * n, t[6], 32.0 * n / (t[6] * 1e-6) / 1e9);
    }
    return 0;
}
