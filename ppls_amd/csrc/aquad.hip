// aquad.hip -- MI355X (gfx950) adaptive trapezoid quadrature: kernels + the C ABI of include/aquad.h.
//
// Reference: /root/reference/aquadPartA.c. Its hot path is the worker task body (:183-202) fed by
// the farmer's LIFO bag of intervals over MPI (:125-173). Here the bag and the workers become one
// persistent launch ("on-device farmer"):
//   * every workgroup (one per CU) owns an LDS-resident interval stack (SoA, 33 B/record);
//   * a round pops up to PT records, evaluates F(mid) for each in FP64 (glibc-exact cosh, aq_libm.h),
//     applies the reference's refine test (:191), and pushes the children back with a wave
//     ballot/mbcnt prefix scan -- no messages, no HBM traffic;
//   * accepted areas are summed per lane in registers and reduced wave -> LDS -> one f64 atomic per
//     workgroup at exit (the farmer's `result += buff[0]`, :149);
//   * load balance (what the bag of tasks is for) goes through an HBM ticket queue of interval
//     chunks: an idle workgroup takes a ticket, busy workgroups donate the bottom (shallowest,
//     largest) part of their stack to waiting tickets, or spill when LDS is full;
//   * termination = the token count (busy workgroups + records in published chunks) reaches zero
//     (the farmer's `!is_empty(bag) || idle_count != workers`, :166).
// Seeding: instead of the single root, each workgroup starts with its own cyclically dealt depth-D
// subtrees (positions j = k*V + vwg, snake order over bands), found by a path walk whose F(mid)
// evaluations are all independent (one parallel round); tasks above depth D are counted once, by
// the owner of their leftmost descendant. Every decision is the reference's own arithmetic on the
// same operands, so the interval tree -- hence tasks and accepted counts -- is bit-identical.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared (ppls_amd/build.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "aquad.h"
#include "aq_exp_table.h"
#include "aq_libm.h"
#include "aq_device.h"
#include "aq_stream.h"
#include "aq_dfs.h"

#pragma clang fp contract(off)

namespace aq {

// ------------------------------------------------------------------------------------------------
// Device result block (one per async slot), zeroed before each call.
// ------------------------------------------------------------------------------------------------
struct DevResults {
    double area;
    unsigned long long tasks;
    unsigned long long leaves;
    unsigned long long spilled;
    unsigned int levels;
    unsigned int error;        // AQ_E* as positive bit flags (see err_bit)
    unsigned int q_tail;       // chunk slots claimed by producers
    unsigned int q_head;       // tickets taken by idle workgroups
    int q_tokens;              // busy workgroups + records in published, unconsumed chunks
    unsigned int pad[3];
    unsigned long long tasks_per_level[AQ_MAX_LEVELS];
    unsigned long long leaves_per_level[AQ_MAX_LEVELS];
    unsigned long long cu_tasks[AQ_CU_SLOTS];
};


// ------------------------------------------------------------------------------------------------
// Parity helper: evaluate F or cosh on an array.
// ------------------------------------------------------------------------------------------------
template <int FID, bool COSH_ONLY>
__global__ __launch_bounds__(256) void k_eval(const double* __restrict__ x, double* __restrict__ out, size_t n,
                                              const ExpEntry* __restrict__ gtab) {
    __shared__ ExpEntry tab[128];
    stage_exp_table(tab, gtab);
    __syncthreads();
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        out[i] = COSH_ONLY ? cosh_glibc(x[i], tab) : integrand<FID>(x[i], tab);
    }
}

// ------------------------------------------------------------------------------------------------
// Level-synchronous breadth-first path: one launch per tree level (debug / cross-check schedule).
// ------------------------------------------------------------------------------------------------
struct Rec {
    double l, r, fl, fr;
};

template <int FID>
__global__ __launch_bounds__(64) void k_root(double a, double b, Rec* out, const ExpEntry* __restrict__ gtab) {
    __shared__ ExpEntry tab[128];
    stage_exp_table(tab, gtab);
    __syncthreads();
    if (threadIdx.x == 0) {
        Rec r;
        r.l = a;
        r.r = b;
        r.fl = integrand<FID>(a, tab);
        r.fr = integrand<FID>(b, tab);
        out[0] = r;
    }
}

template <int FID>
__global__ __launch_bounds__(256) void k_level(const Rec* __restrict__ in, unsigned n_in, Rec* __restrict__ out,
                                               unsigned* __restrict__ n_out, unsigned cap_out, double eps, int depth,
                                               int max_depth, DevResults* __restrict__ res,
                                               const ExpEntry* __restrict__ gtab) {
    __shared__ ExpEntry tab[128];
    __shared__ double s_area[4];
    __shared__ unsigned s_cnt[2][4];
    stage_exp_table(tab, gtab);
    __syncthreads();
    double area = 0.0;
    unsigned tasks = 0, leaves = 0;
    const unsigned stride = gridDim.x * blockDim.x;
    for (unsigned base = blockIdx.x * blockDim.x; base < n_in; base += stride) {
        const unsigned i = base + threadIdx.x;
        const bool active = i < n_in;
        const Rec rc = active ? in[i] : Rec{0.0, 0.0, 0.0, 0.0};
        bool refine = false;
        double mid = 0.0, fmid = 0.0;
        if (active) {
            const Step s = task_step<FID>(rc.l, rc.r, rc.fl, rc.fr, eps, tab);
            mid = s.mid;
            fmid = s.fmid;
            ++tasks;
            if (!s.refine) {
                area += s.larea + s.rarea;  // :199
                ++leaves;
            } else if (depth + 1 >= max_depth) {
                atomicOr(&res->error, ERRB_DEPTH);
            } else {
                refine = true;
            }
        }
        const unsigned long long mask = __ballot(refine);
        const unsigned cnt = __popcll(mask);
        unsigned wbase = 0;
        if (cnt) {
            if (lane_id() == 0) wbase = atomicAdd(n_out, 2u * cnt);
            wbase = __shfl(wbase, 0, 64);
        }
        if (refine) {
            const unsigned pos = wbase + 2u * mbcnt(mask);
            if (pos + 1 < cap_out) {
                out[pos] = Rec{rc.l, mid, rc.fl, fmid};      // [l, mid]  (:192-194)
                out[pos + 1] = Rec{mid, rc.r, fmid, rc.fr};  // [mid, r]  (:195-197)
            } else {
                atomicOr(&res->error, ERRB_OVERFLOW);
            }
        }
    }
    // workgroup reduction -> one atomic per counter
    const unsigned w = threadIdx.x >> 6;
    double wa = wave_sum(area);
    unsigned wt = wave_sum_u(tasks), wl = wave_sum_u(leaves);
    if (lane_id() == 0) {
        s_area[w] = wa;
        s_cnt[0][w] = wt;
        s_cnt[1][w] = wl;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double ba = 0.0;
        unsigned bt = 0, bl = 0;
        for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
            ba += s_area[k];
            bt += s_cnt[0][k];
            bl += s_cnt[1][k];
        }
        if (bt) {
            atomicAdd(&res->area, ba);
            atomicAdd(&res->tasks, (unsigned long long)bt);
            atomicAdd(&res->leaves, (unsigned long long)bl);
            atomicAdd(&res->tasks_per_level[depth], (unsigned long long)bt);
            atomicAdd(&res->leaves_per_level[depth], (unsigned long long)bl);
            atomicAdd(&res->cu_tasks[cu_slot()], (unsigned long long)bt);
            atomicMax(&res->levels, (unsigned)(depth + 1));
        }
    }
}

// Frontier engine step (caller-owned buffers, ppls_amd/frontier.py): one task step per record, the
// refining records' children appended to `out` (wave-aggregated atomic), each block's accepted area
// (double-double), task / accepted counts, error bits and deepest level written to its own partial
// row; k_level_fold (one workgroup) folds the rows, in block order, into the caller's accumulator.
struct LevelPart {
    double hi, lo, tasks, leaves, err, levels, pad0, pad1;
};

template <int FID>
__global__ __launch_bounds__(256) void k_level_step(const Rec* __restrict__ in, unsigned n_in, Rec* __restrict__ out,
                                                    unsigned* __restrict__ n_out, unsigned cap_out, double eps,
                                                    int depth, int max_depth, LevelPart* __restrict__ parts,
                                                    const ExpEntry* __restrict__ gtab) {
    __shared__ ExpEntry tab[128];
    __shared__ double s_h[4], s_l[4];
    __shared__ unsigned s_t[4], s_a[4], s_e[4];
    stage_exp_table(tab, gtab);
    __syncthreads();
    double hi = 0.0, lo = 0.0;
    unsigned tasks = 0, leaves = 0, err = 0;
    const unsigned stride = gridDim.x * blockDim.x;
    for (unsigned base = blockIdx.x * blockDim.x; base < n_in; base += stride) {
        const unsigned i = base + threadIdx.x;
        const bool active = i < n_in;
        const Rec rc = active ? in[i] : Rec{1.0, 1.0, 0.0, 0.0};
        const double x[1] = {(rc.l + rc.r) / 2};                         // :187
        double f[1];
        integrand_k<FID, 1>(x, f, tab);                                  // :188
        const double mid = x[0], fmid = f[0];
        const double lrarea = (rc.fl + rc.fr) * (rc.r - rc.l) / 2;       // :185
        const double larea = (rc.fl + fmid) * (mid - rc.l) / 2;          // :189
        const double rarea = (fmid + rc.fr) * (rc.r - mid) / 2;          // :190
        const bool ref = active && fabs((larea + rarea) - lrarea) > eps; // :191
        bool refine = false;
        if (active) {
            ++tasks;
            if (!ref) {
                dd_add(hi, lo, larea + rarea);                           // :199 -> :149
                ++leaves;
            } else if (depth + 1 >= max_depth) {
                err |= ERRB_DEPTH;
            } else {
                refine = true;
            }
        }
        const unsigned long long mask = __ballot(refine);
        const unsigned cnt = (unsigned)__popcll(mask);
        unsigned wbase = 0;
        if (cnt) {
            if (lane_id() == 0) wbase = atomicAdd(n_out, 2u * cnt);
            wbase = __shfl(wbase, 0, 64);
        }
        if (refine) {
            const unsigned pos = wbase + 2u * mbcnt(mask);
            if (pos + 1 < cap_out) {
                out[pos] = Rec{rc.l, mid, rc.fl, fmid};                  // [l, mid]  (:192-194)
                out[pos + 1] = Rec{mid, rc.r, fmid, rc.fr};              // [mid, r]  (:195-197)
            } else {
                err |= ERRB_OVERFLOW;
            }
        }
    }
    wave_sum_dd(hi, lo);
    const unsigned wt = wave_sum_u(tasks), wl = wave_sum_u(leaves), we = wave_or_u(err);
    const unsigned w = threadIdx.x >> 6;
    if (lane_id() == 0) { s_h[w] = hi; s_l[w] = lo; s_t[w] = wt; s_a[w] = wl; s_e[w] = we; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double H = 0.0, L = 0.0;
        unsigned T = 0, A = 0, E = 0;
        for (int k = 0; k < 4; ++k) { dd_add_dd(H, L, s_h[k], s_l[k]); T += s_t[k]; A += s_a[k]; E |= s_e[k]; }
        LevelPart p;
        p.hi = H; p.lo = L; p.tasks = (double)T; p.leaves = (double)A; p.err = (double)E;
        p.levels = T ? (double)(depth + 1) : 0.0;
        p.pad0 = p.pad1 = 0.0;
        parts[blockIdx.x] = p;
    }
}

__global__ __launch_bounds__(64) void k_level_fold(const LevelPart* __restrict__ parts, int nparts,
                                                   double* __restrict__ acc) {
    if (threadIdx.x != 0) return;
    double H = acc[0], L = acc[1], T = acc[2], A = acc[3], lev = acc[5];
    unsigned E = (unsigned)acc[4];
    for (int i = 0; i < nparts; ++i) {
        const LevelPart& p = parts[i];
        dd_add_dd(H, L, p.hi, p.lo);
        T += p.tasks;
        A += p.leaves;
        E |= (unsigned)p.err;
        lev = fmax(lev, p.levels);
    }
    acc[0] = H; acc[1] = L; acc[2] = T; acc[3] = A; acc[4] = (double)E; acc[5] = lev;
}

template <int FID>
__global__ __launch_bounds__(64) void k_frontier_root(double a, double b, Rec* out, const ExpEntry* __restrict__ gtab) {
    __shared__ ExpEntry tab[128];
    stage_exp_table(tab, gtab);
    __syncthreads();
    if (threadIdx.x == 0) out[0] = Rec{a, b, integrand<FID>(a, tab), integrand<FID>(b, tab)};
}

// The area partials of one slot (block of 256 threads): every thread returns the double-double sum
// of its share, in a fixed order -- thread k takes the listed waves 32k..32k+31 in ascending order
// (a 4096-bit LDS bitmap dedupes the list), or, past TCAP listed waves, the dense stride.
__device__ __forceinline__ void slot_area_share(const Ctl& c, const double2* __restrict__ wa, int wstride,
                                                unsigned* s_bits, double& hi, double& lo) {
    const unsigned n = c.sums.ntouch;
    hi = lo = 0.0;
    if (n <= TCAP && wstride <= 4096) {
        for (int i = threadIdx.x; i < wstride / 32; i += blockDim.x) s_bits[i] = 0u;
        __syncthreads();
        if (threadIdx.x < n) {
            const unsigned w = c.touch[threadIdx.x];
            atomicOr(&s_bits[w >> 5], 1u << (w & 31u));
        }
        __syncthreads();
        for (int k = threadIdx.x; k < wstride / 32; k += blockDim.x) {
            unsigned m = s_bits[k];
            while (m) {
                const int b = __builtin_ctz(m);
                m &= m - 1u;
                const double2 v = wa[32 * k + b];
                dd_add_dd(hi, lo, v.x, v.y);
            }
        }
    } else {
        for (int i = threadIdx.x; i < wstride; i += blockDim.x) dd_add_dd(hi, lo, wa[i].x, wa[i].y);
    }
}

// Gather n slots' totals into a caller device buffer as f64 [area, tasks, accepted, error] rows,
// ready for one collective (counts are exact in f64 below 2^53). One workgroup per slot: counts
// from the slot's sums, the area from the listed wave partials in a fixed order.
__global__ __launch_bounds__(256) void k_gather(const Ctl* __restrict__ ctls, const double2* __restrict__ warea,
                                                int wstride, int first, int n, int nslots, double* __restrict__ out) {
    __shared__ double s_h[4], s_lo[4];
    __shared__ unsigned s_bits[128];
    const int slot = (first + (int)blockIdx.x) % nslots;
    const Ctl& c = ctls[slot];
    double hi, lo;
    slot_area_share(c, warea + (size_t)slot * wstride, wstride, s_bits, hi, lo);
    wave_sum_dd(hi, lo);
    const unsigned wv = threadIdx.x >> 6;
    if (lane_id() == 0) { s_h[wv] = hi; s_lo[wv] = lo; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double H = 0.0, Lo = 0.0;
        for (int k = 0; k < 4; ++k) dd_add_dd(H, Lo, s_h[k], s_lo[k]);
        double* o = out + 4 * blockIdx.x;
        o[0] = H + Lo;
        o[1] = (double)c.sums.tasks;
        o[2] = (double)c.sums.leaves;
        o[3] = (double)c.sums.error;
    }
}

// Return slots [first, first + n) to the all-zero state a launch needs: the listed (or, past TCAP,
// all) area partials, the sums and the queue words; the histograms when they were written.
__global__ __launch_bounds__(256) void k_reset(Ctl* __restrict__ ctls, double2* __restrict__ warea, int wstride,
                                               int first, int zero_hist) {
    const int slot = first + (int)blockIdx.x;
    Ctl& c = ctls[slot];
    double2* wa = warea + (size_t)slot * wstride;
    const unsigned n = c.sums.ntouch;
    if (n <= TCAP) {
        if (threadIdx.x < n) wa[c.touch[threadIdx.x]] = make_double2(0.0, 0.0);
    } else {
        for (int i = threadIdx.x; i < wstride; i += blockDim.x) wa[i] = make_double2(0.0, 0.0);
    }
    if (zero_hist)
        for (int i = threadIdx.x; i < 2 * AQ_MAX_LEVELS; i += blockDim.x) c.hist[i] = 0ull;
    __syncthreads();   // every thread has read ntouch / touch before they are cleared
    if (threadIdx.x == 0) {
        c.sums = SlotSums{};
        c.q_tail.v = 0u; c.q_head.v = 0u; c.q_tokens.v = 0u; c.jobs.v = 0u;
    }
}

}  // namespace aq

// ================================================================================================
// Host side: the C ABI.
// ================================================================================================
using namespace aq;

namespace {

#ifndef AQ_PCU_SW
#define AQ_PCU_SW 4   // measured: one integral at eps=1e-12 94 -> 80 us, eps=1e-10 unchanged
#endif
constexpr int NSLOTS = 65536;
constexpr int NSTAGE = 4;          // pinned bounds staging buffers
constexpr unsigned QCAP = 16384;
constexpr int DFS_MIN_K = 1 << 30;   // auto engine: k_stream (measured faster); k_dfs on request
static_assert(MAXK <= NSLOTS, "a launch's integrals need distinct slots");

#define AQ_HIP(call)                                                                  \
    do {                                                                              \
        hipError_t e_ = (call);                                                       \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "aquad: HIP error %s at %s:%d\n", hipGetErrorString(e_),   \
                    __FILE__, __LINE__);                                              \
            return AQ_EHIP;                                                           \
        }                                                                             \
    } while (0)

int err_from_bits(unsigned bits) {
    if (bits & ERRB_TIMEOUT) return AQ_ETIMEOUT;
    if (bits & ERRB_OVERFLOW) return AQ_EOVERFLOW;
    if (bits & ERRB_DEPTH) return AQ_EDEPTH;
    return AQ_OK;
}

int floor_log2(unsigned long long v) {
    int d = 0;
    while ((2ull << d) <= v) ++d;
    return d;
}

bool bounds_ok(double a, double b) { return std::isfinite(a) && std::isfinite(b) && b >= a; }

int validate(const aq_problem* p) {
    if (!p) return AQ_EINVAL;
    if (p->integrand != AQ_F_COSH4 && p->integrand != AQ_F_SIN_RECIP) return AQ_EINVAL;
    if (!bounds_ok(p->a, p->b)) return AQ_EINVAL;
    if (!(p->eps >= 0.0)) return AQ_EINVAL;
    if (p->max_depth < 0 || p->max_depth > AQ_MAX_LEVELS - 1) return AQ_EINVAL;
    return AQ_OK;
}

// Host view of one finished integral, whichever path produced it.
struct HostOut {
    double area = 0.0;
    unsigned long long tasks = 0, leaves = 0, spilled = 0;
    unsigned levels = 0, error = 0;
    unsigned long long hist[2 * AQ_MAX_LEVELS] = {};
    unsigned long long cu[AQ_CU_SLOTS] = {};
};

}  // namespace

struct aq_ctx {
    int device = 0;
    int num_cus = 0;
    int grid = 0;                      // persistent workgroups per launch (one per CU)
    bool histograms = true;
    hipStream_t stream = nullptr;
    ExpEntry* d_tab = nullptr;
    Ctl* d_ctl = nullptr;              // NSLOTS control blocks (queue + per-integral histograms)
    WgPart* d_parts = nullptr;         // NSLOTS x grid per-workgroup partials
    double2* d_warea = nullptr;        // NSLOTS x grid*NW per-wave double-double areas
    double2* h_warea = nullptr;        // pinned, grid*NW entries
    bool dirty[NSLOTS] = {};           // slot's sums / area partials used since they were last reset
    bool parts_dirty[NSLOTS] = {};     // slot's per-workgroup partials written (per-CU launches)
    bool slot_hist[NSLOTS] = {};
    double2* d_bounds = nullptr;       // NSLOTS {a, b}
    double2* h_bounds = nullptr;       // pinned staging ring, NSTAGE x NSLOTS (a launch's copy may still be
                                       // pending when the host queues the next launch)
    hipEvent_t stage_ev[NSTAGE] = {};  // recorded after each staging copy
    int stage = 0;
    Chunk* d_chunks = nullptr;
    Cellar* d_cellar = nullptr;        // grid * NW per-wave HBM overflow stacks
    unsigned* d_ready = nullptr;
    unsigned epoch = 0;
    int engine = AQ_ENGINE_AUTO;       // aq_set_engine
    int wstride = 0;                   // warea entries per slot: max waves of either engine's grid
    double2* d_stk = nullptr;          // k_dfs lane stacks, grid * DW * SDEPTH * 64 entries
    LaunchHint* d_hint = nullptr;      // job-size hint carried from launch to launch
    bool hint_valid = false;           // the workload the hint was measured on
    int hint_fid = -1, hint_nshards = 0;
    double hint_eps = 0.0;
    int gsplit_env = 0;                // AQ_GSPLIT: waves per job of a multi-integral launch (0 = default)
    // level path
    DevResults* d_lres = nullptr;
    Rec* d_front[2] = {nullptr, nullptr};
    size_t front_cap = 0;
    unsigned* d_count = nullptr;
    // eval buffers
    LevelPart* d_lparts = nullptr;     // frontier engine: per-block partials of one level step
    double* d_batch = nullptr;         // batch front end: MAXK x {area, tasks, accepted, error}
    double* h_batch = nullptr;         // pinned, batch_cap rows
    size_t batch_cap = 0;
    double* d_x = nullptr;
    double* d_y = nullptr;
    size_t eval_cap = 0;
    // host staging
    WgPart* h_parts = nullptr;         // pinned, grid entries
    SlotSums* h_sums = nullptr;        // pinned, one
    unsigned long long* h_hist = nullptr;  // pinned, 2 * AQ_MAX_LEVELS
    DevResults* h_lres = nullptr;      // pinned
    HostOut last;
    bool last_valid = false;
    // diagnostics
    unsigned long long* d_diag = nullptr;
    // timing
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_free;
    double timed_ms = 0.0;
    unsigned long long timed_launches = 0;
};

namespace {

// Return slots [s, s+k) to the all-zero state if any was used since it was last reset: k_reset
// clears only what the slots' lists name (sums, queue words, listed area partials), so a reset
// costs bytes per touched wave, not 64 KiB per slot; per-workgroup partials (per-CU launches only)
// are cleared with a memset of just those slots.
int ensure_clean(aq_ctx* c, int s, int k) {
    bool need = false, hist = false;
    for (int i = s; i < s + k; ++i) {
        need |= c->dirty[i];
        hist |= c->dirty[i] && c->slot_hist[i];
    }
    if (need) {
        hipLaunchKernelGGL(k_reset, dim3(k), dim3(256), 0, c->stream, c->d_ctl, c->d_warea, c->wstride, s, hist ? 1 : 0);
        AQ_HIP(hipGetLastError());
        for (int i = s; i < s + k; ++i) c->dirty[i] = false;
    }
    for (int i = s; i < s + k;) {
        if (!c->parts_dirty[i]) { ++i; continue; }
        int j = i;
        while (j < s + k && c->parts_dirty[j]) c->parts_dirty[j++] = false;
        AQ_HIP(hipMemsetAsync(c->d_parts + (size_t)i * c->grid, 0, sizeof(WgPart) * (size_t)(j - i) * c->grid,
                              c->stream));
        i = j;
    }
    return AQ_OK;
}

// The engine a launch of k integrals runs on: the lane-DFS kernel for multi-integral launches (many
// jobs, the throughput path), the streaming pair kernel (HBM work queue) for a lone integral.
bool use_dfs(const aq_ctx* ctx, int k) {
    if (ctx->engine == AQ_ENGINE_DFS) return true;
    if (ctx->engine == AQ_ENGINE_STREAM) return false;
    return k >= DFS_MIN_K;
}

int engine_waves(const aq_ctx* ctx, bool dfs) { return ctx->grid * (dfs ? DW : NW); }

template <int FID, bool HIST>
int launch_stream(aq_ctx* ctx, int k, const double* a, const double* b, double eps, int max_depth, int shard,
                  int nshards, int first_slot) {
    const int G = ctx->grid;
    const bool dfs = use_dfs(ctx, k);
    const int W = engine_waves(ctx, dfs);
    int rc = ensure_clean(ctx, first_slot, k);
    if (rc) return rc;
    const int st = ctx->stage;
    ctx->stage = (st + 1) % NSTAGE;
    AQ_HIP(hipEventSynchronize(ctx->stage_ev[st]));   // the copy that last used this buffer is done
    double2* hb = ctx->h_bounds + (size_t)st * NSLOTS;
    for (int i = 0; i < k; ++i) hb[i] = make_double2(a[i], b[i]);
    AQ_HIP(hipMemcpyAsync(ctx->d_bounds + first_slot, hb, sizeof(double2) * (size_t)k,
                          hipMemcpyHostToDevice, ctx->stream));
    AQ_HIP(hipEventRecord(ctx->stage_ev[st], ctx->stream));
    StreamParams P{};
    P.bounds = ctx->d_bounds + first_slot;
    P.nprob = k;
    P.first_slot = first_slot;
    P.eps = eps;
    P.max_depth = max_depth ? max_depth : AQ_DEFAULT_MAX_DEPTH;
    P.shard = shard;
    P.nshards = nshards;
    // jobs: one integral is split into one share per wave (the partition the oracle restates); a
    // multi-integral launch uses gsplit-times larger shares, so one seeding pass feeds more rounds.
    // A shard of N holds 1/N of each integral: its shares are N times fewer, so a job (and its
    // seeding overhead) stays the same size whatever N (strong scaling).
    int gs = k >= 16 ? DEFAULT_GSPLIT * std::max(1, nshards) : 1;
    gs = std::min(gs, W);
    if (ctx->gsplit_env > 0) gs = ctx->gsplit_env;
    while (gs > 1 && W % gs != 0) gs >>= 1;
    P.shares = W / gs;
    // a lone unsharded integral (one share per wave) seeds deeper: more, smaller positions per
    // share even out the shares' subtrees (only the totals of such a launch are compared)
    P.D = floor_log2((unsigned long long)P.shares * (unsigned long long)nshards) +
          ((k < PCU_MAXK && nshards == 1 && !dfs) ? AQ_PCU_SW : S_W);
    {   // seeding keeps F and flags of every path node of a share in the wave's ring (WCAP slots)
        const unsigned long long V = (unsigned long long)P.shares * (unsigned long long)nshards;
        const unsigned long long nb = ((1ull << P.D) + V - 1) / V;
        if (!dfs && (unsigned long long)(P.D + 1) * nb + 2 > (unsigned long long)WCAP) return AQ_EINVAL;
    }
    P.epoch = ++ctx->epoch;
    if (P.epoch == 0) P.epoch = ++ctx->epoch;
    P.qcap = QCAP;
    P.timeout_ticks = 100000000ull * 20ull;  // 20 s of the 100 MHz realtime clock
    P.ctls = ctx->d_ctl;
    P.parts = ctx->d_parts;
    P.warea = ctx->d_warea;
    P.diag = ctx->d_diag;
    P.chunks = ctx->d_chunks;
    P.cellar = ctx->d_cellar;
    P.ready = ctx->d_ready;
    P.gtab = ctx->d_tab;
    P.stk = ctx->d_stk;
    P.wstride = (unsigned)ctx->wstride;
    P.hint = ctx->d_hint;
    P.per_cu = k < PCU_MAXK ? 1 : 0;   // per-CU task counts for lone integrals (the reference's per-worker printout)
    // multi-integral stream launches size their jobs from the previous launch's tasks per integral,
    // when that launch integrated the same integrand at the same tolerance (a context that switches
    // workload starts from the default shares and a fresh hint). Not for shards: every shard of an
    // integral must use the same partition (shares, seed depth), and each rank's hint would come
    // from its own, slightly different, share of the work.
    P.adaptive = 0;
    if (!dfs && k >= 16 && ctx->gsplit_env <= 0 && nshards == 1) {
        const bool same = ctx->hint_valid && ctx->hint_fid == FID && ctx->hint_eps == eps &&
                          ctx->hint_nshards == nshards;
        P.adaptive = same ? 3 : 2;
        ctx->hint_valid = true;
        ctx->hint_fid = FID;
        ctx->hint_eps = eps;
        ctx->hint_nshards = nshards;
    }
    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    if (ctx->timing) {
        if (!ctx->ev_free.empty()) {
            ev = ctx->ev_free.back();
            ctx->ev_free.pop_back();
        } else {
            AQ_HIP(hipEventCreate(&ev.first));
            AQ_HIP(hipEventCreate(&ev.second));
        }
        AQ_HIP(hipEventRecord(ev.first, ctx->stream));
    }
    if (dfs) {
        if (P.diag)
            hipLaunchKernelGGL((k_dfs<FID, HIST, true>), dim3(G), dim3(DPT), 0, ctx->stream, P);
        else
            hipLaunchKernelGGL((k_dfs<FID, HIST, false>), dim3(G), dim3(DPT), 0, ctx->stream, P);
    } else if (P.diag) {
        if (P.per_cu)
            hipLaunchKernelGGL((k_stream<FID, HIST, true, true>), dim3(G), dim3(PT), 0, ctx->stream, P);
        else
            hipLaunchKernelGGL((k_stream<FID, HIST, true, false>), dim3(G), dim3(PT), 0, ctx->stream, P);
    } else {
        if (P.per_cu)
            hipLaunchKernelGGL((k_stream<FID, HIST, false, true>), dim3(G), dim3(PT), 0, ctx->stream, P);
        else
            hipLaunchKernelGGL((k_stream<FID, HIST, false, false>), dim3(G), dim3(PT), 0, ctx->stream, P);
    }
    AQ_HIP(hipGetLastError());
    if (ctx->timing) {
        AQ_HIP(hipEventRecord(ev.second, ctx->stream));
        ctx->ev_pending.push_back(ev);
    }
    for (int i = first_slot; i < first_slot + k; ++i) {
        ctx->dirty[i] = true;
        ctx->parts_dirty[i] = ctx->parts_dirty[i] || P.per_cu;
        ctx->slot_hist[i] = HIST;
    }
    return AQ_OK;
}

void fill_result(const HostOut& h, aq_result* out) {
    if (!out) return;
    out->area = h.area;
    out->tasks = h.tasks;
    out->accepted = h.leaves;
    out->levels = h.levels;
    out->spilled = h.spilled;
    unsigned n = 0;
    for (int i = 0; i < AQ_CU_SLOTS; ++i) n += h.cu[i] ? 1u : 0u;
    out->n_cu = n;
}

int fetch_slot(aq_ctx* ctx, int slot, aq_result* out) {
    if (ctx->parts_dirty[slot])
        AQ_HIP(hipMemcpyAsync(ctx->h_parts, ctx->d_parts + (size_t)slot * ctx->grid,
                              sizeof(WgPart) * (size_t)ctx->grid, hipMemcpyDeviceToHost, ctx->stream));
    AQ_HIP(hipMemcpyAsync(ctx->h_sums, &ctx->d_ctl[slot].sums, sizeof(SlotSums), hipMemcpyDeviceToHost, ctx->stream));
    const size_t nw = (size_t)ctx->wstride;
    AQ_HIP(hipMemcpyAsync(ctx->h_warea, ctx->d_warea + (size_t)slot * nw, sizeof(double2) * nw, hipMemcpyDeviceToHost,
                          ctx->stream));
    if (ctx->slot_hist[slot])
        AQ_HIP(hipMemcpyAsync(ctx->h_hist, ctx->d_ctl[slot].hist, sizeof(unsigned long long) * 2 * AQ_MAX_LEVELS,
                              hipMemcpyDeviceToHost, ctx->stream));
    AQ_HIP(hipStreamSynchronize(ctx->stream));
    HostOut& h = ctx->last;
    h = HostOut();
    double hi = 0.0, lo = 0.0;
    for (size_t i = 0; i < nw; ++i) dd_add_dd(hi, lo, ctx->h_warea[i].x, ctx->h_warea[i].y);
    h.area = hi + lo;
    const SlotSums& sm = *ctx->h_sums;
    h.tasks = sm.tasks;
    h.leaves = sm.leaves;
    h.spilled = sm.spilled;
    h.levels = sm.levels;
    h.error = sm.error;
    if (ctx->parts_dirty[slot]) {   // per-CU counts: lone-integral launches keep per-workgroup partials
        for (int i = 0; i < ctx->grid; ++i) {
            const WgPart& w = ctx->h_parts[i];
            if (w.tasks) h.cu[w.cu % AQ_CU_SLOTS] += w.tasks;
        }
    }
    if (ctx->slot_hist[slot]) memcpy(h.hist, ctx->h_hist, sizeof(h.hist));
    ctx->last_valid = true;
    fill_result(h, out);
    return err_from_bits(h.error);
}

int launch_any(aq_ctx* ctx, int integrand, int k, const double* a, const double* b, double eps, int max_depth,
               int shard, int nshards, int first_slot) {
    const bool h = ctx->histograms;
    if (integrand == AQ_F_COSH4)
        return h ? launch_stream<F_COSH4, true>(ctx, k, a, b, eps, max_depth, shard, nshards, first_slot)
                 : launch_stream<F_COSH4, false>(ctx, k, a, b, eps, max_depth, shard, nshards, first_slot);
    return h ? launch_stream<F_SIN_RECIP, true>(ctx, k, a, b, eps, max_depth, shard, nshards, first_slot)
             : launch_stream<F_SIN_RECIP, false>(ctx, k, a, b, eps, max_depth, shard, nshards, first_slot);
}

}  // namespace

extern "C" {

const char* aq_strerror(int code) {
    switch (code) {
        case AQ_OK: return "ok";
        case AQ_EINVAL: return "invalid argument";
        case AQ_EHIP: return "HIP runtime error";
        case AQ_ETIMEOUT: return "on-device wait timed out";
        case AQ_EOVERFLOW: return "frontier / work-queue capacity exceeded";
        case AQ_EDEPTH: return "maximum refinement depth reached";
        case AQ_ENOMEM: return "out of memory";
        case AQ_ENODEV: return "no HIP device";
        default: return "unknown error";
    }
}

int aq_device_count(int* count) {
    if (!count) return AQ_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return n > 0 ? AQ_OK : AQ_ENODEV;
}

int aq_ctx_create(int device, aq_ctx** out) {
    if (!out) return AQ_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return AQ_ENODEV;
    if (device < 0 || device >= n) return AQ_EINVAL;
    aq_ctx* c = new aq_ctx();
    c->device = device;
    AQ_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    AQ_HIP(hipGetDeviceProperties(&prop, device));
    c->num_cus = prop.multiProcessorCount;
    int occ = 0;
    AQ_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k_stream<F_COSH4, true, false, false>, PT, 0));
    if (occ < 1) {
        delete c;
        return AQ_ENODEV;
    }
    // One workgroup per CU (the LDS rings take most of a CU's LDS); the whole grid must be
    // resident, because idle workgroups wait on the queue for busy ones.
    c->grid = std::min(c->num_cus, MAXG);
    c->wstride = c->grid * std::max(NW, DW);
    if (const char* e = getenv("AQ_ENGINE")) {
        if (!strcmp(e, "stream")) c->engine = AQ_ENGINE_STREAM;
        else if (!strcmp(e, "dfs")) c->engine = AQ_ENGINE_DFS;
    }
    if (const char* e = getenv("AQ_GSPLIT")) c->gsplit_env = atoi(e);
    AQ_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    AQ_HIP(hipMalloc(&c->d_tab, sizeof(ExpEntry) * 128));
    AQ_HIP(hipMemcpy(c->d_tab, aq_exp_tab_host, sizeof(ExpEntry) * 128, hipMemcpyHostToDevice));
    AQ_HIP(hipMalloc(&c->d_ctl, sizeof(Ctl) * NSLOTS));
    AQ_HIP(hipMemset(c->d_ctl, 0, sizeof(Ctl) * NSLOTS));
    AQ_HIP(hipMalloc(&c->d_parts, sizeof(WgPart) * (size_t)NSLOTS * c->grid));
    AQ_HIP(hipMemset(c->d_parts, 0, sizeof(WgPart) * (size_t)NSLOTS * c->grid));
    AQ_HIP(hipMalloc(&c->d_warea, sizeof(double2) * (size_t)NSLOTS * c->wstride));
    AQ_HIP(hipMemset(c->d_warea, 0, sizeof(double2) * (size_t)NSLOTS * c->wstride));
    AQ_HIP(hipHostMalloc(&c->h_warea, sizeof(double2) * (size_t)c->wstride, hipHostMallocDefault));
    AQ_HIP(hipMalloc(&c->d_stk, sizeof(double2) * (size_t)c->grid * DW * SDEPTH * 64));
    AQ_HIP(hipMalloc(&c->d_bounds, sizeof(double2) * NSLOTS));
    AQ_HIP(hipMalloc(&c->d_hint, sizeof(LaunchHint)));
    AQ_HIP(hipMemset(c->d_hint, 0, sizeof(LaunchHint)));
    AQ_HIP(hipHostMalloc(&c->h_bounds, sizeof(double2) * NSLOTS * NSTAGE, hipHostMallocDefault));
    for (int i = 0; i < NSTAGE; ++i) {
        AQ_HIP(hipEventCreateWithFlags(&c->stage_ev[i], hipEventDisableTiming));
        AQ_HIP(hipEventRecord(c->stage_ev[i], c->stream));
    }
    AQ_HIP(hipMalloc(&c->d_chunks, sizeof(Chunk) * (size_t)QCAP));
    AQ_HIP(hipMalloc(&c->d_cellar, sizeof(Cellar) * (size_t)c->grid * NW));
    AQ_HIP(hipMalloc(&c->d_ready, sizeof(unsigned) * (size_t)QCAP * READY_STRIDE));
    AQ_HIP(hipMemset(c->d_ready, 0, sizeof(unsigned) * (size_t)QCAP * READY_STRIDE));
    AQ_HIP(hipHostMalloc(&c->h_parts, sizeof(WgPart) * (size_t)c->grid, hipHostMallocDefault));
    AQ_HIP(hipHostMalloc(&c->h_sums, sizeof(SlotSums), hipHostMallocDefault));
    AQ_HIP(hipHostMalloc(&c->h_hist, sizeof(unsigned long long) * 2 * AQ_MAX_LEVELS, hipHostMallocDefault));
    AQ_HIP(hipHostMalloc(&c->h_lres, sizeof(DevResults), hipHostMallocDefault));
    AQ_HIP(hipMalloc(&c->d_lres, sizeof(DevResults)));
    AQ_HIP(hipMalloc(&c->d_count, sizeof(unsigned) * (AQ_MAX_LEVELS + 2)));
    AQ_HIP(hipDeviceSynchronize());
    *out = c;
    return AQ_OK;
}

void aq_ctx_destroy(aq_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& e : c->ev_pending) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
    for (auto& e : c->ev_free) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
    (void)hipFree(c->d_tab);
    (void)hipFree(c->d_ctl);
    (void)hipFree(c->d_parts);
    (void)hipFree(c->d_warea);
    (void)hipFree(c->d_bounds);
    (void)hipFree(c->d_hint);
    (void)hipFree(c->d_chunks);
    (void)hipFree(c->d_cellar);
    (void)hipFree(c->d_stk);
    (void)hipFree(c->d_ready);
    (void)hipFree(c->d_lres);
    (void)hipFree(c->d_diag);
    (void)hipFree(c->d_front[0]);
    (void)hipFree(c->d_front[1]);
    (void)hipFree(c->d_count);
    (void)hipFree(c->d_x);
    (void)hipFree(c->d_batch);
    (void)hipFree(c->d_lparts);
    if (c->h_batch) (void)hipHostFree(c->h_batch);
    (void)hipFree(c->d_y);
    if (c->h_bounds) (void)hipHostFree(c->h_bounds);
    for (int i = 0; i < NSTAGE; ++i)
        if (c->stage_ev[i]) (void)hipEventDestroy(c->stage_ev[i]);
    if (c->h_parts) (void)hipHostFree(c->h_parts);
    if (c->h_sums) (void)hipHostFree(c->h_sums);
    if (c->h_warea) (void)hipHostFree(c->h_warea);
    if (c->h_hist) (void)hipHostFree(c->h_hist);
    if (c->h_lres) (void)hipHostFree(c->h_lres);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int aq_ctx_num_cus(const aq_ctx* c) { return c ? c->num_cus : 0; }
int aq_ctx_num_workers(const aq_ctx* c) { return c ? engine_waves(c, use_dfs(c, 1)) : 0; }

int aq_set_engine(aq_ctx* c, int engine) {
    if (!c || engine < AQ_ENGINE_AUTO || engine > AQ_ENGINE_DFS) return AQ_EINVAL;
    c->engine = engine;
    return AQ_OK;
}

int aq_set_level_histograms(aq_ctx* c, int enable) {
    if (!c) return AQ_EINVAL;
    c->histograms = enable != 0;
    return AQ_OK;
}

int aq_set_diagnostics(aq_ctx* c, int enable) {
    if (!c) return AQ_EINVAL;
    AQ_HIP(hipSetDevice(c->device));
    AQ_HIP(hipStreamSynchronize(c->stream));
    if (enable && !c->d_diag) {
        AQ_HIP(hipMalloc(&c->d_diag, sizeof(unsigned long long) * DIAG_WORDS * MAXG));
        AQ_HIP(hipMemset(c->d_diag, 0, sizeof(unsigned long long) * DIAG_WORDS * MAXG));
    } else if (!enable && c->d_diag) {
        (void)hipFree(c->d_diag);
        c->d_diag = nullptr;
    }
    return AQ_OK;
}

int aq_diagnostics(aq_ctx* c, uint64_t* out, int cap_words) {
    if (!c || !out || !c->d_diag) return AQ_EINVAL;
    AQ_HIP(hipSetDevice(c->device));
    const size_t words = std::min<size_t>((size_t)cap_words, (size_t)DIAG_WORDS * c->grid);
    AQ_HIP(hipStreamSynchronize(c->stream));
    AQ_HIP(hipMemcpy(out, c->d_diag, words * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return (int)(words / DIAG_WORDS);
}

int aq_async_slots(void) { return NSLOTS; }

int aq_max_integrals_per_launch(void) { return MAXK; }

int aq_integrate_many_async(aq_ctx* ctx, int integrand, int k, const double* a, const double* b, double eps,
                            int max_depth, int shard, int nshards, int first_slot) {
    if (!ctx || k < 1 || k > MAXK || !a || !b) return AQ_EINVAL;
    if (integrand != AQ_F_COSH4 && integrand != AQ_F_SIN_RECIP) return AQ_EINVAL;
    if (!(eps >= 0.0) || max_depth < 0 || max_depth > AQ_MAX_LEVELS - 1) return AQ_EINVAL;
    if (nshards < 1 || shard < 0 || shard >= nshards || nshards > 64) return AQ_EINVAL;
    if (first_slot < 0 || first_slot + k > NSLOTS) return AQ_EINVAL;
    for (int i = 0; i < k; ++i)
        if (!bounds_ok(a[i], b[i])) return AQ_EINVAL;
    AQ_HIP(hipSetDevice(ctx->device));
    return launch_any(ctx, integrand, k, a, b, eps, max_depth, shard, nshards, first_slot);
}

int aq_integrate_async(aq_ctx* ctx, const aq_problem* p, int shard, int nshards, int slot) {
    if (!ctx) return AQ_EINVAL;
    int rc = validate(p);
    if (rc) return rc;
    return aq_integrate_many_async(ctx, p->integrand, 1, &p->a, &p->b, p->eps, p->max_depth, shard, nshards, slot);
}

int aq_gather_results(aq_ctx* ctx, int first_slot, int n, void* d_out) {
    if (!ctx || !d_out || n < 0 || n > NSLOTS || first_slot < 0 || first_slot >= NSLOTS) return AQ_EINVAL;
    if (n == 0) return AQ_OK;
    AQ_HIP(hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_gather, dim3(n), dim3(256), 0, ctx->stream, ctx->d_ctl, ctx->d_warea, ctx->wstride,
                       first_slot, n, NSLOTS, (double*)d_out);
    AQ_HIP(hipGetLastError());
    return AQ_OK;
}

int aq_fetch(aq_ctx* ctx, int slot, aq_result* res) {
    if (!ctx || slot < 0 || slot >= NSLOTS) return AQ_EINVAL;
    AQ_HIP(hipSetDevice(ctx->device));
    return fetch_slot(ctx, slot, res);
}

int aq_synchronize(aq_ctx* ctx) {
    if (!ctx) return AQ_EINVAL;
    AQ_HIP(hipSetDevice(ctx->device));
    AQ_HIP(hipStreamSynchronize(ctx->stream));
    return AQ_OK;
}

int aq_integrate_shard(aq_ctx* ctx, const aq_problem* p, int shard, int nshards, aq_result* res) {
    int rc = aq_integrate_async(ctx, p, shard, nshards, 0);
    if (rc) return rc;
    return aq_fetch(ctx, 0, res);
}

int aq_integrate(aq_ctx* ctx, const aq_problem* p, aq_result* res) { return aq_integrate_shard(ctx, p, 0, 1, res); }

int aq_level_histogram(aq_ctx* ctx, uint64_t* tpl, uint64_t* lpl, int maxlev) {
    if (!ctx || maxlev < 0 || !ctx->last_valid) return AQ_EINVAL;
    for (int i = 0; i < maxlev; ++i) {
        const bool in = i < AQ_MAX_LEVELS;
        if (tpl) tpl[i] = in ? ctx->last.hist[i] : 0;
        if (lpl) lpl[i] = in ? ctx->last.hist[AQ_MAX_LEVELS + i] : 0;
    }
    return AQ_OK;
}

int aq_tasks_per_cu(aq_ctx* ctx, uint64_t* out, int cap) {
    if (!ctx || !ctx->last_valid) return AQ_EINVAL;
    int n = 0;
    for (int i = 0; i < AQ_CU_SLOTS; ++i) {
        if (out && i < cap) out[i] = ctx->last.cu[i];
        n += ctx->last.cu[i] ? 1 : 0;
    }
    return n;
}

int aq_integrate_levels(aq_ctx* ctx, const aq_problem* p, aq_result* res, uint64_t* tpl, uint64_t* lpl,
                        int maxlev) {
    if (!ctx) return AQ_EINVAL;
    int rc = validate(p);
    if (rc) return rc;
    AQ_HIP(hipSetDevice(ctx->device));
    const int max_depth = p->max_depth ? p->max_depth : AQ_DEFAULT_MAX_DEPTH;
    if (!ctx->d_front[0]) {
        size_t cap = (size_t)1 << 24;  // 16 M records (512 MiB) per buffer
        AQ_HIP(hipMalloc(&ctx->d_front[0], cap * sizeof(Rec)));
        AQ_HIP(hipMalloc(&ctx->d_front[1], cap * sizeof(Rec)));
        ctx->front_cap = cap;
    }
    DevResults* dres = ctx->d_lres;
    AQ_HIP(hipMemsetAsync(dres, 0, sizeof(DevResults), ctx->stream));
    AQ_HIP(hipMemsetAsync(ctx->d_count, 0, sizeof(unsigned) * (AQ_MAX_LEVELS + 2), ctx->stream));
    if (p->integrand == AQ_F_COSH4)
        hipLaunchKernelGGL((k_root<F_COSH4>), dim3(1), dim3(64), 0, ctx->stream, p->a, p->b, ctx->d_front[0], ctx->d_tab);
    else
        hipLaunchKernelGGL((k_root<F_SIN_RECIP>), dim3(1), dim3(64), 0, ctx->stream, p->a, p->b, ctx->d_front[0], ctx->d_tab);
    AQ_HIP(hipGetLastError());
    unsigned n = 1;
    int depth = 0;
    for (; n > 0 && depth < AQ_MAX_LEVELS; ++depth) {
        Rec* in = ctx->d_front[depth & 1];
        Rec* outb = ctx->d_front[(depth + 1) & 1];
        unsigned* n_out = ctx->d_count + depth + 1;
        const unsigned grid = (unsigned)std::min<size_t>((n + 255) / 256, 8192);
        if (p->integrand == AQ_F_COSH4)
            hipLaunchKernelGGL((k_level<F_COSH4>), dim3(grid), dim3(256), 0, ctx->stream, in, n, outb, n_out,
                               (unsigned)ctx->front_cap, p->eps, depth, max_depth, dres, ctx->d_tab);
        else
            hipLaunchKernelGGL((k_level<F_SIN_RECIP>), dim3(grid), dim3(256), 0, ctx->stream, in, n, outb, n_out,
                               (unsigned)ctx->front_cap, p->eps, depth, max_depth, dres, ctx->d_tab);
        AQ_HIP(hipGetLastError());
        AQ_HIP(hipMemcpyAsync(ctx->h_lres, n_out, sizeof(unsigned), hipMemcpyDeviceToHost, ctx->stream));
        AQ_HIP(hipStreamSynchronize(ctx->stream));
        unsigned next = 0;
        memcpy(&next, ctx->h_lres, sizeof(unsigned));
        if (next > ctx->front_cap) next = (unsigned)ctx->front_cap;  // overflow flagged in res->error
        n = next;
    }
    AQ_HIP(hipMemcpyAsync(ctx->h_lres, dres, sizeof(DevResults), hipMemcpyDeviceToHost, ctx->stream));
    AQ_HIP(hipStreamSynchronize(ctx->stream));
    const DevResults& d = *ctx->h_lres;
    HostOut& h = ctx->last;
    h = HostOut();
    h.area = d.area;
    h.tasks = d.tasks;
    h.leaves = d.leaves;
    h.levels = d.levels;
    h.error = d.error;
    for (int i = 0; i < AQ_MAX_LEVELS; ++i) {
        h.hist[i] = d.tasks_per_level[i];
        h.hist[AQ_MAX_LEVELS + i] = d.leaves_per_level[i];
    }
    for (int i = 0; i < AQ_CU_SLOTS; ++i) h.cu[i] = d.cu_tasks[i];
    ctx->last_valid = true;
    fill_result(h, res);
    rc = err_from_bits(h.error);
    if (rc) return rc;
    if (n > 0) return AQ_EDEPTH;
    return aq_level_histogram(ctx, tpl, lpl, maxlev);
}

static int ensure_eval(aq_ctx* ctx, size_t n) {
    if (ctx->eval_cap >= n) return AQ_OK;
    (void)hipFree(ctx->d_x);
    (void)hipFree(ctx->d_y);
    ctx->d_x = ctx->d_y = nullptr;
    AQ_HIP(hipMalloc(&ctx->d_x, n * sizeof(double)));
    AQ_HIP(hipMalloc(&ctx->d_y, n * sizeof(double)));
    ctx->eval_cap = n;
    return AQ_OK;
}

static int eval_common(aq_ctx* ctx, int integrand, bool cosh_only, size_t n, const double* x, double* out) {
    if (!ctx || (!x && n) || (!out && n)) return AQ_EINVAL;
    if (integrand != AQ_F_COSH4 && integrand != AQ_F_SIN_RECIP) return AQ_EINVAL;
    if (n == 0) return AQ_OK;
    AQ_HIP(hipSetDevice(ctx->device));
    int rc = ensure_eval(ctx, n);
    if (rc) return rc;
    AQ_HIP(hipMemcpyAsync(ctx->d_x, x, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    const unsigned grid = (unsigned)std::min<size_t>((n + 255) / 256, 4096);
    if (cosh_only)
        hipLaunchKernelGGL((k_eval<F_COSH4, true>), dim3(grid), dim3(256), 0, ctx->stream, ctx->d_x, ctx->d_y, n, ctx->d_tab);
    else if (integrand == AQ_F_COSH4)
        hipLaunchKernelGGL((k_eval<F_COSH4, false>), dim3(grid), dim3(256), 0, ctx->stream, ctx->d_x, ctx->d_y, n, ctx->d_tab);
    else
        hipLaunchKernelGGL((k_eval<F_SIN_RECIP, false>), dim3(grid), dim3(256), 0, ctx->stream, ctx->d_x, ctx->d_y, n, ctx->d_tab);
    AQ_HIP(hipGetLastError());
    AQ_HIP(hipMemcpyAsync(out, ctx->d_y, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    AQ_HIP(hipStreamSynchronize(ctx->stream));
    return AQ_OK;
}

int aq_eval_integrand(aq_ctx* ctx, int integrand, size_t n, const double* x, double* out) {
    return eval_common(ctx, integrand, false, n, x, out);
}

int aq_eval_cosh(aq_ctx* ctx, size_t n, const double* x, double* out) {
    return eval_common(ctx, AQ_F_COSH4, true, n, x, out);
}

int aq_integrate_batch(aq_ctx* ctx, int integrand, size_t n, const double* a, const double* b, double eps,
                       double* area, uint64_t* tasks, uint64_t* accepted) {
    // Batch front end (SURVEY config 3): MAXK integrals per persistent launch, every integral with
    // its own slot; each launch's slots are gathered on the device into one row block that is
    // copied back asynchronously, so launches, gathers and copies stream back to back with one
    // host synchronisation at the end.
    if (!ctx || (n && (!a || !b))) return AQ_EINVAL;
    if (integrand != AQ_F_COSH4 && integrand != AQ_F_SIN_RECIP) return AQ_EINVAL;
    if (!(eps >= 0.0)) return AQ_EINVAL;
    for (size_t i = 0; i < n; ++i)
        if (!bounds_ok(a[i], b[i])) return AQ_EINVAL;
    if (n == 0) return AQ_OK;
    AQ_HIP(hipSetDevice(ctx->device));
    if (!ctx->d_batch) AQ_HIP(hipMalloc(&ctx->d_batch, sizeof(double) * 4 * MAXK));
    if (ctx->batch_cap < n) {
        if (ctx->h_batch) AQ_HIP(hipHostFree(ctx->h_batch));
        ctx->h_batch = nullptr;
        AQ_HIP(hipHostMalloc(&ctx->h_batch, sizeof(double) * 4 * n, hipHostMallocDefault));
        ctx->batch_cap = n;
    }
    const bool hist = ctx->histograms;
    ctx->histograms = false;
    int rc = AQ_OK;
    for (size_t done = 0; done < n && rc == AQ_OK;) {
        const int m = (int)std::min<size_t>(n - done, (size_t)MAXK);
        rc = aq_integrate_many_async(ctx, integrand, m, a + done, b + done, eps, 0, 0, 1, 0);
        if (rc) break;
        rc = aq_gather_results(ctx, 0, m, ctx->d_batch);
        if (rc) break;
        if (hipMemcpyAsync(ctx->h_batch + 4 * done, ctx->d_batch, sizeof(double) * 4 * (size_t)m,
                           hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) {
            rc = AQ_EHIP;
            break;
        }
        done += (size_t)m;
    }
    ctx->histograms = hist;
    if (hipStreamSynchronize(ctx->stream) != hipSuccess && rc == AQ_OK) rc = AQ_EHIP;
    if (rc) return rc;
    unsigned errbits = 0;
    for (size_t i = 0; i < n; ++i) {
        const double* row = ctx->h_batch + 4 * i;
        if (area) area[i] = row[0];
        if (tasks) tasks[i] = (uint64_t)row[1];
        if (accepted) accepted[i] = (uint64_t)row[2];
        errbits |= (unsigned)row[3];
    }
    return err_from_bits(errbits);
}

int aq_frontier_root(aq_ctx* ctx, int integrand, double a, double b, double* d_out) {
    if (!ctx || !d_out || !bounds_ok(a, b)) return AQ_EINVAL;
    if (integrand != AQ_F_COSH4 && integrand != AQ_F_SIN_RECIP) return AQ_EINVAL;
    AQ_HIP(hipSetDevice(ctx->device));
    if (integrand == AQ_F_COSH4)
        hipLaunchKernelGGL((k_frontier_root<F_COSH4>), dim3(1), dim3(64), 0, ctx->stream, a, b, (Rec*)d_out, ctx->d_tab);
    else
        hipLaunchKernelGGL((k_frontier_root<F_SIN_RECIP>), dim3(1), dim3(64), 0, ctx->stream, a, b, (Rec*)d_out,
                           ctx->d_tab);
    AQ_HIP(hipGetLastError());
    return AQ_OK;
}

int aq_level_step(aq_ctx* ctx, int integrand, const double* d_in, uint32_t n_in, double* d_out, uint32_t cap_out,
                  double eps, int depth, int max_depth, uint32_t* d_n_out, double* d_acc) {
    constexpr int MAXB = 8192;   // level-step grid cap (grid-stride beyond)
    if (!ctx || !d_n_out || !d_acc || (n_in && (!d_in || !d_out))) return AQ_EINVAL;
    if (integrand != AQ_F_COSH4 && integrand != AQ_F_SIN_RECIP) return AQ_EINVAL;
    if (!(eps >= 0.0) || depth < 0 || max_depth < 1 || max_depth > AQ_MAX_LEVELS - 1) return AQ_EINVAL;
    AQ_HIP(hipSetDevice(ctx->device));
    if (!ctx->d_lparts) AQ_HIP(hipMalloc(&ctx->d_lparts, sizeof(LevelPart) * MAXB));
    AQ_HIP(hipMemsetAsync(d_n_out, 0, sizeof(uint32_t), ctx->stream));
    if (n_in == 0) return AQ_OK;
    const int grid = (int)std::min<size_t>(((size_t)n_in + 255) / 256, (size_t)MAXB);
    if (integrand == AQ_F_COSH4)
        hipLaunchKernelGGL((k_level_step<F_COSH4>), dim3(grid), dim3(256), 0, ctx->stream, (const Rec*)d_in, n_in,
                           (Rec*)d_out, d_n_out, cap_out, eps, depth, max_depth, ctx->d_lparts, ctx->d_tab);
    else
        hipLaunchKernelGGL((k_level_step<F_SIN_RECIP>), dim3(grid), dim3(256), 0, ctx->stream, (const Rec*)d_in, n_in,
                           (Rec*)d_out, d_n_out, cap_out, eps, depth, max_depth, ctx->d_lparts, ctx->d_tab);
    AQ_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_level_fold, dim3(1), dim3(64), 0, ctx->stream, ctx->d_lparts, grid, d_acc);
    AQ_HIP(hipGetLastError());
    return AQ_OK;
}

int aq_kernel_timing(aq_ctx* ctx, int enable) {
    if (!ctx) return AQ_EINVAL;
    AQ_HIP(hipSetDevice(ctx->device));
    AQ_HIP(hipStreamSynchronize(ctx->stream));
    for (auto& e : ctx->ev_pending) ctx->ev_free.push_back(e);
    ctx->ev_pending.clear();
    ctx->timing = enable != 0;
    ctx->timed_ms = 0.0;
    ctx->timed_launches = 0;
    return AQ_OK;
}

int aq_kernel_time(aq_ctx* ctx, double* total_ms, uint64_t* launches) {
    if (!ctx) return AQ_EINVAL;
    AQ_HIP(hipSetDevice(ctx->device));
    AQ_HIP(hipStreamSynchronize(ctx->stream));
    for (auto& e : ctx->ev_pending) {
        float ms = 0.f;
        AQ_HIP(hipEventElapsedTime(&ms, e.first, e.second));
        ctx->timed_ms += ms;
        ctx->timed_launches += 1;
        ctx->ev_free.push_back(e);
    }
    ctx->ev_pending.clear();
    if (total_ms) *total_ms = ctx->timed_ms;
    if (launches) *launches = ctx->timed_launches;
    return AQ_OK;
}

void aq_print_reference(FILE* f, double area, const uint64_t* tpp, int nprocs) {
    if (!f) f = stdout;
    fprintf(f, "Area=%lf\n", area);             // :108
    fprintf(f, "\nTasks Per Process\n");         // :109
    for (int i = 0; i < nprocs; ++i) fprintf(f, "%d\t", i);                               // :110-112
    fprintf(f, "\n");
    for (int i = 0; i < nprocs; ++i) fprintf(f, "%llu\t", (unsigned long long)(tpp ? tpp[i] : 0));  // :114-116
    fprintf(f, "\n");
}

}  // extern "C"
