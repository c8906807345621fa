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
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "aquad.h"
#include "aq_exp_table.h"
#include "aq_libm.h"
#include "aq_device.h"
#include "aq_stream.h"
#include "aq_host_pool.h"

#include <rccl/rccl.h>

#pragma clang fp contract(off)

namespace aq {

// ------------------------------------------------------------------------------------------------
// Result block of the level-synchronous path (aq_integrate_levels), zeroed before each call.
// ------------------------------------------------------------------------------------------------
struct DevResults {
    double area;
    unsigned long long tasks;
    unsigned long long leaves;
    unsigned long long spilled;
    unsigned int levels;
    unsigned int error;        // AQ_E* as positive bit flags (see err_bit)
    unsigned long long tasks_per_level[AQ_MAX_LEVELS];
    unsigned long long leaves_per_level[AQ_MAX_LEVELS];
    unsigned long long cu_tasks[AQ_CU_SLOTS];
};


// ------------------------------------------------------------------------------------------------
// Parity helper: evaluate F or cosh on an array.
// ------------------------------------------------------------------------------------------------
template <int FID, bool COSH_ONLY>
__global__ __launch_bounds__(256) void k_eval(const double* __restrict__ x, double* __restrict__ out, size_t n,
                                              const ExpPair* __restrict__ gtab) {
    constexpr int TF = COSH_ONLY ? F_COSH4 : FID;
    __shared__ ExpEntry tab[ftab_entries<TF>()];
    stage_f_table<TF>(tab, gtab);
    __syncthreads();
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    if constexpr (FID == F_COSH4 && !COSH_ONLY) {
        // F through the persistent kernel's batched path (integrand_k: two interleaved cosh chains,
        // 2 cosh and 16 F), two points per lane; aq_eval_cosh keeps the scalar one
        const ExpConsts kk = pinned_exp_consts();
        for (size_t i = 2 * gid; i < n; i += 2 * stride) {
            const double xx[2] = {x[i], x[i + 1 < n ? i + 1 : i]};
            double ff[2];
            integrand_k<F_COSH4, 2, true>(xx, ff, tab, kk);   // 16 F, as k_stream's rounds (exact /16)
            out[i] = ff[0] / f_scale<F_COSH4>();
            if (i + 1 < n) out[i + 1] = ff[1] / f_scale<F_COSH4>();
        }
    } else {
        for (size_t i = gid; i < n; i += stride) out[i] = COSH_ONLY ? cosh_glibc(x[i], tab) : integrand<FID>(x[i], tab);
    }
}

// ------------------------------------------------------------------------------------------------
// Batch ordering (aq_integrate_batch, r05): a launch of whole tiny trees ends when its last-claimed jobs
// do, so the batch front end hands its launches their integrals largest first. The size of a tree is
// predicted from its top: the reference's task body (:185-191) on the 15 nodes of depths 0..3 -- F at
// the 17 points of a 1/16 grid by recursive midpoints -- and, for every depth-3 node the tree reaches
// and refines, (|diff| / eps)^(1/3) (trapezoid error ~ h^3, so the leaves a subtree needs scale like
// the cube root of its top error). Over 20 000 C3 integrals this predicts the task count with
// correlation 0.9996 (Spearman 0.9995; an offline check with the host integrand). Only the ORDER
// uses it: the counts and areas of every integral are those of its own tree whatever the order.
// ------------------------------------------------------------------------------------------------
// Size classes: key 0 = largest, EST_PER_OCTAVE classes per doubling of 1 + est, so the 256 classes span
// 2^32 (r06: 64 classes at 6 per octave ran out at est ~ 1 450, ~4 000 tasks -- at eps=1e-10 187 of the
// 200 golden C3 integrals shared key 0 and the chunk ran unsorted; 8 per octave over 256 classes order
// them with no pair more than 30 % out of order)
constexpr int EST_KEYS = 256;
constexpr double EST_PER_OCTAVE = 8.0;
// tasks per unit of the estimate: 2.77-2.90 over cosh4 [0,5] at eps = 1e-3 ... 1e-12 and 2.84 for C3's
// mean at 1e-3 and 1e-10 (an offline check with the host integrand), so a fresh workload's first launch
// can size its jobs from it (k_batch_scatter)
constexpr double EST_TASKS = 2.84;
template <int FID>
__global__ __launch_bounds__(256) void k_batch_estimate(const double2* __restrict__ bounds, int n, double eps,
                                                        unsigned* __restrict__ key_of, unsigned* __restrict__ counts,
                                                        double* __restrict__ est_sum, const ExpPair* __restrict__ gtab) {
    __shared__ ExpEntry tab[ftab_entries<FID>()];
    __shared__ unsigned s_cnt[EST_KEYS];
    __shared__ double s_est[4];
    stage_f_table<FID>(tab, gtab);
    if (threadIdx.x < EST_KEYS) s_cnt[threadIdx.x] = 0u;
    __syncthreads();
    double est = 0.0;
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < n) {
        const double2 ab = bounds[i];
        double x[17], f[17];
        x[0] = ab.x;
        x[16] = ab.y;
#pragma unroll
        for (int s = 8; s >= 1; s >>= 1)           // midpoints, level by level (:187)
#pragma unroll
            for (int k = s; k < 16; k += 2 * s) x[k] = (x[k - s] + x[k + s]) / 2;
#pragma unroll
        for (int k = 0; k < 17; ++k) f[k] = integrand<FID>(x[k], tab);   // :188
        bool alive[16] = {true};
#pragma unroll
        for (int d = 0, s = 16; d < 4; ++d, s >>= 1) {
#pragma unroll
            for (int k = 0; k < (1 << d); ++k) {
                const int lo = k * s, hi = lo + s, md = lo + s / 2;
                const double lrarea = (f[lo] + f[hi]) * (x[hi] - x[lo]) / 2;    // :185
                const double larea = (f[lo] + f[md]) * (x[md] - x[lo]) / 2;     // :189
                const double rarea = (f[md] + f[hi]) * (x[hi] - x[md]) / 2;     // :190
                const double diff = fabs((larea + rarea) - lrarea);
                const bool refine = alive[k << (3 - d)] && diff > eps;           // :191
                if (d < 3) {
                    alive[k << (3 - d)] = refine;                                // the children's slots
                    alive[(2 * k + 1) << (2 - d)] = refine;
                } else if (refine) {
                    est += cbrt(diff / eps);
                }
            }
        }
        const double lg = EST_PER_OCTAVE * log2(1.0 + est);
        const unsigned key = (unsigned)(EST_KEYS - 1) - (unsigned)min((double)(EST_KEYS - 1), lg);
        key_of[i] = key;
        atomicAdd(&s_cnt[key], 1u);
    }
    // the block's sum of the estimates (one atomic per block)
    for (int o = 32; o >= 1; o >>= 1) est += __shfl_xor(est, o, 64);
    if ((threadIdx.x & 63u) == 0u) s_est[threadIdx.x >> 6] = est;
    __syncthreads();
    if (threadIdx.x < EST_KEYS && s_cnt[threadIdx.x]) atomicAdd(&counts[threadIdx.x], s_cnt[threadIdx.x]);
    if (threadIdx.x == 0) atomicAdd(est_sum, (s_est[0] + s_est[1]) + (s_est[2] + s_est[3]));
}

// Scatter the chunk into size order: sorted[pos] = bounds[i], perm[pos] = i, pos = the key's offset (an
// exclusive scan of counts) + this block's reserved range + the thread's rank within it. Block 0 also
// zeroes `next` / `next_est` (the other chunk parity's counts, cursors and estimate sum: the next
// chunk's estimate adds into them; the previous chunk's scatter is done with them) and, for a fresh
// workload (hint != null), sets the launch's job size from the chunk's mean estimate: shares per
// integral for ~TASKS_PER_JOB tasks per job, as the end of an adaptive launch does from its measured
// tasks (a first launch of tiny trees with the default 16 shares had been seeding-bound, profiles/r05w).
__global__ __launch_bounds__(256) void k_batch_scatter(const double2* __restrict__ bounds, const unsigned* __restrict__ key_of,
                                                       int n, const unsigned* __restrict__ counts,
                                                       unsigned* __restrict__ cursor, double2* __restrict__ sorted,
                                                       unsigned* __restrict__ perm, unsigned* __restrict__ next,
                                                       const double* __restrict__ est_sum, double* __restrict__ next_est,
                                                       LaunchHint* __restrict__ hint, unsigned max_shares) {
    static_assert(EST_KEYS == 256, "one class per thread of the block (the scan below)");
    __shared__ unsigned s_off[EST_KEYS], s_cnt[EST_KEYS], s_base[EST_KEYS];
    const unsigned t = threadIdx.x;
    if (blockIdx.x == 0) {
        for (unsigned i = t; i < 2u * EST_KEYS; i += blockDim.x) next[i] = 0u;
        if (t == 0) {
            *next_est = 0.0;
            if (hint) {
                const double per = EST_TASKS * *est_sum / (double)max(n, 1);   // predicted tasks per integral
                const double sh = floor((per + 0.5 * TASKS_PER_JOB) / TASKS_PER_JOB);
                hint->shares_next = (unsigned)fmin(fmax(sh, 1.0), (double)max_shares);
                hint->per_next = (unsigned long long)fmax(per, 0.0);
            }
        }
    }
    // the classes' offsets: an exclusive scan of the counts, one class per thread (Hillis-Steele in LDS)
    s_cnt[t] = 0u;
    s_off[t] = counts[t];
    __syncthreads();
    for (unsigned d = 1; d < (unsigned)EST_KEYS; d <<= 1) {
        const unsigned v = t >= d ? s_off[t - d] : 0u;
        __syncthreads();
        s_off[t] += v;
        __syncthreads();
    }
    s_base[t] = t ? s_off[t - 1] : 0u;   // inclusive -> exclusive
    __syncthreads();
    s_off[t] = s_base[t];
    __syncthreads();
    const int i = (int)(blockIdx.x * blockDim.x + t);
    unsigned key = 0, rank = 0;
    if (i < n) {
        key = key_of[i];
        rank = atomicAdd(&s_cnt[key], 1u);
    }
    __syncthreads();
    if (t < EST_KEYS && s_cnt[t]) s_base[t] = s_off[t] + atomicAdd(&cursor[t], s_cnt[t]);
    __syncthreads();
    if (i < n) {
        const unsigned pos = s_base[key] + rank;
        sorted[pos] = bounds[i];
        perm[pos] = (unsigned)i;
    }
}

// ------------------------------------------------------------------------------------------------
// Level-synchronous breadth-first path: one launch per tree level (debug / cross-check schedule).
// ------------------------------------------------------------------------------------------------
struct Rec {
    double l, r, fl, fr;
};

template <int FID>
__global__ __launch_bounds__(64) void k_root(double a, double b, Rec* out, const ExpPair* __restrict__ gtab) {
    __shared__ ExpEntry tab[ftab_entries<FID>()];
    stage_f_table<FID>(tab, gtab);
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
                                               const ExpPair* __restrict__ gtab) {
    __shared__ ExpEntry tab[ftab_entries<FID>()];
    __shared__ double s_area[4];
    __shared__ unsigned s_cnt[2][4];
    stage_f_table<FID>(tab, gtab);
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

// Children are appended with ONE atomic per workgroup and chunk of LEVEL_R x 256 records: a wave-level
// atomic per 64 records had made the wide levels a serial fan-in on the one counter (cosh4 eps=1e-12,
// 1.65 M records: 25.8 k atomics, 202 us = 0.5 TB/s; profiles/r02t). Each lane takes LEVEL_R records
// of the chunk (coalesced, LEVEL_R F chains interleaved); the block's wave counts meet in LDS
// (double-buffered by chunk parity, so two barriers per chunk suffice).
#ifndef AQ_LEVEL_R
#define AQ_LEVEL_R 4
#endif
constexpr int LEVEL_R = AQ_LEVEL_R;
// Threads per block (a chunk of LEVEL_T x LEVEL_R records per append). r03 A/B over cosh4 eps=1e-12
// under rocprofv3 (tools/frontier_ab.sh; profiles/r03_ab/frontier_ab.txt): widest level 256 threads
// 33.5 us, 512 33.2, 1024 37.6, 1024 x 8 records 54.4; a decoupled look-back scan in place of the
// atomic (chunk-ordered output, wave-parallel look-back) 40.4 us -- the PRE frontier advances ~64
// chunks per L2 round trip while all 1.6 k chunks finish at once, slower than the atomics' fan-in.
#ifndef AQ_LEVEL_T
#define AQ_LEVEL_T 256
#endif
constexpr int LEVEL_T = AQ_LEVEL_T;
#ifndef AQ_LEVEL_HOIST
#define AQ_LEVEL_HOIST 0   // r03 A/B (profiles/r03q/front_ab.txt): widest level 32.4 -> 35.4 us with it -- off
#endif
constexpr int LEVEL_NW = LEVEL_T / 64;

template <int FID>
__global__ __launch_bounds__(LEVEL_T) void k_level_step(const Rec* __restrict__ in, unsigned n_in, Rec* __restrict__ out,
                                                    unsigned* __restrict__ n_out, unsigned cap_out, double eps,
                                                    int depth, int max_depth, LevelPart* __restrict__ parts,
                                                    const ExpPair* __restrict__ gtab,
                                                    const unsigned* __restrict__ n_in_dev) {
    constexpr int R = LEVEL_R;
    // chained levels: the count a previous step appended (read once; uniform), clamped to n_in = the
    // host's bound (<= the input buffer's capacity; a count beyond it was flagged as an overflow)
    if (n_in_dev) n_in = min(*n_in_dev, n_in);
    __shared__ ExpEntry tab[ftab_entries<FID>()];
    __shared__ double s_h[LEVEL_NW], s_l[LEVEL_NW];
    __shared__ unsigned s_t[LEVEL_NW], s_a[LEVEL_NW], s_e[LEVEL_NW];
    __shared__ unsigned s_wc[2][LEVEL_NW], s_base[2];
    const unsigned chunk = (unsigned)LEVEL_T * R;
    // the first chunk's records are requested BEFORE the exp table is staged (AQ_LEVEL_HOIST): a block
    // of a wide level runs one chunk, and the table's global read (then the barrier) had preceded every
    // record load, adding its latency to every block's
    Rec rn[R];
    bool an[R];
    auto load_chunk = [&](unsigned base) {
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const unsigned i = base + (unsigned)k * (unsigned)LEVEL_T + threadIdx.x;
            an[k] = i < n_in;
            rn[k] = an[k] ? in[i] : Rec{1.0, 1.0, 0.0, 0.0};
        }
    };
    if (AQ_LEVEL_HOIST && blockIdx.x * chunk < n_in) load_chunk(blockIdx.x * chunk);
    stage_f_table<FID>(tab, gtab);
    __syncthreads();
    double hi = 0.0, lo = 0.0;
    unsigned tasks = 0, leaves = 0, err = 0;
    const unsigned w = threadIdx.x >> 6;
    unsigned parity = 0;
    // the loop bound depends on blockIdx only: every thread of the block runs every chunk (barriers)
    for (unsigned base = blockIdx.x * chunk; base < n_in; base += gridDim.x * chunk, parity ^= 1u) {
        Rec rc[R];
        bool active[R];
        double x[R], f[R];
        if (!AQ_LEVEL_HOIST || base != blockIdx.x * chunk) load_chunk(base);
#pragma unroll
        for (int k = 0; k < R; ++k) {
            active[k] = an[k];
            rc[k] = rn[k];
            x[k] = (rc[k].l + rc[k].r) / 2;                              // :187
        }
        integrand_k<FID, R>(x, f, tab);                                  // :188
        bool refine[R];
        unsigned long long m[R];
        unsigned c[R + 1];
        c[0] = 0;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const double mid = x[k], fmid = f[k];
            const double lrarea = (rc[k].fl + rc[k].fr) * (rc[k].r - rc[k].l) / 2;   // :185
            const double larea = (rc[k].fl + fmid) * (mid - rc[k].l) / 2;            // :189
            const double rarea = (fmid + rc[k].fr) * (rc[k].r - mid) / 2;            // :190
            const bool ref = active[k] && fabs((larea + rarea) - lrarea) > eps;       // :191
            refine[k] = false;
            if (active[k]) {
                ++tasks;
                if (!ref) {
                    dd_add(hi, lo, larea + rarea);                       // :199 -> :149
                    ++leaves;
                } else if (depth + 1 >= max_depth) {
                    err |= ERRB_DEPTH;
                } else {
                    refine[k] = true;
                }
            }
            m[k] = __ballot(refine[k]);
            c[k + 1] = c[k] + (unsigned)__popcll(m[k]);
        }
        // the chunk's offset: one atomic per block and chunk
        if (lane_id() == 0) s_wc[parity][w] = c[R];
        __syncthreads();
        if (threadIdx.x == 0) {   // one atomic for the block's chunk
            unsigned tot = 0;
            for (int v = 0; v < LEVEL_NW; ++v) tot += s_wc[parity][v];
            s_base[parity] = tot ? atomicAdd(n_out, 2u * tot) : 0u;
        }
        __syncthreads();
        unsigned off = s_base[parity];
        for (unsigned v = 0; v < w; ++v) off += 2u * s_wc[parity][v];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            if (refine[k]) {
                const unsigned pos = off + 2u * (c[k] + mbcnt(m[k]));
                if (pos + 1 < cap_out) {
                    out[pos] = Rec{rc[k].l, x[k], rc[k].fl, f[k]};       // [l, mid]  (:192-194)
                    out[pos + 1] = Rec{x[k], rc[k].r, f[k], rc[k].fr};   // [mid, r]  (:195-197)
                } else {
                    err |= ERRB_OVERFLOW;
                }
            }
        }
    }
    wave_sum_dd(hi, lo);
    const unsigned wt = wave_sum_u(tasks), wl = wave_sum_u(leaves), we = wave_or_u(err);
    if (lane_id() == 0) { s_h[w] = hi; s_l[w] = lo; s_t[w] = wt; s_a[w] = wl; s_e[w] = we; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double H = 0.0, L = 0.0;
        unsigned T = 0, A = 0, E = 0;
        for (int k = 0; k < LEVEL_NW; ++k) { dd_add_dd(H, L, s_h[k], s_l[k]); T += s_t[k]; A += s_a[k]; E |= s_e[k]; }
        LevelPart p;
        p.hi = H; p.lo = L; p.tasks = (double)T; p.leaves = (double)A; p.err = (double)E;
        p.levels = T ? (double)(depth + 1) : 0.0;
        p.pad0 = p.pad1 = 0.0;
        parts[blockIdx.x] = p;
    }
}

// 256 threads each fold an interleaved share of the rows in row order, then a fixed pairwise tree
// (strides 128 .. 1) folds the 256 partials: the same order for a given row count (deterministic).
// One thread folding every row had cost 1.1 ms for the 4096 rows of a chained wide level, a serial
// fold of the 256 partials 18 us per level (profiles/r02u, r02v).
constexpr int FOLD_T = 256;
__global__ __launch_bounds__(FOLD_T) void k_level_fold(const LevelPart* __restrict__ parts, int nparts,
                                                       double* __restrict__ acc) {
    __shared__ double s_h[FOLD_T], s_l[FOLD_T], s_t[FOLD_T], s_a[FOLD_T], s_v[FOLD_T];
    __shared__ unsigned s_e[FOLD_T];
    const int t = threadIdx.x;
    double H = 0.0, L = 0.0, T = 0.0, A = 0.0, lev = 0.0;
    unsigned E = 0;
    for (int i = t; i < nparts; i += FOLD_T) {
        const LevelPart p = parts[i];
        dd_add_dd(H, L, p.hi, p.lo);
        T += p.tasks;
        A += p.leaves;
        E |= (unsigned)p.err;
        lev = fmax(lev, p.levels);
    }
    s_h[t] = H; s_l[t] = L; s_t[t] = T; s_a[t] = A; s_v[t] = lev; s_e[t] = E;
    __syncthreads();
    for (int s = FOLD_T / 2; s > 0; s >>= 1) {
        if (t < s) {
            double h = s_h[t], l = s_l[t];
            dd_add_dd(h, l, s_h[t + s], s_l[t + s]);
            s_h[t] = h; s_l[t] = l;
            s_t[t] += s_t[t + s];
            s_a[t] += s_a[t + s];
            s_v[t] = fmax(s_v[t], s_v[t + s]);
            s_e[t] |= s_e[t + s];
        }
        __syncthreads();
    }
    if (t != 0) return;
    H = acc[0]; L = acc[1];
    dd_add_dd(H, L, s_h[0], s_l[0]);
    acc[0] = H; acc[1] = L; acc[2] += s_t[0]; acc[3] += s_a[0];
    acc[4] = (double)((unsigned)acc[4] | s_e[0]);
    acc[5] = fmax(acc[5], s_v[0]);
}

// The frontier's narrow levels in ONE launch: a single workgroup runs `levels`
// consecutive levels, level depth + k reading counts[depth + k] records from buf[k & 1] and writing
// its children to buf[(k + 1) & 1] and their number to counts[depth + k + 1]. The appends need no
// global atomic (one block: a block-wide prefix of the wave counts in LDS), the levels no host round
// trip and no launch each (the tree's first ~13 levels hold <= 8 k records: launch- and
// latency-bound as one launch per level, 2 launches each with the fold). The block's accumulators go
// into d_acc once at the end, as k_level_fold's would.
constexpr int NARROW_T = 1024;
template <int FID>
__global__ __launch_bounds__(NARROW_T) void k_level_narrow(Rec* __restrict__ buf0, Rec* __restrict__ buf1, unsigned cap,
                                                           unsigned* __restrict__ counts, int d0, int levels, double eps,
                                                           int max_depth, double* __restrict__ acc,
                                                           const ExpPair* __restrict__ gtab) {
    constexpr int NWV = NARROW_T / 64;
    __shared__ ExpEntry tab[ftab_entries<FID>()];
    __shared__ unsigned s_wc[NWV];
    __shared__ unsigned s_n;
    __shared__ double s_h[NWV], s_l[NWV];
    __shared__ unsigned s_t[NWV], s_a[NWV], s_e[NWV], s_v[NWV];
    stage_f_table<FID>(tab, gtab);
    if (threadIdx.x == 0) s_n = min(counts[d0], cap);
    __syncthreads();
    double hi = 0.0, lo = 0.0;
    unsigned tasks = 0, leaves = 0, err = 0, lev = 0;
    const unsigned w = threadIdx.x >> 6;
    for (int k = 0; k < levels; ++k) {
        const int depth = d0 + k;
        const Rec* __restrict__ in = (k & 1) ? buf1 : buf0;
        Rec* __restrict__ out = (k & 1) ? buf0 : buf1;
        const unsigned n_in = s_n;
        unsigned n_ref = 0;   // refining records of this level so far (block-uniform)
        for (unsigned base = 0; base < n_in; base += NARROW_T) {
            const unsigned i = base + threadIdx.x;
            const bool active = i < n_in;
            const Rec rc = active ? in[i] : Rec{1.0, 1.0, 0.0, 0.0};
            double x[1] = {(rc.l + rc.r) / 2}, f[1];                       // :187
            integrand_k<FID, 1>(x, f, tab);                                 // :188
            const double lrarea = (rc.fl + rc.fr) * (rc.r - rc.l) / 2;      // :185
            const double larea = (rc.fl + f[0]) * (x[0] - rc.l) / 2;        // :189
            const double rarea = (f[0] + rc.fr) * (rc.r - x[0]) / 2;        // :190
            bool refine = false;
            if (active) {
                ++tasks;
                lev = max(lev, (unsigned)depth + 1u);
                if (!(fabs((larea + rarea) - lrarea) > eps)) {              // :191
                    dd_add(hi, lo, larea + rarea);                          // :199 -> :149
                    ++leaves;
                } else if (depth + 1 >= max_depth) {
                    err |= ERRB_DEPTH;
                } else {
                    refine = true;
                }
            }
            const unsigned long long m = __ballot(refine);
            if (lane_id() == 0) s_wc[w] = (unsigned)__popcll(m);
            __syncthreads();
            unsigned off = n_ref, tot = 0;
            for (unsigned v = 0; v < (unsigned)NWV; ++v) {
                const unsigned c = s_wc[v];
                off += v < w ? c : 0u;
                tot += c;
            }
            __syncthreads();   // s_wc is rewritten by the next chunk
            if (refine) {
                const unsigned pos = 2u * (off + mbcnt(m));
                if (pos + 1 < cap) {
                    out[pos] = Rec{rc.l, x[0], rc.fl, f[0]};        // [l, mid]  (:192-194)
                    out[pos + 1] = Rec{x[0], rc.r, f[0], rc.fr};    // [mid, r]  (:195-197)
                } else {
                    err |= ERRB_OVERFLOW;
                }
            }
            n_ref += tot;
        }
        __syncthreads();   // the level's children are written (and visible to the block) before the next reads them
        if (threadIdx.x == 0) {
            counts[depth + 1] = 2u * n_ref;
            s_n = min(2u * n_ref, cap);
        }
        __syncthreads();
    }
    wave_sum_dd(hi, lo);
    const unsigned wt = wave_sum_u(tasks), wl = wave_sum_u(leaves), we = wave_or_u(err), wv = wave_max_u(lev);
    if (lane_id() == 0) { s_h[w] = hi; s_l[w] = lo; s_t[w] = wt; s_a[w] = wl; s_e[w] = we; s_v[w] = wv; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double H = acc[0], L = acc[1];
        unsigned T = 0, A = 0, E = 0, V = 0;
        for (int v = 0; v < NWV; ++v) {
            dd_add_dd(H, L, s_h[v], s_l[v]);
            T += s_t[v]; A += s_a[v]; E |= s_e[v]; V = max(V, s_v[v]);
        }
        acc[0] = H; acc[1] = L; acc[2] += (double)T; acc[3] += (double)A;
        acc[4] = (double)((unsigned)acc[4] | E);
        acc[5] = fmax(acc[5], (double)V);
    }
}

template <int FID>
__global__ __launch_bounds__(64) void k_frontier_root(double a, double b, Rec* out, const ExpPair* __restrict__ gtab) {
    __shared__ ExpEntry tab[ftab_entries<FID>()];
    stage_f_table<FID>(tab, gtab);
    __syncthreads();
    if (threadIdx.x == 0) out[0] = Rec{a, b, integrand<FID>(a, tab), integrand<FID>(b, tab)};
}

// Gather n slots' totals into a caller device buffer as f64 [area, tasks, accepted, error] rows,
// ready for one collective (counts are exact in f64 below 2^53). One thread per slot: the area is
// the correctly rounded value of the slot's exact accumulator.
__global__ __launch_bounds__(64) void k_gather(const Ctl* __restrict__ ctls, const unsigned long long* __restrict__ parts,
                                               int grid, int first, int n, int nslots, double* __restrict__ out) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const int slot = (first + i) % nslots;
    const Ctl& c = ctls[slot];
    const Counts k = slot_counts(c.sums, parts + 2 * parts_row(slot) * grid, grid);
    double* o = out + 4 * (size_t)i;
    o[0] = xs_round(c.area);
    o[1] = (double)k.tasks;
    o[2] = (double)k.leaves;
    o[3] = (double)c.sums.error;
}

// The batch front end's gather (aq_integrate_batch): k_gather's rows, then every slot back to the
// all-zero state the next launch needs -- its sums and the limbs of its window, the only ones any flush
// added to (SlotSums win_lo_not / win_hi) -- so no k_reset runs before the next chunk's launch on the
// same slots, and only a slot's touched lines are read and written (k_gather + k_reset read and wrote
// all 68 limbs of every slot: 115 + 76 us per 262144-slot chunk, profiles/r05a/c3_timeline_r04code.json).
constexpr int GATHER_WIN = 16;   // limbs a window may span to take the short path (a cosh4 tree: ~4-6)
// perm (size-ordered batch chunks): slot i holds integral perm[i], whose row it writes.
__global__ __launch_bounds__(64) void k_gather_reset(Ctl* __restrict__ ctls, const unsigned long long* __restrict__ parts,
                                                     int grid, int first, int n, double* __restrict__ out,
                                                     const unsigned* __restrict__ perm) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const int slot = first + i;
    Ctl& c = ctls[slot];
    const SlotSums sm = c.sums;
    const Counts k = slot_counts(sm, parts + 2 * parts_row(slot) * grid, grid);
    const int lo = sm.win_hi ? (int)~sm.win_lo_not : 0;
    const int hi = sm.win_hi ? min((int)sm.win_hi, XS_LIMBS) : 0;
    double area;
    if (hi - lo <= GATHER_WIN) {
        long long w[GATHER_WIN];
#pragma unroll
        for (int j = 0; j < GATHER_WIN; ++j) w[j] = lo + j < hi ? c.area.limb[lo + j] : 0ll;
        area = xs_round_span<GATHER_WIN>(w, hi - lo, XS_E0 + 32 * lo);
#pragma unroll
        for (int j = 0; j < GATHER_WIN; ++j)
            if (lo + j < hi) c.area.limb[lo + j] = 0ll;
    } else {
        area = xs_round(c.area);
        for (int j = 0; j < XS_LIMBS; ++j) c.area.limb[j] = 0ll;
    }
    double* o = out + 4 * (size_t)(perm ? perm[i] : (unsigned)i);
    o[0] = area;
    o[1] = (double)k.tasks;
    o[2] = (double)k.leaves;
    o[3] = (double)sm.error;
    c.sums = SlotSums{};
}

// The same slots as exact int64 rows (AQ_EXACT_ROW each): limbs, tasks, accepted, spilled,
// levels | error << 32. Sums of such rows (an int64 all-reduce) keep the area exact.
__global__ __launch_bounds__(64) void k_gather_exact(const Ctl* __restrict__ ctls,
                                                     const unsigned long long* __restrict__ parts, int grid, int first,
                                                     int n, int nslots, long long* __restrict__ out) {
    const int i = (int)blockIdx.x;
    if (i >= n) return;
    const int slot = (first + i) % nslots;
    const Ctl& c = ctls[slot];
    long long* o = out + (size_t)AQ_EXACT_ROW * i;
    for (int k = threadIdx.x; k < XS_LIMBS; k += blockDim.x) o[k] = c.area.limb[k];
    if (threadIdx.x == 0) {
        const Counts k = slot_counts(c.sums, parts + 2 * parts_row(slot) * grid, grid);
        o[XS_LIMBS] = (long long)k.tasks;
        o[XS_LIMBS + 1] = (long long)k.leaves;
        o[XS_LIMBS + 2] = (long long)c.sums.spilled;
        o[XS_LIMBS + 3] = (long long)k.levels | ((long long)c.sums.error << 32);
    }
}

// PCU_AREA (aq_stream.h): add the exact sum of a per-CU launch's workgroup area words -- 2 x grid doubles,
// one double-double per workgroup -- to sx[XS_LIMBS] (block-shared). Every thread of the block calls it
// between barriers; LDS int64 atomics keep the sum exact in any order.
__device__ __forceinline__ void add_wg_area(long long* sx, const double* __restrict__ pa, int grid) {
    for (int i = threadIdx.x; i < 2 * grid; i += blockDim.x) {
        XDigits g;
        if (xs_digits(pa[i], g)) {
#pragma unroll
            for (int k = 0; k < 3; ++k)
                if (g.d[k]) atomicAdd(reinterpret_cast<unsigned long long*>(&sx[g.i + k]), (unsigned long long)g.d[k]);
        }
    }
}

// After an asynchronous per-CU launch of k integrals (slots first .. first + k - 1; pa: the launch's area
// row, integral b's words at pa + 2 * b * grid): each slot's workgroup areas into its exact accumulator,
// one workgroup per slot -- every reader (k_gather*, aq_fetch*) then sees the whole area in the slot.
__global__ __launch_bounds__(256) void k_fold_parts(Ctl* __restrict__ ctls, const double* __restrict__ pa, int grid,
                                                    int first) {
    __shared__ long long sx[XS_LIMBS];
    for (int i = threadIdx.x; i < XS_LIMBS; i += blockDim.x) sx[i] = 0;
    __syncthreads();
    add_wg_area(sx, pa + 2 * (size_t)blockIdx.x * grid, grid);
    __syncthreads();
    Ctl& c = ctls[first + (int)blockIdx.x];
    for (int i = threadIdx.x; i < XS_LIMBS; i += blockDim.x)
        if (sx[i]) c.area.limb[i] += sx[i];
}

// Return slots [first, first + n) to the all-zero state a launch needs: sums and the exact area
// accumulator; the histograms when they were written.
__global__ __launch_bounds__(128) void k_reset(Ctl* __restrict__ ctls, int first, int zero_hist) {
    Ctl& c = ctls[first + (int)blockIdx.x];
    for (int i = threadIdx.x; i < XS_LIMBS; i += blockDim.x) c.area.limb[i] = 0;
    if (zero_hist)
        for (int i = threadIdx.x; i < 2 * AQ_MAX_LEVELS; i += blockDim.x) c.hist[i] = 0ull;
    if (threadIdx.x == 0) {
        c.sums = SlotSums{};
    }
}

// The synchronous path's read-back (aq_integrate / aq_integrate_shard): one workgroup copies the
// internal sync slot's result -- sums, exact limbs, the per-workgroup words of a per-CU launch, the
// histograms when written -- straight into pinned host memory, then zeroes the slot for the next
// call. One small launch in place of a reset kernel, a memset and three or four device-to-host
// copies around every call.
struct SyncOut {
    unsigned long long seq;   // the call's sequence number, stored last (the host waits on it)
    SlotSums sums;
    XSum area;
    unsigned long long hist[2 * AQ_MAX_LEVELS];
    unsigned long long parts[2 * MAXG];
};
__global__ __launch_bounds__(256) void k_fetch_sync(Ctl* __restrict__ c, unsigned long long* __restrict__ parts,
                                                    const double* __restrict__ parea, int grid, int with_parts,
                                                    int with_hist, SyncOut* __restrict__ out,
                                                    unsigned long long seq) {
    const int t = threadIdx.x;
    __shared__ long long sx[XS_LIMBS];
    if (t == 0) out->sums = c->sums;
    for (int i = t; i < XS_LIMBS; i += blockDim.x) sx[i] = c->area.limb[i];
    __syncthreads();
    if (with_parts) add_wg_area(sx, parea, grid);   // a per-CU launch's workgroup areas (PCU_AREA)
    __syncthreads();
    for (int i = t; i < XS_LIMBS; i += blockDim.x) out->area.limb[i] = sx[i];
    if (with_hist)
        for (int i = t; i < 2 * AQ_MAX_LEVELS; i += blockDim.x) out->hist[i] = c->hist[i];
    if (with_parts)
        for (int i = t; i < 2 * grid; i += blockDim.x) out->parts[i] = parts[i];
    __syncthreads();   // every read precedes the zeroing
    if (t == 0) c->sums = SlotSums{};
    for (int i = t; i < XS_LIMBS; i += blockDim.x) c->area.limb[i] = 0;
    if (with_hist)
        for (int i = t; i < 2 * AQ_MAX_LEVELS; i += blockDim.x) c->hist[i] = 0ull;
    if (with_parts)
        for (int i = t; i < 2 * grid; i += blockDim.x) parts[i] = 0ull;
    // the result is complete in host memory: every thread's stores made visible system-wide, then the
    // sequence number released. The host sees it before the kernel's completion signal would arrive
    __threadfence_system();
    __syncthreads();
    if (t == 0) __hip_atomic_store(&out->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// aq_integrate_group: one rank's contribution to the RCCL exchange. sum_row (int64, summed over
// ranks): limbs, tasks, accepted, spilled. info (gathered from every rank): tasks, levels, error,
// then the rank's per-workgroup pack_cu words (grid of them; zero when not kept).
__global__ __launch_bounds__(256) void k_pack_group(const Ctl* __restrict__ ctls, const unsigned long long* parts,
                                                    const double* __restrict__ parea, int slot, int grid, int with_parts,
                                                    long long* __restrict__ sum_row, unsigned long long* __restrict__ info) {
    const Ctl& c = ctls[slot];
    const unsigned long long* wp = parts + 2 * parts_row(slot) * grid;
    __shared__ long long sx[XS_LIMBS];
    for (int k = threadIdx.x; k < XS_LIMBS; k += blockDim.x) sx[k] = c.area.limb[k];
    __syncthreads();
    if (with_parts) add_wg_area(sx, parea + 2 * parts_row(slot) * grid, grid);   // PCU_AREA
    __syncthreads();
    for (int k = threadIdx.x; k < XS_LIMBS; k += blockDim.x) sum_row[k] = sx[k];
    for (int k = threadIdx.x; k < grid; k += blockDim.x) info[3 + k] = with_parts ? wp[2 * k] : 0ull;
    if (threadIdx.x == 0) {
        const Counts k = slot_counts(c.sums, wp, grid);
        sum_row[XS_LIMBS] = (long long)k.tasks;
        sum_row[XS_LIMBS + 1] = (long long)k.leaves;
        sum_row[XS_LIMBS + 2] = (long long)c.sums.spilled;
        info[0] = k.tasks;
        info[1] = k.levels;
        info[2] = c.sums.error;
    }
}

}  // namespace aq

#include "aq_abi.inc"   // host side: the C ABI (include/aquad.h)
