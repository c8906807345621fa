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

enum : unsigned { ERRB_TIMEOUT = 1, ERRB_OVERFLOW = 2, ERRB_DEPTH = 4 };

// Persistent-path control block (one per context). Valid between launches: the last workgroup
// of every launch publishes the totals into the launch's SlotOut and resets this block, so a
// launch needs no memset in front of it (each memset would be one more dispatch per integral).
struct Ctl {
    unsigned q_tail;           // chunk slots claimed by producers
    unsigned q_head;           // tickets taken by idle workgroups
    int q_tokens;              // busy workgroups + records in published, unconsumed chunks (= G at launch)
    unsigned exited;           // workgroups that have flushed their accumulators
    double area;
    unsigned long long tasks;
    unsigned long long leaves;
    unsigned long long spilled;
    unsigned levels;
    unsigned error;
    unsigned pad[2];
    unsigned long long hist[2 * AQ_MAX_LEVELS];   // [0,L): tasks per level, [L,2L): accepted per level
};

constexpr int MAXG = 2048;     // max persistent workgroups per launch
struct SlotOut {               // fully rewritten by every launch that targets the slot
    double area;
    unsigned long long tasks;
    unsigned long long leaves;
    unsigned long long spilled;
    unsigned levels;
    unsigned error;
    unsigned nwg;
    unsigned epoch;
    unsigned long long hist[2 * AQ_MAX_LEVELS];
    unsigned wg_cu[MAXG];                         // hardware CU slot of workgroup i
    unsigned long long wg_tasks[MAXG];            // tasks evaluated by workgroup i
};

// Hardware CU slot of the executing wave: xcc*256 + (se*2 + sh)*16 + cu (HW_ID / XCC_ID registers).
__device__ __forceinline__ unsigned cu_slot() {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID, 32 bits
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID, bits 3:0
    const unsigned cu = (hw >> 8) & 15u, sh = (hw >> 12) & 1u, se = (hw >> 13) & 7u;
    return ((xcc & 7u) << 8) | (((se << 1) | sh) << 4) | cu;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ unsigned wave_sum_u(unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ unsigned wave_max_u(unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (unsigned)__shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ unsigned lane_id() { return __lane_id(); }
__device__ __forceinline__ unsigned mbcnt(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// One trapezoid step of the reference (aquadPartA.c:185-191) on a record that carries F(l), F(r).
// The operand order and association are the reference's; '/2' is exact (scaling by 2^-1).
struct Step {
    double mid, fmid, larea, rarea;
    bool refine;
};
template <int FID>
__device__ __forceinline__ Step task_step(double l, double r, double fl, double fr, double eps,
                                          const ExpEntry* __restrict__ tab) {
    Step s;
    const double lrarea = (fl + fr) * (r - l) / 2;   // :185
    s.mid = (l + r) / 2;                             // :187
    s.fmid = integrand<FID>(s.mid, tab);             // :188
    s.larea = (fl + s.fmid) * (s.mid - l) / 2;       // :189
    s.rarea = (s.fmid + fr) * (r - s.mid) / 2;       // :190
    s.refine = fabs((s.larea + s.rarea) - lrarea) > eps;  // :191 (strict >)
    return s;
}

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

// ------------------------------------------------------------------------------------------------
// Persistent on-device farmer.
// ------------------------------------------------------------------------------------------------
constexpr int PT = 512;             // threads per workgroup (8 waves, 2 per SIMD)
constexpr int PW = PT / 64;         // waves per workgroup
constexpr int CAP = 4096;           // LDS ring capacity, records (power of two)
constexpr int CMASK = CAP - 1;
constexpr int CH = 512;             // records per HBM queue chunk
constexpr int S_POS = 5;            // 2^S_POS seed positions per virtual worker (32..63 dealt)
constexpr int DONATE_MIN = 64;      // a busy workgroup donates only from stacks at least this deep

struct Chunk {                      // SoA, one queue slot
    double l[CH], r[CH], fl[CH], fr[CH];
    unsigned char d[CH];
    unsigned count;
    unsigned pad[15];
};

struct PersistParams {
    double a, b, eps, fa_unused;
    int max_depth;
    int shard, nshards;
    int D;                          // seed depth
    unsigned epoch;                 // tags queue slots of this call (ready[s] == epoch)
    unsigned qcap;                  // queue slots
    unsigned long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
    Ctl* ctl;
    SlotOut* out;
    Chunk* chunks;
    unsigned* ready;
    const ExpEntry* gtab;
};

__device__ __forceinline__ unsigned long long rtc() { return __builtin_amdgcn_s_memrealtime(); }

template <int FID, bool HIST>
__global__ __launch_bounds__(PT) void k_persist(PersistParams P) {
    __shared__ double s_l[CAP], s_r[CAP], s_fl[CAP], s_fr[CAP];
    __shared__ unsigned char s_d[CAP];
    __shared__ ExpEntry tab[128];
    __shared__ unsigned s_wcnt[PW];
    __shared__ int s_cmd[4];
    __shared__ double s_red[PW];
    __shared__ unsigned s_redu[3][PW];
    __shared__ unsigned s_hist[HIST ? 2 * AQ_MAX_LEVELS : 1];

    const unsigned tid = threadIdx.x;
    const unsigned lane = lane_id();
    const unsigned wid = tid >> 6;
    Ctl* __restrict__ ctl = P.ctl;
    stage_exp_table(tab, P.gtab);
    if (HIST)
        for (unsigned i = tid; i < 2 * AQ_MAX_LEVELS; i += PT) s_hist[i] = 0;

    const double eps = P.eps;
    const int max_depth = P.max_depth;
    double my_area = 0.0;
    unsigned my_tasks = 0, my_leaves = 0, my_maxd = 0;
    unsigned err = 0;

    // ---------------- seeding: path walk to this worker's depth-D positions ----------------
    const unsigned V = gridDim.x * (unsigned)P.nshards;
    const unsigned vwg = blockIdx.x * (unsigned)P.nshards + (unsigned)P.shard;
    const int D = P.D;
    const unsigned long long npos_total = 1ull << D;
    const unsigned nbands = (unsigned)((npos_total + V - 1) / V);
    // position of band k (snake order): k*V + (k odd ? V-1-vwg : vwg), valid if < 2^D
    auto position = [&](unsigned k, bool& valid) -> unsigned long long {
        const unsigned long long o = (k & 1u) ? (unsigned long long)(V - 1 - vwg) : (unsigned long long)vwg;
        const unsigned long long j = (unsigned long long)k * V + o;
        valid = j < npos_total;
        return j;
    };
    double* fm = s_fl;  // F(mid) of ancestor (d, k) at fm[d*nbands + k]; stack is empty now
    __syncthreads();
    double fa, fb;
    {
        // F(A), F(B): every lane needs them in the decision pass; lane-redundant evaluation is
        // cheaper than a broadcast round.
        fa = integrand<FID>(P.a, tab);
        fb = integrand<FID>(P.b, tab);
    }
    for (unsigned q = tid; q < (unsigned)D * nbands; q += PT) {
        const unsigned d = q / nbands, k = q % nbands;
        bool valid;
        const unsigned long long p = position(k, valid);
        double x = 0.0;
        if (valid) {
            const unsigned long long anc = p >> (D - (int)d);
            double l = P.a, r = P.b;
            for (int i = 0; i < (int)d; ++i) {
                const double m = (l + r) / 2;
                if ((anc >> (d - 1 - i)) & 1ull) l = m; else r = m;
            }
            x = integrand<FID>((l + r) / 2, tab);
        }
        fm[q] = x;
    }
    __syncthreads();
    // decision pass: wave 0, lane k = band k (nbands <= 64)
    bool seed_alive = false;
    double sl = 0, sr = 0, sfl = 0, sfr = 0;
    if (wid == 0) {
        const unsigned k = lane;
        bool valid = false;
        const unsigned long long p = (k < nbands) ? position(k, valid) : 0ull;
        bool alive = valid;
        double l = P.a, r = P.b, fl = fa, fr = fb;
        for (int d = 0; d < D; ++d) {
            if (alive) {
                const double mid = (l + r) / 2;
                const double fmid = fm[(unsigned)d * nbands + k];
                const double lrarea = (fl + fr) * (r - l) / 2;
                const double larea = (fl + fmid) * (mid - l) / 2;
                const double rarea = (fmid + fr) * (r - mid) / 2;
                const bool refine = fabs((larea + rarea) - lrarea) > eps;
                const bool owner = (p & ((1ull << (D - d)) - 1ull)) == 0ull;
                if (owner) {
                    ++my_tasks;
                    my_maxd = max(my_maxd, (unsigned)d + 1u);
                    if (HIST) atomicAdd(&s_hist[d], 1u);
                }
                if (!refine) {
                    if (owner) {
                        my_area += larea + rarea;
                        ++my_leaves;
                        if (HIST) atomicAdd(&s_hist[AQ_MAX_LEVELS + d], 1u);
                    }
                    alive = false;
                } else if (d + 1 >= max_depth) {
                    if (owner) err |= ERRB_DEPTH;
                    alive = false;
                } else if ((p >> (D - 1 - d)) & 1ull) {
                    l = mid;
                    fl = fmid;
                } else {
                    r = mid;
                    fr = fmid;
                }
            }
        }
        seed_alive = alive;
        sl = l; sr = r; sfl = fl; sfr = fr;
    }
    __syncthreads();  // fm (aliases s_fl) fully consumed
    unsigned top = 0, bot = 0;  // ring indices (uniform across the workgroup)
    if (wid == 0) {
        const unsigned long long m = __ballot(seed_alive);
        if (seed_alive) {
            const unsigned pos = mbcnt(m);
            s_l[pos] = sl; s_r[pos] = sr; s_fl[pos] = sfl; s_fr[pos] = sfr;
            s_d[pos] = (unsigned char)D;
        }
        if (lane == 0) s_cmd[0] = (int)__popcll(m);
    }
    __syncthreads();
    top = (unsigned)s_cmd[0];

    // ---------------- main loop ----------------
    const unsigned long long t0 = rtc();
    unsigned seen_head = 0, seen_tail = 0;   // thread 0 only
    unsigned long long spilled = 0;         // thread 0 only
    bool busy = true;                       // holds a token
    const unsigned my_slot = cu_slot();
    (void)my_slot;

    for (;;) {
        unsigned size = top - bot;
        if (size == 0) {
            // ---- idle: take a ticket, wait for a chunk or for global termination ----
            if (tid == 0) {
                if (busy) {
                    __hip_atomic_fetch_add(&ctl->q_tokens, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    busy = false;
                }
                const unsigned h = __hip_atomic_fetch_add(&ctl->q_head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                int cmd = -1;  // -1 exit, -2 error exit, else slot
                for (unsigned spins = 0;; ++spins) {
                    if (h < P.qcap) {
                        const unsigned v = __hip_atomic_load(&P.ready[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (v == P.epoch) { cmd = (int)h; break; }
                    }
                    const int tk = __hip_atomic_load(&ctl->q_tokens, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (tk == 0) { cmd = -1; break; }
                    if ((spins & 63u) == 63u && rtc() - t0 > P.timeout_ticks) { err |= ERRB_TIMEOUT; cmd = -2; break; }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (cmd >= 0) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    s_cmd[1] = (int)P.chunks[cmd].count;
                }
                s_cmd[0] = cmd;
            }
            __syncthreads();
            const int cmd = s_cmd[0];
            if (cmd < 0) break;
            const unsigned k = (unsigned)s_cmd[1];
            const Chunk* __restrict__ c = P.chunks + cmd;
            for (unsigned i = tid; i < k; i += PT) {
                s_l[i] = c->l[i]; s_r[i] = c->r[i]; s_fl[i] = c->fl[i]; s_fr[i] = c->fr[i]; s_d[i] = c->d[i];
            }
            bot = 0;
            top = k;
            if (tid == 0) {
                // take one token for being busy, release the chunk's k record tokens
                __hip_atomic_fetch_add(&ctl->q_tokens, 1 - (int)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                busy = true;
            }
            __syncthreads();
            continue;
        }

        // ---- busy: decide whether to hand out work (spill when full, donate to waiters) ----
        if (tid == 0) {
            int cmd = -1;
            unsigned k = 0;
            if (size > (unsigned)(CAP - PT)) {
                const unsigned s = __hip_atomic_fetch_add(&ctl->q_tail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                k = min((unsigned)CH, size - (unsigned)(CAP - PT) + (unsigned)PT);
                k = min(k, size);
                if (s < P.qcap) cmd = (int)s; else { err |= ERRB_OVERFLOW; cmd = -3; }
            } else if ((int)(seen_head - seen_tail) > 0 && size >= (unsigned)DONATE_MIN) {
                unsigned expect = seen_tail;
                if (__hip_atomic_compare_exchange_strong(&ctl->q_tail, &expect, seen_tail + 1u, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    k = min((unsigned)CH, size / 2u);
                    if (seen_tail < P.qcap) cmd = (int)seen_tail; else { err |= ERRB_OVERFLOW; cmd = -3; }
                }
            }
            if (cmd >= 0) {
                // tokens for the k records before the chunk becomes visible
                __hip_atomic_fetch_add(&ctl->q_tokens, (int)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                spilled += k;
            }
            s_cmd[2] = cmd;
            s_cmd[3] = (int)k;
            // refresh the queue view for the next decision (consumed at the next round's start)
            seen_head = __hip_atomic_load(&ctl->q_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            seen_tail = __hip_atomic_load(&ctl->q_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        {
            const int cmd = s_cmd[2];
            const unsigned k = (unsigned)s_cmd[3];
            if (cmd >= 0) {
                Chunk* __restrict__ c = P.chunks + cmd;
                for (unsigned i = tid; i < k; i += PT) {
                    const unsigned j = (bot + i) & CMASK;
                    c->l[i] = s_l[j]; c->r[i] = s_r[j]; c->fl[i] = s_fl[j]; c->fr[i] = s_fr[j]; c->d[i] = s_d[j];
                }
                if (tid == 0) c->count = k;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (tid == 0) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_store(&P.ready[cmd], P.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                bot += k;
                continue;  // re-evaluate size
            } else if (cmd == -3) {
                // queue overflow: drop records (result invalid, error reported)
                bot += k;
                continue;
            }
        }

        // ---- one round: pop up to PT records from the top, evaluate, push children ----
        const unsigned n = min(size, (unsigned)PT);
        const unsigned b0 = top - n;
        double l = 0, r = 0, fl = 0, fr = 0;
        unsigned d = 0;
        const bool active = tid < n;
        if (active) {
            const unsigned j = (b0 + tid) & CMASK;
            l = s_l[j]; r = s_r[j]; fl = s_fl[j]; fr = s_fr[j]; d = s_d[j];
        }
        __syncthreads();  // popped region read before children overwrite it
        bool refine = false;
        double mid = 0, fmid = 0;
        if (active) {
            const Step s = task_step<FID>(l, r, fl, fr, eps, tab);
            mid = s.mid;
            fmid = s.fmid;
            ++my_tasks;
            my_maxd = max(my_maxd, d + 1u);
            if (HIST) atomicAdd(&s_hist[d], 1u);
            if (s.refine) {
                if ((int)d + 1 >= max_depth) {
                    err |= ERRB_DEPTH;
                } else {
                    refine = true;
                }
            } else {
                my_area += s.larea + s.rarea;  // :199 -> :149
                ++my_leaves;
                if (HIST) atomicAdd(&s_hist[AQ_MAX_LEVELS + d], 1u);
            }
        }
        const unsigned long long mask = __ballot(refine);
        if (lane == 0) s_wcnt[wid] = (unsigned)__popcll(mask);
        __syncthreads();
        unsigned pre = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < PW; ++w) {
            const unsigned c = s_wcnt[w];
            pre += (w < (int)wid) ? c : 0u;
            tot += c;
        }
        if (refine) {
            const unsigned pos = b0 + 2u * (pre + mbcnt(mask));
            const unsigned j0 = pos & CMASK, j1 = (pos + 1u) & CMASK;
            const unsigned char cd = (unsigned char)(d + 1u);
            s_l[j0] = l;   s_r[j0] = mid; s_fl[j0] = fl;   s_fr[j0] = fmid; s_d[j0] = cd;  // [l,mid]  :192-194
            s_l[j1] = mid; s_r[j1] = r;   s_fl[j1] = fmid; s_fr[j1] = fr;   s_d[j1] = cd;  // [mid,r]  :195-197
        }
        top = b0 + 2u * tot;
        __syncthreads();
    }

    // ---------------- exit: flush this workgroup's accumulators ----------------
    const double wa = wave_sum(my_area);
    const unsigned wt = wave_sum_u(my_tasks), wl = wave_sum_u(my_leaves), wm = wave_max_u(my_maxd);
    if (lane == 0) {
        s_red[wid] = wa;
        s_redu[0][wid] = wt;
        s_redu[1][wid] = wl;
        s_redu[2][wid] = wm;
    }
    if (err) atomicOr(&ctl->error, err);
    __syncthreads();
    if (tid == 0) {
        double ba = 0.0;
        unsigned bt = 0, bl = 0, bm = 0;
        for (int w = 0; w < PW; ++w) {
            ba += s_red[w];
            bt += s_redu[0][w];
            bl += s_redu[1][w];
            bm = max(bm, s_redu[2][w]);
        }
        if (bt) {
            atomicAdd(&ctl->area, ba);
            atomicAdd(&ctl->tasks, (unsigned long long)bt);
            atomicAdd(&ctl->leaves, (unsigned long long)bl);
            atomicMax(&ctl->levels, bm);
        }
        if (spilled) atomicAdd(&ctl->spilled, spilled);
        P.out->wg_cu[blockIdx.x] = cu_slot();
        P.out->wg_tasks[blockIdx.x] = bt;
    }
    if (HIST) {
        for (unsigned i = tid; i < 2 * AQ_MAX_LEVELS; i += PT) {
            const unsigned v = s_hist[i];
            if (v) atomicAdd(&ctl->hist[i], (unsigned long long)v);
        }
    }
    // last workgroup out publishes the totals and resets the control block for the next launch
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(&ctl->exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_cmd[0] = (old == gridDim.x - 1u) ? 1 : 0;
        if (old == gridDim.x - 1u) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (s_cmd[0]) {
        SlotOut* __restrict__ o = P.out;
        if (HIST) {
            for (unsigned i = tid; i < 2 * AQ_MAX_LEVELS; i += PT) {
                o->hist[i] = __hip_atomic_load(&ctl->hist[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&ctl->hist[i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (tid == 0) {
            unsigned long long* area_bits = reinterpret_cast<unsigned long long*>(&ctl->area);
            o->area = __longlong_as_double(
                (long long)__hip_atomic_load(area_bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            o->tasks = __hip_atomic_load(&ctl->tasks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            o->leaves = __hip_atomic_load(&ctl->leaves, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            o->spilled = __hip_atomic_load(&ctl->spilled, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            o->levels = __hip_atomic_load(&ctl->levels, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            o->error = __hip_atomic_load(&ctl->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            o->nwg = gridDim.x;
            o->epoch = P.epoch;
            __hip_atomic_store(area_bits, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl->tasks, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl->leaves, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl->spilled, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl->levels, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl->error, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl->q_tail, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl->q_head, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl->q_tokens, (int)gridDim.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl->exited, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Gather n slots' totals into a caller device buffer as f64 [area, tasks, accepted, error] rows,
// ready for one collective (counts are exact in f64 below 2^53).
__global__ __launch_bounds__(256) void k_gather(const SlotOut* __restrict__ slots, int first, int n, int nslots,
                                                double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const SlotOut& s = slots[(first + i) % nslots];
        out[4 * i + 0] = s.area;
        out[4 * i + 1] = (double)s.tasks;
        out[4 * i + 2] = (double)s.leaves;
        out[4 * i + 3] = (double)s.error;
    }
}

}  // namespace aq

// ================================================================================================
// Host side: the C ABI.
// ================================================================================================
using namespace aq;

namespace {

constexpr int NSLOTS = 256;
constexpr unsigned QCAP = 16384;  // HBM queue slots (16384 x 17 KiB = 273 MiB)

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

int ceil_log2(unsigned v) {
    int d = 0;
    while ((1u << d) < v) ++d;
    return d;
}

int validate(const aq_problem* p) {
    if (!p) return AQ_EINVAL;
    if (p->integrand != AQ_F_COSH4 && p->integrand != AQ_F_SIN_RECIP) return AQ_EINVAL;
    if (!std::isfinite(p->a) || !std::isfinite(p->b) || !(p->b >= p->a)) return AQ_EINVAL;
    if (!(p->eps >= 0.0)) return AQ_EINVAL;
    if (p->max_depth < 0 || p->max_depth > AQ_MAX_LEVELS - 1) return AQ_EINVAL;
    return AQ_OK;
}

// Host view of one finished call, whichever path produced it.
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
    int persist_grid = 0;
    bool histograms = true;
    hipStream_t stream = nullptr;
    ExpEntry* d_tab = nullptr;
    Ctl* d_ctl = nullptr;
    SlotOut* d_out = nullptr;          // NSLOTS
    bool slot_hist[NSLOTS] = {};
    Chunk* d_chunks = nullptr;
    unsigned* d_ready = nullptr;
    unsigned epoch = 0;
    // level path
    DevResults* d_lres = nullptr;
    Rec* d_front[2] = {nullptr, nullptr};
    size_t front_cap = 0;
    unsigned* d_count = nullptr;
    // eval buffers
    double* d_x = nullptr;
    double* d_y = nullptr;
    size_t eval_cap = 0;
    // host staging
    SlotOut* h_slot = nullptr;         // pinned
    DevResults* h_lres = nullptr;      // pinned
    HostOut last;
    bool last_valid = false;
    // timing
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_free;
    double timed_ms = 0.0;
    unsigned long long timed_launches = 0;
};

namespace {

int reset_ctl(aq_ctx* c) {
    Ctl h{};
    h.q_tokens = c->persist_grid;
    AQ_HIP(hipMemcpyAsync(c->d_ctl, &h, sizeof(Ctl), hipMemcpyHostToDevice, c->stream));
    AQ_HIP(hipStreamSynchronize(c->stream));
    return AQ_OK;
}

template <int FID, bool HIST>
int launch_persist(aq_ctx* ctx, const aq_problem* p, int shard, int nshards, int slot) {
    const int G = ctx->persist_grid;
    PersistParams P{};
    P.a = p->a;
    P.b = p->b;
    P.eps = p->eps;
    P.max_depth = p->max_depth ? p->max_depth : AQ_DEFAULT_MAX_DEPTH;
    P.shard = shard;
    P.nshards = nshards;
    const unsigned V = (unsigned)G * (unsigned)nshards;
    P.D = ceil_log2(V) + S_POS;
    P.epoch = ++ctx->epoch;
    if (P.epoch == 0) P.epoch = ++ctx->epoch;
    P.qcap = QCAP;
    P.timeout_ticks = 100000000ull * 20ull;  // 20 s of the 100 MHz realtime clock
    P.ctl = ctx->d_ctl;
    P.out = ctx->d_out + slot;
    P.chunks = ctx->d_chunks;
    P.ready = ctx->d_ready;
    P.gtab = ctx->d_tab;
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
    hipLaunchKernelGGL((k_persist<FID, HIST>), dim3(G), dim3(PT), 0, ctx->stream, P);
    AQ_HIP(hipGetLastError());
    if (ctx->timing) {
        AQ_HIP(hipEventRecord(ev.second, ctx->stream));
        ctx->ev_pending.push_back(ev);
    }
    ctx->slot_hist[slot] = HIST;
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
    AQ_HIP(hipMemcpyAsync(ctx->h_slot, ctx->d_out + slot, sizeof(SlotOut), hipMemcpyDeviceToHost, ctx->stream));
    AQ_HIP(hipStreamSynchronize(ctx->stream));
    const SlotOut& s = *ctx->h_slot;
    HostOut& h = ctx->last;
    h = HostOut();
    h.area = s.area;
    h.tasks = s.tasks;
    h.leaves = s.leaves;
    h.spilled = s.spilled;
    h.levels = s.levels;
    h.error = s.error;
    if (ctx->slot_hist[slot]) memcpy(h.hist, s.hist, sizeof(h.hist));
    const unsigned nwg = std::min<unsigned>(s.nwg, MAXG);
    for (unsigned i = 0; i < nwg; ++i) {
        if (s.wg_tasks[i]) h.cu[s.wg_cu[i] % AQ_CU_SLOTS] += s.wg_tasks[i];
    }
    ctx->last_valid = true;
    fill_result(h, out);
    return err_from_bits(h.error);
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
    AQ_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k_persist<F_COSH4, true>, PT, 0));
    if (occ < 1) {
        delete c;
        return AQ_ENODEV;
    }
    // One workgroup per CU: the LDS stack takes most of the CU's LDS; residency of the whole grid
    // is required by the token protocol (idle workgroups wait for busy ones).
    c->persist_grid = std::min(c->num_cus, MAXG);
    AQ_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    AQ_HIP(hipMalloc(&c->d_tab, sizeof(ExpEntry) * 128));
    AQ_HIP(hipMemcpy(c->d_tab, aq_exp_tab_host, sizeof(ExpEntry) * 128, hipMemcpyHostToDevice));
    AQ_HIP(hipMalloc(&c->d_ctl, sizeof(Ctl)));
    AQ_HIP(hipMalloc(&c->d_out, sizeof(SlotOut) * NSLOTS));
    AQ_HIP(hipMemset(c->d_out, 0, sizeof(SlotOut) * NSLOTS));
    AQ_HIP(hipMalloc(&c->d_chunks, sizeof(Chunk) * (size_t)QCAP));
    AQ_HIP(hipMalloc(&c->d_ready, sizeof(unsigned) * (size_t)QCAP));
    AQ_HIP(hipMemset(c->d_ready, 0, sizeof(unsigned) * (size_t)QCAP));
    AQ_HIP(hipHostMalloc(&c->h_slot, sizeof(SlotOut), hipHostMallocDefault));
    AQ_HIP(hipHostMalloc(&c->h_lres, sizeof(DevResults), hipHostMallocDefault));
    AQ_HIP(hipMalloc(&c->d_lres, sizeof(DevResults)));
    AQ_HIP(hipMalloc(&c->d_count, sizeof(unsigned) * (AQ_MAX_LEVELS + 2)));
    int rc = reset_ctl(c);
    if (rc) return rc;
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
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_chunks);
    (void)hipFree(c->d_ready);
    (void)hipFree(c->d_lres);
    (void)hipFree(c->d_front[0]);
    (void)hipFree(c->d_front[1]);
    (void)hipFree(c->d_count);
    (void)hipFree(c->d_x);
    (void)hipFree(c->d_y);
    if (c->h_slot) (void)hipHostFree(c->h_slot);
    if (c->h_lres) (void)hipHostFree(c->h_lres);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int aq_ctx_num_cus(const aq_ctx* c) { return c ? c->num_cus : 0; }

int aq_set_level_histograms(aq_ctx* c, int enable) {
    if (!c) return AQ_EINVAL;
    c->histograms = enable != 0;
    return AQ_OK;
}

int aq_async_slots(void) { return NSLOTS; }

int aq_integrate_async(aq_ctx* ctx, const aq_problem* p, int shard, int nshards, int slot) {
    if (!ctx) return AQ_EINVAL;
    int rc = validate(p);
    if (rc) return rc;
    if (nshards < 1 || shard < 0 || shard >= nshards || nshards > 64) return AQ_EINVAL;
    if (slot < 0 || slot >= NSLOTS) return AQ_EINVAL;
    AQ_HIP(hipSetDevice(ctx->device));
    if (p->integrand == AQ_F_COSH4)
        return ctx->histograms ? launch_persist<F_COSH4, true>(ctx, p, shard, nshards, slot)
                               : launch_persist<F_COSH4, false>(ctx, p, shard, nshards, slot);
    return ctx->histograms ? launch_persist<F_SIN_RECIP, true>(ctx, p, shard, nshards, slot)
                           : launch_persist<F_SIN_RECIP, false>(ctx, p, shard, nshards, slot);
}

int aq_gather_results(aq_ctx* ctx, int first_slot, int n, void* d_out) {
    if (!ctx || !d_out || n < 0 || n > NSLOTS || first_slot < 0 || first_slot >= NSLOTS) return AQ_EINVAL;
    if (n == 0) return AQ_OK;
    AQ_HIP(hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_gather, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_out, first_slot, n, NSLOTS,
                       (double*)d_out);
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
    // Round-1 batch front end: the integrals are pipelined through the persistent path, up to
    // NSLOTS launches in flight, no host synchronisation between them.
    if (!ctx || (n && (!a || !b))) return AQ_EINVAL;
    const bool hist = ctx->histograms;
    ctx->histograms = false;
    int rc = AQ_OK;
    size_t done = 0;
    while (done < n && rc == AQ_OK) {
        const size_t m = std::min<size_t>(n - done, NSLOTS);
        for (size_t i = 0; i < m && rc == AQ_OK; ++i) {
            aq_problem p{integrand, 0, a[done + i], b[done + i], eps};
            rc = aq_integrate_async(ctx, &p, 0, 1, (int)i);
        }
        for (size_t i = 0; i < m && rc == AQ_OK; ++i) {
            aq_result r{};
            rc = aq_fetch(ctx, (int)i, &r);
            if (rc) break;
            if (area) area[done + i] = r.area;
            if (tasks) tasks[done + i] = r.tasks;
            if (accepted) accepted[done + i] = r.accepted;
        }
        done += m;
    }
    ctx->histograms = hist;
    return rc;
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
