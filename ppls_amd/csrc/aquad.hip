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

// Persistent-path control block, one per async slot. It must be all-zero when a launch starts;
// the host zeroes slots lazily in batches (one memset per 64 launches in sequential use) so a
// launch needs no memset of its own. q_tokens stores (tokens - G): the HBM-queue protocol's
// token count starts at G (every workgroup busy) and the run is over when it reaches 0.
struct alignas(128) Line { unsigned v; unsigned pad[31]; };
struct Ctl {
    Line q_tail;               // chunk slots claimed by producers
    Line q_head;               // tickets taken by idle workgroups
    Line q_tokens;             // tokens - G
    Line spare;
    unsigned long long hist[2 * AQ_MAX_LEVELS];   // [0,L): tasks per level, [L,2L): accepted per level
};

constexpr int MAXG = 2048;     // max persistent workgroups per launch
struct WgPart {                // one workgroup's share of a launch, plain stores at exit
    double area;
    unsigned long long tasks;
    unsigned long long leaves;
    unsigned long long spilled;
    unsigned levels;
    unsigned error;
    unsigned cu;               // hardware CU slot
    unsigned pad;
};
struct SlotOut {               // fully rewritten by every launch that targets the slot
    unsigned nwg;
    unsigned epoch;
    unsigned pad[2];
    WgPart wg[MAXG];
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
//
// Work unit = an interval record {l, r, F(l), F(r), depth}. Worker = a WAVEFRONT: each of the NW
// waves of a workgroup owns a ring of WCAP records in LDS and runs rounds of "pop <= 64 records,
// evaluate F(mid) for each (aquadPartA.c:183-191), push the children (:192-197) with a ballot /
// mbcnt compaction" with no workgroup barrier at all. Waves share work through a locked LDS pool
// (overflow in, idle waves out); workgroups share work through an HBM ticket queue driven by one
// elected leader wave per workgroup.
// ------------------------------------------------------------------------------------------------
constexpr int PT = 512;             // threads per workgroup
constexpr int NW = PT / 64;         // waves (workers) per workgroup: 8, two per SIMD
constexpr int WCAP = 256;           // per-wave LDS ring, records (power of two)
constexpr int PCAP = 2048;          // per-workgroup LDS pool ring, records (power of two)
constexpr int LREC = NW * WCAP + PCAP;   // LDS record slots: 4096 x 33 B = 132 KiB
constexpr int POOL0 = NW * WCAP;    // first pool slot
constexpr int CH = 512;             // records per HBM queue chunk
constexpr int S_POS = 5;            // 2^S_POS seed positions per virtual worker (32..63 dealt)
constexpr int GIVE_MIN = 96;        // a busy wave feeds the pool for idle siblings only above this depth
constexpr int DONATE_MIN = 128;     // records needed before a workgroup donates to another CU
constexpr int POLL_ROUNDS = 32;     // a busy wave refreshes its view of the HBM queue every POLL_ROUNDS rounds

// Write-through (sc1) global accesses for the chunk hand-off: the producer stores every payload
// byte sc1 and drains vmcnt before one lane's sc1 flag store; the consumer polls the flag and
// reads the payload with sc1 loads only (MI355X_MICROARCH.md, "Valid forms", row 1) -- no
// release / acquire fences, whose L2 write-back / invalidate cost microseconds.
__device__ __forceinline__ void st_wt(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load(
        reinterpret_cast<unsigned long long*>(const_cast<double*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ unsigned ld_wt(const unsigned* p) {
    return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int g_add(int* p, int v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned g_add(unsigned* p, unsigned v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned g_ld(unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Diagnostics record per workgroup (aq_set_diagnostics), accumulated in LDS by every wave:
// realtime stamps are s_memrealtime ticks (100 MHz), cycle counts are s_memtime shader cycles.
enum : int {
    DG_T_START = 0, DG_T_SEEDED, DG_T_FIRST_LEAD, DG_T_EXIT, DG_ROUNDS, DG_TASKS, DG_CHUNKS_OUT, DG_CHUNKS_IN,
    DG_RECORDS_OUT, DG_T_WAIT, DG_LEADS, DG_SEEDS, DG_POOL_PUSH, DG_CU, DG_RECORDS_IN, DG_ACTIVE_LANES,
    DG_C_ROUND, DG_C_EVAL, DG_POOL_TAKE, DG_LOCK_SPINS, DG_T_LAST_ROUND, DG_SPILL_RECORDS, DG_MAX_RING, DG_C_SEED,
    DIAG_WORDS = 24
};

__device__ __forceinline__ unsigned long long clk() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    return t;
}

struct Chunk {                      // SoA, one queue slot
    double l[CH], r[CH], fl[CH], fr[CH];
    unsigned d[CH];
    unsigned count;
    unsigned pad[31];
};

struct PersistParams {
    double a, b, eps, pad0;
    int max_depth;
    int shard, nshards;
    int D;                          // seed depth
    unsigned epoch;                 // tags queue slots of this call (ready[s] == epoch)
    unsigned qcap;                  // queue slots
    unsigned long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
    Ctl* ctl;
    SlotOut* out;
    unsigned long long* diag;          // optional per-workgroup timeline (DIAG_WORDS each), or null
    Chunk* chunks;
    unsigned* ready;
    const ExpEntry* gtab;
};

__device__ __forceinline__ unsigned long long rtc() { return __builtin_amdgcn_s_memrealtime(); }

// Shared (LDS) state of one workgroup.
struct WgState {
    int lock;            // pool lock (lane 0 of the holding wave)
    unsigned pbot, ptop; // pool ring, monotonic indices
    int idle;            // waves with no records that are counted idle
    int phase;           // 0 running, 1 a leader wave is at the HBM queue, 2 exit
    int busy_token;      // the workgroup holds one token of the HBM-queue protocol
    int err;
    int pad;
    unsigned top0[NW];   // seeded ring tops
};

// LDS record arrays (SoA), one per field.
struct LdsRecs {
    double* l;
    double* r;
    double* fl;
    double* fr;
    unsigned char* d;
};

__device__ __forceinline__ void wave_lock(int* lock, unsigned lane, unsigned long long& spins) {
    if (lane == 0) {
        int expect = 0;
        while (!__hip_atomic_compare_exchange_strong(lock, &expect, 1, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP)) {
            expect = 0;
            ++spins;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ void wave_unlock(int* lock, unsigned lane) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) __hip_atomic_store(lock, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Copy one record (LDS slot i -> LDS slot j).
__device__ __forceinline__ void copy_rec(const LdsRecs& R, unsigned i, unsigned j) {
    const double l = R.l[i], r = R.r[i], fl = R.fl[i], fr = R.fr[i];
    const unsigned char d = R.d[i];
    R.l[j] = l; R.r[j] = r; R.fl[j] = fl; R.fr[j] = fr; R.d[j] = d;
}

// Publish k records (LDS slots src(i), i < k, i.e. base..) as HBM chunk `slot` (caller: one whole wave).
template <typename SrcIdx>
__device__ __forceinline__ void publish_chunk(const PersistParams& P, const LdsRecs& R, unsigned slot, unsigned k,
                                              SrcIdx src, unsigned lane) {
    Chunk* __restrict__ c = P.chunks + slot;
    for (unsigned i = lane; i < k; i += 64) {
        const unsigned j = src(i);
        st_wt(&c->l[i], R.l[j]); st_wt(&c->r[i], R.r[j]); st_wt(&c->fl[i], R.fl[j]);
        st_wt(&c->fr[i], R.fr[j]); st_wt(&c->d[i], (unsigned)R.d[j]);
    }
    if (lane == 0) st_wt(&c->count, k);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the single storing wave drains
    if (lane == 0) st_wt(&P.ready[slot], P.epoch);
}

template <int FID, bool HIST, bool DIAG>
__global__ __launch_bounds__(PT) void k_persist(PersistParams P) {
    __shared__ double s_l[LREC], s_r[LREC], s_fl[LREC], s_fr[LREC];
    __shared__ unsigned char s_d[LREC];
    __shared__ ExpEntry tab[128];
    __shared__ WgState S;
    __shared__ double s_red[NW];
    __shared__ unsigned s_redu[3][NW];
    __shared__ unsigned long long s_spill[NW];
    __shared__ unsigned s_hist[HIST ? 2 * AQ_MAX_LEVELS : 1];

    const unsigned tid = threadIdx.x;
    const unsigned lane = lane_id();
    const unsigned wid = tid >> 6;
    Ctl* __restrict__ ctl = P.ctl;
    const LdsRecs R{s_l, s_r, s_fl, s_fr, s_d};
    const unsigned long long t_entry = rtc();
    const unsigned long long c_entry = DIAG ? clk() : 0ull;
    __shared__ unsigned long long s_dg[DIAG ? DIAG_WORDS : 1];  // diagnostics (DIAG builds only)
    if (DIAG) {
        for (unsigned i = tid; i < DIAG_WORDS; i += PT) s_dg[i] = (i == DG_T_FIRST_LEAD) ? ~0ull : 0ull;
    }
    stage_exp_table(tab, P.gtab);
    if (HIST)
        for (unsigned i = tid; i < 2 * AQ_MAX_LEVELS; i += PT) s_hist[i] = 0;
    if (tid == 0) {
        S.lock = 0; S.pbot = 0; S.ptop = 0; S.idle = 0; S.phase = 0; S.busy_token = 1; S.err = 0;
    }

    const double eps = P.eps;
    const int max_depth = P.max_depth;
    double my_area = 0.0;
    unsigned my_tasks = 0, my_leaves = 0, my_maxd = 0;
    unsigned err = 0;

    // ---------------- seeding: this worker's depth-D positions, all F evaluations in one pass ----
    // Virtual worker vwg of V owns positions j = k*V + (k odd ? V-1-vwg : vwg) < 2^D (snake order
    // over bands). Every ancestor of every position is a task; its decision is the reference's
    // arithmetic on (l, r, F(l), F(r), F(mid)), all of which are F at mids of the position's own
    // path or at A/B. A task above depth D is counted by the owner of its leftmost descendant.
    const unsigned V = gridDim.x * (unsigned)P.nshards;
    const unsigned vwg = blockIdx.x * (unsigned)P.nshards + (unsigned)P.shard;
    const int D = P.D;
    const unsigned long long npos_total = 1ull << D;
    const unsigned nb = (unsigned)((npos_total + V - 1) / V);  // bands = positions per worker (<= 64)
    const unsigned npairs = (unsigned)D * nb;
    auto position = [&](unsigned k, bool& valid) -> unsigned long long {
        const unsigned long long o = (k & 1u) ? (unsigned long long)(V - 1 - vwg) : (unsigned long long)vwg;
        const unsigned long long j = (unsigned long long)k * V + o;
        valid = j < npos_total;
        return j;
    };
    // scratch in the (still empty) pool region
    double* fm = s_l + POOL0;          // [npairs + 2]: F(mid of node (d,k)) at d*nb+k, then F(A), F(B)
    double* leafa = s_r + POOL0;       // [npairs]: larea + rarea of node (d,k)
    unsigned char* flag = s_d + POOL0; // [npairs]: node (d,k) refines
    for (unsigned q = tid; q < npairs + 2; q += PT) {
        double x;
        if (q < npairs) {
            const unsigned d = q / nb, k = q % nb;
            bool valid;
            const unsigned long long p = position(k, valid);
            const unsigned long long anc = valid ? (p >> (D - (int)d)) : 0ull;
            double l = P.a, r = P.b;
            for (unsigned i = 0; i < d; ++i) {
                const double m = (l + r) / 2;
                if ((anc >> (d - 1 - i)) & 1ull) l = m; else r = m;
            }
            x = (l + r) / 2;
        } else {
            x = (q == npairs) ? P.a : P.b;
        }
        fm[q] = x;
    }
    __syncthreads();  // exp table staged
    for (unsigned q = tid; q < npairs + 2; q += PT) fm[q] = integrand<FID>(fm[q], tab);
    __syncthreads();
    for (unsigned q = tid; q < npairs; q += PT) {
        const unsigned d = q / nb, k = q % nb;
        bool valid;
        const unsigned long long p = position(k, valid);
        const unsigned long long anc = valid ? (p >> (D - (int)d)) : 0ull;
        double l = P.a, r = P.b;
        unsigned li = npairs, ri = npairs + 1;
        for (unsigned i = 0; i < d; ++i) {
            const double m = (l + r) / 2;
            if ((anc >> (d - 1 - i)) & 1ull) { l = m; li = i * nb + k; } else { r = m; ri = i * nb + k; }
        }
        const double fl = fm[li], fr = fm[ri], fmid = fm[q];
        const double mid = (l + r) / 2;
        const double lrarea = (fl + fr) * (r - l) / 2;        // :185
        const double larea = (fl + fmid) * (mid - l) / 2;     // :189
        const double rarea = (fmid + fr) * (r - mid) / 2;     // :190
        flag[q] = fabs((larea + rarea) - lrarea) > eps;      // :191
        leafa[q] = larea + rarea;                             // :199
    }
    __syncthreads();
    if (wid == 0) {
        const unsigned k = lane;
        bool valid = false;
        const unsigned long long p = (k < nb) ? position(k, valid) : 0ull;
        // every flag of this position's path in one batch of independent LDS reads
        unsigned long long fmask = 0;
        for (int d = 0; d < D; ++d)
            fmask |= (unsigned long long)(flag[(unsigned)d * nb + (k < nb ? k : 0)] ? 1u : 0u) << d;
        const int dstar = (int)__builtin_ctzll(~fmask);   // first depth that does not refine (D if none)
        bool alive = valid;
        if (valid) {
            const int dlast = min(dstar, D - 1);
            for (int d = 0; d <= dlast; ++d) {
                const bool owner = (p & ((1ull << (D - d)) - 1ull)) == 0ull;
                if (owner) {
                    ++my_tasks;
                    my_maxd = max(my_maxd, (unsigned)d + 1u);
                    if (HIST) atomicAdd(&s_hist[d], 1u);
                    if (d == dstar) {
                        my_area += leafa[(unsigned)d * nb + k];
                        ++my_leaves;
                        if (HIST) atomicAdd(&s_hist[AQ_MAX_LEVELS + d], 1u);
                    } else if (d + 1 >= max_depth) {
                        err |= ERRB_DEPTH;
                    }
                }
            }
            alive = dstar >= D && D < max_depth;
        }
        double l = P.a, r = P.b, fl = 0.0, fr = 0.0;
        if (alive) {
            unsigned li = npairs, ri = npairs + 1;
            for (int i = 0; i < D; ++i) {
                const double m = (l + r) / 2;
                if ((p >> (D - 1 - i)) & 1ull) { l = m; li = (unsigned)i * nb + k; } else { r = m; ri = (unsigned)i * nb + k; }
            }
            fl = fm[li];
            fr = fm[ri];
        }
        // seed k goes to wave k % NW
        for (unsigned w = 0; w < NW; ++w) {
            const unsigned long long m = __ballot(alive && (k % NW) == w);
            if (alive && (k % NW) == w) {
                const unsigned j = w * WCAP + mbcnt(m);
                s_l[j] = l; s_r[j] = r; s_fl[j] = fl; s_fr[j] = fr; s_d[j] = (unsigned char)D;
            }
            if (lane == 0) S.top0[w] = (unsigned)__popcll(m);
        }
    }
    __syncthreads();

    // ---------------- main loop: every wave is an independent worker ----------------
    const unsigned base = wid * WCAP;            // this wave's ring
    unsigned top = S.top0[wid], bot = 0;         // wave-uniform
    if constexpr (DIAG) {
        if (tid == 0) {
            s_dg[DG_T_START] = t_entry;
            s_dg[DG_T_SEEDED] = rtc();
            s_dg[DG_C_SEED] = clk() - c_entry;
            unsigned n = 0;
            for (int w = 0; w < NW; ++w) n += S.top0[w];
            s_dg[DG_SEEDS] = n;
        }
    }
    const unsigned long long t0 = rtc();
    bool counted_idle = false;                    // wave-uniform
    unsigned poll_ctr = wid * (POLL_ROUNDS / NW);
    unsigned seen_head = 0, seen_tail = 0;        // lane 0's view of the HBM queue
    unsigned long long spilled = 0;               // records this wave sent to HBM (lane 0)
    unsigned long long lock_spins = 0;

    for (;;) {
        unsigned size = top - bot;

        if (size == 0) {
            // ---- out of records: take from the pool, else idle / lead the workgroup to the HBM queue
            if (counted_idle) {
                // already counted idle: peek without the lock (the wave whose increment made every
                // wave idle is the one that leads, so a counted wave only waits here)
                const unsigned pt = __hip_atomic_load(&S.ptop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const unsigned pb = __hip_atomic_load(&S.pbot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const int ph = __hip_atomic_load(&S.phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (pt == pb) {
                    if (ph == 2) break;
                    __builtin_amdgcn_s_sleep(4);
                    continue;
                }
            }
            wave_lock(&S.lock, lane, lock_spins);
            const unsigned avail = S.ptop - S.pbot;
            const int phase = S.phase;
            unsigned k = 0;
            bool lead = false;
            if (avail > 0) {
                k = min(avail, 64u);
                const unsigned pb = S.pbot;
                if (lane < k) copy_rec(R, POOL0 + ((pb + lane) & (PCAP - 1)), base + lane);
                if (lane == 0) {
                    S.pbot = pb + k;
                    if (counted_idle) S.idle -= 1;
                }
                counted_idle = false;
            } else {
                if (!counted_idle) {
                    if (lane == 0) S.idle += 1;
                    counted_idle = true;
                }
                __builtin_amdgcn_wave_barrier();
                if (phase == 0 && S.idle == NW) {   // every wave idle and the pool empty
                    lead = true;
                    if (lane == 0) S.phase = 1;
                }
            }
            wave_unlock(&S.lock, lane);
            if constexpr (DIAG) { if (lane == 0 && k) atomicAdd(&s_dg[DG_POOL_TAKE], (unsigned long long)k); }
            if (k) {
                bot = 0;
                top = k;
                continue;
            }
            if (phase == 2) break;
            if (!lead) {
                __builtin_amdgcn_s_sleep(4);
                continue;
            }
            // ---- leader: this workgroup has no work; hand its token back and wait for a chunk
            unsigned long long tl = DIAG ? rtc() : 0ull;
            if constexpr (DIAG) {
                if (lane == 0) {
                    atomicMin(&s_dg[DG_T_FIRST_LEAD], tl);
                    atomicAdd(&s_dg[DG_LEADS], 1ull);
                }
            }
            int cmd = -1;   // >= 0 chunk slot, -1 exit, -2 error
            unsigned cnt = 0;
            if (lane == 0) {
                if (S.busy_token) {
                    g_add((int*)&ctl->q_tokens.v, -1);
                    S.busy_token = 0;
                }
                const unsigned h = g_add(&ctl->q_head.v, 1u);
                for (unsigned spins = 0;; ++spins) {
                    if (h < P.qcap && ld_wt(&P.ready[h]) == P.epoch) { cmd = (int)h; break; }
                    if ((spins & 3u) == 0u &&
                            __hip_atomic_load((int*)&ctl->q_tokens.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                            -(int)gridDim.x) {
                        cmd = -1;
                        break;
                    }
                    if ((spins & 63u) == 63u && rtc() - t0 > P.timeout_ticks) { err |= ERRB_TIMEOUT; cmd = -2; break; }
                    __builtin_amdgcn_s_sleep(8);
                }
                if (cmd >= 0) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only
                    cnt = ld_wt(&P.chunks[cmd].count);
                }
            }
            cmd = __shfl(cmd, 0, 64);
            cnt = __shfl(cnt, 0, 64);
            if (cmd < 0) {
                wave_lock(&S.lock, lane, lock_spins);
                if (lane == 0) S.phase = 2;
                wave_unlock(&S.lock, lane);
                break;
            }
            // load the chunk into the (empty) pool, take this workgroup's token back
            const Chunk* __restrict__ c = P.chunks + cmd;
            wave_lock(&S.lock, lane, lock_spins);
            const unsigned pt = S.ptop;
            for (unsigned i = lane; i < cnt; i += 64) {
                const unsigned j = POOL0 + ((pt + i) & (PCAP - 1));
                s_l[j] = ld_wt(&c->l[i]); s_r[j] = ld_wt(&c->r[i]); s_fl[j] = ld_wt(&c->fl[i]);
                s_fr[j] = ld_wt(&c->fr[i]); s_d[j] = (unsigned char)ld_wt(&c->d[i]);
            }
            if (lane == 0) {
                S.ptop = pt + cnt;
                S.phase = 0;
                S.busy_token = 1;
                S.idle -= 1;   // the leader un-counts itself, so an empty chunk leads to a new leader
                g_add((int*)&ctl->q_tokens.v, 1 - (int)cnt);
            }
            counted_idle = false;
            wave_unlock(&S.lock, lane);
            if constexpr (DIAG) {
                if (lane == 0) {
                    atomicAdd(&s_dg[DG_CHUNKS_IN], 1ull);
                    atomicAdd(&s_dg[DG_RECORDS_IN], (unsigned long long)cnt);
                    atomicAdd(&s_dg[DG_T_WAIT], rtc() - tl);
                }
            }
            continue;
        }

        // ---- keep the ring from overflowing: move its bottom 64 records to the pool, else to HBM
        if (size > (unsigned)(WCAP - 64)) {
            wave_lock(&S.lock, lane, lock_spins);
            const unsigned pt = S.ptop;
            const bool fits = (pt - S.pbot) + 64u <= (unsigned)PCAP;
            if (fits) {
                copy_rec(R, base + ((bot + lane) & (WCAP - 1)), POOL0 + ((pt + lane) & (PCAP - 1)));
                if (lane == 0) S.ptop = pt + 64u;
            }
            wave_unlock(&S.lock, lane);
            if (!fits) {
                // pool full: spill 64 records to an HBM chunk (tokens first, then publish)
                unsigned slot = 0;
                if (lane == 0) {
                    slot = g_add(&ctl->q_tail.v, 1u);
                    if (slot < P.qcap) g_add((int*)&ctl->q_tokens.v, 64);
                    spilled += 64;
                }
                slot = __shfl(slot, 0, 64);
                if (slot < P.qcap) {
                    const unsigned b = bot;
                    publish_chunk(P, R, slot, 64u, [&](unsigned i) { return base + ((b + i) & (WCAP - 1)); }, lane);
                } else {
                    err |= ERRB_OVERFLOW;   // records dropped: result invalid, error reported
                }
            }
            if constexpr (DIAG) { if (lane == 0) atomicAdd(&s_dg[DG_POOL_PUSH], 64ull); }
            bot += 64;
            continue;
        }

        // ---- feed idle sibling waves / donate to starving workgroups
        if (size >= (unsigned)GIVE_MIN && S.idle > 0 && S.ptop == S.pbot) {
            const unsigned k = size / 2u;   // <= 128
            wave_lock(&S.lock, lane, lock_spins);
            const unsigned pt = S.ptop;
            const bool fits = (pt - S.pbot) + k <= (unsigned)PCAP;
            if (fits) {
                for (unsigned i = lane; i < k; i += 64)
                    copy_rec(R, base + ((bot + i) & (WCAP - 1)), POOL0 + ((pt + i) & (PCAP - 1)));
                if (lane == 0) S.ptop = pt + k;
            }
            wave_unlock(&S.lock, lane);
            if (fits) {
                bot += k;
                continue;
            }
        }
        if (((++poll_ctr) % POLL_ROUNDS) == 0) {
            // another CU waits on the HBM queue and this workgroup has plenty: donate from the pool
            // (its oldest, i.e. shallowest, records) or from the bottom of this ring
            unsigned slot = 0xffffffffu;
            if (lane == 0) {
                if ((int)(seen_head - seen_tail) > 0) {
                    unsigned expect = seen_tail;
                    if (__hip_atomic_compare_exchange_strong(&ctl->q_tail.v, &expect, seen_tail + 1u, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                        slot = seen_tail;
                }
                seen_head = g_ld(&ctl->q_head.v);
                seen_tail = g_ld(&ctl->q_tail.v);
            }
            slot = __shfl(slot, 0, 64);
            if (slot != 0xffffffffu) {
                if (slot >= P.qcap) {
                    err |= ERRB_OVERFLOW;
                } else {
                    wave_lock(&S.lock, lane, lock_spins);
                    const unsigned pavail = S.ptop - S.pbot;
                    unsigned k;
                    if (pavail >= (unsigned)DONATE_MIN) {
                        k = min((unsigned)CH, pavail / 2u);
                        const unsigned pb = S.pbot;
                        if (lane == 0) g_add((int*)&ctl->q_tokens.v, (int)k);
                        publish_chunk(P, R, slot, k, [&](unsigned i) { return POOL0 + ((pb + i) & (PCAP - 1)); }, lane);
                        if (lane == 0) S.pbot = pb + k;
                        wave_unlock(&S.lock, lane);
                    } else {
                        wave_unlock(&S.lock, lane);
                        k = size / 2u;   // may be 0: an empty chunk is harmless
                        if (lane == 0) g_add((int*)&ctl->q_tokens.v, (int)k);
                        const unsigned b = bot;
                        publish_chunk(P, R, slot, k, [&](unsigned i) { return base + ((b + i) & (WCAP - 1)); }, lane);
                        bot += k;
                    }
                    if (lane == 0) spilled += k;
                    if constexpr (DIAG) {
                        if (lane == 0) {
                            atomicAdd(&s_dg[DG_CHUNKS_OUT], 1ull);
                            atomicAdd(&s_dg[DG_RECORDS_OUT], (unsigned long long)k);
                        }
                    }
                    continue;
                }
            }
        }

        // ---- one round: pop up to 64 records from the top of this wave's ring
        unsigned long long c0 = 0, c1 = 0;
        if constexpr (DIAG) c0 = clk();
        const unsigned n = min(size, 64u);
        const unsigned b0 = top - n;
        const bool active = lane < n;
        double l = 0, r = 0, fl = 0, fr = 0;
        unsigned d = 0;
        if (active) {
            const unsigned j = base + ((b0 + lane) & (WCAP - 1));
            l = s_l[j]; r = s_r[j]; fl = s_fl[j]; fr = s_fr[j]; d = s_d[j];
        }
        bool refine = false;
        double mid = 0, fmid = 0;
        if (active) {
            const Step st = task_step<FID>(l, r, fl, fr, eps, tab);
            mid = st.mid;
            fmid = st.fmid;
            ++my_tasks;
            my_maxd = max(my_maxd, d + 1u);
            if (HIST) atomicAdd(&s_hist[d], 1u);
            if (st.refine) {
                if ((int)d + 1 >= max_depth) err |= ERRB_DEPTH;
                else refine = true;
            } else {
                my_area += st.larea + st.rarea;  // :199 -> :149
                ++my_leaves;
                if (HIST) atomicAdd(&s_hist[AQ_MAX_LEVELS + d], 1u);
            }
        }
        if constexpr (DIAG) c1 = clk();
        const unsigned long long mask = __ballot(refine);
        if (refine) {
            const unsigned pos = b0 + 2u * mbcnt(mask);
            const unsigned j0 = base + (pos & (WCAP - 1)), j1 = base + ((pos + 1u) & (WCAP - 1));
            const unsigned char cd = (unsigned char)(d + 1u);
            s_l[j0] = l;   s_r[j0] = mid; s_fl[j0] = fl;   s_fr[j0] = fmid; s_d[j0] = cd;  // [l,mid]  :192-194
            s_l[j1] = mid; s_r[j1] = r;   s_fl[j1] = fmid; s_fr[j1] = fr;   s_d[j1] = cd;  // [mid,r]  :195-197
        }
        top = b0 + 2u * (unsigned)__popcll(mask);
        if constexpr (DIAG) {
            if (lane == 0) {
                const unsigned long long c2 = clk();
                atomicAdd(&s_dg[DG_ROUNDS], 1ull);
                atomicAdd(&s_dg[DG_ACTIVE_LANES], (unsigned long long)n);
                atomicAdd(&s_dg[DG_C_ROUND], c2 - c0);
                atomicAdd(&s_dg[DG_C_EVAL], c1 - c0);
                atomicMax(&s_dg[DG_MAX_RING], (unsigned long long)size);
                atomicMax(&s_dg[DG_T_LAST_ROUND], rtc());
            }
        }
    }

    // ---------------- exit: this workgroup's partial results, plain stores (no contention) ------
    const double wa = wave_sum(my_area);
    const unsigned wt = wave_sum_u(my_tasks), wl = wave_sum_u(my_leaves), wm = wave_max_u(my_maxd);
    unsigned we = err;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) we |= (unsigned)__shfl_xor((int)we, o, 64);
    if (lane == 0) {
        s_red[wid] = wa;
        s_redu[0][wid] = wt;
        s_redu[1][wid] = wl;
        s_redu[2][wid] = wm;
        s_spill[wid] = spilled | ((unsigned long long)we << 48);
        if constexpr (DIAG) {
            atomicAdd(&s_dg[DG_LOCK_SPINS], lock_spins);
            atomicAdd(&s_dg[DG_SPILL_RECORDS], spilled);
        }
    }
    __syncthreads();
    if (tid == 0) {
        double ba = 0.0;
        unsigned bt = 0, bl = 0, bm = 0, be = 0;
        unsigned long long bs = 0;
        for (int w = 0; w < NW; ++w) {
            ba += s_red[w];
            bt += s_redu[0][w];
            bl += s_redu[1][w];
            bm = max(bm, s_redu[2][w]);
            bs += s_spill[w] & 0xffffffffffffull;
            be |= (unsigned)(s_spill[w] >> 48);
        }
        WgPart* o = &P.out->wg[blockIdx.x];
        o->area = ba;
        o->tasks = bt;
        o->leaves = bl;
        o->spilled = bs;
        o->levels = bm;
        o->error = be;
        o->cu = cu_slot();
        if (blockIdx.x == 0) {
            P.out->nwg = gridDim.x;
            P.out->epoch = P.epoch;
        }
        if constexpr (DIAG) {
            s_dg[DG_T_EXIT] = rtc();
            s_dg[DG_CU] = cu_slot();
            s_dg[DG_TASKS] = bt;
            unsigned long long* d = P.diag + (size_t)blockIdx.x * DIAG_WORDS;
            for (int i = 0; i < DIAG_WORDS; ++i) d[i] = s_dg[i];
        }
    }
    if (HIST) {
        for (unsigned i = tid; i < 2 * AQ_MAX_LEVELS; i += PT) {
            const unsigned v = s_hist[i];
            if (v) atomicAdd(&ctl->hist[i], (unsigned long long)v);
        }
    }
}

// Gather n slots' totals into a caller device buffer as f64 [area, tasks, accepted, error] rows,
// ready for one collective (counts are exact in f64 below 2^53). One workgroup per slot sums the
// slot's per-workgroup partials in a fixed order.
__global__ __launch_bounds__(256) void k_gather(const SlotOut* __restrict__ slots, int first, int n, int nslots,
                                                double* __restrict__ out) {
    __shared__ double s_a[4];
    __shared__ unsigned long long s_t[4], s_l[4];
    __shared__ unsigned s_e[4];
    const SlotOut& s = slots[(first + (int)blockIdx.x) % nslots];
    const unsigned nwg = min(s.nwg, (unsigned)MAXG);
    double a = 0.0;
    unsigned long long t = 0, l = 0;
    unsigned e = 0;
    for (unsigned i = threadIdx.x; i < nwg; i += blockDim.x) {
        a += s.wg[i].area;
        t += s.wg[i].tasks;
        l += s.wg[i].leaves;
        e |= s.wg[i].error;
    }
    a = wave_sum(a);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        t += __shfl_xor(t, o, 64);
        l += __shfl_xor(l, o, 64);
        e |= (unsigned)__shfl_xor((int)e, o, 64);
    }
    const unsigned w = threadIdx.x >> 6;
    if (lane_id() == 0) { s_a[w] = a; s_t[w] = t; s_l[w] = l; s_e[w] = e; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double A = 0.0;
        unsigned long long T = 0, L = 0;
        unsigned E = 0;
        for (int k = 0; k < 4; ++k) { A += s_a[k]; T += s_t[k]; L += s_l[k]; E |= s_e[k]; }
        double* o = out + 4 * blockIdx.x;
        o[0] = A;
        o[1] = (double)T;
        o[2] = (double)L;
        o[3] = (double)E;
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
    Ctl* d_ctl = nullptr;              // NSLOTS control blocks
    bool ctl_dirty[NSLOTS] = {};       // slot's control block used since it was last zeroed
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

// Zero the control block of `slot` (and of the following slots up to a batch of 64) if it has
// been used since it was last zeroed: one memset per 64 launches when slots are used in order.
int ensure_clean(aq_ctx* c, int slot) {
    if (!c->ctl_dirty[slot]) return AQ_OK;
    int n = 0;
    while (slot + n < NSLOTS && n < 64) c->ctl_dirty[slot + n++] = false;
    AQ_HIP(hipMemsetAsync(c->d_ctl + slot, 0, sizeof(Ctl) * (size_t)n, c->stream));
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
    int rc = ensure_clean(ctx, slot);
    if (rc) return rc;
    P.ctl = ctx->d_ctl + slot;
    P.out = ctx->d_out + slot;
    P.chunks = ctx->d_chunks;
    P.ready = ctx->d_ready;
    P.gtab = ctx->d_tab;
    P.diag = ctx->d_diag;
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
    if (P.diag)
        hipLaunchKernelGGL((k_persist<FID, HIST, true>), dim3(G), dim3(PT), 0, ctx->stream, P);
    else
        hipLaunchKernelGGL((k_persist<FID, HIST, false>), dim3(G), dim3(PT), 0, ctx->stream, P);
    AQ_HIP(hipGetLastError());
    if (ctx->timing) {
        AQ_HIP(hipEventRecord(ev.second, ctx->stream));
        ctx->ev_pending.push_back(ev);
    }
    ctx->slot_hist[slot] = HIST;
    ctx->ctl_dirty[slot] = true;
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
    const size_t nbytes = offsetof(SlotOut, wg) + sizeof(WgPart) * (size_t)ctx->persist_grid;
    AQ_HIP(hipMemcpyAsync(ctx->h_slot, ctx->d_out + slot, nbytes, hipMemcpyDeviceToHost, ctx->stream));
    if (ctx->slot_hist[slot])
        AQ_HIP(hipMemcpyAsync(ctx->h_hist, ctx->d_ctl[slot].hist, sizeof(unsigned long long) * 2 * AQ_MAX_LEVELS,
                              hipMemcpyDeviceToHost, ctx->stream));
    AQ_HIP(hipStreamSynchronize(ctx->stream));
    const SlotOut& s = *ctx->h_slot;
    HostOut& h = ctx->last;
    h = HostOut();
    const unsigned nwg = std::min<unsigned>(s.nwg, MAXG);
    for (unsigned i = 0; i < nwg; ++i) {
        const WgPart& w = s.wg[i];
        h.area += w.area;
        h.tasks += w.tasks;
        h.leaves += w.leaves;
        h.spilled += w.spilled;
        h.levels = std::max(h.levels, w.levels);
        h.error |= w.error;
        if (w.tasks) h.cu[w.cu % AQ_CU_SLOTS] += w.tasks;
    }
    if (ctx->slot_hist[slot]) memcpy(h.hist, ctx->h_hist, sizeof(h.hist));
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
    AQ_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k_persist<F_COSH4, true, false>, PT, 0));
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
    AQ_HIP(hipMalloc(&c->d_ctl, sizeof(Ctl) * NSLOTS));
    AQ_HIP(hipMemset(c->d_ctl, 0, sizeof(Ctl) * NSLOTS));
    AQ_HIP(hipMalloc(&c->d_out, sizeof(SlotOut) * NSLOTS));
    AQ_HIP(hipMemset(c->d_out, 0, sizeof(SlotOut) * NSLOTS));
    AQ_HIP(hipMalloc(&c->d_chunks, sizeof(Chunk) * (size_t)QCAP));
    AQ_HIP(hipMalloc(&c->d_ready, sizeof(unsigned) * (size_t)QCAP));
    AQ_HIP(hipMemset(c->d_ready, 0, sizeof(unsigned) * (size_t)QCAP));
    AQ_HIP(hipHostMalloc(&c->h_slot, sizeof(SlotOut), hipHostMallocDefault));
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
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_chunks);
    (void)hipFree(c->d_ready);
    (void)hipFree(c->d_lres);
    (void)hipFree(c->d_diag);
    (void)hipFree(c->d_front[0]);
    (void)hipFree(c->d_front[1]);
    (void)hipFree(c->d_count);
    (void)hipFree(c->d_x);
    (void)hipFree(c->d_y);
    if (c->h_slot) (void)hipHostFree(c->h_slot);
    if (c->h_hist) (void)hipHostFree(c->h_hist);
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
    const size_t words = std::min<size_t>((size_t)cap_words, (size_t)DIAG_WORDS * c->persist_grid);
    AQ_HIP(hipStreamSynchronize(c->stream));
    AQ_HIP(hipMemcpy(out, c->d_diag, words * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return (int)(words / DIAG_WORDS);
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
    hipLaunchKernelGGL(k_gather, dim3(n), dim3(256), 0, ctx->stream, ctx->d_out, first_slot, n, NSLOTS,
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
