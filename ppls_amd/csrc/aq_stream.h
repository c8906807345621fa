// aq_stream.h -- the persistent on-device farmer: K integrals per launch, one wavefront per worker.
//
// Reference: /root/reference/aquadPartA.c. The farmer's LIFO bag (:125-173) and the workers' task
// body (:183-202) become one persistent launch:
//   * worker = WAVEFRONT. Each of the NW waves of a workgroup owns an LDS ring of interval records
//     {l, r, F(l), F(r), depth | integral<<8}. A round pops <= 64 records, evaluates F(mid) for each
//     in FP64 (glibc-exact cosh, aq_libm.h), applies the reference's refine test (:191) and pushes the
//     children (:192-197) back with a ballot / mbcnt compaction: no workgroup barrier, no HBM traffic.
//   * work sharing inside a CU: a locked LDS pool (ring overflow in, idle waves out);
//   * work sharing across CUs (what the bag of tasks is for): an HBM ticket queue of record chunks,
//     driven by one elected leader wave per workgroup; busy waves donate to waiting tickets;
//   * seeding is WAVE-LOCAL: virtual worker vw = ((wg*NW + wave)*nshards + shard) of V owns the
//     depth-D positions j = k*V + (k odd ? V-1-vw : vw) (snake order). All F evaluations of the
//     positions' ancestors are independent (pure (l+r)/2 recursion), so one wave evaluates them in one
//     pass, decides every ancestor in a second pass and keeps the surviving positions as its first
//     records. A task above depth D is counted by the owner of its leftmost descendant position.
//   * a wave that runs out of records takes from the pool, else seeds its share of the NEXT
//     integral of the launch -- the tail of one integral overlaps the start of the next, which is
//     what keeps all lanes busy (a single integral's frontier is too narrow to fill a CU).
//   * accepted areas / task counts accumulate per lane in registers per integral and are flushed
//     (wave reduction + one set of uncontended atomics into this workgroup's partial of that
//     integral) when a wave switches integral or exits (the farmer's `result += buff[0]`, :149).
// Every decision is the reference's own arithmetic on the same operands, so the interval tree --
// tasks and accepted counts -- is bit-identical whatever the schedule.
#pragma once
#include <type_traits>

#include "aq_device.h"

namespace aq {

constexpr int PT = 512;             // threads per workgroup
constexpr int NW = PT / 64;         // waves (workers) per workgroup: 8, two per SIMD
constexpr int MAX_ILP = 2;          // records per lane per round, at most (two interleaved evaluations)
constexpr int RB = 64 * MAX_ILP;    // records per round, at most
constexpr int WCAP = 384;           // per-wave LDS ring, records: a round pops RB, pushes <= 2*RB
constexpr int PCAP = 1024;          // per-workgroup LDS pool ring, records (power of two)
constexpr int LREC = NW * WCAP + PCAP;   // LDS record slots: 4096 x 36 B = 144 KiB
constexpr int POOL0 = NW * WCAP;    // first pool slot
constexpr int CH = 512;             // records per HBM queue chunk
constexpr int S_W = 2;              // 2^S_W seed positions per wave (4..7 dealt)
constexpr int GIVE_MIN = 192;       // a busy wave feeds the pool for idle siblings only above this depth
constexpr int DONATE_MIN = 128;     // pool records needed before a workgroup donates from its pool
constexpr int POLL_ROUNDS = 32;     // a busy wave refreshes its view of the HBM queue every POLL_ROUNDS rounds
constexpr int READY_STRIDE = 32;    // one ready flag per 128-B line: pollers never share a line
constexpr int MAXG = 2048;          // max persistent workgroups per launch
constexpr int MAXK = 256;           // max integrals per launch
constexpr int CCAP = 4096;          // records per wave cellar (private HBM overflow stack, 144 KiB)
constexpr int REFILL = 192;         // records a wave takes back from its cellar at once
constexpr int DEFAULT_GSPLIT = 8;   // a multi-integral launch's job = the share of this many waves
constexpr int DEFAULT_ILP = 1;      // records per lane per round

// Queue control block (HBM ticket queue) and per-integral histogram accumulators. One per async
// slot; it must be all-zero when a launch starts -- the host zeroes slots lazily in batches.
// q_tokens stores (tokens - G): the protocol's token count starts at G (every workgroup busy) and
// the run is over when it reaches 0.
struct alignas(128) Line {
    unsigned v;
    unsigned pad[31];
};
struct Ctl {
    Line q_tail;               // chunk slots claimed by producers
    Line q_head;               // tickets taken by idle workgroups
    Line q_tokens;             // tokens - G
    Line spare;
    unsigned long long hist[2 * AQ_MAX_LEVELS];   // [0,L): tasks per level, [L,2L): accepted per level
};

// One workgroup's share of one integral, accumulated with uncontended atomics (zeroed per slot).
struct WgPart {
    double area;
    unsigned long long tasks;
    unsigned long long leaves;
    unsigned long long spilled;
    unsigned levels;
    unsigned error;
    unsigned cu;               // hardware CU slot
    unsigned pad;
};

struct Chunk {                      // SoA, one queue slot
    double l[CH], r[CH], fl[CH], fr[CH];
    unsigned dt[CH];                // depth | integral << 8
    unsigned count;
    unsigned pad[31];
};

// A wave's private HBM overflow stack: the bottom (oldest, shallowest) records of a full ring go
// down here without any lock; the wave takes them back when its ring runs dry, before it looks at
// the shared pool or seeds new work, so the cellar is empty whenever the wave reports idle. Only
// the owning wave touches it (one CU, one L2), so it stays on-die.
struct Cellar {
    double l[CCAP], r[CCAP], fl[CCAP], fr[CCAP];
    unsigned dt[CCAP];
};

struct StreamParams {
    const double2* bounds;          // [nprob] {a, b} per integral
    int nprob;
    int first_slot;                 // integral p -> slot first_slot + p
    double eps;
    int max_depth;
    int shard, nshards;
    int D;                          // seed depth
    int shares;                     // jobs per integral: job j = share j % shares of integral j / shares
    int ilp;                        // records per lane per round (1 or 2)
    unsigned epoch;                 // tags queue slots of this launch (ready[s] == epoch)
    unsigned qcap;                  // queue slots
    unsigned long long timeout_ticks;  // s_memrealtime ticks (100 MHz)
    Ctl* ctls;                      // per-slot control blocks; the queue uses ctls[first_slot]
    WgPart* parts;                  // [slot * gridDim.x + wg]
    unsigned long long* diag;       // optional per-workgroup timeline (DIAG_WORDS each)
    Chunk* chunks;
    Cellar* cellar;                 // [gridDim.x * NW]
    unsigned* ready;
    const ExpEntry* gtab;
};

// Diagnostics record per workgroup (aq_set_diagnostics), accumulated in LDS by every wave:
// realtime stamps are s_memrealtime ticks (100 MHz), cycle counts are s_memtime shader cycles.
enum : int {
    DG_T_START = 0, DG_T_SEEDED, DG_T_FIRST_LEAD, DG_T_EXIT, DG_ROUNDS, DG_TASKS, DG_CHUNKS_OUT, DG_CHUNKS_IN,
    DG_RECORDS_OUT, DG_T_WAIT, DG_LEADS, DG_SEEDS, DG_POOL_PUSH, DG_CU, DG_RECORDS_IN, DG_ACTIVE_LANES,
    DG_C_ROUND, DG_C_EVAL, DG_POOL_TAKE, DG_LOCK_SPINS, DG_T_LAST_ROUND, DG_SPILL_RECORDS, DG_MAX_RING, DG_C_SEED,
    DG_SEED_CALLS, DG_FLUSHES, DG_MIXED_ROUNDS, DG_C_IDLE, DG_C_LOCK, DG_C_SHARE, DG_GIVE, DG_CELLAR_IN,
    DG_CELLAR_OUT, DG_PAD33, DG_PAD34, DG_PAD35, DG_PAD36, DG_PAD37, DG_PAD38, DG_PAD39,
    DIAG_WORDS = 40
};

// Shared (LDS) state of one workgroup.
struct WgState {
    int lock;            // pool lock (lane 0 of the holding wave)
    unsigned pbot, ptop; // pool ring, monotonic indices
    int idle;            // waves with nothing left (no records, pool empty, nothing to seed)
    int phase;           // 0 running, 1 a leader wave is at the HBM queue, 2 exit
    int busy_token;      // the workgroup holds one token of the HBM-queue protocol
    int pad[2];
};

// LDS record arrays (SoA), one per field.
struct LdsRecs {
    double* l;
    double* r;
    double* fl;
    double* fr;
    unsigned* dt;
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

__device__ __forceinline__ void copy_rec(const LdsRecs& R, unsigned i, unsigned j) {
    const double l = R.l[i], r = R.r[i], fl = R.fl[i], fr = R.fr[i];
    const unsigned dt = R.dt[i];
    R.l[j] = l; R.r[j] = r; R.fl[j] = fl; R.fr[j] = fr; R.dt[j] = dt;
}

// Publish k records (LDS slots src(i), i < k) as HBM chunk `slot` (caller: one whole wave).
template <typename SrcIdx>
__device__ __forceinline__ void publish_chunk(const StreamParams& P, const LdsRecs& R, unsigned slot, unsigned k,
                                              SrcIdx src, unsigned lane) {
    Chunk* __restrict__ c = P.chunks + slot;
    for (unsigned i = lane; i < k; i += 64) {
        const unsigned j = src(i);
        st_wt(&c->l[i], R.l[j]); st_wt(&c->r[i], R.r[j]); st_wt(&c->fl[i], R.fl[j]);
        st_wt(&c->fr[i], R.fr[j]); st_wt(&c->dt[i], R.dt[j]);
    }
    if (lane == 0) st_wt(&c->count, k);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the single storing wave drains
    if (lane == 0) st_wt(&P.ready[(size_t)slot * READY_STRIDE], P.epoch);
}

// Per-wave accumulators of the integral currently being summed (`tag`).
struct Acc {
    double area;
    unsigned tasks, leaves, maxd;
};

// Flush a wave's accumulators for integral `tag` into this workgroup's partial (one lane, three
// to five uncontended atomics), and reset them.
__device__ __forceinline__ void flush_acc(const StreamParams& P, Acc& a, int tag, unsigned lane) {
    const double s = wave_sum(a.area);
    const unsigned t = wave_sum_u(a.tasks), l = wave_sum_u(a.leaves), m = wave_max_u(a.maxd);
    if (lane == 0 && t) {
        WgPart* w = P.parts + (size_t)(P.first_slot + tag) * gridDim.x + blockIdx.x;
        atomicAdd(&w->area, s);
        atomicAdd(&w->tasks, (unsigned long long)t);
        atomicAdd(&w->leaves, (unsigned long long)l);
        atomicMax(&w->levels, m);
    }
    a.area = 0.0;
    a.tasks = a.leaves = a.maxd = 0;
}

// Ring slot of monotonic ring index i (WCAP is not a power of two).
__device__ __forceinline__ unsigned ring_slot(unsigned i) { return i % (unsigned)WCAP; }

template <int FID, bool HIST, bool DIAG>
__global__ __launch_bounds__(PT) void k_stream(StreamParams P) {
    __shared__ double s_l[LREC], s_r[LREC], s_fl[LREC], s_fr[LREC];
    __shared__ unsigned s_dt[LREC];
    __shared__ ExpEntry tab[128];
    __shared__ WgState S;
    __shared__ unsigned long long s_dg[DIAG ? DIAG_WORDS : 1];
    __shared__ double2 s_bounds[MAXK];   // {a, b} of every integral of the launch

    const unsigned tid = threadIdx.x;
    const unsigned lane = lane_id();
    const unsigned wid = tid >> 6;
    Ctl* __restrict__ qctl = P.ctls + P.first_slot;
    const LdsRecs R{s_l, s_r, s_fl, s_fr, s_dt};
    const unsigned long long t_entry = rtc();
    stage_exp_table(tab, P.gtab);
    if (tid == 0) {
        S.lock = 0; S.pbot = 0; S.ptop = 0; S.idle = 0; S.phase = 0; S.busy_token = 1;
    }
    if (DIAG) {
        for (unsigned i = tid; i < DIAG_WORDS; i += PT) s_dg[i] = (i == DG_T_FIRST_LEAD) ? ~0ull : 0ull;
    }
    if (tid < (unsigned)P.nprob && tid < (unsigned)MAXK) {
        P.parts[(size_t)(P.first_slot + tid) * gridDim.x + blockIdx.x].cu = cu_slot();
        s_bounds[tid] = P.bounds[tid];
    }
    __syncthreads();   // the only workgroup barrier before the exit

    const double eps = P.eps;
    const int max_depth = P.max_depth;
    const int D = P.D;
    // jobs: job j seeds share j % shares of integral j / shares (integrals in launch order). Wave w
    // does job w first; later jobs are claimed from a counter, one claim in flight per wave, so the
    // waves that draw light shares simply take more of them.
    const unsigned W = gridDim.x * (unsigned)NW;
    const unsigned w_all = blockIdx.x * (unsigned)NW + wid;
    const unsigned shares = (unsigned)P.shares;
    const unsigned total_jobs = (unsigned)P.nprob * shares;
    const unsigned V = shares * (unsigned)P.nshards;
    const unsigned long long npos_total = 1ull << D;
    const unsigned nb = (unsigned)((npos_total + V - 1) / V);   // positions per wave (<= 8)
    const unsigned npairs = (unsigned)D * nb;
    const unsigned base = wid * WCAP;                            // this wave's ring
    // seeding fast path (npairs <= 64): lane q = d*nb + kk; colmask = the lanes of this lane's kk
    unsigned long long colmask = 0;
    if (npairs <= 64) {
        const unsigned kk = lane % nb;
        for (int d = 0; d < D; ++d)
            if ((unsigned)d * nb + kk < 64u) colmask |= 1ull << ((unsigned)d * nb + kk);
    }

    Acc acc{0.0, 0u, 0u, 0u};
    int tag = 0;                  // integral the accumulators belong to (wave-uniform)
    unsigned ctop = 0;            // records in this wave's cellar (wave-uniform)
    Cellar* __restrict__ cel = P.cellar + w_all;
    unsigned job = w_all;         // the job this wave seeds next (wave-uniform)
    bool job_pending = false;     // `job` is still in flight in lane 0's `claim`
    unsigned claim = 0;           // lane 0: the prefetched claim
    unsigned err = 0;
    unsigned top = 0, bot = 0;    // ring indices (wave-uniform)
    bool counted_idle = false;
    unsigned poll_ctr = wid * (POLL_ROUNDS / NW);
    unsigned seen_head = 0, seen_tail = 0;   // lane 0's view of the HBM queue
    unsigned long long spilled = 0;          // records this wave sent to HBM (lane 0)
    unsigned long long lock_spins = 0;
    const unsigned long long t0 = rtc();
    if constexpr (DIAG) {
        if (tid == 0) s_dg[DG_T_START] = t_entry;
    }

    for (;;) {
        unsigned size = top - bot;

        if (size == 0) {
            // ---- out of records: own cellar, then the pool, then the next job's seeds, else idle / lead
            if (ctop > 0) {
                const unsigned k = min(ctop, (unsigned)REFILL), c0 = ctop - k;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's own spills have landed
                for (unsigned q = lane; q < k; q += 64) {
                    const unsigned i = c0 + q, j = base + q;
                    s_l[j] = ld_wt(&cel->l[i]); s_r[j] = ld_wt(&cel->r[i]); s_fl[j] = ld_wt(&cel->fl[i]);
                    s_fr[j] = ld_wt(&cel->fr[i]); s_dt[j] = ld_wt(&cel->dt[i]);
                }
                ctop = c0;
                bot = 0;
                top = k;
                if constexpr (DIAG) { if (lane == 0) atomicAdd(&s_dg[DG_CELLAR_IN], (unsigned long long)k); }
                continue;
            }
            unsigned long long ci = 0;
            if constexpr (DIAG) ci = clk();
            if (counted_idle) {
                const unsigned pt = __hip_atomic_load(&S.ptop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const unsigned pb = __hip_atomic_load(&S.pbot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const int ph = __hip_atomic_load(&S.phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (pt == pb) {
                    if (ph == 2) break;
                    __builtin_amdgcn_s_sleep(4);
                    if constexpr (DIAG) { if (lane == 0) atomicAdd(&s_dg[DG_C_IDLE], clk() - ci); }
                    continue;
                }
            }
            if (job_pending) {
                job = __shfl(claim, 0, 64);
                job_pending = false;
            }
            unsigned k = 0;
            bool lead = false, seed = false;
            int phase;
            wave_lock(&S.lock, lane, lock_spins);
            {
                const unsigned avail = S.ptop - S.pbot;
                phase = S.phase;
                if (avail > 0) {
                    k = min(avail, (unsigned)RB);
                    const unsigned pb = S.pbot;
                    for (unsigned i = lane; i < k; i += 64) copy_rec(R, POOL0 + ((pb + i) & (PCAP - 1)), base + i);
                    if (lane == 0) {
                        S.pbot = pb + k;
                        if (counted_idle) S.idle -= 1;
                    }
                    counted_idle = false;
                } else if (job < total_jobs) {
                    seed = true;
                } else {
                    if (!counted_idle) {
                        if (lane == 0) S.idle += 1;
                        counted_idle = true;
                    }
                    __builtin_amdgcn_wave_barrier();
                    if (phase == 0 && S.idle == NW) {   // every wave idle, pool empty, nothing to seed
                        lead = true;
                        if (lane == 0) S.phase = 1;
                    }
                }
            }
            wave_unlock(&S.lock, lane);
            if constexpr (DIAG) {
                if (lane == 0) {
                    if (k) atomicAdd(&s_dg[DG_POOL_TAKE], (unsigned long long)k);
                    atomicAdd(&s_dg[DG_C_IDLE], clk() - ci);
                }
            }
            if (k) {
                bot = 0;
                top = k;
                continue;
            }

            if (seed) {
                // ---- wave-local seeding of job `job` (see the file header)
                unsigned long long cs = 0;
                if constexpr (DIAG) cs = clk();
                const int p = (int)(job / shares);
                const unsigned vw = (job % shares) * (unsigned)P.nshards + (unsigned)P.shard;
                if (lane == 0) claim = W + g_add(&qctl->spare.v, 1u);   // next job: latency hides behind this one
                job_pending = true;
                if (p != tag) {
                    flush_acc(P, acc, tag, lane);
                    tag = p;
                }
                const double2 ab = s_bounds[p];
                const double A = ab.x, B = ab.y;
                double* fm = s_l + base;          // [npairs + 2]: F(mid of (d,k)) at d*nb+k, then F(A), F(B)
                double* leafa = s_r + base;       // [npairs]: larea + rarea of node (d,k)
                unsigned* flag = s_dt + base;     // [npairs]: node (d,k) refines
                auto position = [&](unsigned kk, bool& valid) -> unsigned long long {
                    const unsigned long long o = (kk & 1u) ? (unsigned long long)(V - 1 - vw) : (unsigned long long)vw;
                    const unsigned long long j = (unsigned long long)kk * V + o;
                    valid = j < npos_total;
                    return j;
                };
                unsigned long long cp1 = 0, cp2 = 0;
                bool alive = false;
                double l = A, r = B, fl = 0.0, fr = 0.0;
                if (npairs <= 64) {
                    // fast path: lane q = d*nb + kk owns node (d, kk) -- its path walk, its F(mid), its
                    // decision; the first leaf depth of every position comes from ONE ballot
                    const unsigned q = lane;
                    const bool isnode = q < npairs;
                    const unsigned d = isnode ? q / nb : 0u, kk = isnode ? q - d * nb : 0u;
                    bool valid = false;
                    const unsigned long long pp = isnode ? position(kk, valid) : 0ull;
                    const unsigned long long anc = valid ? (pp >> (D - (int)d)) : 0ull;
                    unsigned li = npairs, ri = npairs + 1;
                    for (unsigned i = 0; i < d; ++i) {
                        const double m = (l + r) / 2;
                        if ((anc >> (d - 1 - i)) & 1ull) { l = m; li = i * nb + kk; } else { r = m; ri = i * nb + kk; }
                    }
                    const double mid = (l + r) / 2;                           // :187
                    const unsigned fq = npairs + 2 <= 64 ? q : (q < npairs ? q : 64u);
                    double fmid = 0.0;
                    if (fq < npairs + 2)
                        fmid = integrand<FID>(isnode ? mid : (q == npairs ? A : B), tab);   // :188
                    if (fq < npairs + 2) fm[q] = fmid;
                    if (npairs + 2 > 64 && lane < 2) fm[npairs + lane] = integrand<FID>(lane == 0 ? A : B, tab);
                    if constexpr (DIAG) cp1 = clk();
                    bool refine = false;
                    double leafarea = 0.0;
                    if (isnode) {
                        fl = fm[li];
                        fr = fm[ri];
                        const double lrarea = (fl + fr) * (r - l) / 2;        // :185
                        const double larea = (fl + fmid) * (mid - l) / 2;     // :189
                        const double rarea = (fmid + fr) * (r - mid) / 2;     // :190
                        refine = fabs((larea + rarea) - lrarea) > eps;       // :191
                        leafarea = larea + rarea;                             // :199
                    }
                    const unsigned long long leafm = __ballot(isnode && valid && !refine) & colmask;
                    const unsigned dstar = leafm ? (unsigned)__builtin_ctzll(leafm) / nb : (unsigned)D;
                    if (isnode && valid && d <= dstar && (pp & ((1ull << (D - (int)d)) - 1ull)) == 0ull) {
                        ++acc.tasks;                                          // owner of node (d, kk)
                        acc.maxd = max(acc.maxd, d + 1u);
                        if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[d], 1ull);
                        if (d == dstar) {
                            acc.area += leafarea;                             // :199 -> :149
                            ++acc.leaves;
                            if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[AQ_MAX_LEVELS + d], 1ull);
                        } else if ((int)d + 1 >= max_depth) {
                            err |= ERRB_DEPTH;
                        }
                    }
                    // the depth-(D-1) node of a surviving path emits the position's depth-D record
                    alive = isnode && valid && (int)d == D - 1 && dstar >= (unsigned)D && D < max_depth;
                    if (alive) {
                        if (pp & 1ull) { l = mid; fl = fmid; } else { r = mid; fr = fmid; }
                    }
                    if constexpr (DIAG) cp2 = clk();
                } else {
                    for (unsigned q0 = 0; q0 < npairs + 2; q0 += 64) {
                        const unsigned q = q0 + lane;
                        if (q < npairs + 2) {
                            double x;
                            if (q < npairs) {
                                const unsigned d = q / nb, kk = q % nb;
                                bool valid;
                                const unsigned long long pp = position(kk, valid);
                                const unsigned long long anc = valid ? (pp >> (D - (int)d)) : 0ull;
                                double ll = A, rr = B;
                                for (unsigned i = 0; i < d; ++i) {
                                    const double m = (ll + rr) / 2;
                                    if ((anc >> (d - 1 - i)) & 1ull) ll = m; else rr = m;
                                }
                                x = (ll + rr) / 2;
                            } else {
                                x = (q == npairs) ? A : B;
                            }
                            fm[q] = integrand<FID>(x, tab);
                        }
                    }
                    if constexpr (DIAG) cp1 = clk();
                    for (unsigned q0 = 0; q0 < npairs; q0 += 64) {
                        const unsigned q = q0 + lane;
                        if (q < npairs) {
                            const unsigned d = q / nb, kk = q % nb;
                            bool valid;
                            const unsigned long long pp = position(kk, valid);
                            const unsigned long long anc = valid ? (pp >> (D - (int)d)) : 0ull;
                            double ll = A, rr = B;
                            unsigned li = npairs, ri = npairs + 1;
                            for (unsigned i = 0; i < d; ++i) {
                                const double m = (ll + rr) / 2;
                                if ((anc >> (d - 1 - i)) & 1ull) { ll = m; li = i * nb + kk; } else { rr = m; ri = i * nb + kk; }
                            }
                            const double fll = fm[li], frr = fm[ri], fmid = fm[q];
                            const double mid = (ll + rr) / 2;
                            const double lrarea = (fll + frr) * (rr - ll) / 2;    // :185
                            const double larea = (fll + fmid) * (mid - ll) / 2;   // :189
                            const double rarea = (fmid + frr) * (rr - mid) / 2;   // :190
                            flag[q] = fabs((larea + rarea) - lrarea) > eps ? 1u : 0u;   // :191
                            leafa[q] = larea + rarea;                             // :199
                        }
                    }
                    if constexpr (DIAG) cp2 = clk();
                    // resolve: lane kk < nb follows position kk down its path
                    const unsigned kk = lane;
                    bool valid = false;
                    const unsigned long long pp = (kk < nb) ? position(kk, valid) : 0ull;
                    unsigned long long fmask = 0;
                    for (int d = 0; d < D; ++d)
                        fmask |= (unsigned long long)(flag[(unsigned)d * nb + (kk < nb ? kk : 0u)] & 1u) << d;
                    const int dstar = (int)__builtin_ctzll(~fmask);   // first depth that does not refine (D if none)
                    if (valid) {
                        const int dlast = min(dstar, D - 1);
                        for (int d = 0; d <= dlast; ++d) {
                            if ((pp & ((1ull << (D - d)) - 1ull)) == 0ull) {   // owner of node (d, kk)
                                ++acc.tasks;
                                acc.maxd = max(acc.maxd, (unsigned)d + 1u);
                                if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[d], 1ull);
                                if (d == dstar) {
                                    acc.area += leafa[(unsigned)d * nb + kk];          // :199 -> :149
                                    ++acc.leaves;
                                    if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[AQ_MAX_LEVELS + d], 1ull);
                                } else if (d + 1 >= max_depth) {
                                    err |= ERRB_DEPTH;
                                }
                            }
                        }
                        alive = dstar >= D && D < max_depth;
                        if (alive) {
                            unsigned li = npairs, ri = npairs + 1;
                            for (int i = 0; i < D; ++i) {
                                const double m = (l + r) / 2;
                                if ((pp >> (D - 1 - i)) & 1ull) { l = m; li = (unsigned)i * nb + kk; } else { r = m; ri = (unsigned)i * nb + kk; }
                            }
                            fl = fm[li];
                            fr = fm[ri];
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();   // every read of the scratch precedes the seed writes
                const unsigned long long am = __ballot(alive);
                if (alive) {
                    const unsigned j = base + mbcnt(am);
                    s_l[j] = l; s_r[j] = r; s_fl[j] = fl; s_fr[j] = fr; s_dt[j] = (unsigned)D | ((unsigned)p << 8);
                }
                bot = 0;
                top = (unsigned)__popcll(am);
                if constexpr (DIAG) {
                    if (lane == 0) {
                        atomicAdd(&s_dg[DG_SEED_CALLS], 1ull);
                        atomicAdd(&s_dg[DG_C_LOCK], cp1 - cs);
                        atomicAdd(&s_dg[DG_C_SHARE], cp2 - cp1);
                        atomicAdd(&s_dg[DG_FLUSHES], clk() - cp2);
                        atomicAdd(&s_dg[DG_SEEDS], (unsigned long long)top);
                        atomicAdd(&s_dg[DG_C_SEED], clk() - cs);
                        atomicMax(&s_dg[DG_T_SEEDED], rtc());
                    }
                }
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
                    g_add((int*)&qctl->q_tokens.v, -1);
                    S.busy_token = 0;
                }
                const unsigned h = g_add(&qctl->q_head.v, 1u);
                for (unsigned spins = 0;; ++spins) {
                    // both words are read every spin, issued together (one latency per spin)
                    const unsigned rv = h < P.qcap ? ld_wt(&P.ready[(size_t)h * READY_STRIDE]) : 0u;
                    const int tk = g_ld((int*)&qctl->q_tokens.v);
                    if (rv == P.epoch) { cmd = (int)h; break; }
                    if (tk == -(int)gridDim.x) { cmd = -1; break; }
                    if ((spins & 63u) == 63u && rtc() - t0 > P.timeout_ticks) { err |= ERRB_TIMEOUT; cmd = -2; break; }
                    __builtin_amdgcn_s_sleep(2);
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
                s_fr[j] = ld_wt(&c->fr[i]); s_dt[j] = ld_wt(&c->dt[i]);
            }
            if (lane == 0) {
                S.ptop = pt + cnt;
                S.phase = 0;
                S.busy_token = 1;
                S.idle -= 1;   // the leader un-counts itself, so an empty chunk leads to a new leader
                g_add((int*)&qctl->q_tokens.v, 1 - (int)cnt);
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
        if (size > (unsigned)WCAP - 64u * (unsigned)P.ilp) {
            if (ctop + 64u <= (unsigned)CCAP) {
                // the ring's bottom 64 records go down to this wave's cellar (no lock)
                const unsigned i = ctop + lane, j = base + ring_slot(bot + lane);
                cel->l[i] = s_l[j]; cel->r[i] = s_r[j]; cel->fl[i] = s_fl[j]; cel->fr[i] = s_fr[j]; cel->dt[i] = s_dt[j];
                ctop += 64u;
                bot += 64u;
                if constexpr (DIAG) { if (lane == 0) atomicAdd(&s_dg[DG_CELLAR_OUT], 64ull); }
                continue;
            }
            wave_lock(&S.lock, lane, lock_spins);
            const unsigned pt = S.ptop;
            const bool fits = (pt - S.pbot) + 64u <= (unsigned)PCAP;
            if (fits) {
                copy_rec(R, base + ring_slot(bot + lane), POOL0 + ((pt + lane) & (PCAP - 1)));
                if (lane == 0) S.ptop = pt + 64u;
            }
            wave_unlock(&S.lock, lane);
            if (!fits) {
                // pool full: spill 64 records to an HBM chunk (tokens first, then publish)
                unsigned slot = 0;
                if (lane == 0) {
                    slot = g_add(&qctl->q_tail.v, 1u);
                    if (slot < P.qcap) g_add((int*)&qctl->q_tokens.v, 64);
                    spilled += 64;
                }
                slot = __shfl(slot, 0, 64);
                if (slot < P.qcap) {
                    const unsigned b = bot;
                    publish_chunk(P, R, slot, 64u, [&](unsigned i) { return base + ring_slot(b + i); }, lane);
                } else {
                    err |= ERRB_OVERFLOW;   // records dropped: result invalid, error reported
                }
            }
            if constexpr (DIAG) { if (lane == 0) atomicAdd(&s_dg[DG_POOL_PUSH], 64ull); }
            bot += 64;
            continue;
        }

        // ---- feed idle sibling waves
        if (size >= (unsigned)GIVE_MIN && S.idle > 0 && S.ptop == S.pbot) {
            const unsigned k = size / 2u;   // <= WCAP / 2
            wave_lock(&S.lock, lane, lock_spins);
            const unsigned pt = S.ptop;
            const bool fits = (pt - S.pbot) + k <= (unsigned)PCAP;
            if (fits) {
                for (unsigned i = lane; i < k; i += 64)
                    copy_rec(R, base + ring_slot(bot + i), POOL0 + ((pt + i) & (PCAP - 1)));
                if (lane == 0) S.ptop = pt + k;
            }
            wave_unlock(&S.lock, lane);
            if constexpr (DIAG) { if (lane == 0) atomicAdd(&s_dg[DG_GIVE], (unsigned long long)(fits ? k : 0u)); }
            if (fits) {
                bot += k;
                continue;
            }
        }
        // ---- donate to starving workgroups (another CU waits on the HBM queue)
        if (((++poll_ctr) % POLL_ROUNDS) == 0) {
            unsigned slot = 0xffffffffu;
            if (lane == 0) {
                if ((int)(seen_head - seen_tail) > 0) {
                    unsigned expect = seen_tail;
                    if (__hip_atomic_compare_exchange_strong(&qctl->q_tail.v, &expect, seen_tail + 1u, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                        slot = seen_tail;
                }
                seen_head = g_ld(&qctl->q_head.v);
                seen_tail = g_ld(&qctl->q_tail.v);
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
                        if (lane == 0) g_add((int*)&qctl->q_tokens.v, (int)k);
                        publish_chunk(P, R, slot, k, [&](unsigned i) { return POOL0 + ((pb + i) & (PCAP - 1)); }, lane);
                        if (lane == 0) S.pbot = pb + k;
                        wave_unlock(&S.lock, lane);
                    } else {
                        wave_unlock(&S.lock, lane);
                        k = size / 2u;   // may be 0: an empty chunk is harmless
                        if (lane == 0) g_add((int*)&qctl->q_tokens.v, (int)k);
                        const unsigned b = bot;
                        publish_chunk(P, R, slot, k, [&](unsigned i) { return base + ring_slot(b + i); }, lane);
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

        // ---- one round: pop up to 64*K records from the top of this wave's ring, K per lane
        unsigned long long c0 = 0, c1 = 0;
        if constexpr (DIAG) c0 = clk();
        auto do_round = [&](auto kc) -> unsigned {
            constexpr int K = decltype(kc)::value;
            const unsigned n = min(size, 64u * K);
            const unsigned b0 = top - n;
            double l[K], r[K], fl[K], fr[K];
            unsigned dt[K];
            bool act[K], solo[K], refine[K];
            bool mixed = false;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                act[k] = lane + 64u * k < n;
                l[k] = 1.0; r[k] = 1.0; fl[k] = 0.0; fr[k] = 0.0; dt[k] = 0;
                if (act[k]) {
                    const unsigned j = base + ring_slot(b0 + 64u * k + lane);
                    l[k] = s_l[j]; r[k] = s_r[j]; fl[k] = s_fl[j]; fr[k] = s_fr[j]; dt[k] = s_dt[j];
                }
                mixed |= act[k] && (int)(dt[k] >> 8) != tag;
                solo[k] = false;
                refine[k] = false;
            }
            // records of another integral than the accumulators': flush, then follow lane 0's
            // integral; records still of a third one account for themselves (rare: pool/queue moves)
            if (__ballot(mixed)) {
                flush_acc(P, acc, tag, lane);
                tag = __shfl((int)(dt[0] >> 8), 0, 64);
#pragma unroll
                for (int k = 0; k < K; ++k) solo[k] = act[k] && (int)(dt[k] >> 8) != tag;
                if constexpr (DIAG) { if (lane == 0) atomicAdd(&s_dg[DG_MIXED_ROUNDS], 1ull); }
            }
            Step st[K];
            task_step_k<FID, K>(l, r, fl, fr, eps, tab, st);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (!act[k]) continue;
                const unsigned d = dt[k] & 255u;
                const int rtag = (int)(dt[k] >> 8);
                if (HIST) atomicAdd(&P.ctls[P.first_slot + rtag].hist[d], 1ull);
                const bool leaf = !st[k].refine;
                if (st[k].refine) {
                    if ((int)d + 1 >= max_depth) err |= ERRB_DEPTH;
                    else refine[k] = true;
                } else if (HIST) {
                    atomicAdd(&P.ctls[P.first_slot + rtag].hist[AQ_MAX_LEVELS + d], 1ull);
                }
                if (!solo[k]) {
                    ++acc.tasks;
                    acc.maxd = max(acc.maxd, d + 1u);
                    if (leaf) {
                        acc.area += st[k].larea + st[k].rarea;  // :199 -> :149
                        ++acc.leaves;
                    }
                } else {
                    WgPart* w = P.parts + (size_t)(P.first_slot + rtag) * gridDim.x + blockIdx.x;
                    atomicAdd(&w->tasks, 1ull);
                    atomicMax(&w->levels, d + 1u);
                    if (leaf) {
                        atomicAdd(&w->area, st[k].larea + st[k].rarea);
                        atomicAdd(&w->leaves, 1ull);
                    }
                }
            }
            if constexpr (DIAG) c1 = clk();
            unsigned pushed = 0;   // children pairs so far this round
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const unsigned long long mask = __ballot(refine[k]);
                if (refine[k]) {
                    const unsigned pos = b0 + 2u * (pushed + mbcnt(mask));
                    const unsigned j0 = base + ring_slot(pos), j1 = base + ring_slot(pos + 1u);
                    const unsigned cdt = dt[k] + 1u;   // depth + 1, same integral
                    s_l[j0] = l[k];      s_r[j0] = st[k].mid; s_fl[j0] = fl[k];      s_fr[j0] = st[k].fmid; s_dt[j0] = cdt;  // :192-194
                    s_l[j1] = st[k].mid; s_r[j1] = r[k];      s_fl[j1] = st[k].fmid; s_fr[j1] = fr[k];      s_dt[j1] = cdt;  // :195-197
                }
                pushed += (unsigned)__popcll(mask);
            }
            top = b0 + 2u * pushed;
            return n;
        };
        const unsigned n = P.ilp == 2 ? do_round(std::integral_constant<int, 2>{}) : do_round(std::integral_constant<int, 1>{});
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

    // ---------------- exit: flush this wave's accumulators (no workgroup barrier needed) --------
    flush_acc(P, acc, tag, lane);
    const unsigned werr = wave_or_u(err);
    if (lane == 0) {
        if (werr) {
            for (int p = 0; p < P.nprob; ++p)
                atomicOr(&P.parts[(size_t)(P.first_slot + p) * gridDim.x + blockIdx.x].error, werr);
        }
        if (spilled) atomicAdd(&P.parts[(size_t)P.first_slot * gridDim.x + blockIdx.x].spilled, spilled);
        if constexpr (DIAG) {
            atomicAdd(&s_dg[DG_LOCK_SPINS], lock_spins);
            atomicAdd(&s_dg[DG_SPILL_RECORDS], spilled);
        }
    }
    if constexpr (DIAG) {
        __syncthreads();
        if (tid == 0) {
            s_dg[DG_T_EXIT] = rtc();
            s_dg[DG_CU] = cu_slot();
            unsigned long long tasks = 0;
            for (int p = 0; p < P.nprob; ++p)
                tasks += __hip_atomic_load(&P.parts[(size_t)(P.first_slot + p) * gridDim.x + blockIdx.x].tasks,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_dg[DG_TASKS] = tasks;
            unsigned long long* o = P.diag + (size_t)blockIdx.x * DIAG_WORDS;
            for (int i = 0; i < DIAG_WORDS; ++i) o[i] = s_dg[i];
        }
    }
}

}  // namespace aq
