// aq_dfs.h -- the lane-DFS persistent kernel: every lane walks its own subtree depth first.
//
// Reference: /root/reference/aquadPartA.c. The worker's task body (:183-202) is applied by every
// lane to its own current interval, and the farmer's LIFO bag (:152-165) becomes, per lane, the
// depth-first continuation of the reference's recursion:
//   * a refining task (:191-197) continues with its LEFT child [l, mid] and pushes the right end
//     point {r, F(r)} of the pending right child [mid, r] on the lane's stack (16 B, HBM, L2-resident:
//     a push is one store; the top entry is re-read into registers at the end of every iteration,
//     so a pop finds it there one F evaluation later);
//   * an accepted task (:199-201) adds its area to the lane's accumulator and pops the next pending
//     interval [r, top]: its depth follows from a 64-bit path word (bit = "nothing pending to the
//     right at this level"), so the stack holds end points only;
//   * when the wave's LDS pool runs low, refining lanes DONATE their left child [l, mid] to it and
//     continue with the right child; idle lanes take pool records at the top of every iteration
//     (wave-local ballot / mbcnt, no locks, no atomics);
//   * jobs (share j % S of integral j / S, seeded exactly as k_stream: the partition the oracle
//     restates) are claimed when fewer than DSEED_BELOW lanes are busy, so a new job fills the lanes
//     the previous job's tail leaves idle. A wave accumulates two integrals at once (slot bits 0/1,
//     per-lane area and per-wave counters), flushed when a slot's last interval is done.
// Per task, the only memory traffic is one 16-B stack store (refine) or load (accept); everything
// else stays in registers. Every decision is the reference's own arithmetic on the same operands,
// so the interval tree -- tasks and accepted counts -- is bit-identical whatever the schedule.
#pragma once
#include "aq_stream.h"

namespace aq {

constexpr int DW = 16;                 // waves per workgroup (k_dfs)
constexpr int DPT = DW * 64;           // threads per workgroup
constexpr int DPOOL = 128;             // per-wave LDS pool of interval records
constexpr int DLOW = 48;               // refining lanes donate while the pool holds fewer records
constexpr int DSEED_BELOW = 32;        // seed the next job once fewer lanes are busy (pool empty)
constexpr int SDEPTH = 64;             // lane stack entries (pending right siblings <= 63)
constexpr int DSCR = 96;               // per-wave seeding scratch (nodes + 2)
constexpr int REL_NORM = 60;           // path words are renormalised above this relative depth

struct alignas(16) StkEntry {          // pending right end point of a lane's DFS
    double x, fx;
};

// Shared (LDS) state of one k_dfs workgroup: per-wave pools and seeding scratch.
struct DfsLds {
    double pl[DW][DPOOL], pr[DW][DPOOL], pfl[DW][DPOOL], pfr[DW][DPOOL];
    unsigned pmeta[DW][DPOOL];          // depth | slot bit << 8
    double sfm[DW][DSCR];               // seeding: F(mid) per node, then F(A), F(B)
    double sleaf[DW][DSCR];             // seeding: larea + rarea per node (slow path)
    unsigned sflag[DW][DSCR];           // seeding: node refines (slow path)
};


// Flush one accumulation slot of a wave: per-lane areas reduce in double-double into the wave's own
// partial (plain read-modify-write: no other wave touches it), counts go to this workgroup's
// partial with uncontended atomics.
__device__ __forceinline__ void dfs_flush(const StreamParams& P, int tag, double h, unsigned m, unsigned tasks,
                                          unsigned leaves, unsigned lane, unsigned w_all, unsigned nwaves) {
    double hi = h, lo = 0.0;
    wave_sum_dd(hi, lo);
    const unsigned mx = wave_max_u(m);
    if (lane == 0 && tasks) {
        if (P.per_cu) {
            WgPart* w = P.parts + (size_t)(P.first_slot + tag) * gridDim.x + blockIdx.x;
            atomicAdd(&w->tasks, (unsigned long long)tasks);
            atomicAdd(&w->leaves, (unsigned long long)leaves);
            atomicMax(&w->levels, mx);
        }
        slot_flush(P.ctls[P.first_slot + tag], &P.warea[(size_t)(P.first_slot + tag) * P.wstride + w_all], tasks,
                   leaves, mx, hi, lo, w_all);
    }
    __builtin_amdgcn_wave_barrier();   // reconverge: keeps the caller's wave state out of this join
}

template <int FID, bool HIST, bool DIAG>
__global__ __launch_bounds__(DPT) void k_dfs(StreamParams P) {
    __shared__ DfsLds L;
    __shared__ ExpEntry tab[128];
    __shared__ unsigned long long s_dg[DIAG ? DIAG_WORDS : 1];

    const unsigned tid = threadIdx.x;
    const unsigned lane = lane_id();
    const unsigned wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: keeps the wave state in SGPRs
    const unsigned long long t_entry = rtc();
    stage_exp_table(tab, P.gtab);
    if (DIAG) {
        for (unsigned i = tid; i < DIAG_WORDS; i += DPT) s_dg[i] = 0ull;
    }
    if (P.per_cu)
        for (unsigned p = tid; p < (unsigned)P.nprob; p += blockDim.x)
            P.parts[(size_t)(P.first_slot + p) * gridDim.x + blockIdx.x].cu = cu_slot();
    __syncthreads();   // the only workgroup barrier before the exit

    const double eps = P.eps;
    const int max_depth = P.max_depth;
    const int D = P.D;
    const unsigned nwaves = gridDim.x * (unsigned)DW;
    const unsigned w_all = blockIdx.x * (unsigned)DW + wid;
    const unsigned shares = (unsigned)P.shares;
    const unsigned total_jobs = (unsigned)P.nprob * shares;
    const unsigned V = shares * (unsigned)P.nshards;
    const unsigned long long npos_total = 1ull << D;
    const unsigned nb = (unsigned)((npos_total + V - 1) / V);   // positions per share (<= 4)
    const unsigned nlev = (unsigned)D + 1u;                     // seeding evaluates depths 0..D
    const unsigned nnodes = nlev * nb;
    unsigned long long colmask = 0;   // seeding fast path: the lanes of this lane's position column
    if (nnodes <= 64) {
        const unsigned kk = lane % nb;
        for (unsigned d = 0; d < nlev; ++d)
            if (d * nb + kk < 64u) colmask |= 1ull << (d * nb + kk);
    }
    double* __restrict__ pl = L.pl[wid];
    double* __restrict__ pr = L.pr[wid];
    double* __restrict__ pfl = L.pfl[wid];
    double* __restrict__ pfr = L.pfr[wid];
    unsigned* __restrict__ pmeta = L.pmeta[wid];
#ifndef AQ_STK_LANE_MAJOR
    StkEntry* __restrict__ stk = reinterpret_cast<StkEntry*>(P.stk) + (size_t)w_all * SDEPTH * 64 + lane;
    constexpr unsigned SSTRIDE = 64u;
#else
    StkEntry* __restrict__ stk = reinterpret_cast<StkEntry*>(P.stk) + ((size_t)w_all * 64 + lane) * SDEPTH;
    constexpr unsigned SSTRIDE = 1u;
#endif

    // ---- lane state: the current interval and its DFS continuation
    bool act = false;
    unsigned sb = 0;                  // accumulation slot of the lane's interval (0 / 1)
    double l = 1.0, r = 1.0, fl = 0.0, fr = 0.0;
    unsigned dd = 0, d0 = 0, ns = 0;  // depth, root depth of the walk, stack entries (top also in tx/tfx)
    unsigned long long path = 0;      // bit k: nothing pending to the right at depth dd - k
    double tx = 0.0, tfx = 0.0;
    double h0 = 0.0, h1 = 0.0;        // per-lane area of slot 0 / 1
    unsigned m0 = 0, m1 = 0;          // per-lane max level of slot 0 / 1
    unsigned err = 0;
    // ---- wave state (uniform)
    int tag0 = -1, tag1 = -1;         // integral of slot 0 / 1 (-1: free)
    unsigned ct0 = 0, ct1 = 0, cl0 = 0, cl1 = 0;   // tasks / accepted of slot 0 / 1
    unsigned pool_n = 0;
    unsigned job = w_all;             // the job this wave seeds next
    bool job_pending = false;
    unsigned claim = 0;               // lane 0: the prefetched claim
    unsigned long long dg_it = 0, dg_act = 0, dg_don = 0, dg_take = 0, dg_seed = 0, dg_seeds = 0, dg_fl = 0;
    unsigned long long dg_cseed = 0;
    unsigned long long cl_start = 0;
    if constexpr (DIAG) cl_start = clk();

    const unsigned long long t0 = rtc();
    unsigned watch = 0;
    bool running = true;
    do {
        // every wave's loop is bounded in time: a stuck launch reports ERRB_TIMEOUT and drains
        if (__builtin_expect((++watch & 1023u) == 0u, 0) && rtc() - t0 > P.timeout_ticks) {
            err |= ERRB_TIMEOUT;   // drop everything; the loop's single exit below is taken
            act = false;
            pool_n = 0;
            job = total_jobs;
            job_pending = false;
        }
        // the wave state is uniform, but the compiler's uniformity analysis loses track of it across
        // this loop's divergent regions and would keep it in VGPRs (with copies at every join):
        // re-assert it once per iteration
        pool_n = uni(pool_n);
        tag0 = uni(tag0);
        tag1 = uni(tag1);
        ct0 = uni(ct0); ct1 = uni(ct1); cl0 = uni(cl0); cl1 = uni(cl1);
        job = uni(job);
        job_pending = uni((unsigned)job_pending) != 0u;
        // ---- 1. idle lanes take records from the wave pool (LIFO)
        unsigned long long actm = __ballot(act);
        if (pool_n != 0u && actm != ~0ull) {
            const unsigned long long idlem = ~actm;
            const unsigned k = min((unsigned)__popcll(idlem), pool_n);
            const unsigned rank = mbcnt(idlem);
            if (!act && rank < k) {
                const unsigned i = pool_n - 1u - rank;
                l = pl[i]; r = pr[i]; fl = pfl[i]; fr = pfr[i];
                const unsigned meta = pmeta[i];
                dd = d0 = meta & 255u;
                sb = meta >> 8;
                path = 0;
                ns = 0;
                act = true;
            }
            pool_n -= k;
            if constexpr (DIAG) dg_take += k;
            actm = __ballot(act);
        }
        // ---- 2. few busy lanes and nothing pooled: retire finished slots, seed the next job
        bool seeded = false;
        if (pool_n == 0u && (unsigned)__popcll(actm) < (unsigned)DSEED_BELOW) {
            const unsigned long long s1m = __ballot(act && sb);
            if ((actm & ~s1m) == 0ull && tag0 >= 0) {
                dfs_flush(P, tag0, h0, m0, ct0, cl0, lane, w_all, nwaves);
                h0 = 0.0; m0 = 0; ct0 = cl0 = 0; tag0 = -1;
                if constexpr (DIAG) ++dg_fl;
            }
            if (s1m == 0ull && tag1 >= 0) {
                dfs_flush(P, tag1, h1, m1, ct1, cl1, lane, w_all, nwaves);
                h1 = 0.0; m1 = 0; ct1 = cl1 = 0; tag1 = -1;
                if constexpr (DIAG) ++dg_fl;
            }
            if (job_pending) {
                job = uni(__shfl(claim, 0, 64));
                job_pending = false;
            }
            const int p = job < total_jobs ? (int)(job / shares) : -1;
            int s = -1;
            if (p >= 0) {
                if (tag0 == p) s = 0;
                else if (tag1 == p) s = 1;
                else if (tag0 < 0) s = 0;
                else if (tag1 < 0) s = 1;
            }
            if (s >= 0) {
                // ---- wave-local seeding of job `job` into slot s (the partition of k_stream)
                unsigned long long cs = 0;
                if constexpr (DIAG) cs = clk();
                if (s == 0) tag0 = p; else tag1 = p;
                const unsigned vw = (job % shares) * (unsigned)P.nshards + (unsigned)P.shard;
                if (lane == 0) claim = nwaves + g_add(&P.ctls[P.first_slot].jobs.v, 1u);
                job_pending = true;
                const double2 ab = P.bounds[p];   // once per job (HBM / L2)
                const double A = ab.x, B = ab.y;
                double* fm = L.sfm[wid];
                auto position = [&](unsigned kk, bool& valid) -> unsigned long long {
                    const unsigned long long o = (kk & 1u) ? (unsigned long long)(V - 1 - vw) : (unsigned long long)vw;
                    const unsigned long long j = (unsigned long long)kk * V + o;
                    valid = j < npos_total;
                    return j;
                };
                bool alive = false;
                double ql = A, qr = B, qfl = 0.0, qfr = 0.0, qmid = 0.0, qfmid = 0.0;
                unsigned long long ownm = 0, leafm_own = 0;
                double myleaf = 0.0;
                unsigned myd = 0;
                if (nnodes <= 64) {
                    // lane q = d*nb + kk owns node (d, kk): its path walk, its F(mid), its decision;
                    // the first leaf depth of every position comes from ONE ballot
                    const unsigned q = lane;
                    const bool isnode = q < nnodes;
                    const unsigned d = isnode ? q / nb : 0u, kk = isnode ? q - d * nb : 0u;
                    bool valid = false;
                    const unsigned long long pp = isnode ? position(kk, valid) : 0ull;
                    const unsigned long long anc = valid ? (pp >> (D - (int)d)) : 0ull;
                    unsigned li = nnodes, ri = nnodes + 1;
                    // uniform trip count (a lane-dependent one makes the whole wave state divergent)
                    for (unsigned i = 0; i + 1u < nlev; ++i) {
                        if (i < d) {
                            const double mm = (ql + qr) / 2;
                            if ((anc >> (d - 1 - i)) & 1ull) { ql = mm; li = i * nb + kk; } else { qr = mm; ri = i * nb + kk; }
                        }
                    }
                    qmid = (ql + qr) / 2;                                       // :187
                    {   // F at every node's midpoint, lanes nnodes / nnodes+1: F(A), F(B) (:188)
                        const double x[1] = {isnode ? qmid : (q == nnodes ? A : (q == nnodes + 1 ? B : 1.0))};
                        double f[1];
                        integrand_k<FID, 1>(x, f, tab);
                        qfmid = f[0];
                        if (q < nnodes + 2) fm[q] = qfmid;
                        if (nnodes + 2 > 64) {
                            const double y[1] = {lane == 0 ? A : (lane == 1 ? B : 1.0)};
                            integrand_k<FID, 1>(y, f, tab);
                            if (lane < 2) fm[nnodes + lane] = f[0];
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    bool refine = false;
                    double leafarea = 0.0;
                    if (isnode) {
                        qfl = fm[li];
                        qfr = fm[ri];
                        const double lrarea = (qfl + qfr) * (qr - ql) / 2;        // :185
                        const double larea = (qfl + qfmid) * (qmid - ql) / 2;     // :189
                        const double rarea = (qfmid + qfr) * (qr - qmid) / 2;     // :190
                        refine = fabs((larea + rarea) - lrarea) > eps;           // :191
                        leafarea = larea + rarea;                                 // :199
                    }
                    const unsigned long long leafm = __ballot(isnode && valid && !refine) & colmask;
                    const unsigned dstar = leafm ? (unsigned)__builtin_ctzll(leafm) / nb : nlev;
                    const bool own = isnode && valid && d <= dstar && (pp & ((1ull << (D - (int)d)) - 1ull)) == 0ull;
                    const bool ownleaf = own && d == dstar;
                    if (own && d != dstar && (int)d + 1 >= max_depth) err |= ERRB_DEPTH;
                    ownm = __ballot(own);
                    leafm_own = __ballot(ownleaf);
                    if (ownleaf) { myleaf = leafarea; myd = d + 1u; }
                    if (HIST && own) {
                        atomicAdd(&P.ctls[P.first_slot + p].hist[d], 1ull);
                        if (ownleaf) atomicAdd(&P.ctls[P.first_slot + p].hist[AQ_MAX_LEVELS + d], 1ull);
                    }
                    alive = isnode && valid && (int)d == D && dstar >= nlev && D + 1 < max_depth;
                } else {
                    double* leafa = L.sleaf[wid];
                    unsigned* flag = L.sflag[wid];
                    for (unsigned q0 = 0; q0 < nnodes + 2; q0 += 64) {
                        const unsigned q = q0 + lane;
                        if (q < nnodes + 2) {
                            double x;
                            if (q < nnodes) {
                                const unsigned d = q / nb, kk = q % nb;
                                bool valid;
                                const unsigned long long pp = position(kk, valid);
                                const unsigned long long anc = valid ? (pp >> (D - (int)d)) : 0ull;
                                double ll = A, rr = B;
                                for (unsigned i = 0; i + 1u < nlev; ++i) {
                                    if (i < d) {
                                        const double mm = (ll + rr) / 2;
                                        if ((anc >> (d - 1 - i)) & 1ull) ll = mm; else rr = mm;
                                    }
                                }
                                x = (ll + rr) / 2;
                            } else {
                                x = (q == nnodes) ? A : B;
                            }
                            fm[q] = integrand<FID>(x, tab);
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    for (unsigned q0 = 0; q0 < nnodes; q0 += 64) {
                        const unsigned q = q0 + lane;
                        if (q < nnodes) {
                            const unsigned d = q / nb, kk = q % nb;
                            bool valid;
                            const unsigned long long pp = position(kk, valid);
                            const unsigned long long anc = valid ? (pp >> (D - (int)d)) : 0ull;
                            double ll = A, rr = B;
                            unsigned li = nnodes, ri = nnodes + 1;
                            for (unsigned i = 0; i + 1u < nlev; ++i) {
                                if (i < d) {
                                    const double mm = (ll + rr) / 2;
                                    if ((anc >> (d - 1 - i)) & 1ull) { ll = mm; li = i * nb + kk; } else { rr = mm; ri = i * nb + kk; }
                                }
                            }
                            const double fll = fm[li], frr = fm[ri], fmd = fm[q];
                            const double mm = (ll + rr) / 2;
                            const double lrarea = (fll + frr) * (rr - ll) / 2;    // :185
                            const double larea = (fll + fmd) * (mm - ll) / 2;     // :189
                            const double rarea = (fmd + frr) * (rr - mm) / 2;     // :190
                            flag[q] = fabs((larea + rarea) - lrarea) > eps ? 1u : 0u;   // :191
                            leafa[q] = larea + rarea;                             // :199
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    // resolve: lane kk < nb follows position kk down its path; its owned nodes are
                    // counted here, one lane per position (a lane may own several nodes)
                    const unsigned kk = lane;
                    bool valid = false;
                    const unsigned long long pp = (kk < nb) ? position(kk, valid) : 0ull;
                    unsigned long long fmask = 0;
                    for (unsigned d = 0; d < nlev; ++d)
                        fmask |= (unsigned long long)(flag[d * nb + (kk < nb ? kk : 0u)] & 1u) << d;
                    const unsigned dstar = (unsigned)__builtin_ctzll(~fmask);   // first depth that does not refine
                    unsigned owned = 0;
                    if (valid) {
                        const unsigned dlast = min(dstar, (unsigned)D);
                        for (unsigned d = 0; d < nlev; ++d) {
                            if (d <= dlast && (pp & ((1ull << (D - (int)d)) - 1ull)) == 0ull) {   // owner of node (d, kk)
                                ++owned;
                                if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[d], 1ull);
                                if (d == dstar) {
                                    myleaf = leafa[d * nb + kk];                  // :199 -> :149
                                    myd = d + 1u;
                                    if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[AQ_MAX_LEVELS + d], 1ull);
                                } else if ((int)d + 1 >= max_depth) {
                                    err |= ERRB_DEPTH;
                                }
                            }
                        }
                        alive = dstar >= nlev && D + 1 < max_depth;
                        if (alive) {
                            unsigned li = nnodes, ri = nnodes + 1;
                            for (int i = 0; i < D; ++i) {
                                const double mm = (ql + qr) / 2;
                                if ((pp >> (D - 1 - i)) & 1ull) { ql = mm; li = (unsigned)i * nb + kk; } else { qr = mm; ri = (unsigned)i * nb + kk; }
                            }
                            qfl = fm[li];
                            qfr = fm[ri];
                            qmid = (ql + qr) / 2;
                            qfmid = fm[(unsigned)D * nb + kk];
                        }
                    }
                    // counts: a per-lane number of owned nodes -> wave sum
                    const unsigned towned = uni(wave_sum_u(owned));
                    ownm = 0;
                    leafm_own = __ballot(myd != 0u);
                    if (s == 0) ct0 += towned; else ct1 += towned;
                }
                if (nnodes <= 64) {
                    if (s == 0) ct0 += (unsigned)__popcll(ownm); else ct1 += (unsigned)__popcll(ownm);
                }
                if (s == 0) cl0 += (unsigned)__popcll(leafm_own); else cl1 += (unsigned)__popcll(leafm_own);
                if (myd) {
                    if (s == 0) { h0 += myleaf; m0 = max(m0, myd); } else { h1 += myleaf; m1 = max(m1, myd); }
                }
                // a surviving position node hands its two children (depth D + 1) to the pool (:192-197)
                __builtin_amdgcn_wave_barrier();
                const unsigned long long am = __ballot(alive);
                if (alive) {
                    const unsigned i = pool_n + 2u * mbcnt(am);
                    const unsigned meta = (unsigned)(D + 1) | ((unsigned)s << 8);
                    pl[i] = ql; pr[i] = qmid; pfl[i] = qfl; pfr[i] = qfmid; pmeta[i] = meta;
                    pl[i + 1] = qmid; pr[i + 1] = qr; pfl[i + 1] = qfmid; pfr[i + 1] = qfr; pmeta[i + 1] = meta;
                }
                pool_n += 2u * (unsigned)__popcll(am);
                if constexpr (DIAG) {
                    ++dg_seed;
                    dg_seeds += (unsigned)__popcll(am);
                    dg_cseed += clk() - cs;
                }
                __builtin_amdgcn_wave_barrier();
                seeded = true;
            } else if (actm == 0ull) {
                running = false;   // the loop's only exit: no interval left and no job to seed
                seeded = true;
            }
        }

        // ---- 3. one DFS step on every busy lane (:183-202)
        if (!seeded) {
        if constexpr (DIAG) {
            ++dg_it;
            dg_act += (unsigned)__popcll(actm);
        }
        double mid = (l + r) / 2;                                             // :187
        {
            const double x[1] = {act ? mid : 1.0};
            double f[1];
            integrand_k<FID, 1>(x, f, tab);                                   // :188
            const double fmid = f[0];
            const double lrarea = (fl + fr) * (r - l) / 2;                    // :185
            const double larea = (fl + fmid) * (mid - l) / 2;                 // :189
            const double rarea = (fmid + fr) * (r - mid) / 2;                 // :190
            const bool ref = act && fabs((larea + rarea) - lrarea) > eps;     // :191 (strict >)
            const bool deep = ref && (int)dd + 1 >= max_depth;
            if (deep) err |= ERRB_DEPTH;                                      // dropped: the result is invalid
            bool refine = ref && !deep;
            const bool leaf = act && !ref;
            // counts per slot (wave-level), area per lane (:199 -> :149)
            const unsigned long long s1m = __ballot(sb != 0u);
            const unsigned long long lm = __ballot(leaf);
            ct0 += (unsigned)__popcll(actm & ~s1m);
            ct1 += (unsigned)__popcll(actm & s1m);
            cl0 += (unsigned)__popcll(lm & ~s1m);
            cl1 += (unsigned)__popcll(lm & s1m);
            if (leaf) {
                const double v = larea + rarea;
                if (sb) { h1 += v; m1 = max(m1, dd + 1u); } else { h0 += v; m0 = max(m0, dd + 1u); }
            }
            if (HIST && act) {
                const int t = sb ? tag1 : tag0;
                atomicAdd(&P.ctls[P.first_slot + t].hist[dd], 1ull);
                if (leaf) atomicAdd(&P.ctls[P.first_slot + t].hist[AQ_MAX_LEVELS + dd], 1ull);
            }
            // path words stay below 64 bits: drop levels above the shallowest pending entry
            if (__builtin_expect(__ballot(refine && dd - d0 >= (unsigned)REL_NORM) != 0ull, 0)) {
                if (refine && dd - d0 >= (unsigned)REL_NORM) {
                    const unsigned rel = dd - d0;
                    const unsigned long long zeros = ~path & ((1ull << rel) - 1ull);
                    if (zeros == 0ull) {
                        d0 = dd;
                        path = 0;
                    } else {
                        const unsigned h = 63u - (unsigned)__builtin_clzll(zeros);
                        d0 = dd - h - 1u;
                        path &= (h >= 63u) ? ~0ull : ((2ull << h) - 1ull);
                    }
                    if (dd - d0 >= 63u) {   // a pending interval 63 levels up: cannot be represented
                        err |= ERRB_OVERFLOW;
                        refine = false;
                    }
                }
            }
            // donations: refining lanes hand their left child to a low pool
            bool don = false;
            if (pool_n < (unsigned)DLOW) {
                const unsigned long long rm = __ballot(refine);
                if (rm) {
                    const unsigned need = (unsigned)DLOW - pool_n;
                    const unsigned rank = mbcnt(rm);
                    don = refine && rank < need;
                    if (don) {
                        const unsigned i = pool_n + rank;
                        pl[i] = l; pr[i] = mid; pfl[i] = fl; pfr[i] = fmid;              // [l, mid] (:192-194)
                        pmeta[i] = (dd + 1u) | (sb << 8);
                    }
                    const unsigned nd = min(need, (unsigned)__popcll(rm));
                    pool_n += nd;
                    if constexpr (DIAG) dg_don += nd;
                }
            }
            // advance the walk, branch-free: every lane consumes the stack top loaded last
            // iteration (the wait for it falls here, after F(mid)), stores one entry and re-loads
            // the top, so the compiler sees exactly one store and one load per iteration
            {
                const double Tx = tx, Tfx = tfx;
                const unsigned t = (unsigned)__builtin_ctzll(~path);   // levels with nothing pending
                const bool push = refine && !don;                        // [l, mid] next, {r, F(r)} pending
                const bool pop = act && !refine && t < dd - d0;          // next: the pending [r, top]
                const bool fin = act && !refine && t >= dd - d0;         // this walk is finished
                // pushers write {r, F(r)} at their new entry; every other lane writes the free slot
                // above its top (harmless)
                StkEntry e;
                e.x = r;
                e.fx = fr;
                stk[(size_t)ns * SSTRIDE] = e;                               // :195-197
                l = don ? mid : (pop ? r : l);
                fl = don ? fmid : (pop ? fr : fl);
                r = push ? mid : (pop ? Tx : r);
                fr = push ? fmid : (pop ? Tfx : fr);
                path = refine ? ((path << 1) | (don ? 1ull : 0ull)) : (pop ? ((path >> t) | 1ull) : path);
                dd = refine ? dd + 1u : (pop ? dd - t : dd);
                ns = push ? ns + 1u : (pop ? ns - 1u : ns);
                act = act && !fin;
                // the next top (a pusher's own store above: same-wave accesses to one address stay
                // in order); its latency hides behind the next F(mid)
                const StkEntry n = stk[(size_t)(ns ? ns - 1u : 0u) * SSTRIDE];
                tx = n.x;
                tfx = n.fx;
            }
        }
        // reconverge here, before the loop latch: otherwise the latch joins the divergent branches
        // above with the seeding path, and every piece of wave state (pool size, slot tags,
        // counters) is classed divergent and kept in VGPRs
        __builtin_amdgcn_wave_barrier();
        }
    } while (__builtin_amdgcn_readfirstlane((unsigned)running));   // a uniform exit, by construction

    // ---------------- exit: both slots are flushed; report errors and diagnostics --------------
    if (tag0 >= 0) dfs_flush(P, tag0, h0, m0, ct0, cl0, lane, w_all, nwaves);
    if (tag1 >= 0) dfs_flush(P, tag1, h1, m1, ct1, cl1, lane, w_all, nwaves);
    const unsigned werr = wave_or_u(err);
    if (lane == 0 && werr) {
        for (int p = 0; p < P.nprob; ++p)
            atomicOr(&P.ctls[P.first_slot + p].sums.error, werr);
    }
    if constexpr (DIAG) {
        if (lane == 0) {
            atomicAdd(&s_dg[DG_ROUNDS], dg_it);
            atomicAdd(&s_dg[DG_ACTIVE_LANES], dg_act);
            atomicAdd(&s_dg[DG_ACTIVE_TASKS], dg_act);
            atomicAdd(&s_dg[DG_GIVE], dg_don);
            atomicAdd(&s_dg[DG_POOL_TAKE], dg_take);
            atomicAdd(&s_dg[DG_SEED_CALLS], dg_seed);
            atomicAdd(&s_dg[DG_SEEDS], dg_seeds);
            atomicAdd(&s_dg[DG_FLUSHES], dg_fl);
            atomicAdd(&s_dg[DG_C_SEED], dg_cseed);
            atomicAdd(&s_dg[DG_C_LOOP], clk() - cl_start);
            atomicMax(&s_dg[DG_T_LAST_ROUND], rtc());
        }
        __syncthreads();
        if (tid == 0) {
            s_dg[DG_T_START] = t_entry;
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
