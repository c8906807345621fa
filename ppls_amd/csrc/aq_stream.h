// aq_stream.h -- the persistent on-device farmer: K integrals per launch, one wavefront per worker.
//
// Reference: /root/reference/aquadPartA.c. The farmer's LIFO bag (:125-173) and the workers' task
// body (:183-202) become one persistent launch:
//   * the unit of work is a SIBLING PAIR {a, b, F(a), F(m), F(b), dt} = the two tasks [a,m] and [m,b]
//     a refining parent pushes (:192-197); m = (a+b)/2 is recomputed from the parent's own operands
//     (:187), so it is not stored; dt = depth | integral << 8 | SPAN_BIT (bit 31). A pair is six 8-byte LDS
//     fields for two tasks, and it hands every lane two independent evaluations: the K=2 cosh chains
//     interleave (aq_libm.h cosh_main_k).
//   * worker = WAVEFRONT. Each of the NW waves of a workgroup owns an LDS ring of pairs, and each of its
//     lanes carries one pair in registers. A round fills the idle lanes from the ring, evaluates F at
//     both midpoints of every held pair in FP64 (glibc-exact cosh), applies the reference's refine
//     test (:191) to both tasks, keeps task 0's children as the lane's next pair and pushes task 1's
//     onto the ring, with a ballot / mbcnt compaction: no workgroup barrier, no HBM traffic. Rounds
//     run in bursts with all ring state wave-uniform (SGPRs).
//   * ring overflow goes to the wave's private HBM cellar (no lock; prefetched back when the ring
//     runs low); a locked LDS pool feeds idle sibling waves; an HBM ticket queue of pair chunks moves
//     work across CUs (what the bag of tasks is for), driven by one elected leader wave per idle
//     workgroup; busy waves donate to waiting tickets. Termination: a two-level token count (QCtl).
//   * jobs: job j seeds share j % shares of integral j / shares. Seeding is WAVE-LOCAL: virtual
//     worker vw = share*nshards + shard of V owns the depth-D positions j = k*V + (k odd ? V-1-vw : vw)
//     (snake order). All F evaluations of the positions' paths (depths 0..D) are independent (pure
//     (l+r)/2 recursion), so one wave evaluates them in one pass, decides every node, and keeps the
//     children of each surviving position node as its first pair. A task at depth <= D is counted by
//     the owner of its leftmost descendant position (the partition oracle/aq_oracle.c restates).
//     Launches of many integrals claim jobs from a counter (one claim in flight per wave), so the
//     tail of one integral overlaps the start of the next; launches of few take a static stride.
//   * accepted areas / task counts accumulate per lane in registers per integral and are flushed
//     (DPP wave reduction + device atomics into the integral's slot: counts, and the area into an
//     exact fixed-point accumulator, aq_xsum.h) when a wave switches integral, runs dry or exits
//     (the farmer's `result += buff[0]`, :149).
// Every decision is the reference's own arithmetic on the same operands, so the interval tree --
// tasks and accepted counts -- is bit-identical whatever the schedule.
#pragma once
#include "aq_device.h"
#include "aq_xsum.h"

namespace aq {

typedef double f64x2 __attribute__((ext_vector_type(2)));

#ifndef AQ_PT
#define AQ_PT 768
#endif
#ifndef AQ_WCAP
#define AQ_WCAP 256
#endif
constexpr int PT = AQ_PT;           // threads per workgroup
constexpr int NW = PT / 64;         // waves (workers) per workgroup: 12, three per SIMD
constexpr int WCAP = AQ_WCAP;       // per-wave LDS ring, pairs: a round pops <= 64, pushes <= 128
// LDS pair block, one field per array of LREC slots (SoA): a | b | fa | fm | fb | dt, the pair word
// dt in the low half of an 8-byte field. With LREC = 50 x 64 every field of a slot lies at 0 / 50 /
// 100 / 150 / 200 / 250 x 512 B from the slot's a -- inside the reach of ds_read2st64 /
// ds_write2st64 offsets (8 bits of 512 B): a round's pop is three read2st64 and a push three
// write2st64 from ONE address (r02 A/B, 8192 x eps=1e-10: 26.17 -> 25.85 ms per launch against
// five fields + a 4-byte dt array, which needed a second base for fm / fb and a dt address per
// access; the pool went from 256 to 128 pairs to make room).
constexpr int PCAP = 128;           // per-workgroup LDS pool ring, pairs (power of two)
constexpr int DT_STRIDE = 2;        // dt words per slot (the low word of an 8-byte field)
constexpr int LREC = NW * WCAP + PCAP;   // LDS pair slots: 3200 x 48 B = 150 KiB
constexpr int POOL0 = NW * WCAP;    // first pool slot
constexpr int CH = PCAP;            // pairs per HBM queue chunk (<= PCAP: a chunk lands in an empty pool)
// the pair words of the LDS block: slot j's word at p[DT_STRIDE * j]
struct DtField {
    unsigned* p;
    __device__ __forceinline__ unsigned& operator[](unsigned j) const { return p[DT_STRIDE * j]; }
    __device__ __forceinline__ DtField operator+(unsigned o) const { return DtField{p + DT_STRIDE * o}; }
};
#ifndef AQ_S_W
#define AQ_S_W 2
#endif
constexpr int S_W = AQ_S_W;              // seed depth D = floor(log2 V) + S_W: 3 or 4 positions per share
#ifndef AQ_JOB_RUN_MAX
#define AQ_JOB_RUN_MAX 16
#endif
constexpr int JOB_RUN_MAX = AQ_JOB_RUN_MAX;   // most jobs one claim takes (whole-integral jobs only)
#ifndef AQ_GSS_DIV
#define AQ_GSS_DIV 2
#endif
// Guided claims (r05): a claimed run holds min(JOB_RUN_MAX, jobs left / (GSS_DIV x W)) jobs, so the runs
// shrink to one job as the counter nears the end and the waves run dry together. With fixed runs of 16
// tiny jobs (C3 at eps=1e-3: ~1 400 tasks, ~20 us each) the last runs claimed held the launch ~0.1-0.3
// ms past the others (DIAG: last rounds spread over ~100 us of a 512 us launch, profiles/r05a).
constexpr unsigned GSS_DIV = AQ_GSS_DIV;
#ifndef AQ_S_W1
#define AQ_S_W1 2
#endif
#ifndef AQ_HEAP_SEED
#define AQ_HEAP_SEED 1
#endif
// whole-integral jobs (V = 1) seed the top HEAP_D + 1 levels, one node per lane in heap order: the k_stream
// instance the batch front end launches (HEAPS, aq_abi.inc batch_heap) -- tiny trees of big batches. The
// other instances leave the path out: compiled into the bench's instance, unused there, it had cost the
// bench launch 0.6 % (profiles/r06h: 80.27-80.33 against 79.73-79.91 ms, code placement)
constexpr bool HEAP_SEED = AQ_HEAP_SEED != 0;
constexpr int HEAP_D = 4;
constexpr unsigned HEAP_NODES = (2u << HEAP_D) - 1u;   // 31 nodes + F(A), F(B): 33 lanes
static_assert(HEAP_NODES + 2u <= 64u, "the heap seeding path is one node per lane");
// seed depth of a job: floor(log2 V) + S_W for V = shares x shards virtual workers; a whole-integral
// job (V = 1, tiny trees of big batches) seeds at S_W1 (its partition is the whole tree at any depth)
__host__ __device__ constexpr int seed_depth(unsigned long long V) {
    return V <= 1ull ? AQ_S_W1 : 63 - __builtin_clzll(V) + S_W;
}
// positions per share, ceil(2^D / V): with L = floor(log2 V), 2^D / V lies in (2^(D-L-1), 2^(D-L)], so a
// count-down of at most 2^(D-L-1) steps instead of a 64-bit division (cold code at every seeding)
__host__ __device__ constexpr unsigned seed_nb(int D, unsigned long long V) {
    if (V <= 1ull) return 1u << D;
    unsigned nb = 1u << (D - (63 - __builtin_clzll(V)));
    while (nb > 1u && (unsigned long long)(nb - 1u) * V >= (1ull << D)) --nb;
    return nb;
}
// a job's seed depth: seed_depth(V), one level deeper where the seeding's one-wave fast path
// ((D + 1) levels x nb positions <= 64 nodes) still holds the deeper seeding -- the bench's adaptive
// jobs (V ~ 24: 3 -> 6 positions per share) and whole-integral jobs (V = 1: 4 -> 8 positions); not a
// lone launch (V = 3072: 42 -> 90 nodes). r04n A/B at 32768 integrals: -0.8 %, C3 unchanged
// (profiles/r04n2). The oracle's shard partition restates this rule (tests' device_seed_S).
__host__ __device__ constexpr int seed_depth_job(unsigned long long V) {
    return (unsigned long long)(seed_depth(V) + 2) * seed_nb(seed_depth(V) + 1, V) <= 64ull
        ? seed_depth(V) + 1 : seed_depth(V);
}
// q / nb for small q (seeding's lane -> node map): the float estimate q * rcp(nb), then one
// correction each way (exact whenever the estimate is off by at most one)
__device__ __forceinline__ unsigned div_small(unsigned q, unsigned nb, float rnb) {
    unsigned d = (unsigned)((float)q * rnb);
    d += (d + 1u) * nb <= q ? 1u : 0u;
    d -= d * nb > q ? 1u : 0u;
    return d;
}
#ifndef AQ_GIVE_MIN
#define AQ_GIVE_MIN 96
#endif
constexpr int GIVE_MIN = AQ_GIVE_MIN;        // a busy wave feeds the pool for idle siblings only above this size
constexpr int DONATE_MIN = 64;      // pool pairs needed before a workgroup donates from its pool
#ifndef AQ_POLL_ROUNDS
// A/B r01q (8192 integrals, eps 1e-10): 16 34.26, 32 33.35, 64 32.95 ms per launch; r03 (in-burst
// moves, wave priority; the bench's 32768-integral launch, profiles/r03x): 128 with GIVE 64; r04: 256
// with GIVE 128 (below; 128 is the largest give period the depth byte allows at AQ_MAX_LEVELS 128)
#define AQ_POLL_ROUNDS 256
#endif
constexpr int POLL_ROUNDS = AQ_POLL_ROUNDS;     // a busy wave refreshes its view of the HBM queue every POLL_ROUNDS rounds
#ifndef AQ_GIVE_ROUNDS
// r02 (burst loop, PF_BELOW 64): 8 -> 16 -> 32 rounds 28.15 -> 27.93 ms... 64 slower; C3 unchanged.
// r03 (bursts no longer end at cellar moves, so the give / poll round is their main end): 64 / 128 with
// 60 k-task jobs -1.8 % on the bench launch (profiles/r03x), 16 +1.5 %, 128 / 256 -0.5 %; r04 (carried
// pairs: a burst's end pushes the held pairs back, so longer bursts pay): 128 / 256 -0.8 % against
// 64 / 128 on the bench's 32768-integral launch (profiles/r04k2/ab.txt)
#define AQ_GIVE_ROUNDS 128
#endif
constexpr int GIVE_ROUNDS = AQ_GIVE_ROUNDS;      // ... and looks for idle siblings every GIVE_ROUNDS rounds
#ifndef AQ_SKEWED_GIVE
#define AQ_SKEWED_GIVE 4
#endif
constexpr int SKEWED_GIVE = AQ_SKEWED_GIVE;   // give rounds for the skewed built-in integrand (sin(1/x))
#ifndef AQ_SKEWED_POLL
#define AQ_SKEWED_POLL 64   // (the measured sin(1/x) setting, kept when cosh4's poll went to 128)
#endif
constexpr int SKEWED_POLL = AQ_SKEWED_POLL;
#ifndef AQ_SKEWED_GIVE_MIN
#define AQ_SKEWED_GIVE_MIN AQ_GIVE_MIN
#endif
constexpr int SKEWED_GIVE_MIN = AQ_SKEWED_GIVE_MIN;
// (lone-integral launches, whose waves run only ~3-13 rounds of one share, measured with give /
// poll intervals of 2-16 rounds and GIVE_MIN 32-64: all slower, 1e-10 up to 2x -- HBM donations
// and bursts cut short cost more than the balance they buy; profiles/r02_ab)
#ifndef AQ_LEAD_SLEEP
#define AQ_LEAD_SLEEP 2     // s_sleep units (64 clocks) between a waiting leader's polls
#endif
// AQ_STAMPS=1 (diagnostic builds only, tools/stamps_single.py): every wave of the plain instance
// keeps the 100 MHz realtime clock at a few points of its life in registers and stores them once at
// its exit (g_aq_stamps, read back by aq_debug_stamps) -- the lone launch's timeline without the DIAG
// instance's LDS atomics
#ifndef AQ_WIDE_TAB
#define AQ_WIDE_TAB 1   // the bulk cosh4 instance's 256-entry exp table (k_stream WIDE)
#endif
#ifndef AQ_STAMPS
#define AQ_STAMPS 0
#endif
#ifndef AQ_X_NOFOLD
#define AQ_X_NOFOLD 0   // timing experiments only (wrong areas): per-CU launches skip the exit's area fold
#endif
#ifndef AQ_X_NOCUACC
#define AQ_X_NOCUACC 0  // timing experiments only: no per-CU task counter atomic at exit
#endif
#ifndef AQ_FLUSHX
#define AQ_FLUSHX 0   // timing experiments on the flush (stamps builds only): 1 no reductions, 2 no atomics,
                      // 3 no double-double reduction, 4 no integer reductions
#endif
// Per-CU (lone) launches: a new leader first polls only its group's end flag, for up to LAZY_TICKET
// spins, before it takes a queue ticket -- at a lone launch's end 255 leaders drawing tickets from one
// counter (~12 ns each, MI355X_MICROARCH.md "fanin") held the last of them ~3 us past the end (r04j/k)
constexpr unsigned LAZY_TICKET = 64;
// Per-CU launches of the skewed integrand (sin(1/x): one region holds nearly all of the tree): a burst
// that starts with at least HEAVY_S pairs runs its rounds at priority 3 throughout; the others start
// at 1 and drop to 0 after their F chains -- the waves holding the most work win the SIMD's issue
// (config-4 lone 80.6 -> 76.8 us; for cosh4 no gain at thresholds 32 / 64 / 128, r04p)
constexpr unsigned HEAVY_S = 64;
// (ST_CB .. ST_NR are sums, not stamps: shader cycles inside bursts and in the wave's loop, bursts
// and rounds -- where a long launch's wave time goes, tools/stamps_burst.py)
// (ST_CS: cycles in seeding passes, ST_CF: in their flushes of the previous integral, ST_CBD: in their
// bounds loads, ST_NS: seeding passes)
enum : int { ST_ENTRY = 0, ST_INIT, ST_SEED_IN, ST_SEEDED, ST_IDLE, ST_LEAD, ST_BROKE, ST_FLUSHED, ST_EXIT,
             ST_XCC, ST_PRE, ST_CLASS, ST_FEVAL, ST_DONE, ST_KARG, ST_CB, ST_CL, ST_NB, ST_NR, ST_CS, ST_CF,
             ST_CBD, ST_NS, ST_N, ST_STRIDE = 24 };
constexpr int READY_STRIDE = 32;    // one ready flag per 128-B line: pollers never share a line
constexpr int MAXG = 2048;          // max persistent workgroups per launch
constexpr unsigned SHARE_ROT = 1021;   // static-job launches: share offset from one integral to the next
// launches of fewer integrals keep per-workgroup (per-CU) counts and LDS exact accumulators (the LDS
// left beside the pair block holds 12)
constexpr int PCU_MAXK = 12;
constexpr int PCU_ROW = PCU_MAXK - 1;   // per-CU LDS rows: tags < k < PCU_MAXK
constexpr int STATIC_MAXK = 16;     // sharded launches of fewer integrals: one share per wave, static stride
                                    // (unsharded: below PCU_MAXK, aq_abi.inc launch_stream)
// The pair word dt: bits 0-7 the pair's depth (the depth of its two tasks), bits 8-30 the integral
// (tag), bit 31 SPAN_BIT. SPAN_BIT (cosh4): the pair's interval lies where glibc's cosh takes its exp
// path (cosh_main_span) -- set at seeding, inherited by the children (sub-intervals), so a round tests
// the word's sign instead of two words.
constexpr unsigned SPAN_BIT = 1u << 31;
constexpr int TAG_SHIFT = 8;
constexpr unsigned TAG_MASK = (1u << 23) - 1u;
__host__ __device__ constexpr unsigned dt_tag(unsigned dt) { return (dt >> TAG_SHIFT) & TAG_MASK; }
// max integrals per launch: 8 x 32768, so that N = 8 ranks holding 1/8 of each integral of a batch
// pack the same work into one launch as one GPU does with the whole batch (r04)
constexpr int MAXK = 1 << 18;
static_assert((unsigned)MAXK - 1u <= TAG_MASK, "the tag field must hold every integral of a launch");
// slots whose per-CU launches keep per-workgroup words (parts), plus one row for the sync slot
// PCU_AREA: a per-CU launch's area is kept per workgroup -- each wave adds its flushes' double-doubles
// into its own LDS pair per integral (flush_acc), the workgroup's last wave sums its waves' into two
// doubles beside the count words (StreamParams::parea) -- and readers add the grid's pairs into the slot's
// exact accumulator: k_fold_parts after an asynchronous per-CU launch, k_fetch_sync / k_pack_group on the
// synchronous and group paths. So the area of a lone integral is the correctly rounded sum of 2 x grid
// doubles, each a double-double of its workgroup's waves' partials (no far atomic at the launch's end).
// (r06: 16384, was 65536 -- with the per-workgroup area words beside the counts, PCU_AREA, the two blocks
// take 134 MB where the counts alone took 268 MB)
constexpr int NPARTS = 16384;
__host__ __device__ __forceinline__ size_t parts_row(int slot) { return slot < NPARTS ? (size_t)slot : (size_t)NPARTS; }
#ifndef AQ_GSPLIT_DEFAULT
// sharded launches / first launch: 16 shares per integral over all shards (2-rank rehearsal, r03: 32 ->
// 1.743e11, 64 -> 1.778e11, 96 -> 1.803e11; r04, per task of a launch of N x 16384 integrals sharded
// N ways, profiles/r04n5/shard_ab.txt: 96 -> 192 = +1.3 / +0.3 / +0 % at N = 2 / 4 / 8, 384 -0.8 % at 8)
#define AQ_GSPLIT_DEFAULT 192
#endif
constexpr int DEFAULT_GSPLIT = AQ_GSPLIT_DEFAULT;  // a multi-integral launch's job = the share of this many waves
#ifndef AQ_LONE_GSPLIT
#define AQ_LONE_GSPLIT 1   // waves per share in launches of < 16 unsharded integrals (host side, aq_abi.inc)
#endif
#ifndef AQ_TASKS_PER_JOB
// A/B at 8192 integrals per launch (r01): 8k 35.4, 15k 33.7, 25k 33.6, 40k 33.1, 60k 33.3, 100k 37.0 ms;
// r03 at the bench's 32768 per launch (profiles/r03x): 60 k -1.8 % with give / poll 64 / 128, 80 k -1.3 %;
// r04n (give / poll 128 / 256, one level deeper seeding, profiles/r04n3) vs 60 k: 90 k -1.0 %,
// 120 k -1.3 %, 180 k -0.9 %, 240 k +0.8 %
#define AQ_TASKS_PER_JOB 120000
#endif
constexpr unsigned TASKS_PER_JOB = AQ_TASKS_PER_JOB;   // adaptive job size: a job holds about this many tasks
#ifndef AQ_CCAP
#define AQ_CCAP 2048
#endif
// pairs per wave cellar (private HBM overflow stack, 96 KiB). The deepest cellar of any wave measured
// 448 pairs at eps=1e-10 and 576 at 1e-12 (DIAG max_cellar, every workgroup, profiles/r05o); 4096 had
// held 604 MB per context for nothing. A wave whose cellar is full spills to the pool / HBM queue.
constexpr int CCAP = AQ_CCAP;
#ifndef AQ_FLUSH_LDS
#define AQ_FLUSH_LDS 0
#endif
// the flush sums the lanes' area digits in an LDS window instead of a double-double wave reduction
constexpr bool FLUSH_LDS = AQ_FLUSH_LDS;
constexpr int REFILL = WCAP - 64;   // pairs a wave with an empty ring takes back from its cellar
#ifndef AQ_PF_BELOW
// r02 A/B (8192-integral launch, GIVE_ROUNDS 32): 112 28.39, 96 27.93, 80 27.57, 64 27.20, 48 28.18,
// 32 30.25 ms, no prefetch 33.37 ms. The old 128 (= WCAP - 128) made a ring that had just spilled
// its bottom 64 pairs (above 192) fetch the same 64 back a few rounds later: a ping-pong of one chunk.
#define AQ_PF_BELOW (WCAP / 4)
#endif
constexpr int PF_BELOW = AQ_PF_BELOW;   // below this ring size a wave prefetches 64 cellar pairs
// Lazy landing (r03). The prefetch used to be issued at <= PF_BELOW pairs and landed one round later,
// inside a one-round burst: the landing's wait for the HBM loads (~2 us under load) stalled the wave
// at nearly every cellar cycle (r03 A/B estimate: ~2.6 us per spill + prefetch, a fifth of the bench
// launch). Now the loads go out at <= PF_ISSUE pairs, the bursts go on with them in flight, and they
// land when the ring is down to <= PF_BELOW (a ring simulator of the bench's jobs, tools/ring_sim.py:
// 80 % of the prefetches then have >= 2 rounds to arrive instead of 1). A ring that overflows while
// they are in flight cancels them (the pairs are still in the cellar: only ctop moved) and spills.
#ifndef AQ_PF_ISSUE
#define AQ_PF_ISSUE 160   // r03 A/B (8192 x eps=1e-10): 96 -0.6 %, 128 -1.8 %, 160 -2.4 % vs landing after one round
#endif
constexpr int PF_ISSUE = AQ_PF_ISSUE;
static_assert(PF_ISSUE >= PF_BELOW && PF_BELOW + 64 <= WCAP - 64, "a landed prefetch must leave the ring below the spill line");
// In-burst cellar moves (r03): a round that leaves the burst's size window at a cellar edge -- above
// the spill line, or down to the prefetch issue / landing line -- moves the chunk inside the burst
// and the burst goes on, where round 2 left the burst for the outer loop (~60 VALU and ~70 SALU of
// re-checks and state moves per exit, 0.24 exits per round: tools/ring_sim.py, PMC r03e).
//
// Wave priority. r03's popped round ran at s_setprio 3 from its pop to the end of its two F chains and
// at 0 for its tail (-0.6..-0.8 %, profiles/r03s-r03u); the carried round is faster WITHOUT it
// (-0.9 %, three A/B rounds, profiles/r04z/ab.txt), so only the sin(1/x) per-CU instance still sets
// priorities (its heaviest waves, below).
//
// Depth cap checked once per burst (r03): a round pushes every refining task's children and keeps, per
// lane, the deepest REFINING pair it saw (masked max, as before over the popped pairs); the burst's
// end tests that against max_depth - 1 -- one compare per burst instead of a compare, two SALU and a
// branch per round. A burst runs at most give_rounds rounds, so pairs past the cap are at most
// give_rounds levels deeper: the depth byte (dt's low 8 bits) cannot carry into the tag while
// (AQ_MAX_LEVELS - 1) + give_rounds < 256 (asserted below). A wave that finds the cap exceeded drops
// its ring and cellar before anything else can see them: nothing deeper than the cap ever reaches the
// pool or the HBM queue. The run is then invalid (ERRB_DEPTH), as before. (The histogram instance
// keeps the per-round test.)
static_assert((AQ_MAX_LEVELS - 1) + (GIVE_ROUNDS > SKEWED_GIVE ? GIVE_ROUNDS : SKEWED_GIVE) < 256,
              "a burst's pairs past the depth cap must not carry the depth byte into the tag");
constexpr int SPILL = 64;   // pairs a ring above WCAP - 64 moves to its cellar at once (r02 A/B: 128 at once
                            // 4.0 % slower at eps 1e-10, 6.5 % at 1e-12: more refills)

struct alignas(128) Line {
    unsigned v;
    unsigned pad[31];
};

// One launch's HBM ticket queue and termination count (a line per word: pollers and atomics never
// share a line). A context keeps two and its launches use them in turn; workgroup 0 of a launch
// zeroes the one the next launch will use (a context's launches run in stream order), so every
// launch starts from zeros without a reset of its own.
//
// Termination (token counting, two levels): the workgroups form NGROUP groups (workgroup b in group
// b % NGROUP); idle[g] counts the idle workgroups of group g, and
//   T = (groups with a busy workgroup) + sum over published, unconsumed chunks of (records + 1).
// T starts at T0 = min(G, NGROUP) (tokens stores T - T0) and the run is over when T reaches 0. A
// workgroup going idle adds 1 to its group's idle count; the one that makes the group all-idle takes
// the group's token out of T. A workgroup taking a chunk (c records) subtracts 1 from its idle
// count and adds (1 if the group was all-idle) - (c + 1) to T in one atomic. Every outstanding chunk
// holds at least one token, so T stays positive while any chunk or busy workgroup exists: between a
// group's 0 -> 1 busy transition and its T update, the taken chunk's own tokens are still counted.
// The atomic that brings T to 0 is unique; its workgroup stores the end into one `done` line per
// group, which that group's waiting leaders poll. (One counter for all 256 workgroups made the final
// 256 idle transitions a ~3 us fan-in on one line, then a poll of that same line by all of them.)
constexpr int NGROUP = 8;
struct QCtl {
    Line tail;                 // chunk slots claimed by producers
    Line head;                 // tickets taken by idle workgroups
    Line tokens;               // T - T0
    Line jobs;                 // job claims beyond the first W
    Line idle[NGROUP];         // idle workgroups per group
    Line done[NGROUP];         // 1: T reached 0, every workgroup exits -- one line per group, polled by
                               // that group's waiting leaders only (32 pollers per line, not 256)
};
// Per-integral totals: device-scope atomics at every flush (the farmer's `result += buff[0]`, :149,
// and tasks_per_process, :162). The area is the exact fixed-point sum of the waves' double-double
// partials (aq_xsum.h): order-independent, rounded once when it is read.
struct alignas(128) SlotSums {
    unsigned long long tasks, leaves, spilled;
    unsigned levels, error;
    unsigned pcu;       // 1: a per-CU launch wrote this slot's counts as per-workgroup words (parts),
                        // not into tasks / leaves / levels -- readers add them (slot_counts)
    unsigned win_lo_not, win_hi;   // the area limbs ever added to: [~win_lo_not, win_hi), both folded by
                                   // max (aq_xsum.h xs_win_lo / xs_win_hi; 0 / 0 = none) -- the batch
                                   // gather reads and re-zeroes only these (k_gather_reset)
};
// Per-integral totals and histogram accumulators, one per async slot; all-zero when a launch starts
// (the host zeroes used slots lazily, in batches).
struct Ctl {
    SlotSums sums;
    XSum area;                 // exact Σ of the accepted areas (larea + rarea, :199)
    unsigned long long hist[2 * AQ_MAX_LEVELS];   // [0,L): tasks per level, [L,2L): accepted per level
};

// Counts of lone-integral (per-CU) launches: two words per (slot, workgroup), plain stores by the
// workgroup's last wave -- [0] tasks << CU_BITS | hardware CU slot, [1] accepted << 8 | levels.
// 256 workgroups adding three counters into one slot line at the same moment cost ~9 us of a 54 us
// lone integral; readers sum the 256 words instead (slot_counts).
constexpr int CU_BITS = 11;   // AQ_CU_SLOTS = 2048
__host__ __device__ __forceinline__ unsigned long long pack_cu(unsigned long long tasks, unsigned cu) {
    return (tasks << CU_BITS) | (unsigned long long)(cu & ((1u << CU_BITS) - 1u));
}
struct Counts {
    unsigned long long tasks, leaves;
    unsigned levels;
};
__host__ __device__ __forceinline__ Counts slot_counts(const SlotSums& sm, const unsigned long long* wg_words, int grid) {
    Counts c{sm.tasks, sm.leaves, sm.levels};
    if (sm.pcu) {
        for (int w = 0; w < grid; ++w) {
            c.tasks += wg_words[2 * w] >> CU_BITS;
            c.leaves += wg_words[2 * w + 1] >> 8;
            c.levels = max(c.levels, (unsigned)(wg_words[2 * w + 1] & 255u));
        }
    }
    return c;
}

// Exact accumulation into a slot's XSum (device atomics: any order, same bits). Returns the first limb
// the value's digits touch (three from there), or -1 for x == 0.
__device__ __forceinline__ int xs_atomic_add(long long* limbs, double x) {
    XDigits g;
    if (!xs_digits(x, g)) return -1;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (g.d[k]) atomicAdd(reinterpret_cast<unsigned long long*>(&limbs[g.i + k]), (unsigned long long)g.d[k]);
    return g.i;
}
// ... and widen the slot's limb window to cover limbs i .. i + 2 of each (i >= 0) add
__device__ __forceinline__ void xs_window_add(SlotSums& sm, int i0, int i1) {
    const int lo = i0 < 0 ? i1 : (i1 < 0 ? i0 : min(i0, i1)), hi = max(i0, i1);
    if (lo < 0) return;
    atomicMax(&sm.win_lo_not, xs_win_lo(lo));
    atomicMax(&sm.win_hi, xs_win_hi(hi));
}

struct Chunk {                      // SoA, one queue slot
    double a[CH], b[CH], fa[CH], fm[CH], fb[CH];
    unsigned dt[CH];
    unsigned count;
    unsigned pad[31];
};

// A wave's private HBM overflow stack: the bottom (oldest, shallowest) pairs of a full ring go
// down here without any lock; the wave takes them back when its ring runs dry, before it looks at
// the shared pool or seeds new work, so the cellar is empty whenever the wave reports idle. Only
// the owning wave touches it; its lines are written back to HBM when the L2 evicts them (the PMC
// passes measure ~13 GB of WRITE_SIZE per 8192-integral launch).
//
// Layout (r03): chunks of 64 pairs, each three 1-KiB planes {a, b} | {fa, fm} | {fb, dt word} of one
// 16-B entry per pair -- the three f64x2 a pair's ds_read2st64 / ds_write2st64 move. A spill or a
// refill of 64 pairs is then three LDS instructions and three global_*_dwordx4 from ONE address
// each (one lane offset, the planes at +0 / +1 KiB / +2 KiB), where the SoA cellar of round 2 took
// six LDS accesses at separate bases and six 64-bit addresses per side. The cellar top (ctop) only
// ever moves by whole chunks (spills are SPILL pairs, prefetches and refills take whole chunks).
struct CellarChunk {
    f64x2 ab[64], ff[64], fd[64];
};
struct Cellar {
    CellarChunk c[CCAP / 64];
};
static_assert(CCAP % 64 == 0, "the cellar moves whole 64-pair chunks");

// Launch-to-launch job-size hint (one per context): every workgroup adds the tasks it ran, the last
// one to exit turns the mean per integral into the next adaptive launch's shares per integral
// (about TASKS_PER_JOB tasks per job) and clears the sums.
struct alignas(128) LaunchHint {
    unsigned long long tasks;
    unsigned exits;
    unsigned shares_next;   // 0: no hint yet (the launch uses StreamParams::shares)
    unsigned long long per_next;   // the tasks per integral shares_next was sized from
};
// A launch of few integrals (fewer than the waves) takes more shares per integral than the hint's
// ~TASKS_PER_JOB jobs would give -- up to one job per wave, with no job below MIN_JOB_TASKS tasks
// (r06, profiles/r06w: 64 sin(1/x) integrals of 56 k tasks had run as 64 whole-integral jobs on 3072
// waves, 842 us; 12 / 24 shares each 190 us; at 4096 integrals more shares only cost)
#ifndef AQ_MIN_JOB_TASKS
#define AQ_MIN_JOB_TASKS 2048
#endif
constexpr unsigned long long MIN_JOB_TASKS = AQ_MIN_JOB_TASKS;

struct StreamParams {
    const double2* bounds;          // [nprob] {a, b} per integral
    const int* shard_of;            // [nprob] per-integral shard of nshards (mixed launches), or null: `shard`
    int nprob;
    int first_slot;                 // integral p -> slot first_slot + p
    double eps;
    int max_depth;
    int shard, nshards;
    int D;                          // seed position depth
    int shares;                     // jobs per integral: job j = share j % shares of integral j / shares
    int tail_from;                  // integrals from here on: tail_mult x shares each (nprob: none)
    int tail_mult;
    unsigned epoch;                 // tags queue slots of this launch (ready[s] == epoch)
    unsigned qcap;                  // queue slots
    unsigned long long stall_ticks; // s_memrealtime ticks (100 MHz) a waiting leader tolerates WITHOUT
                                    // progress (queue head / tail / token count unchanged)
    Ctl* ctls;                      // per-slot control blocks
    QCtl* q;                        // this launch's queue and termination count (all-zero at launch)
    QCtl* q_next;                   // the next launch's: workgroup 0 zeroes it
    unsigned long long* parts;      // per-CU launches' counts (slot_counts): integral p's row at
                                    // [2 * (p * gridDim.x + wg) + 0/1] (the first slot's parts row)
    double* parea;                  // ... and their area, a double-double per workgroup at [2 * (p * gridDim.x
                                    // + wg) + 0/1] (the same row of the area words; PCU_AREA)
    unsigned long long* diag;       // optional per-workgroup timeline (DIAG_WORDS each)
    unsigned long long* cu_acc;     // [AQ_CU_SLOTS] tasks per hardware CU slot, summed over launches
                                    // (every launch: the farmer's tasks_per_process, :162, per CU)
    Chunk* chunks;
    Cellar* cellar;                 // [gridDim.x * NW]
    unsigned* ready;
    LaunchHint* hint;
    int per_cu;                     // also keep per-workgroup partials (per-CU task counts; lone integrals)
    int static_jobs;                // fewer than STATIC_MAXK integrals: static job stride (see k_stream)
    double2 kbounds[PCU_MAXK];      // per-CU launches: the bounds again, as kernel arguments (a scalar load
                                    // with the launch's other arguments, not a cold HBM line at seeding)
    int adaptive;                   // bit 0: take shares per integral from hint->shares_next; bit 1: update it;
                                    // bit 2: hint->per_next belongs to it (the HEAPS instance's fill rule)
};

// Diagnostics record per workgroup (aq_set_diagnostics), accumulated in LDS by every wave:
// realtime stamps are s_memrealtime ticks (100 MHz), cycle counts are s_memtime shader cycles.
enum : int {
    DG_T_START = 0, DG_T_SEEDED, DG_T_FIRST_LEAD, DG_T_EXIT, DG_ROUNDS, DG_TASKS, DG_CHUNKS_OUT, DG_CHUNKS_IN,
    DG_RECORDS_OUT, DG_T_WAIT, DG_LEADS, DG_SEEDS, DG_POOL_PUSH, DG_CU, DG_RECORDS_IN, DG_ACTIVE_LANES,
    DG_C_ROUND, DG_C_EVAL, DG_POOL_TAKE, DG_LOCK_SPINS, DG_T_LAST_ROUND, DG_SPILL_RECORDS, DG_MAX_RING, DG_C_SEED,
    DG_SEED_CALLS, DG_FLUSHES, DG_MAX_CELLAR, DG_C_IDLE, DG_C_LOCK, DG_C_SHARE, DG_GIVE, DG_CELLAR_IN,
    DG_CELLAR_OUT, DG_C_REFILL, DG_C_LOOP, DG_ACTIVE_TASKS, DG_PREFETCH, DG_T_INIT, DG_T_DONE, DG_T_FOLD,
    DG_T_BROKE, DG_T_FLUSHED, DG_C_P1_CLASS, DG_C_P1_WALK, DG_C_P1_F, DG_T_SEED_IN, DG_T_CLASS, DG_POLLS,
    DIAG_WORDS = 48
};

// Shared (LDS) state of one workgroup.
struct WgState {
    int lock;            // pool lock (lane 0 of the holding wave)
    unsigned pbot, ptop; // pool ring, monotonic indices
    int idle;            // waves with nothing left (no pairs, pool empty, nothing to seed)
    int phase;           // 0 running, 1 a leader wave is at the HBM queue, 2 exit
    int busy_token;      // the workgroup holds one token of the HBM-queue protocol
    unsigned exited;     // waves past the loop (adaptive and per-CU launches)
    unsigned long long tasks;   // tasks this workgroup ran (adaptive launches)
};

// LDS pair arrays (SoA), one per field.
struct LdsPairs {
    double* a;
    double* b;
    double* fa;
    double* fm;
    double* fb;
    DtField dt;
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
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void copy_pair(const LdsPairs& R, unsigned i, unsigned j) {
    const double a = R.a[i], b = R.b[i], fa = R.fa[i], fm = R.fm[i], fb = R.fb[i];
    const unsigned dt = R.dt[i];
    R.a[j] = a; R.b[j] = b; R.fa[j] = fa; R.fm[j] = fm; R.fb[j] = fb; R.dt[j] = dt;
}

// Publish k pairs (LDS slots src(i), i < k) as HBM chunk `slot` (caller: one whole wave).
template <typename SrcIdx>
__device__ __forceinline__ void publish_chunk(const StreamParams& P, const LdsPairs& R, unsigned slot, unsigned k,
                                              SrcIdx src, unsigned lane) {
    Chunk* __restrict__ c = P.chunks + slot;
    for (unsigned i = lane; i < k; i += 64) {
        const unsigned j = src(i);
        st_wt(&c->a[i], R.a[j]); st_wt(&c->b[i], R.b[j]);
        st_wt(&c->fa[i], R.fa[j]); st_wt(&c->fm[i], R.fm[j]); st_wt(&c->fb[i], R.fb[j]);
        st_wt(&c->dt[i], R.dt[j]);
    }
    if (lane == 0) st_wt(&c->count, k);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the single storing wave drains
    if (lane == 0) st_wt(&P.ready[(size_t)slot * READY_STRIDE], P.epoch);
}

// Per-wave accumulators of the integral currently being summed (`tag`).
struct Acc {
    double hi, lo;                  // double-double area (aq_device.h two_sum)
    unsigned tasks, leaves, maxd;   // per lane (seeding, mixed rounds)
    unsigned ut, ul;                // wave-uniform task / accepted counts (the rounds' fast path)
    unsigned maxdt;                 // per lane: the deepest pair depth (dt's low byte) a round popped, or
                                    // with the per-burst depth cap the deepest pair a round pushed
    double r = 0.0;                 // per lane: the rounds' accepted areas of the current burst, a plain
                                    // double (one masked add per accepted task), folded into hi / lo
                                    // exactly at every burst's end -- so a lane's rounding error is that of
                                    // a burst's few leaves, not of a whole job's (r03: 60 k-task jobs had
                                    // let two schedules of one batch differ by > 2 ulp)
};

// Flush a wave's accumulators for integral `tag` and reset them: the wave's double-double area (hi
// and lo, each exact) into the integral's exact accumulator; the counts into the slot sums (device
// atomics, spread over the launch's integrals), or -- per-CU launches, where every wave works on the
// same one or few integrals -- into the workgroup's LDS counts and LDS accumulator, folded into the
// slot once per workgroup at exit (3072 waves would otherwise queue on one slot's lines).
// pc: the per-CU instance's LDS counts, [0,16) tasks, [16,32) accepted, [32,48) levels per integral;
// px: its LDS accumulators, one XSum per integral.
template <int FID, bool PCU>
__device__ __forceinline__ void flush_acc(const StreamParams& P, Acc& a, int tag, unsigned lane, WgState& S,
                                          unsigned long long* pc, double2* wdd, int wdd_stride, long long* xsa,
                                          long long* xsb) {
    // (the rounds' lane partial is folded at every burst's end; fold any remainder here too)
    dd_add(a.hi, a.lo, a.r);
    a.r = 0.0;
    // a wave that ran no task of `tag` has nothing to add (idle waves at the exit of a lone launch)
    if (uni(a.ut) != 0u || __ballot(a.tasks != 0u) != 0ull) {
        // the wave accumulates doubled areas for the built-in integrands (exact halving, aq_device.h)
        double hi = area_scale<FID>() * a.hi, lo = area_scale<FID>() * a.lo;
#if AQ_FLUSHX == 1   // (timing experiment only: no reductions -- wrong results)
        const unsigned t = a.ut + 1u, l = a.ul, m = 1u;
#elif AQ_FLUSHX == 3   // (timing experiment only: no double-double reduction)
        const unsigned mdt = wave_max_full(a.maxdt);
        const unsigned t = wave_add_full(a.tasks) + a.ut, l = wave_add_full(a.leaves) + a.ul,
                       m = max(wave_max_full(a.maxd), mdt ? (mdt & 255u) + 1u : 0u);
#elif AQ_FLUSHX == 4   // (timing experiment only: no integer reductions)
        wave_sum_dd_full(hi, lo);
        const unsigned t = a.ut + 1u, l = a.ul, m = 1u;
#else
        if (PCU || !FLUSH_LDS) wave_sum_dd_full(hi, lo);
        // levels: the seeds' per-lane depth + 1, and the deepest popped pair (its depth byte + 1; one
        // integral per ring, so the max over pair words is the max depth of that integral)
        const unsigned mdt = wave_max_full(a.maxdt);
        const unsigned t = wave_add_full(a.tasks) + a.ut, l = wave_add_full(a.leaves) + a.ul,
                       m = max(wave_max_full(a.maxd), mdt ? (mdt & 255u) + 1u : 0u);
#endif
        if constexpr (!PCU && FLUSH_LDS) {
            if (t) {
                // the lanes' (hi, lo) as exact digits (aq_xsum.h) into a per-wave 68-limb window in LDS --
                // limbs 0-63 at xsa[0..63], 64-67 at xsb[0..3]: the top quarter of the wave's ring, free at
                // every flush (the ring is empty, or holds <= REFILL pool pairs at its bottom) -- then its
                // nonzero limbs into the slot: exact, no double-double chain, no serial digit splits
                xsa[lane] = 0ll;
                if (lane < 4u) xsb[lane] = 0ll;
                auto add_digits = [&](double v) {
                    XDigits g;
                    if (!xs_digits(v, g)) return;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const int i = g.i + k;
                        if (g.d[k]) atomicAdd(reinterpret_cast<unsigned long long*>(i < 64 ? &xsa[i] : &xsb[i - 64]),
                                              (unsigned long long)g.d[k]);
                    }
                };
                add_digits(area_scale<FID>() * a.hi);
                add_digits(area_scale<FID>() * a.lo);
                const long long v0 = xsa[lane], v1 = lane < 4u ? xsb[lane] : 0ll;
                Ctl& c = P.ctls[P.first_slot + tag];
                if (v0) atomicAdd(reinterpret_cast<unsigned long long*>(&c.area.limb[lane]), (unsigned long long)v0);
                if (v1) atomicAdd(reinterpret_cast<unsigned long long*>(&c.area.limb[64 + lane]), (unsigned long long)v1);
                const unsigned long long nz0 = __ballot(v0 != 0ll), nz1 = __ballot(v1 != 0ll);
                if ((nz0 | nz1) && lane == 0u) {
                    const int lo_nz = nz0 ? __builtin_ctzll(nz0) : 64 + __builtin_ctzll(nz1);
                    const int hi_nz = nz1 ? 64 + (63 - __builtin_clzll(nz1)) : 63 - __builtin_clzll(nz0);
                    atomicMax(&c.sums.win_lo_not, xs_win_lo(lo_nz));
                    atomicMax(&c.sums.win_hi, (unsigned)(hi_nz + 1));
                }
            }
        }
        if (AQ_FLUSHX != 2 && lane == 0 && t) {
            atomicAdd(&S.tasks, (unsigned long long)t);
            if constexpr (PCU) {
                atomicAdd(&pc[tag], (unsigned long long)t);
                atomicAdd(&pc[PCU_ROW + tag], (unsigned long long)l);
                atomicMax(&pc[2 * PCU_ROW + tag], (unsigned long long)m);
                // the wave's own double-double of this integral (no other wave writes it): the workgroup's
                // last wave sums the waves' at exit into the per-workgroup area words (PCU_AREA)
                double2& w = wdd[tag * wdd_stride];
                double wh = w.x, wl = w.y;
                dd_add_dd(wh, wl, hi, lo);
                w = make_double2(wh, wl);
            } else {
                Ctl& c = P.ctls[P.first_slot + tag];
                atomicAdd(&c.sums.tasks, (unsigned long long)t);
                atomicAdd(&c.sums.leaves, (unsigned long long)l);
                atomicMax(&c.sums.levels, m);
                if constexpr (!FLUSH_LDS) {
                    const int i0 = xs_atomic_add(c.area.limb, hi);
                    const int i1 = xs_atomic_add(c.area.limb, lo);
                    xs_window_add(c.sums, i0, i1);
                }
            }
        }
    }
    a.hi = a.lo = 0.0;
    a.tasks = a.leaves = a.maxd = 0;
    a.ut = a.ul = 0;
    a.maxdt = 0;
    __builtin_amdgcn_wave_barrier();   // reconverge: keeps the caller's wave state out of this join
}

// {a, b} of integral p through the scalar data cache (a READ: s_load; the host wrote the bounds before
// the launch and the scalar cache starts every kernel invalidated). p is wave-uniform.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double2 sload_bounds(const double2* base, int p) {
    const unsigned long long a64 = (unsigned long long)(base + p);
    const unsigned long long addr = ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(a64 >> 32)) << 32) |
                                    (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a64);
    u32x4 r;
    asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(addr) : "memory");
    return make_double2(__hiloint2double((int)r.y, (int)r.x), __hiloint2double((int)r.w, (int)r.z));
}

// One slot's six fields from / to ONE LDS address (the slot's a, in bytes): the fields lie at 0 / 50 /
// 100 / 150 / 200 / 250 x 512 B (LREC = 3200 slots of 8 B per field), the offsets of three
// ds_write2st64_b64 / ds_read2st64_b64 (and of six ds_read_b64 from two bases). The pops wait for
// their own reads (lgkmcnt(0)) inside the asm -- the compiler cannot count LDS operations it does not
// see -- and the "memory" clobbers keep the compiler's own LDS accesses on their side of both.
static_assert(LREC * 8 == 50 * 512, "the pair moves assume 50 x 512 B per field");
// The carried round's LDS moves: a pop into the lanes of mask m only (the other lanes keep
// their registers: "+v"), and a push of one pair from the lanes of m -- exec set around the three
// accesses, no branch.
// The pop reads the six fields as six ds_read_b64 (2 LDS-array cycles each, 256 B/clk; a
// ds_read2st64_b64 takes 8 for two fields, 128 B/clk -- MI355X_MICROARCH.md §LDS) into six
// independent registers (no 4-register tuple for the allocator to assemble each round); the 16-bit
// offset reaches fields 0-2 from addr and 3-5 from addr2 = addr + 150 x 512 B.
__device__ __forceinline__ void lds_pop6_masked(unsigned long long m, unsigned addr, unsigned addr2, double& a,
                                                double& b, double& fa, double& fm, double& fb, double& dw) {
    unsigned long long saved;
    asm volatile(
        "s_mov_b64 %6, exec\n\t"
        "s_mov_b64 exec, %7\n\t"
        "ds_read_b64 %0, %8\n\t"
        "ds_read_b64 %1, %8 offset:25600\n\t"
        "ds_read_b64 %2, %8 offset:51200\n\t"
        "ds_read_b64 %3, %9\n\t"
        "ds_read_b64 %4, %9 offset:25600\n\t"
        "ds_read_b64 %5, %9 offset:51200\n\t"
        "s_mov_b64 exec, %6\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "+v"(a), "+v"(b), "+v"(fa), "+v"(fm), "+v"(fb), "+v"(dw), "=&s"(saved)
        : "s"(m), "v"(addr), "v"(addr2)
        : "memory");
}
__device__ __forceinline__ void lds_push6_masked(unsigned long long m, unsigned addr, double x0, double x1, double x2,
                                                 double x3, double x4, double x5) {
    unsigned long long saved;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_mov_b64 exec, %1\n\t"
        "ds_write2st64_b64 %2, %3, %4 offset1:50\n\t"
        "ds_write2st64_b64 %2, %5, %6 offset0:100 offset1:150\n\t"
        "ds_write2st64_b64 %2, %7, %8 offset0:200 offset1:250\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(saved)
        : "s"(m), "v"(addr), "v"(x0), "v"(x1), "v"(x2), "v"(x3), "v"(x4), "v"(x5)
        : "memory");
}
// One slot's six fields in registers (cellar moves): lds_issue6 only ISSUES the three
// ds_read2st64_b64; lds_wait6 waits for every outstanding LDS access and is the point from which the
// registers hold the pair -- nothing may read them before (the hardware does not interlock a register
// an LDS load is still writing).
struct PairRegs {
    f64x2 ab, ff, fd;   // {a, b}, {fa, fm}, {fb, dt word}
};
__device__ __forceinline__ void lds_issue6(unsigned addr, PairRegs& r) {
    asm volatile(
        "ds_read2st64_b64 %0, %3 offset1:50\n\t"
        "ds_read2st64_b64 %1, %3 offset0:100 offset1:150\n\t"
        "ds_read2st64_b64 %2, %3 offset0:200 offset1:250"
        : "=&v"(r.ab), "=&v"(r.ff), "=&v"(r.fd)
        : "v"(addr)
        : "memory");
}
__device__ __forceinline__ void lds_wait6(PairRegs& r) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r.ab), "+v"(r.ff), "+v"(r.fd) : : "memory");
}
__device__ __forceinline__ void lds_store6(unsigned addr, const PairRegs& r) {
    asm volatile(
        "ds_write2st64_b64 %0, %1, %2 offset1:50\n\t"
        "ds_write2st64_b64 %0, %3, %4 offset0:100 offset1:150\n\t"
        "ds_write2st64_b64 %0, %5, %6 offset0:200 offset1:250"
        :
        : "v"(addr), "v"(r.ab.x), "v"(r.ab.y), "v"(r.ff.x), "v"(r.ff.y), "v"(r.fd.x), "v"(r.fd.y)
        : "memory");
}
// one lane's pair of a cellar chunk (three global_load_dwordx4 / global_store_dwordx4)
__device__ __forceinline__ PairRegs chunk_load(const CellarChunk* ch, unsigned lane) {
    return PairRegs{ch->ab[lane], ch->ff[lane], ch->fd[lane]};
}
__device__ __forceinline__ void chunk_store(CellarChunk* ch, unsigned lane, const PairRegs& r) {
    ch->ab[lane] = r.ab;
    ch->ff[lane] = r.ff;
    ch->fd[lane] = r.fd;
}
// LDS byte address of ring index i of a wave's ring at byte offset ring8 (a multiple of WCAP * 8):
// one shift-add and one and-or. vmask = (WCAP - 1) << 3 held in a VGPR (a gfx9 VOP3 reads one
// scalar operand, so a literal mask and the scalar ring8 would split the and-or in two).
__device__ __forceinline__ unsigned ring_addr(unsigned ring8, unsigned i, unsigned vmask) {
    return ((i << 3) & vmask) | ring8;
}
// Ring slot of monotonic ring index i.
__device__ __forceinline__ unsigned ring_slot(unsigned i) { return i % (unsigned)WCAP; }
// Ring slot of b + k for a slot b < WCAP and k < WCAP: one mask (power-of-two ring) or one
// subtract and one unsigned min.
__device__ __forceinline__ unsigned ring_wrap(unsigned v) {
    if constexpr ((WCAP & (WCAP - 1)) == 0) return v & (unsigned)(WCAP - 1);
    else return min(v, v - (unsigned)WCAP);
}

// PCU: the per-CU instance (launches of < PCU_MAXK integrals, P.per_cu): workgroup counts per
// integral in LDS, folded into the slot sums once at exit -- a lone integral's 3072 waves would
// otherwise queue on one slot's atomics at every flush.
#if AQ_STAMPS
__device__ unsigned long long g_aq_stamps[MAXG * NW * ST_STRIDE];
#endif

// NWT: waves per workgroup -- NW (12: three per SIMD) for every launch but the unsharded lone ones,
// which run AQ_LONE_NW (aq_abi.inc launch_stream): a lone integral's set-up and seeding are VALU-bound
// at three waves per SIMD, and its rounds are bound by one wave's heaviest share.
template <int FID, bool HIST, bool DIAG, bool PCU, int NWT = NW, bool HEAPS = false>
__global__ __launch_bounds__(NWT * 64) void k_stream(StreamParams P) {
    constexpr int PTT = NWT * 64;   // threads per workgroup
    static_assert(NWT >= 4 && NWT <= NW && NWT % 4 == 0, "whole waves per SIMD, within the LDS rings");
    static_assert(NWT <= 16, "the exit's area sum runs over one DPP row of lanes (PCU_AREA)");
    // one SoA block (a | b | fa | fm | fb, LREC doubles each) so that every field of a slot is a
    // constant offset from one address (ds_read2st64 / ds_write2st64 pairs, no per-field adds). A
    // pair stores no midpoint: m = (a + b) / 2 is recomputed with the parent's own operands (:187),
    // bit-identical, so a pair is 44 B and a ring holds 256 pairs.
    // The integrand table first: it must lie in the LDS's first 64 KiB for the round's table reads to
    // carry its base in their offset field (WIDE). WIDE: the bulk cosh4 instance keeps exp's 128
    // entries twice over, indexed by ki's low byte (cosh_main_k TABMASK; the per-CU instance's LDS has
    // no 2 KiB to spare beside its per-integral accumulators)
    constexpr bool WIDE = AQ_WIDE_TAB && FID == F_COSH4 && !PCU;
    // (the compiler places the largest LDS object first: the wide table shares the pair block's array, at
    // its front -- offset 0 -- and the pairs start 4 KiB in, a multiple of a ring's 2 KiB per field)
    constexpr int TAB_FRONT = WIDE ? 256 * 16 / 8 : 0;   // doubles ahead of the pair block
    __shared__ double s_lds[TAB_FRONT + 6 * LREC];
    double* const s_pr = s_lds + TAB_FRONT;
    __shared__ ExpEntry tab_own[WIDE ? 1 : ftab_entries<FID>()];   // exp's, or sin(1/x)'s __sincostab (stage_f_table)
    ExpEntry* const tab = WIDE ? reinterpret_cast<ExpEntry*>(s_lds) : tab_own;
    const DtField s_dt{reinterpret_cast<unsigned*>(s_pr + 5 * LREC)};
    double* const s_a = s_pr;
    double* const s_b = s_pr + LREC;
    double* const s_fa = s_pr + 2 * LREC;
    double* const s_fm = s_pr + 3 * LREC;
    double* const s_fb = s_pr + 4 * LREC;
    __shared__ WgState S;
    __shared__ unsigned long long s_pc[PCU ? 3 * PCU_ROW : 1];
    __shared__ double2 s_wdd[PCU ? PCU_ROW * NWT : 1];   // per-CU launches: each wave's area per integral
    __shared__ unsigned long long s_dg[DIAG ? DIAG_WORDS : 1];

    const unsigned tid = threadIdx.x;
    const unsigned lane = lane_id();
    const unsigned wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: keeps the wave state in SGPRs
    // one read of the workgroup id: two reads merged after a divergent loop would be a "divergent"
    // phi, and through w_all / job every piece of wave state would follow it into VGPRs
    const unsigned bid = __builtin_amdgcn_readfirstlane(blockIdx.x);
    QCtl* __restrict__ qc = P.q;
    const LdsPairs R{s_a, s_b, s_fa, s_fm, s_fb, s_dt};
    const unsigned pr_base = (unsigned)(uintptr_t)s_pr;   // LDS byte offset of the pair block (low word of its flat address)
    const unsigned long long t_entry = (DIAG || AQ_STAMPS) ? rtc() : 0ull;
    unsigned long long stp[ST_N] = {};   // AQ_STAMPS: this wave's timeline (wave-uniform)
    auto stamp = [&](int k) {
        if constexpr (AQ_STAMPS && !DIAG) { if (!stp[k]) stp[k] = rtc(); }
    };
    stp[ST_ENTRY] = t_entry;
    if constexpr (AQ_STAMPS && !DIAG) {
        // the kernel arguments' first arrival (the set-up's and the first seeding's fields)
        asm volatile("" :: "s"(P.eps), "s"(P.shares), "s"(P.nprob), "s"(P.kbounds[0].x));
        stamp(ST_KARG);
    }
    // the exp table's global loads go out first and land in LDS after the other set-up stores: their
    // latency overlaps the set-up instead of preceding it. (The rings are not pre-filled: the carried
    // round reads ring slots only through masked pops of pushed pairs -- the fill's 18 K LDS stores per
    // CU had cost every launch 0.75 us, r04j)
    ExpPair tv{};
    if (FID != F_SIN_RECIP && tid < (WIDE ? 256u : 128u)) tv = reinterpret_cast<const ExpPair*>(kExpTabBits)[tid & 127u];
    static_assert(FID != F_SIN_RECIP || AQ_SINCOS_TAB_N <= PTT, "one sin-table entry per thread");
    double sv = 0.0;
    if (FID == F_SIN_RECIP && tid < (unsigned)AQ_SINCOS_TAB_N) sv = kSinCosTab[tid];
    stamp(ST_PRE);
    if (bid == 0)
        for (unsigned i = tid; i < (unsigned)(sizeof(QCtl) / 4); i += PTT) reinterpret_cast<unsigned*>(P.q_next)[i] = 0u;
    if (tid == 0) {
        S.lock = 0; S.pbot = 0; S.ptop = 0; S.idle = 0; S.phase = 0; S.busy_token = 1;
        S.exited = 0; S.tasks = 0;
    }
    if (PCU && tid < 3u * PCU_ROW) s_pc[tid] = 0ull;
    if (PCU)
        for (unsigned i = tid; i < (unsigned)(PCU_ROW * NWT); i += PTT) s_wdd[i] = make_double2(0.0, 0.0);
    if (DIAG) {
        for (unsigned i = tid; i < DIAG_WORDS; i += PTT) s_dg[i] = (i == DG_T_FIRST_LEAD) ? ~0ull : 0ull;
    }
    if (FID == F_SIN_RECIP) {
        if (tid < (unsigned)AQ_SINCOS_TAB_N) reinterpret_cast<double*>(tab)[tid] = sv;
    } else if (tid < (WIDE ? 256u : 128u)) {
        tab[tid].tail_bits = tv.tail_bits;
        tab[tid].sbits = tv.sbits;
    }
    __syncthreads();   // the only workgroup barrier before the exit
    if constexpr (DIAG) { if (tid == 0) s_dg[DG_T_INIT] = rtc(); }
    stamp(ST_INIT);

    const double eps = P.eps;
    const double eps2 = eps / area_scale<FID>();   // the rounds compare doubled areas of f_scale F (task_step_k)
    const int max_depth = P.max_depth;
    // shares per integral: the host's choice, or the job-size hint the previous adaptive launch left
    unsigned shares_main = (unsigned)P.shares;
    int D_main = P.D;
    unsigned long long per_hint = 0;   // HEAPS: the hint's tasks per integral (0: unknown)
    if (!PCU && (P.adaptive & 1)) {   // (per-CU launches, k < PCU_MAXK, are never adaptive)
        unsigned h = uni(__hip_atomic_load(&P.hint->shares_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (h) {
            if constexpr (HEAPS) {
                // (the few-integral / batch instance only: the bench's instance keeps its code as it was --
                // its speed moves with code placement). Tasks per integral: per_next when the
                // hint's last writer was this instance (adaptive bit 2), else from the hint's own shares
                // when they say more than "one job" (h >= 2: within a factor 1.5)
                const unsigned long long per =
                    (P.adaptive & 4) ? __hip_atomic_load(&P.hint->per_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : (h >= 2u ? (unsigned long long)h * TASKS_PER_JOB : 0ull);
                const unsigned fill = (gridDim.x * (unsigned)NWT + (unsigned)P.nprob - 1u) / (unsigned)P.nprob;
                const unsigned long long cap = per / MIN_JOB_TASKS;
                h = uni(max(h, (unsigned)min((unsigned long long)fill, cap)));
                per_hint = per;
            }
            shares_main = h;
            D_main = seed_depth_job((unsigned long long)h * (unsigned long long)P.nshards);
        }
    }
    const unsigned W = gridDim.x * (unsigned)NWT;
    const unsigned w_all = bid * (unsigned)NWT + wid;
    // termination group (QCtl): its workgroup count, and T0 = the number of groups
    const unsigned grp = bid % (unsigned)NGROUP;
    const unsigned grp_size = (gridDim.x - grp + (unsigned)NGROUP - 1u) / (unsigned)NGROUP;
    const int t0 = (int)min(gridDim.x, (unsigned)NGROUP);
    // the launch's last integrals (from tail_from on) are cut into tail_mult-times more, smaller
    // shares: the jobs the waves draw last are short, so the waves run dry together instead of
    // idling behind the longest last job (each integral keeps ONE partition: the counts are exact)
    // (only where an integral is already several jobs: whole-integral jobs of tiny trees are short)
    // (per-CU launches have no tail: k < 64)
    const unsigned tail_from = (!PCU && shares_main >= 8u) ? (unsigned)P.tail_from : (unsigned)P.nprob;
    const unsigned shares_tail = min(shares_main * (unsigned)P.tail_mult, W);
    const int D_tail = seed_depth_job((unsigned long long)shares_tail * (unsigned long long)P.nshards);
    const unsigned main_jobs = tail_from * shares_main;
    const unsigned total_jobs = main_jobs + ((unsigned)P.nprob - tail_from) * shares_tail;
    const unsigned base = wid * WCAP;                            // this wave's ring
    // the flush's LDS digit window (FLUSH_LDS): the ring's top quarter, slots WCAP - 64 .. WCAP - 1 of its
    // a and b fields (68 limbs), free whenever a flush runs
    long long* const xs_a = reinterpret_cast<long long*>(s_a + base + (WCAP - 64));
    long long* const xs_b = reinterpret_cast<long long*>(s_b + base + (WCAP - 64));
    // its LDS byte offset (the pair block is the kernel's first LDS object, and a ring is WCAP * 8 B of
    // each field: ring8 is a multiple of WCAP * 8, which ring_addr's and-or relies on)
    const unsigned ring8 = pr_base + base * 8u;
    __builtin_assume((ring8 & (unsigned)(WCAP * 8 - 1)) == 0u);
    unsigned ring_vmask = (unsigned)((WCAP - 1) << 3);
    asm volatile("" : "+v"(ring_vmask));   // kept in a VGPR (see ring_addr)

    Acc acc{0.0, 0.0, 0u, 0u, 0u, 0u, 0u, 0u};
    int tag = 0;                  // integral the accumulators belong to (wave-uniform)
    unsigned ctop = 0;            // pairs in this wave's cellar (wave-uniform)
    Cellar* __restrict__ cel = P.cellar + w_all;
    // the job this wave seeds next (wave-uniform). Launches of few integrals (static jobs) number the
    // waves transposed (wave wid of workgroup b seeds share wid * G + b): a workgroup's 12 shares then
    // lie spread over the whole interval instead of side by side, so no workgroup holds only the
    // costly end of it
    const bool static_jobs = PCU || P.static_jobs != 0;
    // (HEAPS, the batch instance: its launches run size-ordered chunks, whose first W jobs would give
    // workgroup 0 the 12 largest trees and the last workgroup the 12 smallest of them -- dealt transposed,
    // every CU gets one job of each size band; r06)
    unsigned job = (static_jobs || HEAPS) ? wid * gridDim.x + bid : w_all;
    bool job_pending = false;     // `job` is still in flight in lane 0's `claim`
    unsigned claim = 0;           // lane 0: the prefetched claim (jobs W + claim .. + jpc - 1)
    // jobs per claim. Whole-integral jobs of a big batch are short (C3 at eps=1e-3: ~1 400 tasks), and
    // one claim each made the job counter a serial fan-in (65536 claims on one line, ~10 ns each: a
    // static deal of the same launch ran 815 -> 543 us). Such launches claim a run of consecutive
    // jobs at once -- at least 4 claims per wave stay, for the balance -- one job otherwise.
    // (HEAPS: a run holds at most ~TASKS_PER_JOB tasks by the hint's tasks per integral -- in a size-
    // ordered chunk consecutive jobs are alike, and runs of 10 of its largest 66 k-task trees had made a
    // 262144-integral eps=1e-8 batch launch 8 % slower than the same integrals unsorted, r06)
    unsigned jpc = (!static_jobs && shares_main == 1u && P.nshards == 1 && JOB_RUN_MAX > 1)
                       ? max(1u, min((unsigned)JOB_RUN_MAX, total_jobs / (4u * W)))
                       : 1u;
    if constexpr (HEAPS) {
        if (per_hint) jpc = uni(max(1u, min(jpc, (unsigned)min((unsigned long long)TASKS_PER_JOB / per_hint, 64ull))));
    }
    unsigned job_end = job + 1u;  // end of the claimed run `job` belongs to
    unsigned claim_n = jpc;       // jobs the claim in flight takes (guided: shrinks near the end)
    unsigned err = 0;
    bool mixed = false;           // a round met pairs of another integral (never expected)
    unsigned top = 0, bot = 0;    // ring indices (wave-uniform)
    bool counted_idle = false;
    bool fresh = true;            // before this wave's first seeding
    // sin(1/x) (config 4) piles nearly all of its tree into one small region: its waves look for idle
    // siblings every SKEWED_GIVE rounds (a lone integral 79 -> 70 us at 4; cosh4 keeps 32, where 4 cost
    // the eps=1e-12 lone tree 47 -> 61 us and the bench 0.6 %; profiles/r02_ab/fast_give_poll*.txt)
    // (a faster cadence for lone launches, give every 4 / 8 rounds: slower, profiles/r03zb)
    // (per-CU launches feeding idle siblings every 4 / 8 / 16 rounds: ε=1e-10 lone 24 -> 35 / 30 / 26 us,
    // the bursts cut short; r04k)
    constexpr unsigned give_rounds = FID == F_SIN_RECIP ? (unsigned)SKEWED_GIVE : (unsigned)GIVE_ROUNDS;
    constexpr unsigned poll_rounds = FID == F_SIN_RECIP ? (unsigned)SKEWED_POLL : (unsigned)POLL_ROUNDS;
    constexpr unsigned give_min = FID == F_SIN_RECIP ? (unsigned)SKEWED_GIVE_MIN : (unsigned)GIVE_MIN;
    unsigned poll_ctr = wid * (poll_rounds / NWT);
    unsigned seen_head = 0, seen_tail = 0;   // lane 0's view of the HBM queue
    unsigned long long spilled = 0;          // pairs this wave sent to HBM chunks (lane 0)
    unsigned long long lock_spins = 0;
    // cellar prefetch in flight: up to 64 pairs, one per lane, landed below the ring's bottom at
    // the top of the next iteration (the loads overlap one round)
    unsigned pf_n = 0;
    PairRegs pf{};
    unsigned long long cl0 = 0;
    if constexpr (DIAG) {
        if (tid == 0) s_dg[DG_T_START] = t_entry;
        cl0 = clk();
    }
    if constexpr (AQ_STAMPS && !DIAG) cl0 = clk();

    // the ring's bottom SPILL pairs (ring index b) to the cellar's chunks from pair c (whole chunks)
    auto spill_to_cellar = [&](unsigned b, unsigned c) {
        for (unsigned q = 0; q < (unsigned)SPILL; q += 64u) {
            PairRegs r;
            lds_issue6(ring_addr(ring8, ring_slot(b + q) + lane, ring_vmask), r);
            lds_wait6(r);
            chunk_store(&cel->c[(c + q) / 64u], lane, r);
        }
        if constexpr (DIAG) {
            if (lane == 0) {
                atomicAdd(&s_dg[DG_CELLAR_OUT], (unsigned long long)SPILL);
                atomicMax(&s_dg[DG_MAX_CELLAR], (unsigned long long)(c + SPILL));   // the deepest cellar of the workgroup
            }
        }
    };
    const ExpConsts kk = pinned_exp_consts();
    // the depth cap per burst (see the file's configuration notes); the histogram instance keeps the
    // per-round test
    constexpr bool burst_cap = !HIST;
    for (;;) {
        // the wave's ring / cellar state, re-asserted uniform once per iteration: the loop's many
        // divergent lane-level blocks (copies, seeding) otherwise leave it in VGPRs, and every check
        // below becomes a v_cmp + exec-mask branch instead of a scalar compare
        top = uni(top);
        bot = uni(bot);
        ctop = uni(ctop);
        pf_n = uni(pf_n);
        poll_ctr = uni(poll_ctr);
        if (pf_n && top - bot <= (unsigned)PF_BELOW) {
            if (bot < 64u) {   // keep ring indices non-negative (slots are index % WCAP)
                bot += (unsigned)WCAP;
                top += (unsigned)WCAP;
            }
            bot -= pf_n;
            if (lane < pf_n) lds_store6(ring_addr(ring8, ring_slot(bot) + lane, ring_vmask), pf);
            if constexpr (DIAG) { if (lane == 0) atomicAdd(&s_dg[DG_PREFETCH], (unsigned long long)pf_n); }   // landed
            __builtin_amdgcn_wave_barrier();   // reconverge here: the ring indices stay wave-uniform
            pf_n = 0;
        }
        unsigned size = top - bot;

        if (size == 0) {
            // ---- out of pairs: own cellar, then the pool, then the next job's seeds, else idle / lead
            if (ctop > 0) {
                unsigned long long cr = 0;
                if constexpr (DIAG) cr = clk();
                const unsigned k = min(ctop, (unsigned)REFILL), c0 = ctop - k;   // whole chunks
                // no wait for this wave's own spills: one wave's accesses to one address stay in
                // order, and only this wave ever touches its cellar
                for (unsigned q = 0; q < k; q += 64)
                    lds_store6(ring_addr(ring8, q + lane, ring_vmask), chunk_load(&cel->c[(c0 + q) / 64u], lane));
                ctop = c0;
                bot = 0;
                top = k;
                if constexpr (DIAG) {
                    if (lane == 0) {
                        atomicAdd(&s_dg[DG_CELLAR_IN], (unsigned long long)k);
                        atomicAdd(&s_dg[DG_C_REFILL], clk() - cr);
                    }
                }
                __builtin_amdgcn_wave_barrier();   // reconverge before the latch (wave state stays uniform)
                continue;
            }
            unsigned long long ci = 0;
            if constexpr (DIAG) ci = clk();
            if (counted_idle) {
                const unsigned pt = uni(__hip_atomic_load(&S.ptop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                const unsigned pb = uni(__hip_atomic_load(&S.pbot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                const int ph = uni(__hip_atomic_load(&S.phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                if (pt == pb) {
                    if (ph == 2) break;
                    __builtin_amdgcn_s_sleep(4);
                    if constexpr (DIAG) { if (lane == 0) atomicAdd(&s_dg[DG_C_IDLE], clk() - ci); }
                    __builtin_amdgcn_wave_barrier();
                    continue;
                }
            }
            if (job_pending) {
                job = W + uni(__shfl(claim, 0, 64));   // claims count from W (the first W jobs are dealt)
                job_end = job + claim_n;
                job_pending = false;

            }
            unsigned k = 0;
            int ptag = 0;
            bool lead = false, seed = false;
            int phase = 0;
            // a wave's first job needs no look at the pool (empty until some wave has run rounds):
            // 12 waves would otherwise queue on the lock before their first F evaluation
            // (job_pending: the claim was read into `job` above)
            bool counted_now = false;   // counted idle just now, without the lock, and not the last
            const bool pool_empty = uni(__hip_atomic_load(&S.ptop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) ==
                                    uni(__hip_atomic_load(&S.pbot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (job < total_jobs && (fresh || pool_empty)) {
                // the next job while the pool looks empty: seeded without the lock (pool pairs that
                // arrive meanwhile are taken at this wave's next dry spell). A wave of a tiny-tree batch
                // (C3 at eps=1e-3: a job every ~18 us) had taken the lock before every job
                seed = true;
            } else if (!counted_idle && !job_pending && job >= total_jobs && pool_empty) {
                // nothing to seed, pool empty: count idle with one LDS atomic. Only the wave that makes
                // the count whole takes the lock (the lead check below, pool re-read under it); the
                // others go straight to the lock-free idle poll -- a workgroup's 12 waves running dry
                // together had queued on the lock one after another (1-task tree 16.4 -> 15.3 us, r04h)
                stamp(ST_IDLE);
                unsigned old = 0;
                if (lane == 0) old = __hip_atomic_fetch_add(&S.idle, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                old = uni(__shfl(old, 0, 64));
                counted_idle = true;
                counted_now = old + 1u != (unsigned)NWT;
            }
            if (!seed && !counted_now) {
                wave_lock(&S.lock, lane, lock_spins);
                {
                    const unsigned avail = uni(S.ptop - S.pbot);
                    phase = uni(S.phase);
                    if (avail > 0) {
                        k = min(avail, (unsigned)REFILL);
                        const unsigned pb = S.pbot;
                        // a ring holds pairs of ONE integral (the rounds count without per-lane tags):
                        // take the leading run of pool pairs that share the first pair's integral
                        ptag = (int)uni(dt_tag(s_dt[POOL0 + (pb & (PCAP - 1))]));
                        for (unsigned q0 = 0; q0 < k; q0 += 64) {
                            const unsigned q = q0 + lane;
                            const unsigned long long bad =
                                __ballot(q < k && (int)dt_tag(s_dt[POOL0 + ((pb + q) & (PCAP - 1))]) != ptag);
                            if (bad) {
                                k = q0 + (unsigned)__builtin_ctzll(bad);
                                break;
                            }
                        }
                        for (unsigned i = lane; i < k; i += 64) copy_pair(R, POOL0 + ((pb + i) & (PCAP - 1)), base + i);
                        if (lane == 0) {
                            S.pbot = pb + k;
                            if (counted_idle) __hip_atomic_fetch_add(&S.idle, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                        __builtin_amdgcn_wave_barrier();
                        counted_idle = false;
                    } else if (job < total_jobs) {
                        seed = true;
                    } else {
                        if (!counted_idle) {
                            stamp(ST_IDLE);
                            if (lane == 0) __hip_atomic_fetch_add(&S.idle, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            __builtin_amdgcn_wave_barrier();
                            counted_idle = true;
                        }
                        __builtin_amdgcn_wave_barrier();
                        if (phase == 0 && uni(__hip_atomic_load(&S.idle, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) == NWT) {   // every wave idle, pool empty, nothing to seed
                            lead = true;
                            if (lane == 0) S.phase = 1;
                            __builtin_amdgcn_wave_barrier();
                        }
                    }
                }
                wave_unlock(&S.lock, lane);
            }
            fresh = false;
            if constexpr (DIAG) {
                if (lane == 0) {
                    if (k) atomicAdd(&s_dg[DG_POOL_TAKE], (unsigned long long)k);
                    atomicAdd(&s_dg[DG_C_IDLE], clk() - ci);
                }
            }
            if (k) {
                if (ptag != tag) {     // the ring's new integral
                    flush_acc<FID, PCU>(P, acc, tag, lane, S, s_pc, s_wdd + wid, NWT, xs_a, xs_b);
                    tag = ptag;
                }
                bot = 0;
                top = k;
                __builtin_amdgcn_wave_barrier();
                continue;
            }

            if (seed) {
                // ---- wave-local seeding of job `job` (see the file header)
                unsigned long long cs = 0;
                stamp(ST_SEED_IN);
                unsigned long long cs_st = 0;
                if constexpr (AQ_STAMPS && !DIAG) cs_st = clk();
                if constexpr (DIAG) {
                    cs = clk();
                    if (lane == 0) atomicMax(&s_dg[DG_T_SEED_IN], rtc());
                }
                // the job's class: share `share` of integral p, cut into `shares` (its partition)
                const bool in_tail = job >= main_jobs;
                const unsigned shares = in_tail ? shares_tail : shares_main;
                const int D = in_tail ? D_tail : D_main;
                const unsigned jj = in_tail ? job - main_jobs : job;
                // (per-CU launches: jobs < PCU_MAXK x W, so the float estimate with its correction
                // stands in for the integer divisions -- cold code at every lone launch)
                const float sh_rcp = PCU ? __builtin_amdgcn_rcpf((float)shares) : 0.0f;
                const unsigned pj = PCU ? div_small(jj, shares, sh_rcp) : (shares == 1u ? jj : jj / shares);
                const int p = (int)((in_tail ? tail_from : 0u) + pj);
                const unsigned shard_p = P.shard_of ? (unsigned)uni(P.shard_of[p]) : (unsigned)P.shard;
                unsigned sh = jj - pj * shares;
                // static-job launches rotate the shares from one integral to the next: a wave whose
                // share of one integral is costly gets another part of the next
                if (static_jobs) {
                    const unsigned x = sh + (unsigned)p * SHARE_ROT;
                    sh = PCU ? x - div_small(x, shares, sh_rcp) * shares : x % shares;
                }
                const unsigned vw = sh * (unsigned)P.nshards + shard_p;
                const unsigned V = shares * (unsigned)P.nshards;
                const unsigned long long npos_total = 1ull << D;
                const unsigned nb = seed_nb(D, V);                          // positions per share (<= 8)
                const float nb_rcp = __builtin_amdgcn_rcpf((float)nb);      // div_small's estimate
                const unsigned nlev = (unsigned)D + 1u;                     // seeding evaluates depths 0..D
                const unsigned nnodes = nlev * nb;
                // fast path (nnodes <= 64): lane q = d*nb + kk; colmask = the lanes of this lane's kk
                unsigned long long colmask = 0;
                if (nnodes <= 64) {
                    // column 0's lanes, built once per wave on the scalar unit, shifted to this lane's
                    // column (a per-lane loop of 64-bit shifts had cost the lone start ~0.3 us)
                    unsigned long long col0 = 0;
                    for (unsigned d = 0; d < nlev; ++d) col0 |= 1ull << (d * nb);
                    colmask = uni(col0) << (lane - div_small(lane, nb, nb_rcp) * nb);
                }
                unsigned long long cf0 = 0;
                if constexpr (AQ_STAMPS && !DIAG) cf0 = clk();
                if (p != tag) {
                    flush_acc<FID, PCU>(P, acc, tag, lane, S, s_pc, s_wdd + wid, NWT, xs_a, xs_b);
                    tag = p;
                }
                if constexpr (AQ_STAMPS && !DIAG) {
                    const unsigned long long cf1 = clk();
                    stp[ST_CF] += cf1 - cf0;
                    cf0 = cf1;
                }
                // the bounds load goes out before the claim: waiting for it then leaves the claim (one
                // contended atomic, not needed before the next job) in flight
                // once per job. A scalar load (lgkmcnt), so the wait for it does not also wait for the
                // previous integral's flush atomics and this job's claim (vmcnt, in issue order), which
                // stay in flight while the job seeds (C3 eps=1e-3 A/B: profiles/r02_ab/sload_bounds.txt)
                // (a select between kbounds[0] and kbounds[p] put the whole 400-B argument block in
                // scratch: lone launches +10 us, profiles/r05r)
                const double2 ab = PCU ? P.kbounds[p] : sload_bounds(P.bounds, p);
                if constexpr (AQ_STAMPS && !DIAG) stp[ST_CBD] += clk() - cf0;
                if (static_jobs) {
                    // launches of few integrals cut every integral into one share per wave: wave w seeds share w of
                    // each integral in turn (static stride, no claim). 3072 waves claiming through one
                    // counter cost a 2-integral launch 87 us instead of ~25.
                    job += W;
                } else if (total_jobs > W) {
                    if (job + 1u < job_end) {
                        ++job;   // the next job of this wave's claimed run: no atomic
                    } else {
                        // next run: the latency hides behind this job. The raw counter value is kept (W is
                        // added at the read): any arithmetic on the result here would wait for the atomic
                        // guided size: the jobs left past this one, over GSS_DIV claims per wave
                        const unsigned left = total_jobs > job + 1u ? total_jobs - job - 1u : 0u;
                        claim_n = jpc > 1u && GSS_DIV ? max(1u, min(jpc, left / (GSS_DIV * W))) : jpc;   // (0: fixed runs)
                        if (lane == 0) claim = g_add(&qc->jobs.v, claim_n);
                        job_pending = true;
                    }
                } else {
                    // every job was handed out at launch (job = w_all): no claim, so a lone integral's
                    // 3072 waves do not queue on one atomic before their first F evaluation
                    job = total_jobs;
                }
                const double A = ab.x, B = ab.y;
                if constexpr (AQ_STAMPS && !DIAG) { asm volatile("" :: "s"(A)); stamp(ST_CLASS); }
                double* fm = s_a + base;          // [nnodes + 2]: F(mid of (d,k)) at d*nb+k, then F(A), F(B)
                double* leafa = s_b + base;       // [nnodes]: larea + rarea of node (d,k)
                const DtField flag = s_dt + base;  // [nnodes]: node (d,k) refines
                auto position = [&](unsigned kk, bool& valid) -> unsigned long long {
                    const unsigned long long o = (kk & 1u) ? (unsigned long long)(V - 1 - vw) : (unsigned long long)vw;
                    const unsigned long long j = (unsigned long long)kk * V + o;
                    valid = j < npos_total;
                    return j;
                };
                unsigned long long cp1 = 0, cp2 = 0;
                bool alive = false, alive2 = false;   // alive2: the dual path's second node per lane
                double l = A, r = B, fl = 0.0, fr = 0.0, mid = 0.0, fmid = 0.0;
                double l2 = A, r2 = B, fl2 = 0.0, fr2 = 0.0, fmid2 = 0.0;
                // the depth of the seeded pairs' parents (the heap path seeds one level deeper)
                int Ds = D;
                if (HEAP_SEED && HEAPS && V == 1u) {
                    // Whole-integral job (V = 1: the wave owns the whole tree, tiny trees of big batches).
                    // Lane q < 31 owns node q of the top five levels in heap order (depth d = log2(q + 1),
                    // k = q + 1 - 2^d), lanes 31 / 32 F(A) / F(B): every node ONCE, where the column path's
                    // 32 lanes evaluate the 15 nodes of four levels (each node once per position below it).
                    // One F per lane either way, and the first burst starts with up to 16 pairs instead of
                    // 8 -- one ramp round fewer per tiny tree (C3 at eps=1e-3: ~14 rounds of ~1 400 tasks).
                    Ds = HEAP_D;
                    const unsigned q = lane;
                    const bool isnode = q < HEAP_NODES;
                    const unsigned d = isnode ? 31u - (unsigned)__builtin_clz(q + 1u) : 0u;
                    const unsigned k = isnode ? q + 1u - (1u << d) : 0u;
                    unsigned li = HEAP_NODES, ri = HEAP_NODES + 1u;
                    for (unsigned i = 0; i < d; ++i) {
                        const double mm = (l + r) / 2;                           // :187 on the path
                        const unsigned anc = (1u << i) - 1u + (k >> (d - i));    // the path's node at depth i
                        if ((k >> (d - 1u - i)) & 1u) { l = mm; li = anc; } else { r = mm; ri = anc; }
                    }
                    mid = (l + r) / 2;                                            // :187
                    if (q < HEAP_NODES + 2u) {
                        fmid = integrand<FID>(isnode ? mid : (q == HEAP_NODES ? A : B), tab);   // :188
                        fm[q] = fmid;
                    }
                    __builtin_amdgcn_wave_barrier();
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
                    // a node is a task of the tree iff every ancestor refines (:192-197)
                    const unsigned long long rm = __ballot(isnode && refine);
                    bool ev = isnode;
                    for (unsigned x = q; ev && x > 0u;) {
                        x = (x - 1u) >> 1;
                        ev = ((rm >> x) & 1ull) != 0ull;
                    }
                    if (ev) {
                        ++acc.tasks;
                        acc.maxd = max(acc.maxd, d + 1u);
                        if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[d], 1ull);
                        if (!refine) {
                            dd_add(acc.hi, acc.lo, leafarea / area_scale<FID>());   // :199 -> :149 (doubled, exact)
                            ++acc.leaves;
                            if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[AQ_MAX_LEVELS + d], 1ull);
                        } else if ((int)d + 1 >= max_depth) {
                            err |= ERRB_DEPTH;
                        }
                    }
                    alive = ev && refine && d == (unsigned)HEAP_D && HEAP_D + 1 < max_depth;
                    if (burst_cap && alive) acc.maxd = max(acc.maxd, (unsigned)HEAP_D + 2u);
                    if constexpr (DIAG) { cp1 = clk(); cp2 = cp1; }
                } else if (nnodes <= 64) {
                    // fast path: lane q = d*nb + kk owns node (d, kk) -- its path walk, its F(mid), its
                    // decision; the first leaf depth of every position comes from ONE ballot
                    unsigned long long ca = 0, cb = 0;
                    if constexpr (DIAG) {
                        ca = clk();
                        if (lane == 0) atomicMax(&s_dg[DG_T_CLASS], rtc());
                    }
                    const unsigned q = lane;
                    const bool isnode = q < nnodes;
                    const unsigned d = isnode ? div_small(q, nb, nb_rcp) : 0u, kk = isnode ? q - d * nb : 0u;
                    bool valid = false;
                    const unsigned long long pp = isnode ? position(kk, valid) : 0ull;
                    const unsigned long long anc = valid ? (pp >> (D - (int)d)) : 0ull;
                    unsigned li = nnodes, ri = nnodes + 1;
                    for (unsigned i = 0; i < d; ++i) {
                        const double mm = (l + r) / 2;
                        if ((anc >> (d - 1 - i)) & 1ull) { l = mm; li = i * nb + kk; } else { r = mm; ri = i * nb + kk; }
                    }
                    mid = (l + r) / 2;                                        // :187
                    if constexpr (DIAG) { asm volatile("" :: "v"(mid)); cb = clk(); }
                    const unsigned fq = nnodes + 2 <= 64 ? q : (q < nnodes ? q : 64u);
                    if (fq < nnodes + 2)
                        fmid = integrand<FID>(isnode ? mid : (q == nnodes ? A : B), tab);   // :188
                    if (fq < nnodes + 2) fm[q] = fmid;
                    if constexpr (AQ_STAMPS && !DIAG) { asm volatile("" :: "v"(fmid)); stamp(ST_FEVAL); }
                    if (nnodes + 2 > 64 && lane < 2) fm[nnodes + lane] = integrand<FID>(lane == 0 ? A : B, tab);
                    if constexpr (DIAG) {
                        cp1 = clk();
                        if (lane == 0) {
                            atomicAdd(&s_dg[DG_C_P1_CLASS], ca - cs);
                            atomicAdd(&s_dg[DG_C_P1_WALK], cb - ca);
                            atomicAdd(&s_dg[DG_C_P1_F], cp1 - cb);
                        }
                    }
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
                    const unsigned dstar = leafm ? (unsigned)__builtin_ctzll(leafm) / nb : nlev;
                    if (isnode && valid && d <= dstar && (pp & ((1ull << (D - (int)d)) - 1ull)) == 0ull) {
                        ++acc.tasks;                                          // owner of node (d, kk)
                        acc.maxd = max(acc.maxd, d + 1u);
                        if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[d], 1ull);
                        if (d == dstar) {
                            dd_add(acc.hi, acc.lo, leafarea / area_scale<FID>());   // :199 -> :149 (doubled, exact)
                            ++acc.leaves;
                            if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[AQ_MAX_LEVELS + d], 1ull);
                        } else if ((int)d + 1 >= max_depth) {
                            err |= ERRB_DEPTH;
                        }
                    }
                    // a surviving position node emits its children pair (depth D + 1)
                    alive = isnode && valid && (int)d == D && dstar >= nlev && D + 1 < max_depth;
                    // (the per-burst cap's maxdt counts pushed pairs only: the seeds' depth goes here)
                    if (burst_cap && alive) acc.maxd = max(acc.maxd, (unsigned)D + 2u);
                    if constexpr (DIAG) cp2 = clk();
                } else if (FID == F_SIN_RECIP && nnodes + 2u <= 128u) {
                    // dual path (the skewed integrand's lone launches, seeded one level deeper: aq_abi.inc):
                    // lane q owns nodes q and q + 64 -- the fast path twice over, the two F chains
                    // interleaved, the first leaf depth from two ballots over a 128-bit column mask
                    unsigned long long c0lo = 0, c0hi = 0;   // column 0's nodes (uniform)
                    for (unsigned d = 0; d < nlev; ++d) {
                        const unsigned b = d * nb;
                        if (b < 64u) c0lo |= 1ull << b; else c0hi |= 1ull << (b - 64u);
                    }
                    c0lo = uni(c0lo);
                    c0hi = uni(c0hi);
                    bool isn[2], vld[2], rfn[2];
                    unsigned dd[2], kc[2], lix[2], rix[2];
                    unsigned long long ppx[2];
                    double lx[2], rx[2], mx[2], fx[2], flx[2], frx[2], lax[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const unsigned q = lane + 64u * (unsigned)h;
                        isn[h] = q < nnodes;
                        dd[h] = isn[h] ? div_small(q, nb, nb_rcp) : 0u;
                        kc[h] = isn[h] ? q - dd[h] * nb : 0u;
                        vld[h] = false;
                        ppx[h] = isn[h] ? position(kc[h], vld[h]) : 0ull;
                        const unsigned long long anc = vld[h] ? (ppx[h] >> (D - (int)dd[h])) : 0ull;
                        double ll = A, rr = B;
                        unsigned li = nnodes, ri = nnodes + 1;
                        for (unsigned i = 0; i < dd[h]; ++i) {
                            const double mm = (ll + rr) / 2;
                            if ((anc >> (dd[h] - 1 - i)) & 1ull) { ll = mm; li = i * nb + kc[h]; } else { rr = mm; ri = i * nb + kc[h]; }
                        }
                        lx[h] = ll; rx[h] = rr; lix[h] = li; rix[h] = ri;
                        mx[h] = (ll + rr) / 2;                                    // :187
                    }
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const unsigned q = lane + 64u * (unsigned)h;
                        fx[h] = 0.0;
                        if (q < nnodes + 2u) fx[h] = integrand<FID>(isn[h] ? mx[h] : (q == nnodes ? A : B), tab);   // :188
                    }
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const unsigned q = lane + 64u * (unsigned)h;
                        if (q < nnodes + 2u) fm[q] = fx[h];
                    }
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        rfn[h] = false;
                        lax[h] = 0.0;
                        flx[h] = frx[h] = 0.0;
                        if (isn[h]) {
                            flx[h] = fm[lix[h]];
                            frx[h] = fm[rix[h]];
                            const double lrarea = (flx[h] + frx[h]) * (rx[h] - lx[h]) / 2;   // :185
                            const double larea = (flx[h] + fx[h]) * (mx[h] - lx[h]) / 2;     // :189
                            const double rarea = (fx[h] + frx[h]) * (rx[h] - mx[h]) / 2;     // :190
                            rfn[h] = fabs((larea + rarea) - lrarea) > eps;                   // :191
                            lax[h] = larea + rarea;                                          // :199
                        }
                    }
                    const unsigned long long lm_lo = __ballot(isn[0] && vld[0] && !rfn[0]);
                    const unsigned long long lm_hi = __ballot(isn[1] && vld[1] && !rfn[1]);
                    bool alv[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const unsigned k = kc[h];   // < nb <= 64: the column's 128-bit mask is col0 << k
                        const unsigned long long cl = c0lo << k;
                        const unsigned long long ch = k ? ((c0hi << k) | (c0lo >> (64u - k))) : c0hi;
                        const unsigned long long ml = lm_lo & cl, mh = lm_hi & ch;
                        const unsigned qf = ml ? (unsigned)__builtin_ctzll(ml) : (mh ? 64u + (unsigned)__builtin_ctzll(mh) : ~0u);
                        const unsigned dstar = qf == ~0u ? nlev : div_small(qf, nb, nb_rcp);
                        const unsigned d = dd[h];
                        if (isn[h] && vld[h] && d <= dstar && (ppx[h] & ((1ull << (D - (int)d)) - 1ull)) == 0ull) {
                            ++acc.tasks;                                          // owner of node (d, k)
                            acc.maxd = max(acc.maxd, d + 1u);
                            if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[d], 1ull);
                            if (d == dstar) {
                                dd_add(acc.hi, acc.lo, lax[h] / area_scale<FID>());   // :199 -> :149
                                ++acc.leaves;
                                if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[AQ_MAX_LEVELS + d], 1ull);
                            } else if ((int)d + 1 >= max_depth) {
                                err |= ERRB_DEPTH;
                            }
                        }
                        alv[h] = isn[h] && vld[h] && (int)d == D && dstar >= nlev && D + 1 < max_depth;
                        if (burst_cap && alv[h]) acc.maxd = max(acc.maxd, (unsigned)D + 2u);
                    }
                    alive = alv[0]; l = lx[0]; r = rx[0]; fl = flx[0]; fr = frx[0]; fmid = fx[0];
                    alive2 = alv[1]; l2 = lx[1]; r2 = rx[1]; fl2 = flx[1]; fr2 = frx[1]; fmid2 = fx[1];
                    if constexpr (DIAG) { cp1 = clk(); cp2 = cp1; }
                } else {
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
                                for (unsigned i = 0; i < d; ++i) {
                                    const double mm = (ll + rr) / 2;
                                    if ((anc >> (d - 1 - i)) & 1ull) ll = mm; else rr = mm;
                                }
                                x = (ll + rr) / 2;
                            } else {
                                x = (q == nnodes) ? A : B;
                            }
                            fm[q] = integrand<FID>(x, tab);
                        }
                    }
                    if constexpr (DIAG) cp1 = clk();
                    for (unsigned q0 = 0; q0 < nnodes; q0 += 64) {
                        const unsigned q = q0 + lane;
                        if (q < nnodes) {
                            const unsigned d = q / nb, kk = q % nb;
                            bool valid;
                            const unsigned long long pp = position(kk, valid);
                            const unsigned long long anc = valid ? (pp >> (D - (int)d)) : 0ull;
                            double ll = A, rr = B;
                            unsigned li = nnodes, ri = nnodes + 1;
                            for (unsigned i = 0; i < d; ++i) {
                                const double mm = (ll + rr) / 2;
                                if ((anc >> (d - 1 - i)) & 1ull) { ll = mm; li = i * nb + kk; } else { rr = mm; ri = i * nb + kk; }
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
                    if constexpr (DIAG) cp2 = clk();
                    // resolve: lane kk < nb follows position kk down its path
                    const unsigned kk = lane;
                    bool valid = false;
                    const unsigned long long pp = (kk < nb) ? position(kk, valid) : 0ull;
                    unsigned long long fmask = 0;
                    for (unsigned d = 0; d < nlev; ++d)
                        fmask |= (unsigned long long)(flag[d * nb + (kk < nb ? kk : 0u)] & 1u) << d;
                    const unsigned dstar = (unsigned)__builtin_ctzll(~fmask);   // first depth that does not refine
                    if (valid) {
                        const unsigned dlast = min(dstar, (unsigned)D);
                        for (unsigned d = 0; d <= dlast; ++d) {
                            if ((pp & ((1ull << (D - (int)d)) - 1ull)) == 0ull) {   // owner of node (d, kk)
                                ++acc.tasks;
                                acc.maxd = max(acc.maxd, d + 1u);
                                if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[d], 1ull);
                                if (d == dstar) {
                                    dd_add(acc.hi, acc.lo, leafa[d * nb + kk] / area_scale<FID>());   // :199 -> :149 (doubled)
                                    ++acc.leaves;
                                    if (HIST) atomicAdd(&P.ctls[P.first_slot + p].hist[AQ_MAX_LEVELS + d], 1ull);
                                } else if ((int)d + 1 >= max_depth) {
                                    err |= ERRB_DEPTH;
                                }
                            }
                        }
                        alive = dstar >= nlev && D + 1 < max_depth;
                        if (burst_cap && alive) acc.maxd = max(acc.maxd, (unsigned)D + 2u);
                        if (alive) {
                            unsigned li = nnodes, ri = nnodes + 1;
                            for (int i = 0; i < D; ++i) {
                                const double mm = (l + r) / 2;
                                if ((pp >> (D - 1 - i)) & 1ull) { l = mm; li = (unsigned)i * nb + kk; } else { r = mm; ri = (unsigned)i * nb + kk; }
                            }
                            fl = fm[li];
                            fr = fm[ri];
                            mid = (l + r) / 2;
                            fmid = fm[(unsigned)D * nb + kk];
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();   // every read of the scratch precedes the seed writes
                const unsigned long long am = __ballot(alive);
                constexpr double fs = f_scale<FID>();   // the rounds' F values (exact scaling)
                if (alive) {
                    const unsigned j = base + mbcnt(am);
                    // a pair holds its endpoints halved (aq_device.h pair_step_halves; exact)
                    s_a[j] = 0.5 * l; s_b[j] = 0.5 * r; s_fa[j] = fs * fl; s_fm[j] = fs * fmid; s_fb[j] = fs * fr;   // :192-197
                    const bool span = FID == F_COSH4 && cosh_main_span(l, r);
                    s_dt[j] = (unsigned)(Ds + 1) | (span ? SPAN_BIT : 0u) | ((unsigned)p << TAG_SHIFT);
                }
                unsigned n_seeds = (unsigned)__popcll(am);
                if constexpr (FID == F_SIN_RECIP) {   // the dual path's second nodes
                    const unsigned long long am2 = __ballot(alive2);
                    if (alive2) {
                        const unsigned j = base + n_seeds + mbcnt(am2);
                        s_a[j] = 0.5 * l2; s_b[j] = 0.5 * r2; s_fa[j] = fs * fl2; s_fm[j] = fs * fmid2; s_fb[j] = fs * fr2;
                        s_dt[j] = (unsigned)(D + 1) | ((unsigned)p << TAG_SHIFT);
                    }
                    n_seeds += (unsigned)__popcll(am2);
                }
                bot = 0;
                top = n_seeds;
                stamp(ST_SEEDED);
                if constexpr (AQ_STAMPS && !DIAG) {
                    stp[ST_CS] += clk() - cs_st;
                    stp[ST_NS] += 1ull;
                }
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
                __builtin_amdgcn_wave_barrier();
                continue;
            }

            if (phase == 2) break;
            // a leader hands its workgroup's token back first (the atomic's round trip overlaps the flush)
            unsigned r_idle = 0;
            bool had_token = false;
            if (lead && lane == 0) {
                had_token = S.busy_token != 0;
                if (had_token) {
                    S.busy_token = 0;
                    r_idle = g_add(&qc->idle[grp].v, 1u);
                }
            }
            // a wave that ran dry flushes now, off the run's critical path: the workgroup's other waves
            // while its last still works; the last one (the leader) once the end is stored or while it
            // waits, below (every wave flushing after the end was seen had cost a lone launch ~1 us, r04j)
            if (counted_now) flush_acc<FID, PCU>(P, acc, tag, lane, S, s_pc, s_wdd + wid, NWT, xs_a, xs_b);
            if (!lead) {
                __builtin_amdgcn_s_sleep(4);
                __builtin_amdgcn_wave_barrier();
                continue;
            }
            // ---- leader: this workgroup has no work; wait for a chunk or the end
            unsigned long long tl = DIAG ? rtc() : 0ull;
            stamp(ST_LEAD);
            if constexpr (DIAG) {
                if (lane == 0) {
                    atomicMin(&s_dg[DG_T_FIRST_LEAD], tl);
                    atomicAdd(&s_dg[DG_LEADS], 1ull);
                }
            }
            int cmd = -1;   // >= 0 chunk slot, -1 exit, -2 error
            unsigned cnt = 0;
            bool last = false;   // this workgroup's idle transition ended the run
            if (lane == 0) {
                if (had_token && r_idle + 1u == grp_size)   // the group's last busy workgroup
                    last = g_add((int*)&qc->tokens.v, -1) - 1 == -t0;
                if (last)
                    for (int g = 0; g < NGROUP; ++g) st_wt(&qc->done[g].v, 1u);
            }
            // the leader's flush: behind the end's stores (the run's last leader: the other workgroups
            // see the end meanwhile), or before its wait
            flush_acc<FID, PCU>(P, acc, tag, lane, S, s_pc, s_wdd + wid, NWT, xs_a, xs_b);
            if (lane == 0) {
                if (!last) {
                    // per-CU launches: the end flag alone first (one load per spin, no ticket)
                    bool ended = false;
                    if constexpr (PCU) {
                        for (unsigned spins = 0; spins < LAZY_TICKET; ++spins) {
                            if (ld_wt(&qc->done[grp].v)) { ended = true; break; }
                            __builtin_amdgcn_s_sleep(AQ_LEAD_SLEEP);
                        }
                    }
                    if (ended) cmd = -1;
                    const unsigned h = ended ? 0u : g_add(&qc->head.v, 1u);
                    // the wait is bounded by time WITHOUT PROGRESS, not since launch: while work exists,
                    // busy waves donate to waiting tickets within POLL_ROUNDS rounds, and every donation
                    // or idle / busy transition moves the token count or the queue tail
                    unsigned long long t_prog = rtc();
                    int seen_tk = 0;
                    unsigned seen_tl = ~0u;
                    for (unsigned spins = 0; !ended; ++spins) {
                        // both words are read every spin, issued together (one latency per spin)
                        const unsigned rv = h < P.qcap ? ld_wt(&P.ready[(size_t)h * READY_STRIDE]) : 0u;
                        const unsigned dn = ld_wt(&qc->done[grp].v);
                        if (rv == P.epoch) { cmd = (int)h; break; }
                        if (dn) { cmd = -1; break; }
                        if ((spins & 63u) == 63u) {
                            const int tk = g_ld((int*)&qc->tokens.v);
                            const unsigned tl = g_ld(&qc->tail.v);
                            const unsigned long long now = rtc();
                            if (tk != seen_tk || tl != seen_tl) {
                                seen_tk = tk;
                                seen_tl = tl;
                                t_prog = now;
                            } else if (now - t_prog > P.stall_ticks) {
                                err |= ERRB_TIMEOUT;
                                cmd = -2;
                                break;
                            }
                        }
                        __builtin_amdgcn_s_sleep(AQ_LEAD_SLEEP);
                    }
                }
                if (cmd >= 0) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only
                    cnt = ld_wt(&P.chunks[cmd].count);
                }
            }
            cmd = uni(__shfl(cmd, 0, 64));
            cnt = uni(__shfl(cnt, 0, 64));
            if constexpr (DIAG) { if (lane == 0 && cmd < 0) atomicMax(&s_dg[DG_T_DONE], rtc()); }
            if (cmd < 0) stamp(ST_DONE);
            if (cmd < 0) {
                // the end (or an error): no other wave writes the phase any more (all are idle), so one
                // store, no lock
                if (lane == 0) __hip_atomic_store(&S.phase, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __builtin_amdgcn_wave_barrier();
                break;
            }
            // load the chunk into the (empty) pool, take this workgroup's token back
            const Chunk* __restrict__ c = P.chunks + cmd;
            wave_lock(&S.lock, lane, lock_spins);
            const unsigned pt = uni(S.ptop);
            for (unsigned i = lane; i < cnt; i += 64) {
                const unsigned j = POOL0 + ((pt + i) & (PCAP - 1));
                s_a[j] = ld_wt(&c->a[i]); s_b[j] = ld_wt(&c->b[i]);
                s_fa[j] = ld_wt(&c->fa[i]); s_fm[j] = ld_wt(&c->fm[i]); s_fb[j] = ld_wt(&c->fb[i]);
                s_dt[j] = ld_wt(&c->dt[i]);
            }
            if (lane == 0) {
                S.ptop = pt + cnt;
                S.phase = 0;
                S.busy_token = 1;
                __hip_atomic_fetch_add(&S.idle, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);   // the leader un-counts itself, so an empty chunk leads to a new leader
                // busy again: the group's token comes back if the group was all-idle; the chunk's
                // cnt + 1 tokens go (one atomic, so T never shows the chunk gone before the group back)
                const bool was_all_idle = g_add(&qc->idle[grp].v, ~0u) == grp_size;
                g_add((int*)&qc->tokens.v, (was_all_idle ? 1 : 0) - (int)(cnt + 1u));
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
            __builtin_amdgcn_wave_barrier();
            continue;
        }

        // ---- keep the ring from overflowing: its bottom 64 pairs go to the cellar, else the pool,
        //      else an HBM chunk
        if (size > (unsigned)(WCAP - 64)) {
            if (pf_n) {
                // a prefetch in flight is cancelled: its pairs never left the cellar (the loads land in
                // registers nobody reads; the next spill writes above them)
                ctop += pf_n;
                pf_n = 0;
            }
            if (ctop + (unsigned)SPILL <= (unsigned)CCAP) {
                spill_to_cellar(bot, ctop);
                ctop += (unsigned)SPILL;
                bot += (unsigned)SPILL;
                __builtin_amdgcn_wave_barrier();
                continue;
            }
            wave_lock(&S.lock, lane, lock_spins);
            const unsigned pt = uni(S.ptop);
            const bool fits = (pt - S.pbot) + 64u <= (unsigned)PCAP;
            if (fits) {
                copy_pair(R, base + ring_slot(bot + lane), POOL0 + ((pt + lane) & (PCAP - 1)));
                if (lane == 0) S.ptop = pt + 64u;
            }
            wave_unlock(&S.lock, lane);
            if (!fits) {
                // pool full: spill 64 pairs to an HBM chunk (tokens first, then publish)
                unsigned slot = 0;
                if (lane == 0) {
                    slot = g_add(&qc->tail.v, 1u);
                    if (slot < P.qcap) g_add((int*)&qc->tokens.v, 64 + 1);   // records + 1 per chunk
                    spilled += 64;
                }
                slot = uni(__shfl(slot, 0, 64));
                if (slot < P.qcap) {
                    const unsigned b = bot;
                    publish_chunk(P, R, slot, 64u, [&](unsigned i) { return base + ring_slot(b + i); }, lane);
                } else {
                    err |= ERRB_OVERFLOW;   // pairs dropped: result invalid, error reported
                }
            }
            if constexpr (DIAG) { if (lane == 0) atomicAdd(&s_dg[DG_POOL_PUSH], 64ull); }
            bot += 64;
            __builtin_amdgcn_wave_barrier();
            continue;
        }

        ++poll_ctr;
        // ---- donate to starving workgroups (another CU waits on the HBM queue). Checked before the
        //      sibling give: every poll round is also a give round, and a successful give `continue`s
        //      past the poll (r05: a CU whose waves keep feeding each other then never serves a waiting
        //      one; DIAG of a 262144-integral tiny-tree launch, profiles/r05f-g)
        if ((poll_ctr % poll_rounds) == 0) {
            unsigned slot = 0xffffffffu;
            if (lane == 0) {
                if constexpr (DIAG) atomicAdd(&s_dg[DG_POLLS], 1ull);   // polls (low word) | polls that saw a
                                                                          // waiting ticket (high word)
                if ((int)(seen_head - seen_tail) > 0) {
                    unsigned expect = seen_tail;
                    if (__hip_atomic_compare_exchange_strong(&qc->tail.v, &expect, seen_tail + 1u, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                        slot = seen_tail;
                    if constexpr (DIAG) atomicAdd(&s_dg[DG_POLLS], 1ull << 32);
                }
                seen_head = g_ld(&qc->head.v);
                seen_tail = g_ld(&qc->tail.v);
            }
            slot = uni(__shfl(slot, 0, 64));
            if (slot != 0xffffffffu) {
                if (slot >= P.qcap) {
                    err |= ERRB_OVERFLOW;
                } else {
                    wave_lock(&S.lock, lane, lock_spins);
                    const unsigned pavail = uni(S.ptop - S.pbot);
                    unsigned k;
                    if (pavail >= (unsigned)DONATE_MIN) {
                        k = min((unsigned)CH, pavail / 2u);
                        const unsigned pb = S.pbot;
                        if (lane == 0) g_add((int*)&qc->tokens.v, (int)k + 1);   // records + 1 per chunk
                        publish_chunk(P, R, slot, k, [&](unsigned i) { return POOL0 + ((pb + i) & (PCAP - 1)); }, lane);
                        if (lane == 0) S.pbot = pb + k;
                        wave_unlock(&S.lock, lane);
                    } else {
                        wave_unlock(&S.lock, lane);
                        k = size / 2u;   // may be 0: an empty chunk is harmless
                        if (lane == 0) g_add((int*)&qc->tokens.v, (int)k + 1);   // records + 1 per chunk
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
                    __builtin_amdgcn_wave_barrier();
                    continue;
                }
            }
        }

        // ---- feed idle sibling waves
        if ((poll_ctr % give_rounds) == 0 && size >= give_min &&
            uni(__hip_atomic_load(&S.idle, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) > 0 &&
            uni(__hip_atomic_load(&S.ptop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) ==
                uni(__hip_atomic_load(&S.pbot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) {
            const unsigned k = size / 2u;   // <= WCAP / 2 <= PCAP
            wave_lock(&S.lock, lane, lock_spins);
            const unsigned pt = uni(S.ptop);
            const bool fits = (pt - S.pbot) + k <= (unsigned)PCAP;
            if (fits) {
                for (unsigned i = lane; i < k; i += 64)
                    copy_pair(R, base + ring_slot(bot + i), POOL0 + ((pt + i) & (PCAP - 1)));
                if (lane == 0) S.ptop = pt + k;
            }
            wave_unlock(&S.lock, lane);
            if constexpr (DIAG) { if (lane == 0) atomicAdd(&s_dg[DG_GIVE], (unsigned long long)(fits ? k : 0u)); }
            if (fits) {
                bot += k;
                __builtin_amdgcn_wave_barrier();
                continue;
            }
        }
        // ---- running low: fetch the next 64 cellar pairs now, land them next iteration
        if (ctop > 0 && pf_n == 0 && size <= (unsigned)PF_ISSUE) {
            pf_n = 64u;   // ctop is a whole number of chunks
            ctop -= pf_n;
            // (same-wave, same-address order: no wait for the spills)
            pf = chunk_load(&cel->c[ctop / 64u], lane);
            __builtin_amdgcn_wave_barrier();
        }

        // ---- a burst of rounds: the hot loop. It runs while the wave's pairs (ring + held) neither
        //      run out nor near overflow, no cellar move is due, and the next round is not a give /
        //      poll check round: everything it touches besides the pairs is wave-uniform.
        // the burst's state, re-asserted uniform (readfirstlane) once per burst: the outer loop's many
        // paths leave the compiler unsure, and a "divergent" ring index turns every round's index
        // arithmetic and the loop exit into VALU / exec-mask work
        unsigned long long cb0 = 0;
        if constexpr (AQ_STAMPS && !DIAG) cb0 = clk();
        unsigned b_top = uni(top), b_size = uni(size), b_poll = uni(poll_ctr);
        unsigned b_n = 0;                 // pairs evaluated in this burst (2 tasks each)
        unsigned long long b_dv = 0;      // lanes that met the depth cap with a refining task
        unsigned b_bot = uni(bot), b_ctop = uni(ctop), b_pf = uni(pf_n);
        bool b_mixed = uni(mixed);
        // Carried pairs (r04). Every lane keeps ONE pair in registers from round to round (b_am: the
        // lanes that hold one). A round first fills the idle lanes from the ring's top (one masked
        // pop), evaluates both tasks of every held pair, pushes ONE child pair per lane -- task 1's,
        // when it refines -- and keeps task 0's children as the lane's next pair (a depth-first walk
        // per lane, the ring holding the right siblings). Three pair writes per round where the
        // popped-pairs round made six: the writes' VGPR-to-LDS transfer and LDS-array cycles are the
        // CU's second bottleneck beside the VALU (83 LDS-array cycles per wave-round, active 59 % of
        // the kernel's cycles: profiles/r04_pmc_lds; r04 A/B -6.5 %, profiles/r04_ab). The pop is six
        // ds_read_b64 (12 array cycles) rather than three ds_read2st64_b64 (24). The window, the cellar lines and the accounting
        // count S = ring + held pairs; a burst starts with every pair in the ring and ends by pushing
        // the held ones back on top. Capacity: a round moves at most one pair per active lane into the
        // ring, so the ring never holds more than S at a round's start; S <= WCAP - 64 then leaves
        // room for the round (S grows by <= 64) and the final push.
        unsigned b_S = b_size, b_S0 = b_size;   // ring + held; the accounting base (moves with the cellar)
        unsigned long long b_am = 0;
        double ca = 0.0, cb = 0.0, cfa = 0.0, cfm = 0.0, cfb = 0.0, cdw = 0.0;   // the held pair (cdw: the dt word)
        unsigned b_lo1, b_span;
        auto window = [&]() {
            b_lo1 = (b_pf != 0u ? (unsigned)PF_BELOW : (b_ctop > 0u ? (unsigned)PF_ISSUE : 0u)) + 1u;
            b_span = (unsigned)(WCAP - 64) + 1u - b_lo1;
        };
        window();
        constexpr bool prio_by_load = PCU && FID == F_SIN_RECIP;
        const bool b_heavy = prio_by_load && b_S >= HEAVY_S;
        const unsigned b_max = give_rounds - b_poll % give_rounds;   // rounds up to the give / poll round
        unsigned b_rem = b_max;
        __builtin_amdgcn_s_waitcnt(0xC07F);   // (see below: no wait in front of every round's pop)
        bool b_go;
        for (;;) {
        for (;;) {
            unsigned long long c0 = 0, c1 = 0;
            if constexpr (DIAG) c0 = clk();
            if constexpr (prio_by_load) {
                if (b_heavy) asm volatile("s_setprio 3");
                else asm volatile("s_setprio 1");
            }
            // ---- fill: the idle lanes take the ring's top k pairs (rank j among the idle lanes)
            const unsigned long long need = ~b_am;
            const unsigned k = min((unsigned)__popcll(need), b_top - b_bot);
            const unsigned jr = mbcnt(need);
            const unsigned long long fmsk = __ballot(jr < k) & need;
            b_top -= k;
            const unsigned paddr = ring_addr(ring8, ring_slot(b_top) + jr, ring_vmask);
            lds_pop6_masked(fmsk, paddr, paddr + 3u * 50u * 512u, ca, cb, cfa, cfm, cfb, cdw);
            const unsigned long long am = b_am | fmsk;
            const unsigned na = (unsigned)__popcll(am);
            const double pa = ca, pb = cb, pfa = cfa, pfm = cfm, pfb = cfb;
            const unsigned long long dtw = (unsigned long long)__double_as_longlong(cdw);
            const unsigned dt = (unsigned)dtw;
            Step2 st[2];
            // the lanes whose pair lacks SPAN_BIT (both midpoints lie in the pair's interval, so one
            // sign test of the pair word)
            unsigned long long nospan = 0ull;
            if constexpr (FID == F_COSH4) nospan = __ballot((int)dt >= 0);
            double pm, hm;
            pair_step_halves<FID, WIDE ? 255u : 127u>(pa, pb, pfa, pfm, pfb, eps2, tab, st, pm, hm, kk,
                                                       FID == F_COSH4 ? 2 : -1, nospan & am);
            if constexpr (prio_by_load) { if (!b_heavy) asm volatile("s_setprio 0"); }
            const unsigned long long r0m = __ballot(st[0].refine), r1m = __ballot(st[1].refine);
            unsigned long long okm = am;
            if constexpr (!burst_cap) {
                const unsigned long long dm = __ballot((dt & 255u) < (unsigned)(max_depth - 1));
                okm = am & dm;
                const unsigned long long atcap = am & ~dm;
                if (__builtin_expect(atcap != 0ull, 0)) b_dv |= atcap & (r0m | r1m);
            }
            const unsigned long long l0m = am & ~r0m, l1m = am & ~r1m;
            b_n += na;   // tasks 2 na; accepted: once per burst from the growth of S (below)
            const unsigned long long mask0 = okm & r0m, mask1 = okm & r1m;
            // depth + 1, same integral: a 32-bit add on the word's low half (the depth byte never carries
            // past bit 7, static_assert above); the high half of the 8-byte field is carried unread
            const unsigned cdt = dt + 1u;
            const unsigned long long cdtw = ((dtw >> 32) << 32) | (unsigned long long)cdt;
            masked_acc3(acc.r, st[0].area2, l0m, st[1].area2, l1m, acc.maxdt, burst_cap ? cdt : dt,
                        burst_cap ? (mask0 | mask1) : am);
            if constexpr (DIAG) {
                const int rtag = (int)dt_tag(dt);
                b_mixed |= (__ballot(rtag != tag) & am) != 0ull;
            }
            if (HIST) {
                const unsigned d = dt & 255u;
                if (__builtin_amdgcn_inverse_ballot_w64(am)) {
                    atomicAdd(&P.ctls[P.first_slot + tag].hist[d], 2ull);
                    const unsigned nl = ((l0m >> lane) & 1u) + ((l1m >> lane) & 1u);
                    if (nl) atomicAdd(&P.ctls[P.first_slot + tag].hist[AQ_MAX_LEVELS + d], (unsigned long long)nl);
                }
            }
            if constexpr (DIAG) c1 = clk();
            // ---- task 1's children [m, b] go on the ring (:192-197); task 0's [a, m] stay in the lane
            lds_push6_masked(mask1, ring_addr(ring8, ring_slot(b_top) + mbcnt(mask1), ring_vmask), hm, pb, pfm,
                             st[1].fmid, pfb, __longlong_as_double((long long)cdtw));
            b_top += (unsigned)__popcll(mask1);
            cb = hm;
            cfb = pfm;
            cfm = st[0].fmid;
            cdw = __longlong_as_double((long long)cdtw);
            b_am = mask0;
            if constexpr (DIAG) {
                if (lane == 0) {
                    const unsigned long long c2 = clk();
                    atomicAdd(&s_dg[DG_ROUNDS], 1ull);
                    atomicAdd(&s_dg[DG_ACTIVE_LANES], (unsigned long long)na);
                    atomicAdd(&s_dg[DG_C_ROUND], c2 - c0);
                    atomicAdd(&s_dg[DG_C_EVAL], c1 - c0);
                    atomicMax(&s_dg[DG_MAX_RING], (unsigned long long)b_S);
                    atomicMax(&s_dg[DG_T_LAST_ROUND], rtc());
                    atomicAdd(&s_dg[DG_ACTIVE_TASKS], 2ull * na);
                }
            }
            b_S = (b_top - b_bot) + (unsigned)__popcll(mask0);
            --b_rem;
            unsigned span_r = b_rem != 0u ? b_span : 0u;
            asm("" : "+s"(span_r));
            b_go = b_S - b_lo1 < span_r;
            __builtin_amdgcn_wave_barrier();
            if (!b_go) break;
        }
            unsigned b_re = b_rem;
            asm volatile("" : "+s"(b_re));
            const unsigned sz = b_S;
            if (b_re != 0u && sz != 0u) {
                // a cellar edge: S > WCAP - 64 leaves >= WCAP - 128 >= SPILL pairs in the ring; S <=
                // PF_BELOW leaves the ring room for the landing
                if (sz > (unsigned)(WCAP - 64)) {
                    if (b_ctop + (unsigned)SPILL <= (unsigned)CCAP) {
                        if (b_pf) {
                            b_ctop += b_pf;
                            b_pf = 0;
                        }
                        spill_to_cellar(b_bot, b_ctop);
                        b_ctop += (unsigned)SPILL;
                        b_bot += (unsigned)SPILL;
                        b_S -= (unsigned)SPILL;
                        b_S0 -= (unsigned)SPILL;
                        b_go = true;
                    }
                } else if (b_pf) {
                    if (b_bot < 64u) {
                        b_bot += (unsigned)WCAP;
                        b_top += (unsigned)WCAP;
                    }
                    b_bot -= b_pf;
                    if (lane < b_pf) lds_store6(ring_addr(ring8, ring_slot(b_bot) + lane, ring_vmask), pf);
                    if constexpr (DIAG) { if (lane == 0) atomicAdd(&s_dg[DG_PREFETCH], (unsigned long long)b_pf); }
                    b_S += b_pf;
                    b_S0 += b_pf;
                    b_pf = 0;
                    b_go = true;
                } else if (b_ctop > 0u) {
                    b_pf = 64u;
                    b_ctop -= 64u;
                    pf = chunk_load(&cel->c[b_ctop / 64u], lane);
                    b_go = true;
                }
                if (b_go) window();
            }
            __builtin_amdgcn_wave_barrier();
            if (!b_go) break;
        }
        // (a heavy burst ran at priority 3: back to 0 before the push-back, the outer loop, the locks and
        // the leader's polls -- ADVICE r4)
        if constexpr (prio_by_load) asm volatile("s_setprio 0");
        // the held pairs back on top of the ring
        lds_push6_masked(b_am, ring_addr(ring8, ring_slot(b_top) + mbcnt(b_am), ring_vmask), ca, cb, cfa, cfm, cfb,
                         cdw);
        b_top += (unsigned)__popcll(b_am);
        bot = b_bot;
        ctop = b_ctop;
        pf_n = b_pf;
        b_poll += (b_max - b_rem) - 1u;   // every round but the burst's last advances the give / poll counter
        top = b_top;
        poll_ctr = b_poll;
        // a round with na held pairs evaluates 2 na tasks; each refining task adds one pair to S and
        // each evaluated pair leaves it, so accepted = 2 na - refining = na - (growth of S); summed over
        // the burst: b_n - (S_end - S_start), the cellar moves taken out of S_start as they happen
        acc.ut += 2u * b_n;
        acc.ul += b_n - ((b_top - b_bot) - b_S0);
        dd_add(acc.hi, acc.lo, acc.r);   // the burst's lane partial, exactly into the double-double
        acc.r = 0.0;
        if (b_dv) err |= ERRB_DEPTH;
        if constexpr (burst_cap) {
            // the per-burst depth cap: a pushed pair at depth >= max_depth means a task at the cap
            // refined. The wave drops its ring and cellar (the run is invalid) before anything can hand
            // the pairs on, so nothing past the cap leaves the wave (the configuration notes above)
            if (__builtin_expect(__ballot((acc.maxdt & 255u) >= (unsigned)max_depth) != 0ull, 0)) {
                err |= ERRB_DEPTH;
                top = bot;
                ctop = 0;
                pf_n = 0;
            }
        }
        mixed = b_mixed;
        if constexpr (AQ_STAMPS && !DIAG) {
            stp[ST_CB] += clk() - cb0;
            stp[ST_NB] += 1ull;
            stp[ST_NR] += (unsigned long long)(b_max - b_rem);
        }
        __builtin_amdgcn_wave_barrier();   // reconverge before the loop latch (keeps wave state uniform)
    }

    // ---------------- exit: flush this wave's accumulators (no workgroup barrier needed) --------
    if constexpr (DIAG) { if (lane == 0) atomicMax(&s_dg[DG_T_BROKE], rtc()); }
    stamp(ST_BROKE);
    flush_acc<FID, PCU>(P, acc, tag, lane, S, s_pc, s_wdd + wid, NWT, xs_a, xs_b);
    if constexpr (DIAG) { if (lane == 0) atomicMax(&s_dg[DG_T_FLUSHED], rtc()); }
    stamp(ST_FLUSHED);
    if (mixed) err |= ERRB_OVERFLOW;
    const unsigned werr = wave_or_full(err);
    unsigned last_u = 0;
    if (lane == 0) {
        if (werr) {
            for (int p = 0; p < P.nprob; ++p)
                atomicOr(&P.ctls[P.first_slot + p].sums.error, werr);
        }
        if (spilled) atomicAdd(&P.ctls[P.first_slot].sums.spilled, spilled);
        if constexpr (DIAG) {
            atomicAdd(&s_dg[DG_LOCK_SPINS], lock_spins);
            atomicAdd(&s_dg[DG_SPILL_RECORDS], spilled);
            atomicAdd(&s_dg[DG_C_LOOP], clk() - cl0);
        }
        // job-size hint for the next adaptive launch: the last wave of each workgroup adds the
        // workgroup's tasks, the last workgroup sets shares per integral for ~TASKS_PER_JOB per job
        // (every launch: the workgroup's tasks also go to the context's per-CU counters, below)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // this wave's LDS flushes precede its exit count
        const bool last = atomicAdd(&S.exited, 1u) == (unsigned)NWT - 1u;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        last_u = last ? 1u : 0u;
        if (last) {
            // per-CU task counters on every launch shape: the workgroup's tasks, once,
            // into its hardware CU slot -- one atomic per workgroup and launch, on 256 distinct lines
            const unsigned long long wt = __hip_atomic_load(&S.tasks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (wt && !AQ_X_NOCUACC) __hip_atomic_fetch_add(&P.cu_acc[cu_slot()], wt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if constexpr (DIAG) { if (last) atomicMax(&s_dg[DG_T_FOLD], rtc()); }
        if (PCU && last) {
            // per-CU launch: this workgroup's counts per integral, once -- its per-CU word (a plain
            // store, one writer) and the slot sums (256 workgroups instead of every wave's flushes)
            const unsigned cu = cu_slot();
            for (int p = 0; p < P.nprob; ++p) {
                const unsigned long long t = __hip_atomic_load(&s_pc[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const unsigned long long l = __hip_atomic_load(&s_pc[PCU_ROW + p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const unsigned m = (unsigned)__hip_atomic_load(&s_pc[2 * PCU_ROW + p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                unsigned long long* wp = P.parts + 2 * ((size_t)p * gridDim.x + bid);
                wp[0] = pack_cu(t, cu);
                wp[1] = (l << 8) | (unsigned long long)(m & 255u);
                if (bid == 0) {
                    SlotSums& sm = P.ctls[P.first_slot + p].sums;
                    sm.pcu = 1u;
                    sm.win_lo_not = xs_win_lo(0);   // per-CU slots: the full limb window (a few slots only)
                    sm.win_hi = (unsigned)XS_LIMBS;
                }
            }
        }
        if (!PCU && last && (P.adaptive & 2)) {
            const unsigned long long wt = __hip_atomic_load(&S.tasks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(&P.hint->tasks, wt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned g = __hip_atomic_fetch_add(&P.hint->exits, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (g == gridDim.x - 1u) {
                const unsigned long long tot = __hip_atomic_load(&P.hint->tasks, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long per = tot / (unsigned long long)P.nprob;   // tasks per integral (shard)
                unsigned long long sh = (per + TASKS_PER_JOB / 2) / TASKS_PER_JOB;
                sh = sh < 1ull ? 1ull : (sh > (unsigned long long)W ? (unsigned long long)W : sh);
                __hip_atomic_store(&P.hint->shares_next, (unsigned)sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if constexpr (HEAPS) __hip_atomic_store(&P.hint->per_next, per, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&P.hint->tasks, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&P.hint->exits, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if constexpr (PCU && !AQ_X_NOFOLD) {
        // the workgroup's last wave: the waves' double-doubles of each integral summed (lanes < NWT, one
        // DPP row) into the workgroup's two area words, plain stores beside its count words. Readers add
        // the grid's words exactly (k_fold_parts, k_fetch_sync, k_pack_group). r06: the workgroups had
        // folded an exact LDS accumulator into the slot with far atomics at exit -- ~1 300 atomics on the
        // same one or two limb lines at the launch's end, 2.6 us of a 21 us lone integral (profiles/r06b:
        // the AQ_X_NOFOLD timing build; moving them to the waiting leaders saved nothing, r06c)
        if (uni(__shfl(last_u, 0, 64))) {
            for (int p = 0; p < P.nprob; ++p) {
                double hi = 0.0, lo = 0.0;
                if (lane < (unsigned)NWT) {
                    const double2 w = s_wdd[p * NWT + (int)lane];
                    hi = w.x;
                    lo = w.y;
                }
                row_sum_dd(hi, lo);   // lanes 0-15 (NWT <= 16): every lane of the row holds the sum
                if (lane == 0) {
                    double* pa = P.parea + 2 * ((size_t)p * gridDim.x + bid);
                    pa[0] = hi;
                    pa[1] = lo;
                }
            }
        }
    }
#if AQ_STAMPS
    if constexpr (!DIAG) {
        stamp(ST_EXIT);
        stp[ST_CL] = clk() - cl0;
        stp[ST_XCC] = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;
        if (lane < (unsigned)ST_N) {   // vector stores, one word per lane
            unsigned long long v = 0;
            for (int i = 0; i < ST_N; ++i) v = lane == (unsigned)i ? stp[i] : v;
            g_aq_stamps[(size_t)(bid * (unsigned)NWT + wid) * ST_STRIDE + lane] = v;
        }
    }
#endif
    if constexpr (DIAG) {
        __syncthreads();
        if (tid == 0) {
            s_dg[DG_T_EXIT] = rtc();
            s_dg[DG_CU] = cu_slot();
            s_dg[DG_TASKS] = S.tasks;
            unsigned long long* o = P.diag + (size_t)blockIdx.x * DIAG_WORDS;
            for (int i = 0; i < DIAG_WORDS; ++i) o[i] = s_dg[i];
        }
    }
}

}  // namespace aq
