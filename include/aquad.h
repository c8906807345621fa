/*
 * aquad.h -- C ABI of the MI355X-native adaptive-quadrature engine (libaquad.so).
 *
 * The reference (/root/reference/aquadPartA.c) has no plugin or FFI layer: its boundary is
 * the macro quartet F/A/B/EPSILON (:45-48) plus the farmer/worker message protocol
 * (farmer() :125-173, worker() :175-208) that main() (:78-123) drives. Each entry point below
 * names the reference interface it replaces. Plain C types only: no HIP, RCCL or torch types cross
 * this boundary; every host buffer is caller-owned; device memory, streams, events and RCCL
 * communicators are owned by opaque handles (aq_ctx: one GPU; aq_group: GPUs that combine results
 * over RCCL). No global state; a handle is not re-entrant; calls block unless the name says _async.
 * Errors: 0 on success, a negative AQ_E* code otherwise (the reference's only error is
 * numprocs < 2 -> stderr + exit(1), :86-90; the CLI maps codes to that behaviour).
 *
 * Deviation from SURVEY.md §8b's sketch: every call takes its aq_ctx / aq_group first (the sketch's
 * own "no global state" rule); aq_integrate_batch also returns per-integral task counts.
 */
#ifndef AQUAD_H
#define AQUAD_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AQ_OK 0
#define AQ_EINVAL (-1)     /* bad argument (non-finite bounds, b < a, eps < 0, bad shard, outside the integrand's domain;
                            every integrand: each bound 0 or 2^-900 <= |x| <= 2^900) */
#define AQ_EHIP (-2)       /* a HIP runtime call failed */
#define AQ_ETIMEOUT (-3)   /* an on-device wait saw no progress for the stall bound (aq_set_stall_timeout) */
#define AQ_EOVERFLOW (-4)  /* a frontier / work-queue capacity was exceeded */
#define AQ_EDEPTH (-5)     /* refinement reached max_depth (the reference would not terminate) */
#define AQ_ENOMEM (-6)     /* device or host allocation failed */
#define AQ_ENODEV (-7)     /* no HIP device */
#define AQ_ERCCL (-8)      /* an RCCL call failed (aq_group_*) */
#define AQ_ERESIDENT (-9)  /* the persistent grid cannot be co-resident on the device (its workgroups wait
                            on each other): refused before launch, never a stall */

#define AQ_DEFAULT_MAX_DEPTH 96
#define AQ_MAX_LEVELS 128     /* length of the per-level histograms */
#define AQ_CU_SLOTS 2048      /* hardware CU slot space: xcc*256 + (se*2+sh)*16 + cu */
#define AQ_XS_LIMBS 68        /* exact area accumulator: int64 limbs (aq_fetch_exact / aq_exact_round) */
#define AQ_EXACT_ROW (AQ_XS_LIMBS + 4)   /* limbs, tasks, accepted, spilled, levels | error << 32 */

/* Integrand = the reference's F(arg) macro (aquadPartA.c:46) as a compile-time kernel variant. */
typedef enum {
    AQ_F_COSH4 = 0,     /* cosh(x)*cosh(x)*cosh(x)*cosh(x), glibc-2.35-exact cosh (the reference), |x| <= 170 */
    AQ_F_SIN_RECIP = 1, /* sin(1/x) (SURVEY config 4), glibc-exact for |x| > 9.5e-9 */
    AQ_F_USER = 2       /* the plug-in compiled in from AQ_USER_F_HEADER (aq_user_integrand_name()) */
} aq_integrand;

/* Replaces the compile-time macros EPSILON / F / A / B (aquadPartA.c:45-48) and mpirun -n (:83). */
typedef struct {
    int32_t integrand;  /* aq_integrand */
    int32_t max_depth;  /* refinement cap; 0 -> AQ_DEFAULT_MAX_DEPTH (<= AQ_MAX_LEVELS - 1) */
    double a;           /* A (:47) */
    double b;           /* B (:48) */
    double eps;         /* EPSILON (:45): absolute, strict '>' test (:191) */
    int32_t n_gpus;     /* GPUs the integral is sharded over: 0 or 1 for aq_integrate, the group size
                           (or 0) for aq_integrate_group */
    int32_t reserved;
} aq_problem;

/* Replaces farmer()'s return value and the global tasks_per_process[] (:72, :101, :162). */
typedef struct {
    double area;        /* Σ accepted larea+rarea (:199 sent, :149 summed): the exact sum of the workers'
                           partials (per-lane double sums in the persistent kernel), rounded once -- within
                           a few ulp of the exact leaf sum, last bits schedule-dependent */
    uint64_t tasks;     /* intervals evaluated = Σ tasks_per_process (:162) */
    uint64_t accepted;  /* accepted subintervals (tag-1 area messages, :201) */
    uint32_t levels;    /* 1 + deepest refinement level reached */
    uint32_t n_cu;      /* CUs that evaluated at least one task. Per-CU counts (n_cu, tasks_per_cu) are kept
                           for the synchronous calls and for launches of fewer than 12 integrals into slots
                           below 16384; other launches report n_cu = 0 and zero rows (their per-CU work is
                           still counted by aq_cu_task_counters, which sees every launch) */
    uint64_t spilled;   /* interval pairs moved through the HBM work queue (load balance) */
    uint32_t n_gpus;    /* GPUs that contributed (entries written to tasks_per_gpu) */
    uint32_t reserved;
    uint64_t *tasks_per_gpu;  /* [n_gpus] caller-owned or NULL: tasks per GPU (the workers of :162) */
    uint64_t *tasks_per_cu;   /* [n_gpus * aq_ctx_num_cus()] caller-owned or NULL: tasks per CU, each
                                 GPU's CUs in hardware-slot order (0 where not kept) */
} aq_result;

typedef struct aq_ctx aq_ctx;

/* ---- lifecycle (replaces MPI_Init / MPI_Comm_size / MPI_Finalize, :82-84, :121) ------------- */
int aq_device_count(int *count);
int aq_ctx_create(int device, aq_ctx **out);
void aq_ctx_destroy(aq_ctx *ctx);
const char *aq_strerror(int code);
/* Compute units of the context's device (one persistent workgroup each). */
int aq_ctx_num_cus(const aq_ctx *ctx);
/* Wavefront workers of the on-device farmer (workgroups x 12 waves per workgroup): the partition of
 * sharded and multi-integral launches (aq_integrate_shard documents it). An unsharded launch of ONE
 * integral runs 8 waves per workgroup (its set-up and seeding are issue-bound at three waves per SIMD);
 * launches of 2 or more integrals run 12. */
int aq_ctx_num_workers(const aq_ctx *ctx);
/* Device memory the context holds, bytes. */
int aq_ctx_device_bytes(const aq_ctx *ctx, uint64_t *bytes);
/* Per-level task/accepted histograms on the persistent path (default on; a diagnostic the
 * reference does not produce -- pipelined callers switch it off). */
int aq_set_level_histograms(aq_ctx *ctx, int enable);
/* The persistent kernel's grid is one workgroup per CU (AQ_GRID=<n> in the environment at create time
 * overrides it, e.g. to leave CUs to other work). Its workgroups hand work to each other, so every
 * launch checks -- for the exact kernel instance, block size and LDS -- that the device can hold the
 * whole grid at once, and refuses with AQ_ERESIDENT otherwise. AQ_COOP=1 at create time launches it
 * as a cooperative kernel (the runtime's own co-residency guarantee) instead of a plain launch. */
/* How long a waiting workgroup tolerates NO PROGRESS of the on-device work queue before the launch
 * fails with AQ_ETIMEOUT (default 10 s, or the AQ_STALL_MS environment variable at create time). A
 * bound on stalls, not on run time: launches of any length that keep progressing never time out. */
int aq_set_stall_timeout(aq_ctx *ctx, double ms);
/* Name of the AQ_F_USER plug-in compiled into this library. */
const char *aq_user_integrand_name(void);

/* ---- the hot path ----------------------------------------------------------------------------
 * aq_integrate: farmer(numprocs) + every worker() of one run (:125-208) as ONE persistent HIP
 * launch: wavefronts expand sibling-pair frontiers in LDS (task body :183-202), accumulate accepted
 * areas, and rebalance through an HBM work queue (the bag of tasks, :152-165).
 * Bit-identical interval tree: `tasks` and `accepted` equal the reference's counts exactly.
 * The synchronous calls (aq_integrate, aq_integrate_shard) use an internal result slot, never the
 * caller's async slots, and read it back with one small kernel into pinned host memory.
 */
int aq_integrate(aq_ctx *ctx, const aq_problem *p, aq_result *res);

/* This process's share of a multi-GPU run: the depth-D positions (D = floor(log2(V)) + 2) are
 * dealt in snake order over V = nshards * aq_ctx_num_workers() virtual workers; shard `shard`
 * evaluates its positions' subtrees plus the tasks at depth <= D it owns (each counted by the
 * owner of its leftmost descendant position, so by exactly one shard). Summing
 * area/tasks/accepted over all shards (the caller's all-reduce, or aq_integrate_group) gives
 * exactly the single-GPU result. */
int aq_integrate_shard(aq_ctx *ctx, const aq_problem *p, int shard, int nshards, aq_result *res);
/* The same shard, returned as its exact row (int64[AQ_EXACT_ROW], the layout of aq_fetch_exact): the
 * input of a caller's int64 all-reduce (ppls_amd/dist.py). Blocking, internal slot like
 * aq_integrate_shard; the return code carries the row's error bits (the row is written either way). */
int aq_integrate_shard_exact(aq_ctx *ctx, const aq_problem *p, int shard, int nshards, int64_t *row);

/* ---- multi-GPU over RCCL (replaces the MPI layer, :145-171, and `result += buff[0]`, :149) ----
 * A group is a set of contexts, one per GPU, joined by RCCL communicators over xGMI. Either one
 * process drives n GPUs (aq_group_create: ncclCommInitAll), or every process drives one GPU
 * (the MPI layout: rank 0 makes an id with aq_group_unique_id, the caller broadcasts it -- e.g.
 * MPI_Bcast -- and every rank calls aq_group_join). aq_integrate_group runs rank r's shard r of N
 * on each member, then ONE grouped RCCL exchange: an int64 all-reduce of the exact area limbs and
 * counts (so the area is the correctly rounded exact sum, whatever N) and an all-gather of each
 * rank's task / per-CU counts (tasks_per_gpu, tasks_per_cu). Every member gets the whole result. */
typedef struct aq_group aq_group;
#define AQ_GROUP_ID_BYTES 128
int aq_group_create(aq_ctx *const *ctxs, int n, aq_group **out);
int aq_group_unique_id(void *id /* AQ_GROUP_ID_BYTES */);
int aq_group_join(aq_ctx *ctx, int nranks, int rank, const void *id, aq_group **out);
void aq_group_destroy(aq_group *g);
int aq_group_size(const aq_group *g);
int aq_integrate_group(aq_group *g, const aq_problem *p, aq_result *res);

/* Asynchronous form for pipelined callers (bench): enqueue one integral on the context's stream,
 * results land in device slot `slot` (0 <= slot < aq_async_slots()); aq_fetch blocks for it. */
int aq_async_slots(void);
int aq_integrate_async(aq_ctx *ctx, const aq_problem *p, int shard, int nshards, int slot);
/* K integrals of one integrand / eps / max_depth in ONE persistent launch (K <=
 * aq_max_integrals_per_launch()): integral i has bounds [a[i], b[i]] and lands in slot first_slot+i
 * (first_slot + k <= aq_async_slots()). The integrals share the machine: a wave that runs out of
 * work on one integral seeds its share of the next, so the tail of each overlaps the next. */
int aq_max_integrals_per_launch(void);
int aq_integrate_many_async(aq_ctx *ctx, int integrand, int k, const double *a, const double *b, double eps,
                            int max_depth, int shard, int nshards, int first_slot);
/* Like aq_integrate_many_async with a per-integral shard: integral i is shard shard[i] of nshards
 * (the partition of aq_integrate_shard; every launch of one nshards uses the same partition, so any
 * rank may run any shard of any integral -- the rebalanced multi-GPU batch, ppls_amd/dist.py).
 * nshards == 1 (every shard[i] 0: whole integrals) is an unsharded launch, as aq_integrate_many_async. */
int aq_integrate_mixed_async(aq_ctx *ctx, int integrand, int k, const double *a, const double *b,
                             const int32_t *shard, int nshards, double eps, int max_depth, int first_slot);
int aq_fetch(aq_ctx *ctx, int slot, aq_result *res);
/* The slot's exact row: int64[AQ_EXACT_ROW] = area limbs, tasks, accepted, spilled,
 * levels | error bits << 32 -- summed limb-wise across shards (an int64 all-reduce), the rounded
 * area is the same whatever the partition. */
int aq_fetch_exact(aq_ctx *ctx, int slot, int64_t *row);
/* Correctly rounded double of AQ_XS_LIMBS exact-accumulator limbs (host function). */
double aq_exact_round(const int64_t *limbs);
int aq_synchronize(aq_ctx *ctx);
/* Enqueue (on the context's stream) a copy of n consecutive slots' totals, starting at first_slot
 * (mod aq_async_slots()), into the DEVICE buffer d_out as n rows of 4 doubles
 * {area, tasks, accepted, error bits}: the input of one all-reduce for n pipelined integrals. */
int aq_gather_results(aq_ctx *ctx, int first_slot, int n, void *d_out);
/* The same slots as exact int64 rows (AQ_EXACT_ROW each) into the DEVICE buffer d_out. */
int aq_gather_exact(aq_ctx *ctx, int first_slot, int n, void *d_out);

/* Level-synchronous breadth-first path (one kernel per tree level, host loop): the debug /
 * cross-check schedule. Fills per-level histograms (caller arrays of length maxlev or NULL). */
int aq_integrate_levels(aq_ctx *ctx, const aq_problem *p, aq_result *res, uint64_t *tasks_per_level,
                        uint64_t *leaves_per_level, int maxlev);

/* Frontier engine over caller-owned device buffers (the level-synchronous multi-GPU schedule of
 * ppls_amd/frontier.py). A frontier is n records {l, r, F(l), F(r)} (4 doubles each, row-major) of
 * one tree depth. aq_frontier_root writes the root record of [a, b] to d_out[0].
 * aq_level_step enqueues one task step (aquadPartA.c:183-202) on every record of d_in: refining
 * records append their two children to d_out (at most cap_out records; the number written lands in
 * the device counter *d_n_out, which the call zeroes first), accepted ones add into the device
 * accumulator d_acc[8] = {area hi, area lo (double-double), tasks, accepted, error bits, deepest
 * level, 0, 0}; the caller zeroes d_acc once per integral. Both calls are asynchronous on the
 * context's stream and never read device memory from the host. */
int aq_frontier_root(aq_ctx *ctx, int integrand, double a, double b, double *d_out);
int aq_level_step(aq_ctx *ctx, int integrand, const double *d_in, uint32_t n_in, double *d_out, uint32_t cap_out,
                  double eps, int depth, int max_depth, uint32_t *d_n_out, double *d_acc);
/* The same step with the input count read on the DEVICE from *d_n_in (a counter a previous step
 * wrote), so levels chain on the stream with no host round trip (ppls_amd/frontier.py syncs only
 * every few levels, or at rebalancing levels). n_in_max bounds *d_n_in (it sizes the grid; blocks
 * past the real count exit at once). *d_n_out is NOT zeroed: the caller zeroes the counters once
 * (one array of per-level counts: level d reads counts[d] and appends to counts[d + 1]). */
int aq_level_step_chained(aq_ctx *ctx, int integrand, const double *d_in, const uint32_t *d_n_in, uint32_t n_in_max,
                          double *d_out, uint32_t cap_out, double eps, int depth, int max_depth, uint32_t *d_n_out,
                          double *d_acc);

/* Deferred folds: while enabled, the level steps leave their per-block partial rows pending and ONE
 * fold adds them into the accumulator later -- at aq_synchronize, at a step with another d_acc, or
 * when disabling (the chained engine's levels between two host looks then cost one launch each, not
 * two). d_acc is complete once aq_synchronize returns. */
int aq_level_defer_fold(aq_ctx *ctx, int enable);
/* `levels` consecutive levels in ONE single-workgroup launch (the narrow top of the tree, where a
 * launch per level is launch- and latency-bound): level depth + k reads d_counts[depth + k] records
 * from d_buf{k & 1} and appends its children to d_buf{(k + 1) & 1} (at most cap records), writing
 * their number to d_counts[depth + k + 1]; the accepted areas and counts add into d_acc as
 * aq_level_step's do. The last level's children are in d_buf{levels & 1}. Asynchronous. */
int aq_level_narrow(aq_ctx *ctx, int integrand, double *d_buf0, double *d_buf1, uint32_t cap, uint32_t *d_counts,
                    int depth, int levels, double eps, int max_depth, double *d_acc);

/* The frontier engine on ONE GPU with its host loop in C (ppls_amd/frontier.py's single-rank path):
 * the root, the narrow top (aq_level_narrow), then chained level steps with deferred folds, the
 * frontier size read every sync_every levels. Frontier buffers of cap records each are context-owned
 * (grown on demand). Fills res and the per-level histograms (arrays of maxlev, or NULL). */
int aq_frontier_integrate(aq_ctx *ctx, const aq_problem *p, uint32_t cap, int sync_every, aq_result *res,
                          uint64_t *tasks_per_level, uint64_t *leaves_per_level, int maxlev);

/* Per-level task / accepted histograms of the last aq_integrate* call (levels 0..maxlev-1). */
int aq_level_histogram(aq_ctx *ctx, uint64_t *tasks_per_level, uint64_t *leaves_per_level, int maxlev);

/* Per-CU task counters of the last call (tasks_per_process[] mapped to compute units).
 * out[AQ_CU_SLOTS] indexed by hardware slot; returns the number of non-zero slots. */
int aq_tasks_per_cu(aq_ctx *ctx, uint64_t *out, int cap);
/* Per-CU task counters of EVERY persistent launch (any shape: lone integrals, batches, shards),
 * summed since the context was created or last reset: each workgroup adds its tasks to its hardware
 * CU slot once at exit. out[AQ_CU_SLOTS] by hardware slot (cap entries written); reset != 0 zeroes
 * the counters after the read. Waits for the context's stream. Returns the number of non-zero slots.
 * Σ out == Σ tasks of the launches since the reset (every task is counted by the CU that ran it). */
int aq_cu_task_counters(aq_ctx *ctx, uint64_t *out, int cap, int reset);

/* Batch front end (SURVEY config 3): n independent integrals [a[i], b[i]] of one integrand.
 * Per-integral area / accepted / tasks (any may be NULL). NOTE the output order: accepted BEFORE
 * tasks (round 1's header had a single `accepted` output; both are uint64_t*, so a caller written
 * against another order compiles and gets the arrays swapped). The integrals run in launches of up
 * to aq_max_integrals_per_launch(); each launch's bounds are validated just before it is enqueued,
 * so a bad bound in a later launch returns AQ_EINVAL after the earlier launches ran: the outputs
 * are then unspecified (not all-or-nothing). Each launch runs its integrals largest-first (a device
 * pre-pass estimates every tree's size; only the order changes, never a result); the host checks,
 * stages and unpacks on up to 8 threads (a pool the context keeps, created by its first batch call).
 * Environment: AQ_BATCH_SORT=0 keeps the input order, AQ_HOST_THREADS=<n> bounds the host threads
 * (read when the pool is created), AQ_BATCH_FIRST / AQ_BATCH_LAST set the first / last launch's size
 * (defaults 131072 / no split), AQ_BATCH_TRACE=1 prints the call's host phase times on stderr. */
int aq_integrate_batch(aq_ctx *ctx, size_t n, const double *a, const double *b, double eps, int integrand,
                       double *area, uint64_t *accepted, uint64_t *tasks);

/* Device evaluation of the integrand / of cosh (libm parity checks). */
int aq_eval_integrand(aq_ctx *ctx, int integrand, size_t n, const double *x, double *out);
int aq_eval_cosh(aq_ctx *ctx, size_t n, const double *x, double *out);

/* ---- measurement ----------------------------------------------------------------------------
 * When enabled, HIP events bracket every launch of the persistent kernel on the context's
 * stream; aq_kernel_time returns the summed milliseconds and launch count since the last reset. */
int aq_kernel_timing(aq_ctx *ctx, int enable);
int aq_kernel_time(aq_ctx *ctx, double *total_ms, uint64_t *launches);
/* Per-workgroup timeline of the persistent kernel (48 uint64 words per workgroup: realtime stamps
 * in 100 MHz ticks -- entry, init, first seed, seeded, last round, first idle, termination seen,
 * loop exit, flushed, fold, exit -- rounds, tasks, chunks and records moved through the HBM queue,
 * seeds, max ring size, CU slot, active lanes summed over rounds, shader-clock cycles per round
 * phase and per seeding phase, records moved through the wave cellars; field names in
 * ppls_amd.Context.DIAG_FIELDS).
 * Runs an instrumented kernel variant. aq_diagnostics returns the number of workgroup records. */
int aq_set_diagnostics(aq_ctx *ctx, int enable);
int aq_diagnostics(aq_ctx *ctx, uint64_t *out, int cap_words);

/* ---- observable surface ----------------------------------------------------------------------
 * aq_print_reference prints exactly main()'s output (:107-117) for a result: "Area=%lf\n\nTasks Per
 * Process\n", then the index row and the count row, each entry followed by a tab. Entry 0 is the
 * farmer (always 0), entries 1..n_gpus the GPUs' tasks (res->tasks_per_gpu; one worker when NULL).
 * aq_print_reference_procs prints the same for any tasks_per_process[nprocs] (e.g. CUs dealt over
 * P-1 worker columns, the CLI's `-n P`). */
void aq_print_reference(FILE *f, const aq_result *res);
void aq_print_reference_procs(FILE *f, double area, const uint64_t *tasks_per_process, int nprocs);

#ifdef __cplusplus
}
#endif
#endif /* AQUAD_H */
