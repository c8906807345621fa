/*
 * aquad.h -- C ABI of the MI355X-native adaptive-quadrature engine (libaquad.so).
 *
 * The reference (/root/reference/aquadPartA.c) has no plugin or FFI layer: its boundary is
 * the macro quartet F/A/B/EPSILON (:45-48) plus the farmer/worker message protocol
 * (farmer() :125-173, worker() :175-208) that main() (:78-123) drives. Each entry point below
 * names the reference interface it replaces. Plain C types only: no HIP or torch types cross
 * this boundary; every host buffer is caller-owned; device memory, streams and events are owned
 * by an opaque aq_ctx (one per GPU, not re-entrant, blocking unless the name says _async).
 * Errors: 0 on success, a negative AQ_E* code otherwise (the reference's only error is
 * numprocs < 2 -> stderr + exit(1), :86-90; the CLI maps codes to that behaviour).
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
#define AQ_EINVAL (-1)     /* bad argument (non-finite bounds, b < a, eps < 0, bad shard) */
#define AQ_EHIP (-2)       /* a HIP runtime call failed */
#define AQ_ETIMEOUT (-3)   /* an on-device wait exceeded its bound (never expected) */
#define AQ_EOVERFLOW (-4)  /* a frontier / work-queue capacity was exceeded */
#define AQ_EDEPTH (-5)     /* refinement reached max_depth (the reference would not terminate) */
#define AQ_ENOMEM (-6)     /* device or host allocation failed */
#define AQ_ENODEV (-7)     /* no HIP device */

#define AQ_DEFAULT_MAX_DEPTH 96
#define AQ_MAX_LEVELS 128     /* length of the per-level histograms */
#define AQ_CU_SLOTS 2048      /* per-CU counter slots: xcc*256 + (se*2+sh)*16 + cu */

/* Integrand = the reference's F(arg) macro (aquadPartA.c:46) as a compile-time kernel variant. */
typedef enum {
    AQ_F_COSH4 = 0,     /* cosh(x)*cosh(x)*cosh(x)*cosh(x), glibc-2.35-exact cosh (the reference) */
    AQ_F_SIN_RECIP = 1  /* sin(1/x) (SURVEY config 4) */
} aq_integrand;

/* Replaces the compile-time macros EPSILON / F / A / B (aquadPartA.c:45-48). */
typedef struct {
    int32_t integrand;  /* aq_integrand */
    int32_t max_depth;  /* refinement cap; 0 -> AQ_DEFAULT_MAX_DEPTH (<= AQ_MAX_LEVELS - 1) */
    double a;           /* A (:47) */
    double b;           /* B (:48) */
    double eps;         /* EPSILON (:45): absolute, strict '>' test (:191) */
} aq_problem;

/* Replaces farmer()'s return value and the global tasks_per_process[] (:72, :101, :162). */
typedef struct {
    double area;        /* Σ accepted larea+rarea (:199 sent, :149 summed) */
    uint64_t tasks;     /* intervals evaluated = Σ tasks_per_process (:162) */
    uint64_t accepted;  /* accepted subintervals (tag-1 area messages, :201) */
    uint32_t levels;    /* 1 + deepest refinement level reached */
    uint32_t n_cu;      /* CUs that evaluated at least one task (aq_tasks_per_cu) */
    uint64_t spilled;   /* interval records moved through the HBM work queue (load balance) */
} aq_result;

typedef struct aq_ctx aq_ctx;

/* ---- lifecycle (replaces MPI_Init / MPI_Comm_size / MPI_Finalize, :82-84, :121) ------------- */
int aq_device_count(int *count);
int aq_ctx_create(int device, aq_ctx **out);
void aq_ctx_destroy(aq_ctx *ctx);
const char *aq_strerror(int code);
/* Compute units of the context's device (one persistent workgroup each). */
int aq_ctx_num_cus(const aq_ctx *ctx);
/* Wavefront workers of the on-device farmer (workgroups x waves per workgroup): one integral
 * launched alone is split into this many shares (the partition aq_integrate_shard documents). */
int aq_ctx_num_workers(const aq_ctx *ctx);
/* Per-level task/accepted histograms on the persistent path (default on; a diagnostic the
 * reference does not produce -- pipelined callers switch it off). */
int aq_set_level_histograms(aq_ctx *ctx, int enable);
/* Which persistent kernel runs a launch (no reference counterpart: the reference has one schedule,
 * the MPI bag). AUTO: the lane-DFS kernel for launches of >= 16 integrals, the streaming pair kernel
 * (HBM work queue between CUs) below that. Counts and areas are identical under every engine; the
 * engine only changes the schedule (and aq_ctx_num_workers, the share count of a lone integral).
 * The AQ_ENGINE environment variable ("stream" / "dfs") sets the default of new contexts. */
#define AQ_ENGINE_AUTO 0
#define AQ_ENGINE_STREAM 1
#define AQ_ENGINE_DFS 2
int aq_set_engine(aq_ctx *ctx, int engine);

/* ---- the hot path ----------------------------------------------------------------------------
 * aq_integrate: farmer(numprocs) + every worker() of one run (:125-208) as ONE persistent HIP
 * launch: workgroups expand interval frontiers in LDS (task body :183-202), accumulate accepted
 * areas, and rebalance through an HBM work queue (the bag of tasks, :152-165).
 * Bit-identical interval tree: `tasks` and `accepted` equal the reference's counts exactly.
 */
int aq_integrate(aq_ctx *ctx, const aq_problem *p, aq_result *res);

/* This process's share of a multi-GPU run: the depth-D positions (D = ceil(log2(V)) + 2) are
 * dealt in snake order over V = nshards * aq_ctx_num_workers() virtual workers; shard `shard`
 * evaluates its positions' subtrees plus the tasks at depth <= D it owns (each counted by the
 * owner of its leftmost descendant position, so by exactly one shard). Summing
 * area/tasks/accepted over all shards (the caller's all-reduce) gives exactly the single-GPU
 * result. */
int aq_integrate_shard(aq_ctx *ctx, const aq_problem *p, int shard, int nshards, aq_result *res);

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
int aq_fetch(aq_ctx *ctx, int slot, aq_result *res);
int aq_synchronize(aq_ctx *ctx);
/* Enqueue (on the context's stream) a copy of n consecutive slots' totals, starting at first_slot
 * (mod aq_async_slots()), into the DEVICE buffer d_out as n rows of 4 doubles
 * {area, tasks, accepted, error bits}: the input of one all-reduce for n pipelined integrals. */
int aq_gather_results(aq_ctx *ctx, int first_slot, int n, void *d_out);

/* Level-synchronous breadth-first path (one kernel per tree level, host loop): the debug /
 * cross-check schedule. Fills per-level histograms (caller arrays of length maxlev or NULL). */
int aq_integrate_levels(aq_ctx *ctx, const aq_problem *p, aq_result *res, uint64_t *tasks_per_level,
                        uint64_t *leaves_per_level, int maxlev);

/* Frontier engine over caller-owned device buffers (the multi-GPU rebalanced schedule of
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

/* Per-level task / accepted histograms of the last aq_integrate* call (levels 0..maxlev-1). */
int aq_level_histogram(aq_ctx *ctx, uint64_t *tasks_per_level, uint64_t *leaves_per_level, int maxlev);

/* Per-CU task counters of the last call (tasks_per_process[] mapped to compute units).
 * out[AQ_CU_SLOTS] indexed by hardware slot; returns the number of non-zero slots. */
int aq_tasks_per_cu(aq_ctx *ctx, uint64_t *out, int cap);

/* Batch front end (SURVEY config 3): n independent integrals [a[i], b[i]] of one integrand.
 * Per-integral area / tasks / accepted (any may be NULL). */
int aq_integrate_batch(aq_ctx *ctx, int integrand, size_t n, const double *a, const double *b, double eps,
                       double *area, uint64_t *tasks, uint64_t *accepted);

/* Device evaluation of the integrand / of cosh (libm parity checks). */
int aq_eval_integrand(aq_ctx *ctx, int integrand, size_t n, const double *x, double *out);
int aq_eval_cosh(aq_ctx *ctx, size_t n, const double *x, double *out);

/* ---- measurement ----------------------------------------------------------------------------
 * When enabled, HIP events bracket every launch of the persistent kernel on the context's
 * stream; aq_kernel_time returns the summed milliseconds and launch count since the last reset. */
int aq_kernel_timing(aq_ctx *ctx, int enable);
int aq_kernel_time(aq_ctx *ctx, double *total_ms, uint64_t *launches);
/* Per-workgroup timeline of the persistent kernel (40 uint64 words per workgroup: realtime stamps
 * at entry / seeded / first idle / exit in 100 MHz ticks, rounds, tasks, chunks and records moved
 * through the HBM queue, produce/idle ticks, seeds, max stack depth, CU slot, records received,
 * active lanes summed over rounds, shader-clock cycles per round phase and for seeding, then
 * records moved through the workgroup's HBM cellar).
 * Runs an instrumented kernel variant. aq_diagnostics returns the number of workgroup records. */
int aq_set_diagnostics(aq_ctx *ctx, int enable);
int aq_diagnostics(aq_ctx *ctx, uint64_t *out, int cap_words);

/* ---- observable surface ----------------------------------------------------------------------
 * Prints exactly main()'s output (:107-117): "Area=%lf\n\nTasks Per Process\n", then the index
 * row and the count row, each entry followed by a tab. Entry 0 is the farmer (always 0). */
void aq_print_reference(FILE *f, double area, const uint64_t *tasks_per_process, int nprocs);

#ifdef __cplusplus
}
#endif
#endif /* AQUAD_H */
