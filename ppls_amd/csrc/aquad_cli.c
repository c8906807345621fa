/*
 * aquad_cli.c -- drop-in for `mpirun -n P ./aquadPartA` (/root/reference/aquadPartA.c main(), :78-123).
 *
 *   aquad [-n P] [--gpus G] [--eps E] [--a A] [--b B] [--f cosh4|sin_recip|user] [--per-cu] [--levels]
 *
 * Same observable surface as the reference: `Area=%lf`, a blank line, `Tasks Per Process`, the index
 * row and the count row (tab-terminated entries). Process 0 is the farmer and always reports 0 tasks
 * (:162 only counts dispatches to workers). Processes 1..P-1 are the on-device workers: every CU of
 * every GPU used, dealt round-robin (GPU-major, CU slot order) over the P-1 columns; P defaults to
 * 1 + G, i.e. one column per GPU. `--per-cu` prints one column per CU. P < 2 reproduces the
 * reference's error exactly (:86-90). Defaults are the reference's macros (:45-48).
 * With G > 1 the run is sharded over an RCCL group (aq_group_create: one host thread drives every
 * GPU; aq_integrate_group combines the shards with one grouped all-reduce / all-gather).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "aquad.h"

static void usage(void) {
    fprintf(stderr,
            "usage: aquad [-n P] [--gpus G] [--eps E] [--a A] [--b B] [--f cosh4|sin_recip|user] [--per-cu] "
            "[--levels]\n");
}

int main(int argc, char **argv) {
    aq_problem p = {AQ_F_COSH4, 0, 0.0, 5.0, 1e-3, 0, 0}; /* aquadPartA.c:45-48 */
    int nprocs = -1, gpus = 1, per_cu = 0, levels = 0;
    for (int i = 1; i < argc; ++i) {
        const char *a = argv[i];
        const char *v = (i + 1 < argc) ? argv[i + 1] : NULL;
        if ((!strcmp(a, "-n") || !strcmp(a, "-c") || !strcmp(a, "-np")) && v) { nprocs = atoi(v); ++i; }
        else if (!strcmp(a, "--gpus") && v) { gpus = atoi(v); ++i; }
        else if (!strcmp(a, "--eps") && v) { p.eps = atof(v); ++i; }
        else if (!strcmp(a, "--a") && v) { p.a = atof(v); ++i; }
        else if (!strcmp(a, "--b") && v) { p.b = atof(v); ++i; }
        else if (!strcmp(a, "--f") && v) {
            if (!strcmp(v, "cosh4")) p.integrand = AQ_F_COSH4;
            else if (!strcmp(v, "sin_recip")) p.integrand = AQ_F_SIN_RECIP;
            else if (!strcmp(v, "user")) p.integrand = AQ_F_USER;
            else { usage(); return 2; }
            ++i;
        } else if (!strcmp(a, "--per-cu")) per_cu = 1;
        else if (!strcmp(a, "--levels")) levels = 1;
        else { usage(); return 2; }
    }
    if (nprocs == -1) nprocs = 1 + gpus;
    if (nprocs < 2) { /* aquadPartA.c:86-90 */
        fprintf(stderr, "ERROR: Must have at least 2 processes to run\n");
        exit(1);
    }
    int ndev = 0;
    if (aq_device_count(&ndev) != AQ_OK || gpus < 1 || gpus > ndev) {
        fprintf(stderr, "aquad: need %d GPU(s), found %d\n", gpus, ndev);
        return 1;
    }
    aq_ctx **ctx = calloc((size_t)gpus, sizeof(*ctx));
    aq_group *grp = NULL;
    int rc = AQ_OK;
    for (int g = 0; g < gpus && rc == AQ_OK; ++g) rc = aq_ctx_create(g, &ctx[g]);
    const int ncu = rc == AQ_OK ? aq_ctx_num_cus(ctx[0]) : 0;
    uint64_t *per_gpu = calloc((size_t)gpus, sizeof(uint64_t));
    uint64_t *cu = calloc((size_t)gpus * (size_t)(ncu > 0 ? ncu : 1), sizeof(uint64_t));
    aq_result res;
    memset(&res, 0, sizeof(res));
    res.tasks_per_gpu = per_gpu;
    res.tasks_per_cu = cu;
    if (rc == AQ_OK) {
        if (gpus == 1) {
            rc = aq_integrate(ctx[0], &p, &res);
        } else {
            p.n_gpus = gpus;
            rc = aq_group_create(ctx, gpus, &grp);
            if (rc == AQ_OK) rc = aq_integrate_group(grp, &p, &res);
        }
    }
    if (rc != AQ_OK) {
        fprintf(stderr, "aquad: %s\n", aq_strerror(rc));
        return 1;
    }
    if (!per_cu && nprocs - 1 == gpus) {
        aq_print_reference(stdout, &res);
    } else {
        int cols = per_cu ? 0 : nprocs - 1;
        if (per_cu)
            for (int k = 0; k < gpus * ncu; ++k) cols += cu[k] ? 1 : 0;
        uint64_t *tpp = calloc((size_t)cols + 1, sizeof(uint64_t));
        int k = 0;
        for (int c = 0; c < gpus * ncu; ++c)
            if (cu[c]) { tpp[1 + (k % cols)] += cu[c]; ++k; }
        aq_print_reference_procs(stdout, res.area, tpp, cols + 1);
        free(tpp);
    }
    if (levels) {
        uint64_t t[AQ_MAX_LEVELS], l[AQ_MAX_LEVELS];
        aq_level_histogram(ctx[0], t, l, AQ_MAX_LEVELS);
        fprintf(stdout, "\nLevel\tTasks\tAccepted\n");
        for (uint32_t d = 0; d < res.levels; ++d)
            fprintf(stdout, "%u\t%llu\t%llu\n", d, (unsigned long long)t[d], (unsigned long long)l[d]);
        fprintf(stdout, "Total\t%llu\t%llu\n", (unsigned long long)res.tasks, (unsigned long long)res.accepted);
    }
    aq_group_destroy(grp);
    for (int g = 0; g < gpus; ++g) aq_ctx_destroy(ctx[g]);
    free(cu);
    free(per_gpu);
    free(ctx);
    return 0;
}
