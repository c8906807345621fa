/*
 * aquad_cli.c -- drop-in for `mpirun -n P ./aquadPartA` (/root/reference/aquadPartA.c main(), :78-123).
 *
 *   aquad [-n P] [--gpus G] [--eps E] [--a A] [--b B] [--f cosh4|sin_recip] [--per-cu] [--levels]
 *
 * Same observable surface as the reference: `Area=%lf`, a blank line, `Tasks Per Process`, the index
 * row and the count row (tab-terminated entries). Process 0 is the farmer and always reports 0 tasks
 * (:162 only counts dispatches to workers). Processes 1..P-1 are the on-device workers: every CU of
 * every GPU used, dealt round-robin (GPU-major, CU slot order) over the P-1 columns; P defaults to
 * 1 + G, i.e. one column per GPU. `--per-cu` prints one column per CU. P < 2 reproduces the
 * reference's error exactly (:86-90). Defaults are the reference's macros (:45-48).
 * With G > 1 the run is sharded: one host thread drives every GPU (aq_integrate_async on each, then
 * aq_fetch) and sums the per-GPU partial results.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "aquad.h"

static void usage(void) {
    fprintf(stderr,
            "usage: aquad [-n P] [--gpus G] [--eps E] [--a A] [--b B] [--f cosh4|sin_recip] [--per-cu] [--levels]\n");
}

int main(int argc, char **argv) {
    aq_problem p = {AQ_F_COSH4, 0, 0.0, 5.0, 1e-3}; /* aquadPartA.c:45-48 */
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
    aq_result *part = calloc((size_t)gpus, sizeof(*part));
    uint64_t *cu = calloc((size_t)gpus * AQ_CU_SLOTS, sizeof(uint64_t));
    int rc = AQ_OK;
    for (int g = 0; g < gpus && rc == AQ_OK; ++g) rc = aq_ctx_create(g, &ctx[g]);
    for (int g = 0; g < gpus && rc == AQ_OK; ++g) rc = aq_integrate_async(ctx[g], &p, g, gpus, 0);
    for (int g = 0; g < gpus && rc == AQ_OK; ++g) {
        rc = aq_fetch(ctx[g], 0, &part[g]);
        if (rc == AQ_OK) aq_tasks_per_cu(ctx[g], cu + (size_t)g * AQ_CU_SLOTS, AQ_CU_SLOTS);
    }
    if (rc != AQ_OK) {
        fprintf(stderr, "aquad: %s\n", aq_strerror(rc));
        return 1;
    }
    double area = 0.0;
    uint64_t tasks = 0, accepted = 0;
    uint32_t lv = 0;
    int ncu = 0;
    for (int g = 0; g < gpus; ++g) {
        area += part[g].area;
        tasks += part[g].tasks;
        accepted += part[g].accepted;
        if (part[g].levels > lv) lv = part[g].levels;
        for (int s = 0; s < AQ_CU_SLOTS; ++s) ncu += cu[(size_t)g * AQ_CU_SLOTS + s] ? 1 : 0;
    }
    if (per_cu) nprocs = 1 + ncu;
    uint64_t *tpp = calloc((size_t)nprocs, sizeof(uint64_t));
    if (!per_cu && nprocs - 1 == gpus) {
        for (int g = 0; g < gpus; ++g) tpp[1 + g] = part[g].tasks;
    } else {
        int k = 0;
        for (int g = 0; g < gpus; ++g)
            for (int s = 0; s < AQ_CU_SLOTS; ++s) {
                uint64_t v = cu[(size_t)g * AQ_CU_SLOTS + s];
                if (v) { tpp[1 + (k % (nprocs - 1))] += v; ++k; }
            }
    }
    aq_print_reference(stdout, area, tpp, nprocs);
    if (levels) {
        uint64_t t[AQ_MAX_LEVELS], l[AQ_MAX_LEVELS];
        uint64_t ts[AQ_MAX_LEVELS] = {0}, ls[AQ_MAX_LEVELS] = {0};
        for (int g = 0; g < gpus; ++g) {
            aq_level_histogram(ctx[g], t, l, AQ_MAX_LEVELS);
            for (int d = 0; d < AQ_MAX_LEVELS; ++d) { ts[d] += t[d]; ls[d] += l[d]; }
        }
        fprintf(stdout, "\nLevel\tTasks\tAccepted\n");
        for (uint32_t d = 0; d < lv; ++d)
            fprintf(stdout, "%u\t%llu\t%llu\n", d, (unsigned long long)ts[d], (unsigned long long)ls[d]);
        fprintf(stdout, "Total\t%llu\t%llu\n", (unsigned long long)tasks, (unsigned long long)accepted);
    }
    for (int g = 0; g < gpus; ++g) aq_ctx_destroy(ctx[g]);
    free(tpp);
    free(cu);
    free(part);
    free(ctx);
    return 0;
}
