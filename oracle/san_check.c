/*
 * oracle/san_check.c -- TEST INFRASTRUCTURE ONLY (SURVEY §5 "sanitizers"): the CPU restatement
 * (aq_oracle.c, compiled into this one translation unit) driven under AddressSanitizer +
 * UndefinedBehaviorSanitizer by `make san`. It walks the trees tests/test_sanitizers.py names and
 * prints one line per case; the test compares the lines with the golden fixtures (which the
 * reference binary pinned) and fails on any sanitizer report.
 *
 *   san_check tree <integrand 0|1|2> <a> <b> <eps>        -> tasks leaves levels area_quad_hi(%a)
 *   san_check shards <integrand> <a> <b> <eps> <nshards>  -> the summed shard counts (same format)
 *   san_check batch <n> <eps>                             -> Σ tasks, Σ leaves of the splitmix64 batch
 */
#include "aq_oracle.c"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int usage(void)
{
    fprintf(stderr, "usage: san_check tree|shards|batch ...\n");
    return 2;
}

int main(int argc, char **argv)
{
    if (argc < 2) return usage();
    const int maxlev = 64;
    if (!strcmp(argv[1], "tree") && argc == 6) {
        aqo_result r;
        uint64_t tl[64], ll[64];
        int rc = aqo_integrate(atoi(argv[2]), AQO_LIBM_RESTATED_FMA, atof(argv[3]), atof(argv[4]), atof(argv[5]), maxlev, &r, tl, ll);
        if (rc) return 10 + rc;
        uint64_t st = 0, sl = 0;
        for (int i = 0; i < maxlev; i++) { st += tl[i]; sl += ll[i]; }
        if (st != r.tasks || sl != r.leaves) return 3;   /* the per-level histograms sum to the totals */
        printf("%llu %llu %d %a\n", (unsigned long long)r.tasks, (unsigned long long)r.leaves, r.levels, r.area_quad_hi);
        return 0;
    }
    if (!strcmp(argv[1], "shards") && argc == 7) {
        const int n = atoi(argv[6]);
        uint64_t tasks = 0, leaves = 0;
        int levels = 0;
        for (int s = 0; s < n; s++) {
            aqo_result r;
            int rc = aqo_integrate_shard(atoi(argv[2]), AQO_LIBM_RESTATED_FMA, atof(argv[3]), atof(argv[4]), atof(argv[5]), maxlev,
                                         256 * 12, 2, s, n, &r, NULL, NULL);
            if (rc) return 10 + rc;
            tasks += r.tasks;
            leaves += r.leaves;
            if (r.levels > levels) levels = r.levels;
        }
        printf("%llu %llu %d\n", (unsigned long long)tasks, (unsigned long long)leaves, levels);
        return 0;
    }
    if (!strcmp(argv[1], "batch") && argc == 4) {
        const long n = atol(argv[2]);
        double *a = malloc(sizeof(double) * (size_t)n), *b = malloc(sizeof(double) * (size_t)n);
        double *area = malloc(sizeof(double) * (size_t)n);
        uint64_t *t = malloc(sizeof(uint64_t) * (size_t)n), *l = malloc(sizeof(uint64_t) * (size_t)n);
        if (!a || !b || !area || !t || !l) return 4;
        aqo_batch_bounds(n, a, b);
        int rc = aqo_integrate_batch(0, AQO_LIBM_RESTATED_FMA, n, a, b, atof(argv[3]), maxlev, area, t, l);
        if (rc) return 10 + rc;
        uint64_t st = 0, sl = 0;
        for (long i = 0; i < n; i++) { st += t[i]; sl += l[i]; }
        printf("%llu %llu\n", (unsigned long long)st, (unsigned long long)sl);
        free(a); free(b); free(area); free(t); free(l);
        return 0;
    }
    return usage();
}
