/*
 * oracle/aq_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity oracle).
 *
 * This file is the CPU restatement of the reference's hot path. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as
 * the checker or the timed CPU baseline. The product (ppls_amd/, include/) never links it.
 *
 * What it restates (all citations into /root/reference/aquadPartA.c):
 *   - the integrand macro  F(arg) cosh(arg)*cosh(arg)*cosh(arg)*cosh(arg)      :46
 *   - the worker task body (trapezoid on [l,r] and both halves, strict '>')   :183-202
 *   - the farmer's accumulation result += area and LIFO bag order            :149, :152-159
 *   - task counting (one task per interval dispatched)                       :162
 * and, because the hot path's transcendental lives in a third-party dependency that is
 * NOT under /root/reference, glibc 2.35 libm (Ubuntu 2.35-0ubuntu3.11):
 *   - __ieee754_cosh   (sysdeps/ieee754/dbl-64/e_cosh.c, fdlibm formula)
 *   - __exp            (sysdeps/ieee754/dbl-64/e_exp.c, N=128 table; FMA and non-FMA ifunc forms)
 *   - __expm1          (sysdeps/ieee754/dbl-64/s_expm1.c, k=0 path, Estrin polynomial)
 *   - __sin            (sysdeps/ieee754/dbl-64/s_sin.c, |x| < 105414350; FMA and non-FMA forms) for
 *                      the config-4 F macro sin(1.0/(arg))
 * Pinning: tests/test_oracle.py checks these bit for bit against the host libm and the
 * whole tree walk against the reference's header known answer (aquadPartA.c:31-36) and
 * against fixtures produced by the compiled reference (oracle/Makefile -> oracle/_ref/).
 *
 * Build: oracle/Makefile -> oracle/_build/liboracle.so (gcc -O2 -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <quadmath.h>

#include "glibc_exp_table.h"

#define AQO_OK 0
#define AQO_EINVAL (-1)
#define AQO_EDEPTH (-5)
#define AQO_ENOMEM (-6)

/* integrand ids: same numbering as include/aquad.h */
#define AQO_F_COSH4 0     /* aquadPartA.c:46 */
#define AQO_F_SIN_RECIP 1 /* sin(1/x): the SURVEY config-4 variant of the F macro */
#define AQO_F_USER 2      /* exp(-(arg)*(arg)): the library's default AQ_F_USER plug-in (the macro at :46 replaced) */

static inline uint64_t asu(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double asd(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

/* ---- glibc 2.35 exp, e_exp.c main path (valid for |x| in [2^-54, 709.78]) -------------- */
static const double InvLn2N = 0x1.71547652b82fep7;
static const double Shift = 0x1.8p52;
static const double NegLn2hiN = -0x1.62e42fefa0000p-8;
static const double NegLn2loN = -0x1.cf79abc9e3b3ap-47;
static const double C2 = 0x1.ffffffffffdbdp-2;
static const double C3 = 0x1.555555555543cp-3;
static const double C4 = 0x1.55555cf172b91p-5;
static const double C5 = 0x1.1111167a4d017p-7;

/*
 * Both ifunc forms of glibc's __exp (e_exp.c), every path: |x| < 2^-54 -> 1 + x; |x| >= 1024 ->
 * 0 / inf / nan; otherwise the N=128 table evaluation, with specialcase() for |x| >= 512 (k > 0:
 * overflow-safe scaling; k < 0: the subnormal range with its hi/lo re-rounding). The FMA form
 * (__exp_fma, what x86_64 hosts with FMA select) is GCC's contraction of the same source:
 * z+Shift, r, tmp, scale+scale*tmp and scale-y+scale*tmp fuse; this file itself builds with
 * -ffp-contract=off, so the non-FMA form below is the source as written.
 */
static double exp_any(double x, int fma_variant)
{
    uint32_t abstop = (uint32_t)(asu(x) >> 52) & 0x7ff;
    int special = 0;
    if (abstop - 0x3c9u >= 0x408u - 0x3c9u) {
        if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + x;       /* tiny */
        if (abstop >= 0x409) {                                     /* |x| >= 1024 */
            if (asu(x) == asu(-INFINITY)) return 0.0;
            if (abstop >= 0x7ff) return 1.0 + x;
            return (asu(x) >> 63) ? 0.0 : INFINITY;
        }
        special = 1;
    }
    double kd, r;
    if (fma_variant) {
        kd = fma(InvLn2N, x, Shift);
    } else {
        double z = InvLn2N * x;
        kd = z + Shift;
    }
    uint64_t ki = asu(kd);
    kd -= Shift;
    if (fma_variant) r = fma(kd, NegLn2loN, fma(kd, NegLn2hiN, x));
    else r = x + kd * NegLn2hiN + kd * NegLn2loN;
    uint64_t idx = 2 * (ki % 128);
    uint64_t top = ki << 45;
    double tail = asd(aqo_exp_tab[idx]);
    uint64_t sbits = aqo_exp_tab[idx + 1] + top;
    double r2 = r * r;
    double tmp;
    if (fma_variant) tmp = fma(r2 * r2, fma(r, C5, C4), fma(r2, fma(r, C3, C2), tail + r));
    else tmp = tail + r + r2 * (C2 + r * C3) + r2 * r2 * (C4 + r * C5);
    if (special) {
        if ((ki & 0x80000000ull) == 0) {                           /* k > 0 */
            sbits -= 1009ull << 52;
            double scale = asd(sbits);
            return 0x1p1009 * (fma_variant ? fma(scale, tmp, scale) : scale + scale * tmp);
        }
        /* k < 0: GCC leaves this branch unfused in the FMA form too (measured against the host
           libm: fusing either line gives 28 / 254 mismatches in 2 M points, unfused 0) */
        sbits += 1022ull << 52;
        double scale = asd(sbits);
        double y = scale + scale * tmp;
        if (y < 1.0) {
            double lo = scale - y + scale * tmp;
            double hi = 1.0 + y;
            lo = 1.0 - hi + y + lo;
            y = (hi + lo) - 1.0;
            if (y == 0.0) y = 0.0;
        }
        return 0x1p-1022 * y;
    }
    double scale = asd(sbits);
    return fma_variant ? fma(scale, tmp, scale) : scale + scale * tmp;
}

double aqo_exp_fma(double x) { return exp_any(x, 1); }
double aqo_exp_nofma(double x) { return exp_any(x, 0); }

/* ---- glibc 2.35 expm1, s_expm1.c, the |x| < 0.5*ln2 (k = 0) path ----------------------- */
static const double Q1 = -3.33333333333331316428e-02;
static const double Q2 = 1.58730158725481460165e-03;
static const double Q3 = -7.93650757867487942473e-05;
static const double Q4 = 4.00821782732936239552e-06;
static const double Q5 = -2.01099218183624371326e-07;

double aqo_expm1_small(double x)
{
    uint32_t hx = (uint32_t)(asu(x) >> 32) & 0x7fffffff;
    if (hx < 0x3c900000) return x; /* |x| < 2^-54 */
    double hfx = 0.5 * x;
    double hxs = x * hfx;
    double R1 = 1.0 + hxs * Q1;
    double h2 = hxs * hxs;
    double R2 = Q2 + hxs * Q3;
    double h4 = h2 * h2;
    double R3 = Q4 + hxs * Q5;
    double r1 = R1 + h2 * R2 + h4 * R3;
    double t = 3.0 - r1 * hfx;
    double e = hxs * ((r1 - t) / (6.0 - x * t));
    return x - (x * e - hxs);
}

/* ---- glibc 2.35 __ieee754_cosh (e_cosh.c) ----------------------------------------------- */
double aqo_cosh(double x, int fma_variant)
{
    uint32_t ix = (uint32_t)(asu(x) >> 32) & 0x7fffffff;
    double ax = fabs(x);
    if (ix < 0x40360000) { /* |x| < 22 */
        if (ix < 0x3fd62e43) { /* |x| < 0.5*ln2 */
            if (ix < 0x3c800000) return 1.0;
            double t = aqo_expm1_small(ax);
            double w = 1.0 + t;
            return 1.0 + (t * t) / (w + w);
        }
        double t = fma_variant ? aqo_exp_fma(ax) : aqo_exp_nofma(ax);
        return 0.5 * t + 0.5 / t;
    }
    if (ix >= 0x7ff00000) return x * x; /* inf / nan */
    if (ix < 0x40862e42) return 0.5 * (fma_variant ? aqo_exp_fma(ax) : aqo_exp_nofma(ax));
    /* |x| in [log(maxdouble), overflowthreshold] */
    if (ax <= 0x1.633ce8fb9f87dp+9) {
        double w = fma_variant ? aqo_exp_fma(0.5 * ax) : aqo_exp_nofma(0.5 * ax);
        double t = 0.5 * w;
        return t * w;
    }
    return INFINITY;
}

/* ---- glibc 2.35 __sin (s_sin.c, IBM Accurate Mathematical Library), |x| < 105414350 -------
 * The config-4 F macro is sin(1.0/(arg)). Both ifunc forms: the FMA one (__sin_fma, what x86_64
 * hosts with FMA select) is GCC's contraction of the same source -- every a*b+c of the Taylor and
 * table-correction polynomials, of the cor sums and of the Cody-Waite reduction fuses, and of the
 * two-product sums it fuses the left product (p*a - 0.5*da, x*dx + xx*(...)); MAC below spells that
 * out (this file builds with -ffp-contract=off). tests/test_oracle.py pins the FMA form to the host
 * libm. Beyond 105414350 glibc reduces with __branred (Payne-Hanek), not restated here: the host
 * sin answers there. */
#include "glibc_sincos_table.h"
static const double Ss1 = -0x1.5555555555555p-3, Ss2 = 0.0083333333333323288, Ss3 = -1.9841269834414642e-04,
                    Ss4 = 2.755729806860771e-06, Ss5 = -2.5022014848318398e-08;
static const double Sn3 = -1.66666666666664880952546298448555E-01, Sn5 = 8.33333214285722277379541354343671E-03,
                    Cs2 = 4.99999999999999999999950396842453E-01, Cs4 = -4.16666666666664434524222570944589E-02,
                    Cs6 = 1.38888874007937613028114285595617E-03;
static const double SBig = 0x1.8p45, SHp0 = 0x1.921FB54442D18p0, SHp1 = 0x1.1A62633145C07p-54,
                    SMp1 = 0x1.921FB58p0, SMp2 = -0x1.DDE973Cp-27, SPp3 = -0x1.CB3B398p-55,
                    SPp4 = -0x1.d747f23e32ed7p-83, SHpinv = 0x1.45F306DC9C883p-1, SToint = 0x1.8p52;
#define MAC(fv, a, b, c) ((fv) ? fma((a), (b), (c)) : (a) * (b) + (c))

static double aqo_sin_do_cos(double x, double dx, int fv)
{
    if (x < 0) dx = -dx;
    double u = SBig + fabs(x);
    x = fabs(x) - (u - SBig) + dx;
    double xx = x * x;
    double s = MAC(fv, x * xx, MAC(fv, xx, Sn5, Sn3), x);
    double c = xx * MAC(fv, xx, MAC(fv, xx, Cs6, Cs4), Cs2);
    int k = (int)(uint32_t)asu(u) << 2;
    double sn = aqo_sincos_tab[k], ssn = aqo_sincos_tab[k + 1], cs = aqo_sincos_tab[k + 2], ccs = aqo_sincos_tab[k + 3];
    double cor = MAC(fv, -sn, s, MAC(fv, -cs, c, MAC(fv, -s, ssn, ccs)));
    return cs + cor;
}

static double aqo_sin_do_sin(double x, double dx, int fv)
{
    double xold = x;
    if (fabs(x) < 0.126) {          /* TAYLOR_SIN (x*x, x, dx) */
        double xx = x * x;
        double p = MAC(fv, MAC(fv, MAC(fv, MAC(fv, Ss5, xx, Ss4), xx, Ss3), xx, Ss2), xx, Ss1);
        double t = MAC(fv, MAC(fv, p, x, -0.5 * dx), xx, dx);
        return x + t;
    }
    if (x <= 0) dx = -dx;
    double u = SBig + fabs(x);
    x = fabs(x) - (u - SBig);
    double xx = x * x;
    double s = x + MAC(fv, x * xx, MAC(fv, xx, Sn5, Sn3), dx);
    double c = MAC(fv, x, dx, xx * MAC(fv, xx, MAC(fv, xx, Cs6, Cs4), Cs2));
    int k = (int)(uint32_t)asu(u) << 2;
    double sn = aqo_sincos_tab[k], ssn = aqo_sincos_tab[k + 1], cs = aqo_sincos_tab[k + 2], ccs = aqo_sincos_tab[k + 3];
    double cor = MAC(fv, cs, s, MAC(fv, -sn, c, MAC(fv, s, ccs, ssn)));
    return copysign(sn + cor, xold);
}

double aqo_sin(double x, int fma_variant)
{
    uint32_t k = (uint32_t)(asu(x) >> 32) & 0x7fffffff;
    if (k < 0x3e500000) return x;                                   /* |x| < 2^-26 */
    if (k < 0x3feb6000) return aqo_sin_do_sin(x, 0.0, fma_variant);  /* |x| < 0.855469 */
    if (k < 0x400368fd) {                                           /* |x| < 2.426265 */
        double t = SHp0 - fabs(x);
        return copysign(aqo_sin_do_cos(t, SHp1, fma_variant), x);
    }
    if (k < 0x419921FB) {                                           /* |x| < 105414350 */
        double t = MAC(fma_variant, x, SHpinv, SToint);
        double xn = t - SToint;
        double y = MAC(fma_variant, -xn, SMp2, MAC(fma_variant, -xn, SMp1, x));
        int n = (int)((uint32_t)asu(t) & 3);
        double t1 = xn * SPp3, t2 = y - t1, db = (y - t2) - t1;
        t1 = xn * SPp4;
        double b = t2 - t1;
        db += (t2 - b) - t1;
        double r = (n & 1) ? aqo_sin_do_cos(b, db, fma_variant) : aqo_sin_do_sin(b, db, fma_variant);
        return (n & 2) ? -r : r;
    }
    return sin(x);                                                  /* __branred range, inf, nan */
}
#undef MAC

/* libm modes for F: restated glibc (FMA / non-FMA ifunc forms) or the host libm itself. */
#define AQO_LIBM_RESTATED_FMA 0
#define AQO_LIBM_RESTATED_NOFMA 1
#define AQO_LIBM_HOST 2

void aqo_sin_array(int mode, long n, const double *x, double *out)
{
    for (long i = 0; i < n; i++) out[i] = mode == AQO_LIBM_HOST ? sin(x[i]) : aqo_sin(x[i], mode == AQO_LIBM_RESTATED_FMA);
}

/* F(arg) exactly as the reference macro expands: cosh(a)*cosh(a)*cosh(a)*cosh(a), left to right. */
static inline double F_eval(int integrand, int mode, double x)
{
    if (integrand == AQO_F_SIN_RECIP)
        return mode == AQO_LIBM_HOST ? sin(1.0 / x) : aqo_sin(1.0 / x, mode == AQO_LIBM_RESTATED_FMA);
    if (integrand == AQO_F_USER) {
        double y = -x * x;                  /* the macro expands to -(arg)*(arg) = (-x)*x */
        if (mode == AQO_LIBM_HOST) return exp(y);
        return mode == AQO_LIBM_RESTATED_FMA ? aqo_exp_fma(y) : aqo_exp_nofma(y);
    }
    double c;
    if (mode == AQO_LIBM_HOST) c = cosh(x);
    else c = aqo_cosh(x, mode == AQO_LIBM_RESTATED_FMA);
    return c * c * c * c;
}

double aqo_F(int integrand, int mode, double x) { return F_eval(integrand, mode, x); }

/* F over an array (the frontier level step's restatement, pyoracle.level_step). */
void aqo_F_array(int integrand, int mode, long n, const double *x, double *out)
{
    for (long i = 0; i < n; i++) out[i] = F_eval(integrand, mode, x[i]);
}

void aqo_cosh_array(int mode, long n, const double *x, double *out)
{
    for (long i = 0; i < n; i++) {
        if (mode == AQO_LIBM_HOST) out[i] = cosh(x[i]);
        else out[i] = aqo_cosh(x[i], mode == AQO_LIBM_RESTATED_FMA);
    }
}

void aqo_exp_array(int mode, long n, const double *x, double *out)
{
    for (long i = 0; i < n; i++) {
        if (mode == AQO_LIBM_HOST) out[i] = exp(x[i]);
        else out[i] = mode == AQO_LIBM_RESTATED_FMA ? aqo_exp_fma(x[i]) : aqo_exp_nofma(x[i]);
    }
}

void aqo_expm1_array(int mode, long n, const double *x, double *out)
{
    for (long i = 0; i < n; i++) out[i] = mode == AQO_LIBM_HOST ? expm1(x[i]) : aqo_expm1_small(x[i]);
}

/* ---- the tree walk --------------------------------------------------------------------- */
typedef struct {
    double area_lifo;     /* Σ leaf areas in the reference's P=2 arrival order (LIFO, :149) */
    double area_quad_hi;  /* exact-ish Σ leaf areas accumulated in __float128, hi part      */
    double area_quad_lo;  /*                                                   lo part      */
    uint64_t tasks;       /* intervals evaluated (= Σ tasks_per_process, :162)              */
    uint64_t leaves;      /* accepted intervals (messages with tag 1 carrying an area, :201) */
    int32_t levels;       /* 1 + deepest depth reached                                       */
    int32_t pad;
} aqo_result;

typedef struct { double l, r, fl, fr; int32_t depth; } rec_t;

typedef struct {
    double area;
    __float128 q;
    int rc;
} acc_t;

static int push_rec(rec_t **st, size_t *n, size_t *cap, rec_t r)
{
    if (*n + 1 > *cap) {
        size_t nc = *cap * 2;
        rec_t *ns = (rec_t *)realloc(*st, nc * sizeof(rec_t));
        if (!ns) return AQO_ENOMEM;
        *st = ns;
        *cap = nc;
    }
    (*st)[(*n)++] = r;
    return AQO_OK;
}

/*
 * Depth-first walk of the subtree rooted at `root`, in exactly the reference's LIFO bag order
 * (aquadPartA.c:152-159: children pushed [l,mid] then [mid,r], so [mid,r] pops first). With one
 * worker (mpirun -n 2) the reference's arrival order is this order, so acc->area is its printed
 * area bit for bit. Records carry (fl, fr): the child's lrarea (:185) is token-for-token the
 * parent's larea / rarea expression (:189-190) with the same operands, so this is bit-exact with
 * the reference's recomputation.
 */
static void walk(int integrand, int mode, rec_t root, double eps, int maxlev, aqo_result *res, acc_t *acc,
                 uint64_t *tpl, uint64_t *lpl)
{
    size_t cap = 256, n = 0;
    rec_t *st = (rec_t *)malloc(cap * sizeof(rec_t));
    if (!st) { acc->rc = AQO_ENOMEM; return; }
    st[n++] = root;
    while (n) {
        rec_t t = st[--n];
        if (t.depth >= maxlev) { acc->rc = AQO_EDEPTH; break; }
        double left = t.l, right = t.r;
        double lrarea = (t.fl + t.fr) * (right - left) / 2;          /* :185 */
        double mid = (left + right) / 2;                              /* :187 */
        double fmid = F_eval(integrand, mode, mid);                   /* :188 */
        double larea = (t.fl + fmid) * (mid - left) / 2;              /* :189 */
        double rarea = (fmid + t.fr) * (right - mid) / 2;             /* :190 */
        res->tasks++;
        if (tpl) tpl[t.depth]++;
        if (t.depth + 1 > res->levels) res->levels = t.depth + 1;
        if (fabs((larea + rarea) - lrarea) > eps) {                   /* :191 */
            if (push_rec(&st, &n, &cap, (rec_t){left, mid, t.fl, fmid, t.depth + 1}) ||   /* :192-194 */
                push_rec(&st, &n, &cap, (rec_t){mid, right, fmid, t.fr, t.depth + 1})) {  /* :195-197 */
                acc->rc = AQO_ENOMEM;
                break;
            }
        } else {
            double v = larea + rarea;                                 /* :199 */
            acc->area += v;                                           /* :149 */
            acc->q += (__float128)v;
            res->leaves++;
            if (lpl) lpl[t.depth]++;
        }
    }
    free(st);
}

static void finish(aqo_result *res, const acc_t *acc)
{
    res->area_lifo = acc->area;
    res->area_quad_hi = (double)acc->q;
    res->area_quad_lo = (double)(acc->q - (__float128)res->area_quad_hi);
}

/* The whole tree from the root [a,b]. tasks_per_level / leaves_per_level: length maxlev or NULL. */
int aqo_integrate(int integrand, int mode, double a, double b, double eps, int maxlev,
                  aqo_result *res, uint64_t *tasks_per_level, uint64_t *leaves_per_level)
{
    if (!res || maxlev <= 0 || maxlev > 4096 || !(b >= a)) return AQO_EINVAL;
    memset(res, 0, sizeof(*res));
    if (tasks_per_level) memset(tasks_per_level, 0, sizeof(uint64_t) * (size_t)maxlev);
    if (leaves_per_level) memset(leaves_per_level, 0, sizeof(uint64_t) * (size_t)maxlev);
    acc_t acc = {0.0, 0, AQO_OK};
    rec_t root = {a, b, F_eval(integrand, mode, a), F_eval(integrand, mode, b), 0};
    walk(integrand, mode, root, eps, maxlev, res, &acc, tasks_per_level, leaves_per_level);
    finish(res, &acc);
    return acc.rc;
}

/*
 * The share of shard `shard` of `nshards` in the device's partition (ppls_amd/csrc/aq_stream.h,
 * k_stream seeding): V = G*nshards virtual workers, seed depth D = floor(log2 V) + S; virtual
 * worker vwg = w*nshards + shard owns the depth-D positions j = k*V + (k odd ? V-1-vwg : vwg) < 2^D;
 * a task above depth D is counted by the owner of its leftmost descendant position. Summing the
 * results of all shards gives aqo_integrate()'s counts exactly (tests check both properties).
 */
int aqo_integrate_shard(int integrand, int mode, double a, double b, double eps, int maxlev, int G, int S,
                        int shard, int nshards, aqo_result *res, uint64_t *tasks_per_level,
                        uint64_t *leaves_per_level)
{
    if (!res || maxlev <= 0 || maxlev > 4096 || !(b >= a) || G < 1 || S < 0 || S > 6 || nshards < 1 ||
        shard < 0 || shard >= nshards)
        return AQO_EINVAL;
    memset(res, 0, sizeof(*res));
    if (tasks_per_level) memset(tasks_per_level, 0, sizeof(uint64_t) * (size_t)maxlev);
    if (leaves_per_level) memset(leaves_per_level, 0, sizeof(uint64_t) * (size_t)maxlev);
    const uint64_t V = (uint64_t)G * (uint64_t)nshards;
    int D = 0;
    while ((2ull << D) <= V) D++;
    D += S;
    const uint64_t npos = 1ull << D;
    const uint64_t nbands = (npos + V - 1) / V;
    const double fa = F_eval(integrand, mode, a), fb = F_eval(integrand, mode, b);
    acc_t acc = {0.0, 0, AQO_OK};
    for (int w = 0; w < G && acc.rc == AQO_OK; w++) {
        const uint64_t vwg = (uint64_t)w * (uint64_t)nshards + (uint64_t)shard;
        for (uint64_t k = 0; k < nbands && acc.rc == AQO_OK; k++) {
            const uint64_t p = k * V + ((k & 1) ? (V - 1 - vwg) : vwg);
            if (p >= npos) continue;
            double l = a, r = b, fl = fa, fr = fb;
            int alive = 1;
            for (int d = 0; d < D; d++) {
                const double mid = (l + r) / 2;
                const double fmid = F_eval(integrand, mode, mid);
                const double lrarea = (fl + fr) * (r - l) / 2;
                const double larea = (fl + fmid) * (mid - l) / 2;
                const double rarea = (fmid + fr) * (r - mid) / 2;
                const int refine = fabs((larea + rarea) - lrarea) > eps;
                const int owner = (p & ((1ull << (D - d)) - 1ull)) == 0ull;
                if (owner) {
                    res->tasks++;
                    if (tasks_per_level) tasks_per_level[d]++;
                    if (d + 1 > res->levels) res->levels = d + 1;
                }
                if (!refine) {
                    if (owner) {
                        double v = larea + rarea;
                        acc.area += v;
                        acc.q += (__float128)v;
                        res->leaves++;
                        if (leaves_per_level) leaves_per_level[d]++;
                    }
                    alive = 0;
                    break;
                }
                if (d + 1 >= maxlev) {
                    if (owner) acc.rc = AQO_EDEPTH;
                    alive = 0;
                    break;
                }
                if ((p >> (D - 1 - d)) & 1ull) { l = mid; fl = fmid; }
                else { r = mid; fr = fmid; }
            }
            if (alive) {
                rec_t root = {l, r, fl, fr, D};
                walk(integrand, mode, root, eps, maxlev, res, &acc, tasks_per_level, leaves_per_level);
            }
        }
    }
    finish(res, &acc);
    return acc.rc;
}

/* Quad sum as a decimal string (for fixtures). */
int aqo_quad_to_string(double hi, double lo, char *buf, int len)
{
    __float128 q = (__float128)hi + (__float128)lo;
    return quadmath_snprintf(buf, (size_t)len, "%.25Qg", q);
}

/* ---- batch: splitmix64 bounds ------------------------------------ */
static inline uint64_t splitmix64_next(uint64_t *state)
{
    uint64_t z = (*state += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* Generate n bounds pairs: a = 5*u1, b = 5*u2, swapped if a > b (state0 = 0x9E3779B97F4A7C15). */
void aqo_batch_bounds(long n, double *a, double *b)
{
    uint64_t s = 0x9E3779B97F4A7C15ULL;
    for (long i = 0; i < n; i++) {
        double u1 = (double)(splitmix64_next(&s) >> 11) * 0x1.0p-53;
        double u2 = (double)(splitmix64_next(&s) >> 11) * 0x1.0p-53;
        double x = 5.0 * u1, y = 5.0 * u2;
        if (x > y) { double t = x; x = y; y = t; }
        a[i] = x;
        b[i] = y;
    }
}

/* Integrate each [a[i], b[i]] independently; per-integral area (quad-accumulated) and counts. */
int aqo_integrate_batch(int integrand, int mode, long n, const double *a, const double *b,
                        double eps, int maxlev, double *area, uint64_t *tasks, uint64_t *leaves)
{
    for (long i = 0; i < n; i++) {
        aqo_result r;
        int rc = aqo_integrate(integrand, mode, a[i], b[i], eps, maxlev, &r, NULL, NULL);
        if (rc) return rc;
        if (area) area[i] = r.area_quad_hi + r.area_quad_lo;
        if (tasks) tasks[i] = r.tasks;
        if (leaves) leaves[i] = r.leaves;
    }
    return AQO_OK;
}
