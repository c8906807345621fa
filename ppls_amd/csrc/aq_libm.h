// aq_libm.h -- device integrands for gfx950, bit-identical to the host the reference runs on.
//
// The reference's integrand is the macro F(arg) cosh(arg)*cosh(arg)*cosh(arg)*cosh(arg)
// (/root/reference/aquadPartA.c:46), evaluated through glibc 2.35 libm. The accepted-interval
// count at EPSILON=1e-10/1e-12 changes under a 1-ulp change of cosh, so the device
// restates glibc's cosh exactly rather than calling OCML:
//   __ieee754_cosh (e_cosh.c, fdlibm formula) over
//   __exp          (e_exp.c, N=128 table, the FMA ifunc form x86_64 hosts with FMA select) and
//   __expm1        (s_expm1.c, k = 0 path, Estrin polynomial, no fusion),
// and, for the config-4 variant of the macro, sin(1.0/(arg)):
//   __sin          (s_sin.c, |x| < 105414350, the FMA ifunc form; table aq_sincos_table.h).
// The kernels that include this header are compiled with -ffp-contract=off: every fusion below
// is an explicit __fma_rn() placed exactly where GCC fused glibc's source.
//
// The 2 KiB exp table lives in LDS (one ds_read_b128 per lookup); kernels stage it at entry
// with aq_stage_exp_table().
#pragma once
#ifndef AQ_PIN_CONSTS
#define AQ_PIN_CONSTS 1
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aq_exp_table.h"
#include "aq_sincos_table.h"

#pragma clang fp contract(off)

namespace aq {

// glibc's __exp_data.tab[2j], tab[2j+1] as the device's global copy holds them.
struct ExpPair {
    uint64_t tail_bits;
    uint64_t sbits;
};
// The exp table in the code object: k_stream's prologue loads it at entry, with no wait for the
// kernel arguments first (a pointer argument put the argument fetch and the table fetch in series
// at every launch).
static __constant__ uint64_t kExpTabBits[256] = {AQ_EXP_TAB_INIT};

// One entry of the LDS copy (stage_exp_table): the same pair, 16-B aligned for one ds_read_b128.
// (r02 A/B, tools/ab.sh: a 32-B entry that also carried 2^(-j/128)'s high word, so that cosh's first
// reciprocal estimate u (1 - tmp) replaced v_rcp_f64 -- exact on 3.4e10 points, but 2 FMAs, 2 integer
// ops and 2 LDS reads more per round -- measured 1.0 % slower: v_rcp_f64, ~3x an FMA's issue cost
// alone (tools/ubench_issue.hip), overlaps the surrounding VALU work. A 256-entry copy indexed by ki's
// low byte through one SDWA shift (2 integer ops fewer per round) read as ds_read2_b64: 0.8 % slower.)
struct alignas(16) ExpEntry {
    uint64_t tail_bits;
    uint64_t sbits;
};

static constexpr double kInvLn2N = 0x1.71547652b82fep7;
static constexpr double kShift = 0x1.8p52;
static constexpr double kNegLn2hiN = -0x1.62e42fefa0000p-8;
static constexpr double kNegLn2loN = -0x1.cf79abc9e3b3ap-47;
static constexpr double kC2 = 0x1.ffffffffffdbdp-2;
static constexpr double kC3 = 0x1.555555555543cp-3;
static constexpr double kC4 = 0x1.55555cf172b91p-5;
static constexpr double kC5 = 0x1.1111167a4d017p-7;

static constexpr double kQ1 = -3.33333333333331316428e-02;
static constexpr double kQ2 = 1.58730158725481460165e-03;
static constexpr double kQ3 = -7.93650757867487942473e-05;
static constexpr double kQ4 = 4.00821782732936239552e-06;
static constexpr double kQ5 = -2.01099218183624371326e-07;

__device__ __forceinline__ uint32_t hi_word(double x) {
    return (uint32_t)((uint64_t)__double_as_longlong(x) >> 32);
}

// glibc __exp_fma main path for x in [2^-54, 709.78]; x >= 512 takes glibc's specialcase scaling.
__device__ __forceinline__ double exp_glibc(double x, const ExpEntry* __restrict__ tab) {
    double kd = __fma_rn(kInvLn2N, x, kShift);
    const uint64_t ki = (uint64_t)__double_as_longlong(kd);
    kd = kd - kShift;
    const double r = __fma_rn(kd, kNegLn2loN, __fma_rn(kd, kNegLn2hiN, x));
    const ExpEntry e = tab[ki & 127];
    const double tail = __longlong_as_double((long long)e.tail_bits);
    uint64_t sbits = e.sbits + (ki << 45);
    const double r2 = r * r;
    const double tmp = __fma_rn(r2 * r2, __fma_rn(r, kC5, kC4), __fma_rn(r2, __fma_rn(r, kC3, kC2), tail + r));
    if (__builtin_expect(x >= 512.0, 0)) {
        if (x > 0x1.62e42fefa39efp+9) return __longlong_as_double(0x7ff0000000000000LL);
        sbits -= 1009ull << 52;
        const double scale = __longlong_as_double((long long)sbits);
        return 0x1p1009 * __fma_rn(scale, tmp, scale);
    }
    const double scale = __longlong_as_double((long long)sbits);
    return __fma_rn(scale, tmp, scale);
}

// glibc __exp (e_exp.c, FMA ifunc form) for every double: the tiny-argument path (|x| < 2^-54:
// 1 + x), the main path, and both specialcase() branches (k > 0: |x| >= 512 overflow scaling; k < 0:
// the subnormal range with its hi/lo re-rounding). Plug-in integrands (AQ_F_USER) call this one.
__device__ __forceinline__ double exp_glibc_any(double x, const ExpEntry* __restrict__ tab) {
    const uint32_t abstop = (uint32_t)((uint64_t)__double_as_longlong(x) >> 52) & 0x7ffu;
    bool special = false;
    if (__builtin_expect(abstop - 0x3c9u >= 0x408u - 0x3c9u, 0)) {   // |x| < 2^-54 or |x| >= 512 (or nan / inf)
        if ((int)(abstop - 0x3c9u) < 0) return 1.0 + x;
        if (abstop >= 0x409u) {                                        // |x| >= 1024
            if (__double_as_longlong(x) == (long long)0xfff0000000000000ull) return 0.0;
            if (abstop >= 0x7ffu) return 1.0 + x;
            return x < 0.0 ? 0.0 : __longlong_as_double(0x7ff0000000000000LL);
        }
        special = true;
    }
    double kd = __fma_rn(kInvLn2N, x, kShift);
    const uint64_t ki = (uint64_t)__double_as_longlong(kd);
    kd = kd - kShift;
    const double r = __fma_rn(kd, kNegLn2loN, __fma_rn(kd, kNegLn2hiN, x));
    const ExpEntry e = tab[ki & 127];
    const double tail = __longlong_as_double((long long)e.tail_bits);
    uint64_t sbits = e.sbits + (ki << 45);
    const double r2 = r * r;
    const double tmp = __fma_rn(r2 * r2, __fma_rn(r, kC5, kC4), __fma_rn(r2, __fma_rn(r, kC3, kC2), tail + r));
    if (__builtin_expect(special, 0)) {
        if ((ki & 0x80000000ull) == 0) {                               // k > 0
            sbits -= 1009ull << 52;
            const double scale = __longlong_as_double((long long)sbits);
            return 0x1p1009 * __fma_rn(scale, tmp, scale);
        }
        // k < 0, the subnormal range: glibc's FMA build leaves this branch unfused (checked against
        // the host libm, oracle/aq_oracle.c exp_any)
        sbits += 1022ull << 52;
        const double scale = __longlong_as_double((long long)sbits);
        double y = scale + scale * tmp;
        if (y < 1.0) {
            double lo = scale - y + scale * tmp;
            const double hi = 1.0 + y;
            lo = 1.0 - hi + y + lo;
            y = (hi + lo) - 1.0;
            if (y == 0.0) y = 0.0;
        }
        return 0x1p-1022 * y;
    }
    const double scale = __longlong_as_double((long long)sbits);
    return __fma_rn(scale, tmp, scale);
}

// glibc __expm1 for |x| < 0.5*ln2 (the only range cosh passes it).
__device__ __forceinline__ double expm1_glibc_small(double x) {
    if ((hi_word(x) & 0x7fffffffu) < 0x3c900000u) return x;
    const double hfx = 0.5 * x;
    const double hxs = x * hfx;
    const double R1 = 1.0 + hxs * kQ1;
    const double h2 = hxs * hxs;
    const double R2 = kQ2 + hxs * kQ3;
    const double h4 = h2 * h2;
    const double R3 = kQ4 + hxs * kQ5;
    const double r1 = R1 + h2 * R2 + h4 * R3;
    const double t = 3.0 - r1 * hfx;
    const double e = hxs * ((r1 - t) / (6.0 - x * t));
    return x - (x * e - hxs);
}

// RN(0.5 / t) for 1 <= t < 2^64 -- the instruction sequence the compiler emits for the IEEE division
// (v_rcp_f64, two Newton steps, quotient, residual, fused correction) without v_div_scale /
// v_div_fmas / v_div_fixup, which are identities in this range (no operand needs rescaling, no
// special value). They are dropped because v_div_scale / v_div_fmas pass a flag through VCC, and
// that single register serialises any two divisions a wave would otherwise overlap.
#ifndef AQ_RCP_NEWTON
#define AQ_RCP_NEWTON 2
#endif
#ifndef AQ_SIN_RECIP_RN
#define AQ_SIN_RECIP_RN 1   // sin(1/x): recip_rn in place of the compiler's division (bit-identical)
#endif
template <int NEWTON = AQ_RCP_NEWTON>
__device__ __forceinline__ double half_recip_n(double t) {
    double y = __builtin_amdgcn_rcp(t);
    if constexpr (NEWTON == 3) {   // second-order step y0 (1 + e + e^2): the error of two Newton steps, one FMA fewer
        const double e = __fma_rn(-t, y, 1.0);
        y = __fma_rn(y, __fma_rn(e, e, e), y);
    } else {
#pragma unroll
        for (int i = 0; i < NEWTON; ++i) {
            const double e = __fma_rn(-t, y, 1.0);
            y = __fma_rn(y, e, y);
        }
    }
    const double q = 0.5 * y;
    const double r = __fma_rn(-t, q, 0.5);
    return __fma_rn(r, y, q);
}
__device__ __forceinline__ double half_recip(double t) { return half_recip_n<>(t); }
// 1.0 / x, correctly rounded, for the config-4 integrand's sin(1.0/(arg)): the same sequence with
// numerator 1 -- the compiler's IEEE division minus its scale / fmas scaling / fixup steps, identities
// while x and 1/x are normal (every nonzero bound is at least 2^-900 and at most 2^900 in magnitude,
// aq_abi.inc bounds_ok; x = 0, a midpoint of a symmetric interval, gives NaN either way). r06: 4 VALU
// fewer per evaluation, sin(1/x) launch times within noise (profiles/r06zj); tests/test_gpu.py
// test_device_sin_recip_bit_exact pins it to host libm.
__device__ __forceinline__ double recip_rn(double x) {
    double y = __builtin_amdgcn_rcp(x);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const double e = __fma_rn(-x, y, 1.0);
        y = __fma_rn(y, e, y);
    }
    const double r = __fma_rn(-x, y, 1.0);
    return __fma_rn(r, y, y);
}

// glibc's `half*t + half/t` is RN(RN(0.5*t) + h) with h = RN(0.5/t); 0.5*t is exact for the
// normal t of this range, so RN(0.5*t + h) -- one fma(t, 0.5, h) -- is the same value, bit for bit,
// one multiply fewer per evaluation.
// glibc __ieee754_cosh.
__device__ __forceinline__ double cosh_glibc(double x, const ExpEntry* __restrict__ tab) {
    const uint32_t ix = hi_word(x) & 0x7fffffffu;
    const double ax = fabs(x);
    if (__builtin_expect(ix < 0x40360000u, 1)) {          // |x| < 22
        if (ix < 0x3fd62e43u) {                             // |x| < 0.5*ln2
            if (ix < 0x3c800000u) return 1.0;
            const double t = expm1_glibc_small(ax);
            const double w = 1.0 + t;
            return 1.0 + (t * t) / (w + w);
        }
        const double t = exp_glibc(ax, tab);
        return __fma_rn(t, 0.5, half_recip(t));   // 0.5*t + 0.5/t (cosh_tail), t in [1.41, 3.6e9]
    }
    if (ix >= 0x7ff00000u) return x * x;
    if (ix < 0x40862e42u) return 0.5 * exp_glibc(ax, tab);
    if (ax <= 0x1.633ce8fb9f87dp+9) {
        const double w = exp_glibc(0.5 * ax, tab);
        const double t = 0.5 * w;
        return t * w;
    }
    return __longlong_as_double(0x7ff0000000000000LL);
}

// glibc 2.35 sin (sysdeps/ieee754/dbl-64/s_sin.c), the config-4 F macro's sin(1.0/(arg)), as the
// x86_64 __sin_fma ifunc variant evaluates it (the host libm the reference runs on): GCC's
// contraction of the source fuses every a*b+c of the polynomials, the cor sums and the Cody-Waite
// reduction, and the left product of p*a - 0.5*da and x*dx + xx*(...); the __fma_rn()s below spell that
// out as __fma_rn (this file builds with -ffp-contract=off). The table {sin, cos} of i/128 as double-doubles
// (aq_sincos_table.h, 3.5 KiB) is staged into the kernel's LDS integrand table (stage_f_table) in
// place of exp's; kSinCosTab is its constant-memory source.
// Exact for |x| < 105414350 (|arg| > 9.5e-9); beyond that glibc's __branred (Payne-Hanek) is not
// restated and the device libm's faithful sin answers.
static __constant__ double kSinCosTab[AQ_SINCOS_TAB_N] = {AQ_SINCOS_TAB_INIT};

namespace sinc {
constexpr double s1 = -0x1.5555555555555p-3, s2 = 0.0083333333333323288, s3 = -1.9841269834414642e-04,
                 s4 = 2.755729806860771e-06, s5 = -2.5022014848318398e-08;
constexpr double sn3 = -1.66666666666664880952546298448555E-01, sn5 = 8.33333214285722277379541354343671E-03,
                 cs2 = 4.99999999999999999999950396842453E-01, cs4 = -4.16666666666664434524222570944589E-02,
                 cs6 = 1.38888874007937613028114285595617E-03;
constexpr double big = 0x1.8p45, hp0 = 0x1.921FB54442D18p0, hp1 = 0x1.1A62633145C07p-54, mp1 = 0x1.921FB58p0,
                 mp2 = -0x1.DDE973Cp-27, pp3 = -0x1.CB3B398p-55, pp4 = -0x1.d747f23e32ed7p-83,
                 hpinv = 0x1.45F306DC9C883p-1, toint = 0x1.8p52;
}  // namespace sinc

__device__ __forceinline__ double sin_tab_cos(double x, double dx, const double* __restrict__ st) {   // s_sin.c do_cos
    using namespace sinc;
    if (x < 0) dx = -dx;
    const double u = big + fabs(x);
    x = fabs(x) - (u - big) + dx;
    const double xx = x * x;
    const double s = __fma_rn(x * xx, __fma_rn(xx, sn5, sn3), x);
    const double c = xx * __fma_rn(xx, __fma_rn(xx, cs6, cs4), cs2);
    const int k = __double2loint(u) << 2;
    const double sn = st[k], ssn = st[k + 1], cs = st[k + 2], ccs = st[k + 3];
    const double cor = __fma_rn(-sn, s, __fma_rn(-cs, c, __fma_rn(-s, ssn, ccs)));
    return cs + cor;
}

__device__ __forceinline__ double sin_tab_sin(double x, double dx, const double* __restrict__ st) {   // s_sin.c do_sin
    using namespace sinc;
    const double xold = x;
    if (fabs(x) < 0.126) {                                               // TAYLOR_SIN (x*x, x, dx)
        const double xx = x * x;
        const double p = __fma_rn(__fma_rn(__fma_rn(__fma_rn(s5, xx, s4), xx, s3), xx, s2), xx, s1);
        return x + __fma_rn(__fma_rn(p, x, -0.5 * dx), xx, dx);
    }
    if (x <= 0) dx = -dx;
    const double u = big + fabs(x);
    x = fabs(x) - (u - big);
    const double xx = x * x;
    const double s = x + __fma_rn(x * xx, __fma_rn(xx, sn5, sn3), dx);
    const double c = __fma_rn(x, dx, xx * __fma_rn(xx, __fma_rn(xx, cs6, cs4), cs2));
    const int k = __double2loint(u) << 2;
    const double sn = st[k], ssn = st[k + 1], cs = st[k + 2], ccs = st[k + 3];
    const double cor = __fma_rn(cs, s, __fma_rn(-sn, c, __fma_rn(s, ccs, ssn)));
    return copysign(sn + cor, xold);
}

__device__ __forceinline__ double sin_glibc(double x, const double* __restrict__ st) {
    using namespace sinc;
    const unsigned k = (unsigned)__double2hiint(x) & 0x7fffffffu;
    if (k < 0x3e500000u) return x;                                       // |x| < 2^-26
    if (k < 0x3feb6000u) return sin_tab_sin(x, 0.0, st);                     // |x| < 0.855469
    if (k < 0x400368fdu) return copysign(sin_tab_cos(hp0 - fabs(x), hp1, st), x);   // |x| < 2.426265
    if (k < 0x419921fbu) {                                               // |x| < 105414350
        const double t = __fma_rn(x, hpinv, toint);
        const double xn = t - toint;
        const double y = __fma_rn(-xn, mp2, __fma_rn(-xn, mp1, x));
        const int n = __double2loint(t) & 3;
        double t1 = xn * pp3;
        const double t2 = y - t1;
        double db = (y - t2) - t1;
        t1 = xn * pp4;
        const double b = t2 - t1;
        db += (t2 - b) - t1;
        const double r = (n & 1) ? sin_tab_cos(b, db, st) : sin_tab_sin(b, db, st);
        return (n & 2) ? -r : r;
    }
    return sin(x);                                                       // __branred range, inf, nan
}

// A kernel's integrand table as __sincostab (its LDS copy, stage_f_table).
__device__ __forceinline__ const double* sin_table(const ExpEntry* tab) { return reinterpret_cast<const double*>(tab); }

// Integrand ids (include/aquad.h aq_integrand).
enum : int { F_COSH4 = 0, F_SIN_RECIP = 1, F_USER = 2 };

}  // namespace aq

// The AQ_F_USER plug-in: the reference's extension point is the F(arg) macro (aquadPartA.c:46);
// here a header, chosen at build time with -DAQ_USER_F_HEADER=<file> (ppls_amd/build.py:
// PPLS_AMD_USER_F=<file>), defines in namespace aq::user
//   constexpr const char* name;                                  -- reported by aq_user_integrand_name()
//   __device__ double F(double x, const aq::ExpEntry* tab);      -- the macro body (tab: LDS exp table
//                                                                   for aq::exp_glibc_any / cosh_glibc)
//   inline bool domain_ok(double a, double b);                   -- host check of [a, b]
// and is compiled into every kernel as integrand id 2. Plug-in trees use the reference's own area
// expressions literally (no doubled-area rescaling), so they are bit-exact for any finite F.
#ifndef AQ_USER_F_HEADER
#define AQ_USER_F_HEADER "plugins/aq_user_gauss.h"
#endif
#include AQ_USER_F_HEADER

namespace aq {

// F(arg) exactly as the reference macro expands (aquadPartA.c:46): ((c*c)*c)*c.
template <int FID>
__device__ __forceinline__ double integrand(double x, const ExpEntry* __restrict__ tab) {
    if constexpr (FID == F_COSH4) {
        const double c = cosh_glibc(x, tab);
        return c * c * c * c;
    } else if constexpr (FID == F_USER) {
        return user::F(x, tab);
    } else {
        return sin_glibc(AQ_SIN_RECIP_RN ? recip_rn(x) : 1.0 / x, sin_table(tab));   // config 4: sin(1.0/(arg))
    }
}

// Constants of the exp main path. gfx9 VOP3 reads at most one scalar operand and takes no 64-bit
// literal, so every evaluation would rebuild them (s_mov pairs, and a v_mov where two meet in one
// FMA). A persistent kernel pins them in VGPRs once (pinned_exp_consts); the default instance lets
// the compiler choose.
struct ExpConsts {
    double shift = kShift, c4 = kC4, c2 = kC2;
    double inv = kInvLn2N, hi = kNegLn2hiN, lo = kNegLn2loN, c5 = kC5, c3 = kC3;
};
__device__ __forceinline__ ExpConsts pinned_exp_consts() {
    ExpConsts k;
#if AQ_PIN_CONSTS
    asm volatile("" : "+v"(k.shift), "+v"(k.c4), "+v"(k.c2));   // opaque: kept in registers
    asm volatile("" : "+v"(k.inv), "+v"(k.hi), "+v"(k.lo), "+v"(k.c5), "+v"(k.c3));
#endif
    return k;
}

// cosh for K independent arguments, written stage by stage so the K dependency chains interleave
// (the main path has no branch). c[k] is exact for 0.5*ln2 <= |x[k]| < 22; the return value is a
// lane flag set when some x[k] is outside that range, for the caller to redo with cosh_glibc.
__device__ __forceinline__ bool cosh_main_range(double x) {
    const uint32_t ix = hi_word(x) & 0x7fffffffu;
    return ix >= 0x3fd62e43u && ix < 0x40360000u;
}
//
// TWICE: c[k] = 2 cosh(x[k]) = RN(t + y3), exactly twice glibc's value. With q = 0.5 y2 (exact) the
// quotient correction's residual fma(-t, q, 0.5) is half the Newton residual e = fma(-t, y2, 1), so
// RN(0.5 / t) = RN(q + r y2) = 0.5 RN(y2 + e y2) = 0.5 y3 (the next Newton iterate), and cosh =
// RN(0.5 t + 0.5 y3) = 0.5 RN(t + y3): every halving is exact in this range. One multiply fewer per
// evaluation and a shorter chain (e, y3, t + y3 against q, r, h, c).
// TABMASK: 127 for the 128-entry LDS table; 255 for a table of its 128 entries twice over (k_stream's
// bulk instance, AQ_WIDE_TAB): the index is then ki's low byte, one SDWA shift (no and, no or of the
// table's base, which the read's offset field carries).
template <int K, bool CHECK = true, bool TWICE = false, unsigned TABMASK = 127u>
__device__ __forceinline__ bool cosh_main_k(const double (&x)[K], double (&c)[K], const ExpEntry* __restrict__ tab,
                                            const ExpConsts& kk) {
    double ax[K], kd[K], r[K], r2[K], tmp[K], t[K];
    uint64_t ki[K];
    ExpEntry e[K];
    bool out = false;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        ax[k] = fabs(x[k]);
        kd[k] = __fma_rn(kk.inv, ax[k], kk.shift);
        ki[k] = (uint64_t)__double_as_longlong(kd[k]);
        e[k] = tab[ki[k] & TABMASK];
        if (CHECK) out |= !cosh_main_range(x[k]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        kd[k] = kd[k] - kk.shift;
        r[k] = __fma_rn(kd[k], kk.lo, __fma_rn(kd[k], kk.hi, ax[k]));
        r2[k] = r[k] * r[k];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const double tail = __longlong_as_double((long long)e[k].tail_bits);
        tmp[k] = __fma_rn(r2[k] * r2[k], __fma_rn(r[k], kk.c5, kk.c4),
                          __fma_rn(r2[k], __fma_rn(r[k], kk.c3, kk.c2), tail + r[k]));
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        // e.sbits + (ki << 45): the addend's low word is zero, so only the high words add (no carry
        // crosses the word boundary) -- one 32-bit shift-add instead of a 64-bit one
        const uint32_t shi = (uint32_t)(e[k].sbits >> 32) + ((uint32_t)ki[k] << 13);
        const double scale = __hiloint2double((int)shi, (int)(uint32_t)e[k].sbits);
        t[k] = __fma_rn(scale, tmp[k], scale);
    }
    double y[K], q[K];
#pragma unroll
    for (int k = 0; k < K; ++k) y[k] = __builtin_amdgcn_rcp(t[k]);
#pragma unroll
    for (int it = 0; it < 2; ++it) {   // two Newton steps (one is not provably enough)
#pragma unroll
        for (int k = 0; k < K; ++k) y[k] = __fma_rn(y[k], __fma_rn(-t[k], y[k], 1.0), y[k]);
    }
    if constexpr (TWICE) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double e = __fma_rn(-t[k], y[k], 1.0);
            c[k] = t[k] + __fma_rn(y[k], e, y[k]);                    // RN(t + y3) = 2 cosh
        }
        (void)q;
        return out;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        q[k] = 0.5 * y[k];
        c[k] = __fma_rn(t[k], 0.5, __fma_rn(__fma_rn(-t[k], q[k], 0.5), y[k], q[k]));   // 0.5*t + half_recip(t)
    }
    return out;
}

// F at K independent points (one round of K records per lane); every lane of the wave calls it.
// A lane whose K points all lie in one interval [lo, hi] may pass range_hint = cosh_main_span(lo,
// hi) (one test for the K points); -1 tests every point; 2: out_mask is the wave mask of the lanes
// whose points may lie outside the exp path (the caller's one test per lane).
__device__ __forceinline__ bool cosh_main_span(double lo, double hi) {
    // lo >= 0.5*ln2 and hi < 22: every point between has a high word between theirs (the word is
    // monotonic for x >= 0), so glibc takes the exp path for all of them. As SIGNED words a negative
    // lo (sign bit set) is below 0x3fd62e43 and fails; then hi needs no lower test (hi >= lo). Two
    // compares, no subtracts.
    return ((int)hi_word(lo) >= 0x3fd62e43) && ((int)hi_word(hi) < 0x40360000);
}
//
// SCALED (cosh^4 only): f[k] = 16 F(x[k]), exactly, as ((s*s)*s)*s with s = 2 cosh (cosh_main_k
// TWICE): every product is the reference's scaled by a power of two (f_scale<FID>(), aq_device.h).
template <int FID, int K, bool SCALED = false, unsigned TABMASK = 127u>
__device__ __forceinline__ void integrand_k(const double (&x)[K], double (&f)[K], const ExpEntry* __restrict__ tab,
                                            const ExpConsts& kk = ExpConsts{}, int range_hint = -1,
                                            unsigned long long out_mask = 0ull) {
    if constexpr (FID == F_COSH4) {
        constexpr double cs = SCALED ? 2.0 : 1.0;   // c[k] holds cs * cosh
        double c[K];
        bool out;
        if (range_hint == 2) {
            cosh_main_k<K, false, SCALED, TABMASK>(x, c, tab, kk);
            if (__builtin_expect(out_mask != 0ull, 0)) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if (!cosh_main_range(x[k])) c[k] = cs * cosh_glibc(x[k], tab);
            }
            out = false;
        } else if (range_hint >= 0) {
            cosh_main_k<K, false, SCALED, TABMASK>(x, c, tab, kk);
            out = range_hint == 0;
        } else {
            out = cosh_main_k<K, true, SCALED, TABMASK>(x, c, tab, kk);
        }
        if (__builtin_expect(__ballot(out) != 0ull, 0)) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (!cosh_main_range(x[k])) c[k] = cs * cosh_glibc(x[k], tab);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) f[k] = c[k] * c[k];           // ((c*c)*c)*c, stage by stage so
#pragma unroll                                                        // the K chains interleave
        for (int k = 0; k < K; ++k) f[k] = f[k] * c[k];
#pragma unroll
        for (int k = 0; k < K; ++k) f[k] = f[k] * c[k];
    } else if constexpr (FID == F_USER) {
#pragma unroll
        for (int k = 0; k < K; ++k) f[k] = user::F(x[k], tab);
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) f[k] = sin_glibc(AQ_SIN_RECIP_RN ? recip_rn(x[k]) : 1.0 / x[k], sin_table(tab));
    }
}

// A kernel's LDS integrand table: glibc exp's 128 entries (cosh^4 and the plug-ins), or for sin(1/x)
// glibc's __sincostab (444 doubles in 222 16-B entries) -- integrand<F_SIN_RECIP> reads `tab` as that.
template <int FID>
constexpr int ftab_entries() { return FID == F_SIN_RECIP ? (AQ_SINCOS_TAB_N + 1) / 2 : 128; }

// Stage the exp table into LDS (call from every thread, then __syncthreads()).
__device__ __forceinline__ void stage_exp_table(ExpEntry* lds, const ExpPair* __restrict__ g) {
    for (int i = threadIdx.x; i < 128; i += blockDim.x) {
        lds[i].tail_bits = g[i].tail_bits;
        lds[i].sbits = g[i].sbits;
    }
}

// Stage FID's integrand table (ftab_entries<FID>() entries) into LDS; then __syncthreads().
template <int FID>
__device__ __forceinline__ void stage_f_table(ExpEntry* lds, const ExpPair* __restrict__ g) {
    if constexpr (FID == F_SIN_RECIP) {
        double* const d = reinterpret_cast<double*>(lds);
        for (int i = threadIdx.x; i < AQ_SINCOS_TAB_N; i += blockDim.x) d[i] = kSinCosTab[i];
    } else {
        stage_exp_table(lds, g);
    }
}

}  // namespace aq
