// aq_device.h -- device building blocks shared by the quadrature kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aquad.h"
#include "aq_libm.h"

#pragma clang fp contract(off)

namespace aq {

enum : unsigned { ERRB_TIMEOUT = 1, ERRB_OVERFLOW = 2, ERRB_DEPTH = 4 };

// Hardware CU slot of the executing wave: xcc*256 + (se*2 + sh)*16 + cu (HW_ID / XCC_ID registers).
__device__ __forceinline__ unsigned cu_slot() {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID, 32 bits
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID, bits 3:0
    const unsigned cu = (hw >> 8) & 15u, sh = (hw >> 12) & 1u, se = (hw >> 13) & 7u;
    return ((xcc & 7u) << 8) | (((se << 1) | sh) << 4) | cu;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ unsigned wave_sum_u(unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ unsigned wave_max_u(unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (unsigned)__shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ unsigned wave_or_u(unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v |= (unsigned)__shfl_xor((int)v, o, 64);
    return v;
}
__device__ __forceinline__ unsigned lane_id() { return __lane_id(); }
__device__ __forceinline__ unsigned mbcnt(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// One trapezoid step of the reference (aquadPartA.c:185-191) on a record that carries F(l), F(r).
// The operand order and association are the reference's; '/2' is exact (scaling by 2^-1).
struct Step {
    double mid, fmid, larea, rarea;
    bool refine;
};
template <int FID>
__device__ __forceinline__ Step task_step(double l, double r, double fl, double fr, double eps,
                                          const ExpEntry* __restrict__ tab) {
    Step s;
    const double lrarea = (fl + fr) * (r - l) / 2;   // :185
    s.mid = (l + r) / 2;                             // :187
    s.fmid = integrand<FID>(s.mid, tab);             // :188
    s.larea = (fl + s.fmid) * (s.mid - l) / 2;       // :189
    s.rarea = (s.fmid + fr) * (r - s.mid) / 2;       // :190
    s.refine = fabs((s.larea + s.rarea) - lrarea) > eps;  // :191 (strict >)
    return s;
}

// K trapezoid steps at once (K records per lane), with every area DOUBLED: the products
// (fl+fr)*(r-l) etc. of :185/:189/:190 without their '/2'. Halving is exact and commutes with
// rounding as long as nothing falls below 2^-1021 (no doubled area or difference of the built
// integrands comes near: |F| >= 1 for cosh^4, and the smallest nonzero |F(l)+F(r)| * width of
// sin(1/x) at the depth cap is > 2^-200), so
//   larea + rarea        == (L2 + R2) / 2           (x/2 + y/2 rounds like (x + y)/2)
//   (larea+rarea)-lrarea == ((L2 + R2) - LR2) / 2
//   |d / 2| > eps        <=> |d| > 2*eps            (2*eps exact)
// -- every decision of :191 is bit-identical and each accepted area is exactly half of `area2`;
// the caller halves its accumulator once (flush). Saves the three '/2' multiplies per task.
// Every lane of the wave calls it (inactive lanes pass a harmless record, e.g. l = r = 1, F = 0).
struct Step2 {
    double fmid, area2;   // F(mid) and 2 * (larea + rarea)
    bool refine;
};
//
// Doubling needs every product to stay normal: the built-in integrands guarantee it on their
// validated domains (aq_abi.inc bounds_ok). A plug-in F (F_USER) can be anything, so its trees use
// the reference's expressions literally, '/2' included: area2 is then the plain larea + rarea and
// the caller passes eps itself (area_scale<FID>() says which).
template <int FID>
__host__ __device__ constexpr bool doubled_areas() { return FID != F_USER; }
// The persistent kernel's F values for cosh^4 are 16 F (integrand_k SCALED: one multiply fewer per
// evaluation); scaling every F by the same power of two scales every product and difference of
// :185-:191 by it exactly (nothing comes near the subnormal or overflow range on the validated
// domain, |x| <= 170), so the decisions hold with eps scaled alike. Seeds scale their F on push.
template <int FID>
__host__ __device__ constexpr double f_scale() { return FID == F_COSH4 ? 16.0 : 1.0; }
// accepted area = area_scale * area2 (doubled areas of 16 F for cosh^4: 1/32)
template <int FID>
__host__ __device__ constexpr double area_scale() { return doubled_areas<FID>() ? 0.5 / f_scale<FID>() : 1.0; }

template <int FID, int K>
__device__ __forceinline__ void task_step_k(const double (&l)[K], const double (&r)[K], const double (&fl)[K],
                                            const double (&fr)[K], double eps2, const ExpEntry* __restrict__ tab,
                                            Step2 (&s)[K], const ExpConsts& kk = ExpConsts{}, int range_hint = -1,
                                            unsigned long long out_mask = 0ull) {
    double mid[K], fmid[K];
#pragma unroll
    for (int k = 0; k < K; ++k) mid[k] = (l[k] + r[k]) / 2;   // :187
    // the parts of the step that do not need F(mid) first: independent work the scheduler can
    // place in the latency gaps of the F chains (r02 A/B: 27.25 -> 27.04 ms per 8192-integral launch)
    double lr2e[K], wl[K], wr[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        lr2e[k] = (fl[k] + fr[k]) * (r[k] - l[k]);
        wl[k] = mid[k] - l[k];
        wr[k] = r[k] - mid[k];
        // computed HERE (volatile: not sunk below the F chains' range-check branch)
        asm volatile("" : "+v"(lr2e[k]), "+v"(wl[k]), "+v"(wr[k]));
    }
    integrand_k<FID, K, (f_scale<FID>() != 1.0)>(mid, fmid, tab, kk, range_hint, out_mask);   // :188 (f_scale F)
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if constexpr (doubled_areas<FID>()) {
            const double lr2 = lr2e[k];                                   // 2 * lrarea, :185
            const double l2 = (fl[k] + fmid[k]) * wl[k];                  // 2 * larea,  :189
            const double r2 = (fmid[k] + fr[k]) * wr[k];                  // 2 * rarea,  :190
            s[k].fmid = fmid[k];
            s[k].area2 = l2 + r2;
            s[k].refine = fabs(s[k].area2 - lr2) > eps2;                  // :191 (strict >)
        } else {   // eps2 is eps here (area_scale 1)
            const double lrarea = (fl[k] + fr[k]) * (r[k] - l[k]) / 2;    // :185
            const double larea = (fl[k] + fmid[k]) * (mid[k] - l[k]) / 2; // :189
            const double rarea = (fmid[k] + fr[k]) * (r[k] - mid[k]) / 2; // :190
            s[k].fmid = fmid[k];
            s[k].area2 = larea + rarea;                                   // :199
            s[k].refine = fabs((larea + rarea) - lrarea) > eps2;          // :191 (strict >)
        }
    }
}

// Both tasks of a sibling pair [a, m], [m, b] (m = (a + b) / 2, the parent's midpoint) from the pair's
// HALVED endpoints ha = a / 2, hb = b / 2, as k_stream's rings store them. With a = 2 ha exactly
// (the validated domain keeps every coordinate's half normal, aq_abi.inc bounds_ok):
//   m    = RN((a + b) / 2) = RN(ha + hb)               hm = m / 2 (exact)
//   midL = RN((a + m) / 2) = RN(ha + hm)               midR = RN(hm + hb)             (:187)
//   m - a = RN(m - 2 ha) = fma(ha, -2, m)              b - m = fma(hb, 2, -m), and alike for
// the widths of :189 / :190 -- the reference's values, one operation each, so the three midpoints
// cost three adds and one multiply where (l + r) / 2 costs an add and a multiply each. The
// children pairs are {ha, hm} and {hm, hb}: already at hand. Returns m and hm for the pushes.
template <int FID, unsigned TABMASK = 127u>
__device__ __forceinline__ void pair_step_halves(double ha, double hb, double fa, double fm, double fb, double eps2,
                                                 const ExpEntry* __restrict__ tab, Step2 (&s)[2], double& m,
                                                 double& hm, const ExpConsts& kk, int range_hint,
                                                 unsigned long long out_mask) {
    m = ha + hb;                                             // the parent's midpoint (:187)
    hm = 0.5 * m;
    const double mid[2] = {ha + hm, hm + hb};                // :187 for [a, m] and [m, b]
    const double fl[2] = {fa, fm}, fr[2] = {fm, fb};
    // the parts that do not need F(mid) first (as task_step_k's)
    double lr2e[2], wl[2], wr[2];
    lr2e[0] = (fa + fm) * __fma_rn(ha, -2.0, m);             // (fl + fr) * (r - l), :185
    lr2e[1] = (fm + fb) * __fma_rn(hb, 2.0, -m);
    wl[0] = __fma_rn(ha, -2.0, mid[0]);                      // mid - l
    wl[1] = mid[1] - m;
    wr[0] = m - mid[0];                                      // r - mid
    wr[1] = __fma_rn(hb, 2.0, -mid[1]);
#pragma unroll
    for (int k = 0; k < 2; ++k) asm volatile("" : "+v"(lr2e[k]), "+v"(wl[k]), "+v"(wr[k]));
    double fmid[2];
    integrand_k<FID, 2, (f_scale<FID>() != 1.0), TABMASK>(mid, fmid, tab, kk, range_hint, out_mask);   // :188
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        s[k].fmid = fmid[k];
        if constexpr (doubled_areas<FID>()) {
            const double l2 = (fl[k] + fmid[k]) * wl[k];     // 2 * larea, :189
            const double r2 = (fmid[k] + fr[k]) * wr[k];     // 2 * rarea, :190
            s[k].area2 = l2 + r2;
            s[k].refine = fabs(s[k].area2 - lr2e[k]) > eps2;   // :191 (strict >)
        } else {
            const double lrarea = lr2e[k] / 2;                // :185
            const double larea = (fl[k] + fmid[k]) * wl[k] / 2;   // :189
            const double rarea = (fmid[k] + fr[k]) * wr[k] / 2;   // :190
            s[k].area2 = larea + rarea;                       // :199
            s[k].refine = fabs((larea + rarea) - lrarea) > eps2;   // :191
        }
    }
}

// pair_step_halves with the parent's doubled areas carried in (doubled-area integrands only). A child's
// lrarea (:185) is token for token its parent's larea / rarea (:189 / :190: the same F values and
// the same width m - a, b - m), so a pair that carries its parent's two products, lr0 = 2 larea and
// lr1 = 2 rarea of the task it came from, needs no (fl + fr) * (r - l) of its own: six FP64 fewer per
// pair. The children's values are each task's own l2 / r2, returned for the push.
struct Step2c {
    double fmid, l2, r2, area2;
    bool refine;
};
template <int FID>
__device__ __forceinline__ void pair_step_carry(double ha, double hb, double fa, double fm, double fb, double lr0,
                                                double lr1, double eps2, const ExpEntry* __restrict__ tab,
                                                Step2c (&s)[2], double& m, double& hm, const ExpConsts& kk,
                                                int range_hint, unsigned long long out_mask) {
    static_assert(doubled_areas<FID>(), "carried areas are doubled areas");
    m = ha + hb;                                             // the parent's midpoint (:187)
    hm = 0.5 * m;
    const double mid[2] = {ha + hm, hm + hb};                // :187 for [a, m] and [m, b]
    const double fl[2] = {fa, fm}, fr[2] = {fm, fb}, lr[2] = {lr0, lr1};
    double wl[2], wr[2];
    wl[0] = __fma_rn(ha, -2.0, mid[0]);                      // mid - l
    wl[1] = mid[1] - m;
    wr[0] = m - mid[0];                                      // r - mid
    wr[1] = __fma_rn(hb, 2.0, -mid[1]);
#pragma unroll
    for (int k = 0; k < 2; ++k) asm volatile("" : "+v"(wl[k]), "+v"(wr[k]));
    double fmid[2];
    integrand_k<FID, 2, (f_scale<FID>() != 1.0)>(mid, fmid, tab, kk, range_hint, out_mask);   // :188
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        s[k].fmid = fmid[k];
        s[k].l2 = (fl[k] + fmid[k]) * wl[k];                // 2 * larea, :189
        s[k].r2 = (fmid[k] + fr[k]) * wr[k];                // 2 * rarea, :190
        s[k].area2 = s[k].l2 + s[k].r2;
        s[k].refine = fabs(s[k].area2 - lr[k]) > eps2;      // :191 against the carried 2 * lrarea (:185)
    }
}

// Double-double (hi + lo) sums of the accepted areas: every leaf area enters a per-lane pair
// exactly (Knuth's TwoSum, six flops), the pairs reduce across the wave and the workers without
// rounding, and only the final hi + lo is rounded -- so the area is the correctly rounded sum of
// the leaf areas whatever the schedule (the order-dependent double sum of the farmer's
// `result += buff[0]`, :149, is within a few ulps of it).
__host__ __device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
    s = a + b;
    const double bb = s - a;
    e = (a - (s - bb)) + (b - bb);
}
__host__ __device__ __forceinline__ void dd_add(double& hi, double& lo, double v) {
    double s, e;
    two_sum(hi, v, s, e);
    hi = s;
    lo += e;
}
__host__ __device__ __forceinline__ void dd_add_dd(double& hi, double& lo, double h2, double l2) {
    double s, e;
    two_sum(hi, h2, s, e);
    e += lo + l2;
    two_sum(s, e, hi, lo);
}
// acc += v on the lanes of `mask` only: one exec-masked v_add_f64 instead of an add and a 64-bit
// select (two v_cndmask) per lane; lanes outside the mask keep their value.
__device__ __forceinline__ void masked_add(double& acc, double v, unsigned long long mask) {
    unsigned long long saved;
    asm("s_and_saveexec_b64 %1, %3\n\t"
        "v_add_f64 %0, %0, %2\n\t"
        "s_mov_b64 exec, %1"
        : "+v"(acc), "=&s"(saved)
        : "v"(v), "s"(mask)
        : "scc");
}

// m = max(m, v) on the lanes of `mask` only (one exec-masked v_max_u32).
__device__ __forceinline__ void masked_max(unsigned& m, unsigned v, unsigned long long mask) {
    unsigned long long saved;
    asm("s_and_saveexec_b64 %1, %3\n\t"
        "v_max_u32 %0, %0, %2\n\t"
        "s_mov_b64 exec, %1"
        : "+v"(m), "=&s"(saved)
        : "v"(v), "s"(mask)
        : "scc");
}

// The round's three masked accumulations in one exec window: hi += a0 on the lanes of l0m, hi += a1
// on l1m, m = max(m, low byte of v) on am -- exec saved once and restored once (5 SALU, not 6).
// Every mask is a ballot taken under the current exec, so each is a subset of it.
__device__ __forceinline__ void masked_acc3(double& hi, double a0, unsigned long long l0m, double a1,
                                            unsigned long long l1m, unsigned& m, unsigned v, unsigned long long am) {
    unsigned long long saved;
    asm("s_mov_b64 %1, exec\n\t"
        "s_mov_b64 exec, %5\n\t"
        "v_add_f64 %0, %0, %3\n\t"
        "s_mov_b64 exec, %6\n\t"
        "v_add_f64 %0, %0, %4\n\t"
        "s_mov_b64 exec, %7\n\t"
        "v_max_u32_sdwa %2, %2, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0\n\t"
        "s_mov_b64 exec, %1"
        : "+v"(hi), "=&s"(saved), "+v"(m)
        : "v"(a0), "v"(a1), "s"(l0m), "s"(l1m), "s"(am), "v"(v));
}

__device__ __forceinline__ void wave_sum_dd(double& hi, double& lo) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double h2 = __shfl_xor(hi, o, 64), l2 = __shfl_xor(lo, o, 64);
        dd_add_dd(hi, lo, h2, l2);
    }
}

// Full-wave reductions without LDS (every lane active): four DPP exchanges inside each row of 16
// lanes (quad_perm xor 1, xor 2, half-row mirror, row mirror) leave every lane holding its row's
// value, and the four rows combine through readlane. A __shfl_xor step is a ds_bpermute round trip
// through LDS; a wave's exit flush made ~36 of them back to back (~2 us of a lone-integral launch).
enum : int { DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140 };
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = dpp_u<CTRL>((unsigned)b), hi = dpp_u<CTRL>((unsigned)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double readlane_d(double v, int l) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l), hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <typename Op>
__device__ __forceinline__ unsigned wave_reduce_u(unsigned v, Op op) {
    v = op(v, dpp_u<DPP_XOR1>(v));
    v = op(v, dpp_u<DPP_XOR2>(v));
    v = op(v, dpp_u<DPP_HALF_MIRROR>(v));
    v = op(v, dpp_u<DPP_MIRROR>(v));
    return op(op(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
              op(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
__device__ __forceinline__ unsigned wave_add_full(unsigned v) {
    return wave_reduce_u(v, [](unsigned x, unsigned y) { return x + y; });
}
__device__ __forceinline__ unsigned wave_max_full(unsigned v) {
    return wave_reduce_u(v, [](unsigned x, unsigned y) { return x > y ? x : y; });
}
__device__ __forceinline__ unsigned wave_or_full(unsigned v) {
    return wave_reduce_u(v, [](unsigned x, unsigned y) { return x | y; });
}
// double-double sum over each row of 16 lanes (every lane active): every lane holds its row's sum
__device__ __forceinline__ void row_sum_dd(double& hi, double& lo) {
    double h2 = dpp_d<DPP_XOR1>(hi), l2 = dpp_d<DPP_XOR1>(lo);
    dd_add_dd(hi, lo, h2, l2);
    h2 = dpp_d<DPP_XOR2>(hi); l2 = dpp_d<DPP_XOR2>(lo);
    dd_add_dd(hi, lo, h2, l2);
    h2 = dpp_d<DPP_HALF_MIRROR>(hi); l2 = dpp_d<DPP_HALF_MIRROR>(lo);
    dd_add_dd(hi, lo, h2, l2);
    h2 = dpp_d<DPP_MIRROR>(hi); l2 = dpp_d<DPP_MIRROR>(lo);
    dd_add_dd(hi, lo, h2, l2);
}
// double-double sum over the wave (every lane active); the result is wave-uniform
__device__ __forceinline__ void wave_sum_dd_full(double& hi, double& lo) {
    double h2 = dpp_d<DPP_XOR1>(hi), l2 = dpp_d<DPP_XOR1>(lo);
    dd_add_dd(hi, lo, h2, l2);
    h2 = dpp_d<DPP_XOR2>(hi); l2 = dpp_d<DPP_XOR2>(lo);
    dd_add_dd(hi, lo, h2, l2);
    h2 = dpp_d<DPP_HALF_MIRROR>(hi); l2 = dpp_d<DPP_HALF_MIRROR>(lo);
    dd_add_dd(hi, lo, h2, l2);
    h2 = dpp_d<DPP_MIRROR>(hi); l2 = dpp_d<DPP_MIRROR>(lo);
    dd_add_dd(hi, lo, h2, l2);
    double h0 = readlane_d(hi, 0), l0 = readlane_d(lo, 0), h1 = readlane_d(hi, 16), l1 = readlane_d(lo, 16);
    double h3 = readlane_d(hi, 32), l3 = readlane_d(lo, 32);
    const double h4 = readlane_d(hi, 48), l4 = readlane_d(lo, 48);
    dd_add_dd(h0, l0, h1, l1);
    dd_add_dd(h3, l3, h4, l4);
    dd_add_dd(h0, l0, h3, l3);
    hi = h0;
    lo = l0;
}

// Wave-uniform values (readfirstlane). The persistent kernels' loops mix divergent regions with
// wave-level state; LLVM's uniformity analysis loses track of that state across the joins and would
// keep it in VGPRs, copied at every join. Re-asserting it once per iteration keeps it in SGPRs.
__device__ __forceinline__ unsigned uni(unsigned v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ unsigned long long uni(unsigned long long v) {
    return ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32)) << 32) |
           (unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)v);
}
__device__ __forceinline__ bool uni(bool v) { return __builtin_amdgcn_readfirstlane((unsigned)v) != 0u; }

__device__ __forceinline__ unsigned long long rtc() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ unsigned long long clk() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    return t;
}

// Write-through (sc1) global accesses for cross-CU hand-offs: the producer stores every payload
// byte sc1 and drains vmcnt before one lane's sc1 flag store; the consumer polls the flag and
// reads the payload with sc1 loads only (MI355X_MICROARCH.md, "Valid forms", row 1) -- no
// release / acquire fences, whose L2 write-back / invalidate cost microseconds.
__device__ __forceinline__ void st_wt(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load(
        reinterpret_cast<unsigned long long*>(const_cast<double*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ unsigned ld_wt(const unsigned* p) {
    return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int g_add(int* p, int v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned g_add(unsigned* p, unsigned v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned g_ld(unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int g_ld(int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace aq
