// aq_xsum.h -- exact (order-independent) sums of doubles: the per-integral area accumulator.
//
// The reference sums accepted areas serially in arrival order, `result += buff[0]`
// (/root/reference/aquadPartA.c:149), so its last bits depend on the MPI schedule. Here every
// partial enters a fixed-point accumulator that holds the EXACT sum of everything added to it:
// XS_LIMBS signed 64-bit limbs, limb i weighing 2^(32 i + XS_E0). A double x = +-m 2^p (53-bit m)
// is split into three 32-bit digits added to three consecutive limbs, so a limb moves by less than
// 2^32 per addition and holds 2^31 additions before it could overflow. Integer addition is
// associative: partials can be added from any wave, in any order, by device atomics or limb-wise
// collectives (int64 ncclSum), and the result is bit-identical. xs_round() returns the correctly
// rounded (nearest-even) double of the exact sum.
//
// The whole double range is covered (2^-1074 .. 2^1024 plus carry headroom): 68 limbs = 544 B per
// integral slot, against 48 KiB of per-wave double-double partials before.
//
// Plain C++ (host and device): the CPU tests compile this header with g++ (tests/test_xsum.py).
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define AQ_HD __host__ __device__ __forceinline__
#else
#define AQ_HD inline
#endif

namespace aq {

constexpr int XS_LIMBS = 68;     // 32 * 68 = 2176 bits from 2^-1088: every finite double, + 2^64 headroom
constexpr int XS_E0 = -1088;     // weight of limb 0's lowest bit (a multiple of 32, <= -1074)

struct XSum {
    long long limb[XS_LIMBS];
};

// The three digit additions that add x: limbs i, i+1, i+2 get d[0], d[1], d[2] (signed). Returns
// false for x == 0 (nothing to add). Non-finite x must not be passed (callers add finite areas).
struct XDigits {
    int i;
    long long d[3];
};
AQ_HD bool xs_digits(double x, XDigits& out) {
    uint64_t u;
    memcpy(&u, &x, 8);
    const unsigned e = (unsigned)(u >> 52) & 0x7ffu;
    uint64_t m = u & ((1ull << 52) - 1ull);
    int p;
    if (e == 0) {
        if (m == 0) return false;
        p = -1074;
    } else {
        m |= 1ull << 52;
        p = (int)e - 1075;
    }
    const int q = p - XS_E0;              // >= 14
    const int s = q & 31;
    out.i = q >> 5;
    const uint64_t lo = m << s;           // low 64 bits of m * 2^s (m < 2^53, s < 32: < 2^85)
    const uint64_t hi = s ? (m >> (64 - s)) : 0ull;
    const long long sg = (u >> 63) ? -1 : 1;
    out.d[0] = sg * (long long)(lo & 0xffffffffull);
    out.d[1] = sg * (long long)(lo >> 32);
    out.d[2] = sg * (long long)hi;
    return true;
}

// Host / single-threaded addition.
AQ_HD void xs_add(XSum& a, double x) {
    XDigits g;
    if (!xs_digits(x, g)) return;
    for (int k = 0; k < 3; ++k) a.limb[g.i + k] += g.d[k];
}

AQ_HD void xs_add_xs(XSum& a, const XSum& b) {
    for (int i = 0; i < XS_LIMBS; ++i) a.limb[i] += b.limb[i];
}

// Correctly rounded (round-to-nearest-even) double of the exact sum of n <= N limbs, limb 0 weighing
// 2^e0: the whole accumulator (N = n = XS_LIMBS, e0 = XS_E0), or a window of it that holds every
// nonzero limb (the batch gather reads only a slot's touched limbs: SlotSums' limb window) -- the
// value, and so its rounding, does not depend on the zero limbs around the window.
template <int N>
AQ_HD double xs_round_span(const long long* limb, int n, int e0) {
    // carry-propagate into base-2^32 digits of the two's complement value
    uint32_t dg[N + 2];
    long long carry = 0;
    for (int i = 0; i < n; ++i) {
        // v = limb + carry cannot overflow: |limb| < 2^63 - 2^33 by the addition budget, |carry| < 2^32
        const long long v = limb[i] + carry;
        dg[i] = (uint32_t)((unsigned long long)v & 0xffffffffull);
        carry = v >> 32;                   // arithmetic shift: floor division
    }
    // carry is now the sign extension (0 or -1 for any representable total)
    const bool neg = carry < 0;
    dg[n] = (uint32_t)carry;
    dg[n + 1] = (uint32_t)(carry >> 32);
    const int nd = n + 2;
    if (neg) {   // magnitude = two's complement negation
        unsigned long long c = 1;
        for (int i = 0; i < nd; ++i) {
            const unsigned long long v = (unsigned long long)(uint32_t)~dg[i] + c;
            dg[i] = (uint32_t)v;
            c = v >> 32;
        }
    }
    int t = nd - 1;
    while (t >= 0 && dg[t] == 0u) --t;
    if (t < 0) return 0.0;
    int lz = 0;
    for (uint32_t v = dg[t]; !(v & 0x80000000u); v <<= 1) ++lz;
    const int b = 32 * t + 31 - lz;        // bit index of the leading one
    const int e = b + e0;               // its binary exponent
    if (e > 1023) return neg ? -__builtin_inf() : __builtin_inf();
    int keep = 53;
    if (e < -1022) keep = e + 1075;        // subnormal: bits down to 2^-1074 (>= 1: the sum is a multiple of 2^-1074)
    const int low = b - keep + 1;          // lowest kept bit
    auto bit = [&](int k) -> unsigned { return k < 0 ? 0u : (dg[k >> 5] >> (k & 31)) & 1u; };
    uint64_t M = 0;
    for (int k = b; k >= low; --k) M = (M << 1) | bit(k);
    const unsigned rb = bit(low - 1);
    bool sticky = false;                   // any one bit below the rounding bit
    if (low - 2 >= 0) {
        const int k = low - 2, w = k >> 5;
        const uint32_t mask = (k & 31) == 31 ? 0xffffffffu : ((1u << ((k & 31) + 1)) - 1u);
        sticky = (dg[w] & mask) != 0u;
        for (int j = w - 1; j >= 0 && !sticky; --j) sticky = dg[j] != 0u;
    }
    if (rb && (sticky || (M & 1ull))) ++M;
    int ex = low + e0;                  // M * 2^ex
    if (M >> keep) {                       // rounding carried into a new bit
        M >>= 1;
        ++ex;
        if (keep == 53 && ex + 52 > 1023) return neg ? -__builtin_inf() : __builtin_inf();
    }
    // M < 2^53: scale exactly by powers of two (two steps keep every factor a normal double)
    double r = (double)M;
    int ex1 = ex / 2, ex2 = ex - ex / 2;
    auto pow2 = [](int k) -> double {
        uint64_t bits = (uint64_t)(k + 1023) << 52;
        double d;
        memcpy(&d, &bits, 8);
        return d;
    };
    r = r * pow2(ex1) * pow2(ex2);
    return neg ? -r : r;
}

AQ_HD double xs_round(const XSum& a) { return xs_round_span<XS_LIMBS>(a.limb, XS_LIMBS, XS_E0); }

// The limbs a value's digits touch, as a window [lo, hi) folded by max (so an all-zero pair of words
// is the empty window): lo_not = ~lo, hi = last + 1. Kept per slot beside its sums.
AQ_HD unsigned xs_win_lo(int i) { return ~(unsigned)i; }
AQ_HD unsigned xs_win_hi(int i) { return (unsigned)i + 3u; }

}  // namespace aq
