// aq_user_gauss.h -- the default AQ_F_USER plug-in (and the template for writing one).
//
// The reference's extension point is its integrand macro, `#define F(arg) cosh(arg)*...`
// (/root/reference/aquadPartA.c:46). This plug-in is that macro with the body
//     #define F(arg) exp(-(arg)*(arg))
// -- the Gaussian -- evaluated exactly as the reference binary built with that line evaluates it:
// (-x)*x rounded once, then glibc 2.35 exp (aq::exp_glibc_any, the FMA ifunc form, bit-exact).
// tests/golden/trees.json holds the reference binary's own output for it (oracle/Makefile builds
// the variant by substituting line 46).
//
// To plug in another integrand, copy this file, change name / F / domain_ok, and rebuild:
//     PPLS_AMD_USER_F=/path/to/my_f.h python ppls_amd/build.py --force
// F runs on the GPU inside the persistent kernels; it may call aq::exp_glibc_any, aq::cosh_glibc
// (both take the LDS exp table `tab`) and the device libm (faithful, not glibc-exact).
#pragma once

namespace aq {
namespace user {

constexpr const char* name = "gauss: exp(-(arg)*(arg))";

__device__ __forceinline__ double F(double x, const ExpEntry* __restrict__ tab) {
    return exp_glibc_any(-x * x, tab);   // unary minus first, as the macro expands: (-(arg))*(arg)
}

// Any finite interval: exp(-x*x) is in [0, 1] (underflowing to 0 beyond |x| ~ 27.3), so no area
// can overflow.
inline bool domain_ok(double a, double b) { return a >= -1e150 && b <= 1e150; }

}  // namespace user
}  // namespace aq
