"""ppls_amd -- MI355X-native adaptive trapezoid quadrature (the hot path of taithenguyen/ppls).

The reference program (/root/reference/aquadPartA.c) integrates F(x)=cosh(x)^4 over [A,B] with an
MPI farmer/worker bag of tasks. This package is a drop-in for that path: the same F/A/B/EPSILON,
the same accepted-interval count, area and `Area=` / `Tasks Per Process` printout, computed by
hand-written HIP kernels for gfx950 behind the C ABI in include/aquad.h.
"""
from .aquad import (  # noqa: F401
    COSH4,
    SIN_RECIP,
    USER,
    AquadError,
    Context,
    Group,
    Problem,
    Result,
    exact_round,
    farmer,
    format_reference,
    integrate,
    user_integrand_name,
)

__all__ = ["COSH4", "SIN_RECIP", "USER", "AquadError", "Context", "Group", "Problem", "Result", "exact_round",
           "farmer", "format_reference", "integrate", "user_integrand_name"]
