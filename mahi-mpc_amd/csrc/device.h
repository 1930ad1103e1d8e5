// device.h -- the qualifier of the device model and solver helpers (inlined into the kernels).
#pragma once
#include <hip/hip_runtime.h>

#define MMPC_HD __device__ __forceinline__

// sqrt(a) and 1/sqrt(a) of a positive normal fp64 number: the hardware reciprocal square root refined by one coupled
// Goldschmidt step and one Newton step for each result (LLVM's own f64 sqrt expansion uses the same refinement plus
// range scaling and special-value fix-ups): 11 VALU instructions instead of a correctly rounded sqrt (~21) and a
// division (~11).  sqrt within 0.5 ulp, 1/sqrt within 1.5 ulp in a host simulation with an initial error up to
// 3e-7; a <= 0 or non-finite gives NaN / inf, which the callers' factorisation checks (s > 0, isfinite) reject first.
MMPC_HD void sqrt_rsqrt(double a, double& sq, double& rs) {
    const double y = __builtin_amdgcn_rsq(a);
    double g = a * y, hh = 0.5 * y;
    const double r = fma(-hh, g, 0.5);
    g = fma(g, r, g);
    hh = fma(hh, r, hh);
    g = fma(fma(-g, g, a), hh, g);
    const double r0 = hh + hh;
    sq = g;
    rs = fma(r0, fma(-g, r0, 1.0), r0);
}
