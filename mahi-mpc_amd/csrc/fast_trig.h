// fast_trig.h -- sin and cos of one fp64 argument for the model evaluations of the solver loops.
//
// The ROCm device library's fp64 sincos handles every finite argument (Payne-Hanek reduction for |x| >= 2^30 on a
// branch, then a two-constant reduction with compensated adds and polynomials whose coefficients are materialised
// by v_mov pairs): ~100 VALU instructions on the small-argument path of gfx950.  The exo model calls it 4 times per
// evaluation and the lane kernel evaluates the model 3 times per stage and SQP iteration, which made it ~13 % of the
// cfg#3 kernel's instructions.  The joint angles of an MPC iterate are far from 2^20, so this version reduces with
// an FMA Cody-Waite split of pi/2 in three parts (x - n pi/2 with one rounding per part, n = rint(x 2/pi)) and
// evaluates the fdlibm kernels (__kernel_sin / __kernel_cos, minimax on |r| <= pi/4, < 1 ulp) on the reduced
// argument: ~40 VALU instructions with the 16 constants read as scalar loads (s_load) from a constant table.
//
// Accuracy: |x| <= 2^20 pi/2: within 1 ulp of libm (absolute error <= 1.2e-16) in tests/test_fast_trig.py (random
// arguments up to 1.6e6 and the multiples of pi/2 up to 1e5 pi/2).  Beyond that the reduction would lose bits: the
// device build returns NaN there (only a diverging iterate gets that far; the solver then reports the instance
// non-finite; the oracle applies the same domain to its model evaluations, oracle/mmpc_oracle.c kTrigDomain), the host
// build switches to libm (NaN and inf too, so the host never converts a NaN quadrant to int).  The quadrant is formed
// without an out-of-range int conversion for every finite x.  NaN and +-inf give NaN, as the device library.
#pragma once
#include <math.h>

#ifndef MMPC_TRIG_FN
#if defined(__HIPCC__)
#define MMPC_TRIG_FN __device__ __forceinline__
#else
#define MMPC_TRIG_FN inline   // host builds of the model headers (oracle/builtin_hess_host.cpp, tests)
#endif
#endif

namespace mmpc {

// 2/pi, pi/2 in three parts (C1 + C2 + C3 = pi/2 to 160 bits), fdlibm S1..S6, C1..C6
#define MMPC_TRIG_CONSTANTS                                                                                        \
    {0.63661977236758134308, 1.5707963267948966, 6.123233995736766e-17, -1.4973849048591698e-33,                 \
     -1.66666666666666324348e-01, 8.33333333332248946124e-03, -1.98412698298579493134e-04,                       \
     2.75573137070700676789e-06, -2.50507602534068634195e-08, 1.58969099521155010221e-10,                        \
     4.16666666666666019037e-02, -1.38888888888741095749e-03, 2.48015872894767294178e-05,                        \
     -2.75573143513906633035e-07, 2.08757232129817482790e-09, -1.13596475577881948265e-11}

#if defined(__HIPCC__)
__constant__ double kTrigConst[16] = MMPC_TRIG_CONSTANTS;
using trig_cptr = __attribute__((address_space(4))) const double*;
// opaque per call (as exo::coef_table): the constants are loaded at their uses, not hoisted out of the solver loops
// into SGPRs that spill
__device__ __forceinline__ trig_cptr trig_table() {
    trig_cptr K = (trig_cptr)kTrigConst;
    asm volatile("" : "+s"(K));
    return K;
}
#else
static const double kTrigConst[16] = MMPC_TRIG_CONSTANTS;
using trig_cptr = const double*;
inline trig_cptr trig_table() { return kTrigConst; }
#endif
#undef MMPC_TRIG_CONSTANTS

// s = sin x, c = cos x; K = trig_table() (one table pointer may serve several calls of one evaluation)
MMPC_TRIG_FN void sincos_fast(trig_cptr K, double x, double* s, double* c) {
#if !defined(__HIPCC__) && !defined(MMPC_TRIG_DEVICE_PATH_ON_HOST)
    if (!(fabs(x) <= 1647099.3291652855)) {   // beyond 2^20 pi/2, and NaN / inf: the host build (checks) uses libm
        *s = sin(x);
        *c = cos(x);
        return;
    }
#endif
    const double n = rint(x * K[0]);
    double r = fma(-n, K[1], x);
    r = fma(-n, K[2], r);
    r = fma(-n, K[3], r);
    // beyond 2^20 pi/2 the reduction loses bits: the result is made NaN (one compare and select, no branch), so the
    // solver reports such an iterate non-finite instead of continuing with inaccurate trig values
    r = fabs(x) <= 1647099.3291652855 ? r : __builtin_nan("");
    const double z = r * r;
    // __kernel_sin(r, 0): r + r^3 (S1 + z (S2 + ... + z S6))
    const double ps = fma(z, fma(z, fma(z, fma(z, K[9], K[8]), K[7]), K[6]), K[5]);
    const double sr = fma(z * r, fma(z, ps, K[4]), r);
    // __kernel_cos(r, 0): w + (((1 - w) - z/2) + z^2 (C1 + ... + z^5 C6)),  w = 1 - z/2
    const double pc = z * fma(z, fma(z, fma(z, fma(z, fma(z, K[15], K[14]), K[13]), K[12]), K[11]), K[10]);
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + z * pc);
    // quadrant n mod 4: sin = (sr, cr, -sr, -cr), cos = (cr, -sr, -cr, sr).  n mod 4 is formed in double (every step
    // exact for |n| < 2^53), so the int conversion sees 0..3 for any finite x: no out-of-range conversion (undefined
    // behaviour on the host, saturation on the device) however large a diverging iterate gets
    const int q = (int)fma(-4.0, floor(0.25 * n), n);
    const bool odd = (q & 1) != 0;
    const double a = odd ? cr : sr, b = odd ? sr : cr;
    *s = (q & 2) ? -a : a;
    *c = ((q + 1) & 2) ? -b : b;
}

}  // namespace mmpc
