// models.h -- built-in device dynamics x_dot = f(x, u).
//
// The reference takes f as a casadi::SX expression supplied by the caller of
// ModelGenerator (include/Mahi/Mpc/ModelGenerator.hpp:23) and code-generates it
// to C (ModelGenerator.cpp:235-259).  Here each model is a device template over
// the scalar type (double or Dual<NX+NU>), compiled into the solver kernel.
#pragma once
#include "dual.h"

namespace mmpc {

// 2-link planar arm / double pendulum of examples/ex_model_generate.cpp:24-43
// (L = m = 1, g = 9.81), state [qA, qB, qA_dot, qB_dot], control [TA, TB].
// The two accelerations restate :36-37 term by term.
struct TwoLinkArm {
    static constexpr int NX = 4;
    static constexpr int NU = 2;

    template <class T>
    MMPC_HD static void xdot(const T* x, const T* u, T* xd) {
        constexpr double L = 1.0, m = 1.0, g = 9.81;
        constexpr double LLm = L * L * m, Lgm = L * g * m;
        const T qA = x[0], qB = x[1], dA = x[2], dB = x[3], TA = u[0], TB = u[1];
        T sB, cB;
        mm_sincos(qB, sB, cB);
        const T cA = mm_cos(qA);
        const T cAB = mm_cos(qA + qB);
        const T dA2 = dA * dA, dB2 = dB * dB, dAdB = dA * dB, cBsB = cB * sB;
        const T inv_den = 1.0 / (LLm * (cB * cB - 2.0));
        const T nA = TA - TB - TB * cB + LLm * (dA2 * sB) + LLm * (dB2 * sB) - (2.0 * Lgm) * cA
                     + LLm * (dA2 * cBsB) + (2.0 * LLm) * (dAdB * sB) + Lgm * (cAB * cB);
        const T nB = TA - 3.0 * TB + TA * cB - 2.0 * (TB * cB) + (2.0 * Lgm) * cAB
                     + (3.0 * LLm) * (dA2 * sB) + LLm * (dB2 * sB) - (2.0 * Lgm) * cA
                     + (2.0 * LLm) * (dA2 * cBsB) + LLm * (dB2 * cBsB) - (2.0 * Lgm) * (cA * cB)
                     + (2.0 * LLm) * (dAdB * sB) + Lgm * (cAB * cB) + (2.0 * LLm) * (dAdB * cBsB);
        xd[0] = dA;
        xd[1] = dB;
        xd[2] = -(nA * inv_den);
        xd[3] = nB * inv_den;
    }
};

// Values and continuous-time Jacobians of any model: fx[NX*NX], fu[NX*NU] row-major.
template <class Model>
MMPC_HD void model_eval_jac(const double* x, const double* u, double* xd, double* fx, double* fu) {
    constexpr int NX = Model::NX, NU = Model::NU, K = NX + NU;
    Dual<K> xv[NX], uv[NU], xdv[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) xv[i] = dual_var<K>(x[i], i);
#pragma unroll
    for (int i = 0; i < NU; ++i) uv[i] = dual_var<K>(u[i], NX + i);
    Model::template xdot<Dual<K>>(xv, uv, xdv);
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        xd[r] = xdv[r].v;
#pragma unroll
        for (int c = 0; c < NX; ++c) fx[r * NX + c] = xdv[r].d[c];
#pragma unroll
        for (int c = 0; c < NU; ++c) fu[r * NU + c] = xdv[r].d[NX + c];
    }
}

template <class Model>
MMPC_HD void model_eval(const double* x, const double* u, double* xd) {
    Model::template xdot<double>(x, u, xd);
}

}  // namespace mmpc
