// models.h -- built-in device dynamics x_dot = f(x, u).
//
// The reference takes f as a casadi::SX expression supplied by the caller of
// ModelGenerator (include/Mahi/Mpc/ModelGenerator.hpp:23) and code-generates it
// to C (ModelGenerator.cpp:235-259).  Here each built-in model is a device struct with closed-form values and
// derivatives (eval, eval_acc_jac, eval_jac, eval_hess), compiled into the solver kernels; SX-generated models
// (host/src/ModelGenerator.cpp) emit the same interface.
#pragma once
#include <type_traits>

#include "device.h"
#include "exo_model_gen.h"
#include "two_link_fast.h"

namespace mmpc {

// 2-link planar arm / double pendulum of examples/ex_model_generate.cpp:24-43
// (L = m = 1, g = 9.81), state [qA, qB, qA_dot, qB_dot], control [TA, TB].
// Values, Jacobian and the weighted Hessian come from the closed form of two_link_fast.h (one sincos per
// angle, quotient rule); the oracle restates :36-37 term by term (tests/test_sx_models.py compares the two).
struct TwoLinkArm {
    static constexpr int NX = 4;
    static constexpr int NU = 2;
    static constexpr int NQ = 2;  // second-order: x = [q; qd], xdot = [qd; acc(x, u)]
    MMPC_HD static void eval(const double* x, const double* u, double* xd) { TwoLinkFast::eval(x, u, xd); }
    MMPC_HD static void eval_jac(const double* x, const double* u, double* xd, double* fx, double* fu) {
        double Fq[4], Fqd[4], Fu[4];
        TwoLinkFast::eval_acc_jac(x, u, xd + 2, Fq, Fqd, Fu);
        xd[0] = x[2];
        xd[1] = x[3];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
#pragma unroll
            for (int c = 0; c < 4; ++c) fx[r * 4 + c] = (c == 2 + r) ? 1.0 : 0.0;
            fu[r * 2] = fu[r * 2 + 1] = 0.0;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                fx[(2 + r) * 4 + c] = Fq[r * 2 + c];
                fx[(2 + r) * 4 + 2 + c] = Fqd[r * 2 + c];
                fu[(2 + r) * 2 + c] = Fu[r * 2 + c];
            }
        }
    }
    // acceleration and its partials d acc/dq [NQ*NQ], d acc/dqd [NQ*NQ], d acc/du [NQ*NU] (row-major)
    MMPC_HD static void eval_acc_jac(const double* x, const double* u, double* acc, double* Fq, double* Fqd,
                                     double* Fu) {
        TwoLinkFast::eval_acc_jac(x, u, acc, Fq, Fqd, Fu);
    }
    // W = sum_s lam[s] d^2 acc_s / d(x, u)^2 (6 x 6 row-major): the dynamics part of the Lagrangian Hessian
    // (CasADi nlp_hess_l, ModelGenerator.cpp:238)
    static constexpr bool kHasHess = true;
    MMPC_HD static void eval_hess(const double* x, const double* u, const double* lam, double* W) {
        TwoLinkFast::eval_hess(x, u, lam, W);
    }
    // acc is affine in the torques (acc = M(q)^-1 (T - ...)), so the u-u block of every W is exactly zero
    static constexpr bool kControlAffine = true;
};

// Second derivatives available (Model::eval_hess): exact-Hessian SQP and mmpc_nlp_hess_batch
template <class M, class = void>
struct HasHess {
    static constexpr bool value = false;
};
template <class M>
struct HasHess<M, std::enable_if_t<M::kHasHess>> {
    static constexpr bool value = true;
};
// Dynamics affine in u (d^2 acc / du^2 == 0): the exact-Hessian sweep skips the u-u block of W_k, which is zero
template <class M, class = void>
struct IsControlAffine {
    static constexpr bool value = false;
};
template <class M>
struct IsControlAffine<M, std::enable_if_t<M::kControlAffine>> {
    static constexpr bool value = true;
};

// Directional derivative without the Jacobian (Model::eval_jvp): the lane kernel's step sweep only needs
// A_k dx_k + B_k du_k and the trial's A d, not the blocks of A_k, B_k
template <class M, class = void>
struct HasJvp {
    static constexpr bool value = false;
};
template <class M>
struct HasJvp<M, std::enable_if_t<M::kHasJvp>> {
    static constexpr bool value = true;
};
// Jacobian blocks already scaled by the step h (Model::eval_acc_jac_h)
template <class M, class = void>
struct HasJacH {
    static constexpr bool value = false;
};
template <class M>
struct HasJacH<M, std::enable_if_t<M::kHasJacH>> {
    static constexpr bool value = true;
};
template <class M>
MMPC_HD void model_acc_jac_h(const double* x, const double* u, double h, double* acc, double* hFq, double* hFqd,
                             double* hFu) {
    if constexpr (HasJacH<M>::value) M::eval_acc_jac_h(x, u, h, acc, hFq, hFqd, hFu);   // callers test HasJacH first
}
template <class M>
MMPC_HD void model_jvp(const double* x, const double* u, const double* vx, const double* vu, double* xd, double* jv) {
    if constexpr (HasJvp<M>::value) M::eval_jvp(x, u, vx, vu, xd, jv);   // callers test HasJvp first
}

// 4-DoF forearm/wrist exo, state [q0..q3, qd0..qd3] (util/testCorrectEquations.py:16-23),
// control tau[4].  xdot = [qd; M(q)^-1 (tau - D qd - G(q))] with M(q) of src/inverseTest.cpp:59-74
// (generated, exo_model_gen.h) and the build-defined gravity G_i = g_i sin q_i and viscous damping D of
// tests/golden/exo_params.json -- the reference defines neither, so these are NOT reference-pinned.
// M^-1 is applied through a 4x4 Cholesky factor; the Jacobian is analytic:
//   d qdd / dq_j   = M^-1 (-dM/dq_j qdd - dG/dq_j e_j),  d qdd / dqd = -M^-1 D,  d qdd / dtau = M^-1,
// with dM/dq_j from the generated symbolic-derivative polynomials.
struct ExoArm {
    static constexpr int NX = 8;
    static constexpr int NU = 4;
    static constexpr int NQ = 4;  // second-order: x = [q; qd], xdot = [qd; acc(x, u)]

    // Cholesky of the upper-packed SPD matrix a (M00 M01 M02 M03 M11 M12 M13 M22 M23 M33):
    // l = lower factor packed (L00 L10 L11 L20 L21 L22 L30 L31 L32 L33), il = 1 / diag (sqrt_rsqrt: no division)
    MMPC_HD static void chol4(const double* a, double* l, double* il) {
        sqrt_rsqrt(a[0], l[0], il[0]);
        l[1] = a[1] * il[0];
        l[3] = a[2] * il[0];
        l[6] = a[3] * il[0];
        sqrt_rsqrt(a[4] - l[1] * l[1], l[2], il[1]);
        l[4] = (a[5] - l[3] * l[1]) * il[1];
        l[7] = (a[6] - l[6] * l[1]) * il[1];
        sqrt_rsqrt(a[7] - l[3] * l[3] - l[4] * l[4], l[5], il[2]);
        l[8] = (a[8] - l[6] * l[3] - l[7] * l[4]) * il[2];
        sqrt_rsqrt(a[9] - l[6] * l[6] - l[7] * l[7] - l[8] * l[8], l[9], il[3]);
    }
    // y = (L L^T)^-1 b
    MMPC_HD static void chol4_solve(const double* l, const double* il, const double* b, double* y) {
        const double z0 = b[0] * il[0];
        const double z1 = (b[1] - l[1] * z0) * il[1];
        const double z2 = (b[2] - l[3] * z0 - l[4] * z1) * il[2];
        const double z3 = (b[3] - l[6] * z0 - l[7] * z1 - l[8] * z2) * il[3];
        y[3] = z3 * il[3];
        y[2] = (z2 - l[8] * y[3]) * il[2];
        y[1] = (z1 - l[4] * y[2] - l[7] * y[3]) * il[1];
        y[0] = (z0 - l[1] * y[1] - l[3] * y[2] - l[6] * y[3]) * il[0];
    }

    MMPC_HD static void eval(const double* x, const double* u, double* xd) {
        double s[4], c[4];
        const trig_cptr TK = trig_table();
#pragma unroll
        for (int i = 0; i < 4; ++i) sincos_fast(TK, x[i], &s[i], &c[i]);
        const exo::TrigPowers tp(c[1], c[2], c[3], s[1], s[2], s[3]);
        double Mu[10];
        exo::mass_upper(tp, Mu);
        double l[10], il[4], w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = u[i] - exo::kDamping[i] * x[4 + i] - exo::kGravityGain[i] * s[i];
        chol4(Mu, l, il);
#pragma unroll
        for (int i = 0; i < 4; ++i) xd[i] = x[4 + i];
        chol4_solve(l, il, w, xd + 4);
    }

    // (dM/dq_J) v for the upper-packed symmetric dM/dq_J
    template <int J>
    MMPC_HD static void dmass_times(const exo::TrigPowers& tp, const double* v, double* out) {
        double dM[10];
        exo::dmass_upper<J>(tp, dM);
        out[0] = fma(dM[0], v[0], fma(dM[1], v[1], fma(dM[2], v[2], dM[3] * v[3])));
        out[1] = fma(dM[1], v[0], fma(dM[4], v[1], fma(dM[5], v[2], dM[6] * v[3])));
        out[2] = fma(dM[2], v[0], fma(dM[5], v[1], fma(dM[7], v[2], dM[8] * v[3])));
        out[3] = fma(dM[3], v[0], fma(dM[6], v[1], fma(dM[8], v[2], dM[9] * v[3])));
    }

    // acceleration and its partials d qdd/dq [4x4], d qdd/dqd [4x4], d qdd/dtau [4x4] (row-major)
    MMPC_HD static void eval_acc_jac(const double* x, const double* u, double* qdd, double* Fq, double* Fqd,
                                     double* Fu) {
        double s[4], c[4];
        const trig_cptr TK = trig_table();
#pragma unroll
        for (int i = 0; i < 4; ++i) sincos_fast(TK, x[i], &s[i], &c[i]);
        const exo::TrigPowers tp(c[1], c[2], c[3], s[1], s[2], s[3]);
        double Mu[10], l[10], il[4], w[4];
        exo::mass_upper(tp, Mu);
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = u[i] - exo::kDamping[i] * x[4 + i] - exo::kGravityGain[i] * s[i];
        chol4(Mu, l, il);
        chol4_solve(l, il, w, qdd);
        // M^-1 (symmetric) = d qdd/dtau
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            double e[4] = {0.0, 0.0, 0.0, 0.0}, col[4];
            e[j] = 1.0;
            chol4_solve(l, il, e, col);
#pragma unroll
            for (int r = 0; r < 4; ++r) Fu[r * 4 + j] = col[r];
        }
        // d qdd/dq_j = M^-1 (-(dM/dq_j) qdd - g_j cos q_j e_j);  d qdd/dqd_j = -M^-1 e_j D_j
        double rhs[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r) rhs[0][r] = 0.0;
        dmass_times<1>(tp, qdd, rhs[1]);
        dmass_times<2>(tp, qdd, rhs[2]);
        dmass_times<3>(tp, qdd, rhs[3]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
            for (int r = 0; r < 4; ++r) rhs[j][r] = -rhs[j][r];
            rhs[j][j] -= exo::kGravityGain[j] * c[j];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double t = 0.0;
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) t = fma(Fu[r * 4 + cc], rhs[j][cc], t);
                Fq[r * 4 + j] = t;
                Fqd[r * 4 + j] = -Fu[r * 4 + j] * exo::kDamping[j];
            }
        }
    }

    // xd = f(x, u) and jv = d qdd / d(x, u) . (vq, vqd, vu) (vx = [vq; vqd]) without forming the Jacobian:
    // differentiating M qdd = tau - D qd - G(q) along the direction, M jv = vu - D vqd - g cos(q) vq - sum_j vq_j (dM/dq_j) qdd
    // (q0 does not enter M): one more Cholesky solve instead of M^-1's four, no 4x4x4 product, no h-scaled blocks
    static constexpr bool kHasJvp = true;
    MMPC_HD static void eval_jvp(const double* x, const double* u, const double* vx, const double* vu, double* xd,
                                 double* jv) {
        double s[4], c[4];
        const trig_cptr TK = trig_table();
#pragma unroll
        for (int i = 0; i < 4; ++i) sincos_fast(TK, x[i], &s[i], &c[i]);
        const exo::TrigPowers tp(c[1], c[2], c[3], s[1], s[2], s[3]);
        double Mu[10], l[10], il[4], w[4];
        exo::mass_upper(tp, Mu);
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = u[i] - exo::kDamping[i] * x[4 + i] - exo::kGravityGain[i] * s[i];
        chol4(Mu, l, il);
#pragma unroll
        for (int i = 0; i < 4; ++i) xd[i] = x[4 + i];
        double* const qdd = xd + 4;
        chol4_solve(l, il, w, qdd);
        double r[4], t1[4], t2[4], t3[4];
        dmass_times<1>(tp, qdd, t1);
        dmass_times<2>(tp, qdd, t2);
        dmass_times<3>(tp, qdd, t3);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            double t = fma(-exo::kDamping[i], vx[4 + i], vu[i]);
            t = fma(-exo::kGravityGain[i] * c[i], vx[i], t);
            t = fma(-vx[1], t1[i], t);
            t = fma(-vx[2], t2[i], t);
            r[i] = fma(-vx[3], t3[i], t);
        }
        chol4_solve(l, il, r, jv);
    }

    // eval_acc_jac with the blocks already scaled by h (hFq = h d qdd/dq, hFqd, hFu), the form the Riccati kernels
    // use: M^-1 = L^-T L^-1 from the inverse Cholesky factor (no solves against unit vectors, whose zeros are not
    // folded) with h folded into one factor (no scaling pass over the 48 entries)
    static constexpr bool kHasJacH = true;
    MMPC_HD static void eval_acc_jac_h(const double* x, const double* u, double h, double* qdd, double* hFq,
                                       double* hFqd, double* hFu) {
        double s[4], c[4];
        const trig_cptr TK = trig_table();
#pragma unroll
        for (int i = 0; i < 4; ++i) sincos_fast(TK, x[i], &s[i], &c[i]);
        const exo::TrigPowers tp(c[1], c[2], c[3], s[1], s[2], s[3]);
        double Mu[10], l[10], il[4], w[4];
        exo::mass_upper(tp, Mu);
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = u[i] - exo::kDamping[i] * x[4 + i] - exo::kGravityGain[i] * s[i];
        chol4(Mu, l, il);
        chol4_solve(l, il, w, qdd);
        // Li = L^-1 (lower), l packed as chol4's L00 L10 L11 L20 L21 L22 L30 L31 L32 L33
        double Li[4][4];
        Li[0][0] = il[0];
        Li[1][1] = il[1];
        Li[2][2] = il[2];
        Li[3][3] = il[3];
        Li[1][0] = -(l[1] * Li[0][0]) * il[1];
        Li[2][1] = -(l[4] * Li[1][1]) * il[2];
        Li[2][0] = -fma(l[3], Li[0][0], l[4] * Li[1][0]) * il[2];
        Li[3][2] = -(l[8] * Li[2][2]) * il[3];
        Li[3][1] = -fma(l[7], Li[1][1], l[8] * Li[2][1]) * il[3];
        Li[3][0] = -fma(l[6], Li[0][0], fma(l[7], Li[1][0], l[8] * Li[2][0])) * il[3];
        // h M^-1 = Li^T (h Li): entry (i, j) sums over the rows k >= max(i, j)
        double hLi[4][4], hMi[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int j = 0; j <= k; ++j) hLi[k][j] = h * Li[k][j];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = i; j < 4; ++j) {
                double t = Li[j][i] * hLi[j][j];
#pragma unroll
                for (int k = j + 1; k < 4; ++k) t = fma(Li[k][i], hLi[k][j], t);
                hMi[i][j] = t;
                hMi[j][i] = t;
            }
        // h d qdd/dq_j = h M^-1 (-(dM/dq_j) qdd - g_j cos q_j e_j) (dM/dq_0 = 0);  h d qdd/dqd_j = -h M^-1 e_j D_j
        double t1[4], t2[4], t3[4];
        dmass_times<1>(tp, qdd, t1);
        dmass_times<2>(tp, qdd, t2);
        dmass_times<3>(tp, qdd, t3);
        const double* const tj[4] = {nullptr, t1, t2, t3};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            hFq[r * 4] = hMi[r][0] * (-exo::kGravityGain[0] * c[0]);
#pragma unroll
            for (int j = 1; j < 4; ++j) {
                double t = hMi[r][j] * (-exo::kGravityGain[j] * c[j]);
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) t = fma(-hMi[r][cc], tj[j][cc], t);
                hFq[r * 4 + j] = t;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                hFu[r * 4 + j] = hMi[r][j];
                hFqd[r * 4 + j] = -hMi[r][j] * exo::kDamping[j];
            }
        }
    }

    // W = sum_s lam[s] d^2 acc_s / d(x, u)^2 (12 x 12 row-major over z = (q, qd, tau)): the dynamics part of the
    // Lagrangian Hessian (CasADi nlp_hess_l, ModelGenerator.cpp:238).  Differentiating M acc = w (w = tau - D qd -
    // G(q)) twice, with mu = M^-1 lam, rho_i = M^-1 (dM/dq_i) mu and beta_j = (dM/dq_j) acc:
    //   W_{q_i q_j}   = delta_ij mu_i g_i sin q_i - mu^T (d^2M/dq_i dq_j) acc + rho_i.beta_j + rho_j.beta_i
    //                   + g_j cos q_j rho_i[j] + g_i cos q_i rho_j[i]
    //   W_{q_i qd_j}  = D_j rho_i[j],   W_{q_i tau_j} = -rho_i[j],   all qd / tau blocks 0
    // (the oracle's oracle_exo_hess states the same with a Gauss-Jordan inverse and dense loops).
    static constexpr bool kHasHess = true;
    static constexpr bool kControlAffine = true;    // d^2 acc / dtau^2 = 0
    static constexpr bool kExactDefault = false;    // AUTO keeps Gauss-Newton: more iterations exact
    MMPC_HD static void eval_hess(const double* x, const double* u, const double* lam, double* W) {
        double s[4], c[4];
        const trig_cptr TK = trig_table();
#pragma unroll
        for (int i = 0; i < 4; ++i) sincos_fast(TK, x[i], &s[i], &c[i]);
        const exo::TrigPowers tp(c[1], c[2], c[3], s[1], s[2], s[3]);
        double Mu[10], l[10], il[4], w[4], acc[4], mu[4];
        exo::mass_upper(tp, Mu);
        chol4(Mu, l, il);
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = u[i] - exo::kDamping[i] * x[4 + i] - exo::kGravityGain[i] * s[i];
        chol4_solve(l, il, w, acc);
        chol4_solve(l, il, lam, mu);
        double beta[4][4], rho[4][4];   // [0] = 0: M does not depend on q0
#pragma unroll
        for (int r = 0; r < 4; ++r) beta[0][r] = rho[0][r] = 0.0;
        {
            double nu[4];
            dmass_times<1>(tp, acc, beta[1]);
            dmass_times<1>(tp, mu, nu);
            chol4_solve(l, il, nu, rho[1]);
            dmass_times<2>(tp, acc, beta[2]);
            dmass_times<2>(tp, mu, nu);
            chol4_solve(l, il, nu, rho[2]);
            dmass_times<3>(tp, acc, beta[3]);
            dmass_times<3>(tp, mu, nu);
            chol4_solve(l, il, nu, rho[3]);
        }
        // mu^T (d^2M/dq_i dq_j) acc for 1 <= i <= j <= 3
        double h2[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) h2[i][j] = 0.0;
        d2_bilinear<1, 1>(tp, mu, acc, h2);
        d2_bilinear<1, 2>(tp, mu, acc, h2);
        d2_bilinear<1, 3>(tp, mu, acc, h2);
        d2_bilinear<2, 2>(tp, mu, acc, h2);
        d2_bilinear<2, 3>(tp, mu, acc, h2);
        d2_bilinear<3, 3>(tp, mu, acc, h2);
#pragma unroll
        for (int i = 0; i < 144; ++i) W[i] = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int j = i; j < 4; ++j) {
                double t = -h2[i][j];
                if (i == j) t = fma(mu[i] * exo::kGravityGain[i], s[i], t);
#pragma unroll
                for (int r = 0; r < 4; ++r) t = fma(rho[i][r], beta[j][r], fma(rho[j][r], beta[i][r], t));
                t = fma(exo::kGravityGain[j] * c[j], rho[i][j], t);
                t = fma(exo::kGravityGain[i] * c[i], rho[j][i], t);
                W[i * 12 + j] = W[j * 12 + i] = t;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                W[i * 12 + 4 + j] = W[(4 + j) * 12 + i] = exo::kDamping[j] * rho[i][j];
                W[i * 12 + 8 + j] = W[(8 + j) * 12 + i] = -rho[i][j];
            }
        }
    }
    // out[I][J] = out[J][I] = a^T (d^2M/dq_I dq_J) b
    template <int I, int J>
    MMPC_HD static void d2_bilinear(const exo::TrigPowers& tp, const double* a, const double* b, double (*out)[4]) {
        double d[10], v[4];
        exo::d2mass_upper<I, J>(tp, d);
        v[0] = fma(d[0], b[0], fma(d[1], b[1], fma(d[2], b[2], d[3] * b[3])));
        v[1] = fma(d[1], b[0], fma(d[4], b[1], fma(d[5], b[2], d[6] * b[3])));
        v[2] = fma(d[2], b[0], fma(d[5], b[1], fma(d[7], b[2], d[8] * b[3])));
        v[3] = fma(d[3], b[0], fma(d[6], b[1], fma(d[8], b[2], d[9] * b[3])));
        out[I][J] = out[J][I] = fma(a[0], v[0], fma(a[1], v[1], fma(a[2], v[2], a[3] * v[3])));
    }

    MMPC_HD static void eval_jac(const double* x, const double* u, double* xd, double* fx, double* fu) {
        double qdd[4], Fq[16], Fqd[16], Fu[16];
        eval_acc_jac(x, u, qdd, Fq, Fqd, Fu);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            xd[r] = x[4 + r];
            xd[4 + r] = qdd[r];
#pragma unroll
            for (int cc = 0; cc < 8; ++cc) fx[r * 8 + cc] = (cc == 4 + r) ? 1.0 : 0.0;
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                fx[(4 + r) * 8 + cc] = Fq[r * 4 + cc];
                fx[(4 + r) * 8 + 4 + cc] = Fqd[r * 4 + cc];
                fu[r * 4 + cc] = 0.0;
                fu[(4 + r) * 4 + cc] = Fu[r * 4 + cc];
            }
        }
    }
};

// Values and continuous-time Jacobians of any model: fx[NX*NX], fu[NX*NU] row-major.
template <class Model>
MMPC_HD void model_eval_jac(const double* x, const double* u, double* xd, double* fx, double* fu) {
    Model::eval_jac(x, u, xd, fx, fu);
}

template <class Model>
MMPC_HD void model_eval(const double* x, const double* u, double* xd) {
    Model::eval(x, u, xd);
}

}  // namespace mmpc
