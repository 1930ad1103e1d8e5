/*
 * mmpc_oracle.c -- CPU fp64 restatement of the mahi-mpc multiple-shooting NLP
 * and of the Gauss-Newton SQP run by the HIP path.  TEST INFRASTRUCTURE ONLY
 * (see mmpc_oracle.h).  Plain C99 + OpenMP, built by oracle/Makefile.
 *
 * What is restated, and from where (paths relative to the reference root):
 *   dynamics      examples/ex_model_generate.cpp:24-43 (2-link arm, L=m=1, g=9.81)
 *                 src/inverseTest.cpp:59-74 (exo M(q), via exo_model_gen.h, with the build-defined
 *                 parameters / gravity / damping of tests/golden/exo_params.json -- not reference-pinned)
 *   Euler step    src/Mahi/Mpc/ModelGenerator.cpp:33-34     F(x,u) = x + h f(x,u)
 *   F_lin         src/Mahi/Mpc/ModelGenerator.cpp:45-48
 *   V layout      src/Mahi/Mpc/ModelGenerator.cpp:61-112    [x0,u0,x1,u1,...,x_{N-1},u_{N-1},xN]
 *   p layout      src/Mahi/Mpc/ModelGenerator.cpp:129-187   [traj | Q | R | Rm | u_prev]
 *   cost J        src/Mahi/Mpc/ModelGenerator.cpp:191-222   (no 1/2, error uses F(x_k,u_k))
 *   defects g     src/Mahi/Mpc/ModelGenerator.cpp:206
 *   x0 pinning    src/Mahi/Mpc/ModelControl.cpp:144-145
 * The IPOPT call (ModelControl.cpp:159) is replaced by the GN-SQP described in
 * DESIGN.md; this file implements it in the plain dense form (explicit Gamma,
 * H = Gamma^T Q Gamma + D^T R D + Rm, textbook Cholesky) so that it shares no
 * code or loop structure with the recursive condensing of the HIP kernel.
 */
#include "mmpc_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "exo_model_gen.h"

/* model context of the calling thread: dimensions and dynamics (set by set_model) */
static _Thread_local int t_model = ORACLE_MODEL_TWO_LINK_ARM, t_nx = 4, t_nu = 2;
#define NX t_nx
#define NU t_nu
#define ND (t_nx + t_nu)
/* dynamics registered by oracle_set_user_model (process-wide; models generated from SX expressions) */
static oracle_user_jac_fn g_user_jac = NULL;
/* mmpc_opts.init_states (process-wide): 1 = x_1..x_N start at x_0 */
static int g_init_hold = 0;
static int g_init_zero = 0;
void oracle_set_init_states(int mode) { g_init_hold = mode == 1; g_init_zero = mode == 2; }
static int g_user_nx = 0, g_user_nu = 0;
static int set_model(int model) {
    if (model == ORACLE_MODEL_TWO_LINK_ARM) { t_model = model; t_nx = 4; t_nu = 2; return 0; }
    if (model == ORACLE_MODEL_EXO_ARM) { t_model = model; t_nx = 8; t_nu = 4; return 0; }
    if (model == ORACLE_MODEL_USER && g_user_jac) { t_model = model; t_nx = g_user_nx; t_nu = g_user_nu; return 0; }
    return -1;
}
int oracle_set_user_model(int nx, int nu, oracle_user_jac_fn jac) {
    if (nx < 1 || nx > ORACLE_MAX_NX || nu < 1 || nu > ORACLE_MAX_NU || !jac) return -1;
    g_user_nx = nx;
    g_user_nu = nu;
    g_user_jac = jac;
    return 0;
}

/* ---------------- forward-mode dual numbers (6 tangents: x then u of the 2-link arm) ---------------- */
#define DK 6
typedef struct { double v; double d[DK]; } dual;

static dual dc(double c) { dual r; r.v = c; memset(r.d, 0, sizeof r.d); return r; }
static dual dvar(double v, int i) { dual r = dc(v); r.d[i] = 1.0; return r; }
static dual dadd(dual a, dual b) { dual r; r.v = a.v + b.v; for (int i = 0; i < DK; ++i) r.d[i] = a.d[i] + b.d[i]; return r; }
static dual dsub(dual a, dual b) { dual r; r.v = a.v - b.v; for (int i = 0; i < DK; ++i) r.d[i] = a.d[i] - b.d[i]; return r; }
static dual dmul(dual a, dual b) { dual r; r.v = a.v * b.v; for (int i = 0; i < DK; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i]; return r; }
static dual dscale(double s, dual a) { dual r; r.v = s * a.v; for (int i = 0; i < DK; ++i) r.d[i] = s * a.d[i]; return r; }
static dual ddiv(dual a, dual b) {
    dual r; r.v = a.v / b.v;
    for (int i = 0; i < DK; ++i) r.d[i] = (a.d[i] - r.v * b.d[i]) / b.v;
    return r;
}
static dual dsin(dual a) { dual r; r.v = sin(a.v); double c = cos(a.v); for (int i = 0; i < DK; ++i) r.d[i] = c * a.d[i]; return r; }
static dual dcos(dual a) { dual r; r.v = cos(a.v); double s = -sin(a.v); for (int i = 0; i < DK; ++i) r.d[i] = s * a.d[i]; return r; }
static dual dneg(dual a) { return dscale(-1.0, a); }

/* 2-link arm ODE right-hand side, restated from examples/ex_model_generate.cpp:36-37
 * term by term (L = 1, m = 1, g = 9.81 at :24-26). */
static void two_link_dual(const dual* x, const dual* u, dual* xd) {
    const double L = 1.0, m = 1.0, g = 9.81;
    dual qA = x[0], qB = x[1], dA = x[2], dB = x[3], TA = u[0], TB = u[1];
    dual cB = dcos(qB), sB = dsin(qB), cA = dcos(qA), cAB = dcos(dadd(qA, qB));
    const double LLm = L * L * m, Lgm = L * g * m;
    dual dA2 = dmul(dA, dA), dB2 = dmul(dB, dB), dAdB = dmul(dA, dB), cBsB = dmul(cB, sB);
    dual den = dscale(LLm, dsub(dmul(cB, cB), dc(2.0)));
    /* qA_ddot numerator, :36 */
    dual nA = dsub(TA, TB);
    nA = dsub(nA, dmul(TB, cB));
    nA = dadd(nA, dscale(LLm, dmul(dA2, sB)));
    nA = dadd(nA, dscale(LLm, dmul(dB2, sB)));
    nA = dsub(nA, dscale(2.0 * Lgm, cA));
    nA = dadd(nA, dscale(LLm, dmul(dA2, cBsB)));
    nA = dadd(nA, dscale(2.0 * LLm, dmul(dAdB, sB)));
    nA = dadd(nA, dscale(Lgm, dmul(cAB, cB)));
    /* qB_ddot numerator, :37 */
    dual nB = dsub(dadd(TA, dc(0.0)), dscale(3.0, TB));
    nB = dadd(nB, dmul(TA, cB));
    nB = dsub(nB, dscale(2.0, dmul(TB, cB)));
    nB = dadd(nB, dscale(2.0 * Lgm, cAB));
    nB = dadd(nB, dscale(3.0 * LLm, dmul(dA2, sB)));
    nB = dadd(nB, dscale(LLm, dmul(dB2, sB)));
    nB = dsub(nB, dscale(2.0 * Lgm, cA));
    nB = dadd(nB, dscale(2.0 * LLm, dmul(dA2, cBsB)));
    nB = dadd(nB, dscale(LLm, dmul(dB2, cBsB)));
    nB = dsub(nB, dscale(2.0 * Lgm, dmul(cA, cB)));
    nB = dadd(nB, dscale(2.0 * LLm, dmul(dAdB, sB)));
    nB = dadd(nB, dscale(Lgm, dmul(cAB, cB)));
    nB = dadd(nB, dscale(2.0 * LLm, dmul(dAdB, cBsB)));
    xd[0] = dA;
    xd[1] = dB;
    xd[2] = dneg(ddiv(nA, den));
    xd[3] = ddiv(nB, den);
}

/* ---------------- second-order forward mode (value, gradient, Hessian over the 6 inputs x | u) ----------------
 * Used for the exact Hessian of the Lagrangian (CasADi's nlp_hess_l, ModelGenerator.cpp:238; IPOPT's default
 * hessian_approximation = exact, ModelControl.cpp:54-59).  Hessian stored full (symmetric) for clarity. */
typedef struct { double v; double d[DK]; double H[DK][DK]; } hdual;

static hdual hc(double c) { hdual r; memset(&r, 0, sizeof r); r.v = c; return r; }
static hdual hvar(double v, int i) { hdual r = hc(v); r.d[i] = 1.0; return r; }
static hdual hadd(hdual a, hdual b) {
    hdual r; r.v = a.v + b.v;
    for (int i = 0; i < DK; ++i) { r.d[i] = a.d[i] + b.d[i]; for (int j = 0; j < DK; ++j) r.H[i][j] = a.H[i][j] + b.H[i][j]; }
    return r;
}
static hdual hscale(double s, hdual a) {
    hdual r; r.v = s * a.v;
    for (int i = 0; i < DK; ++i) { r.d[i] = s * a.d[i]; for (int j = 0; j < DK; ++j) r.H[i][j] = s * a.H[i][j]; }
    return r;
}
static hdual hsub(hdual a, hdual b) { return hadd(a, hscale(-1.0, b)); }
static hdual hmul(hdual a, hdual b) {
    hdual r; r.v = a.v * b.v;
    for (int i = 0; i < DK; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i];
    for (int i = 0; i < DK; ++i)
        for (int j = 0; j < DK; ++j)
            r.H[i][j] = a.H[i][j] * b.v + a.v * b.H[i][j] + a.d[i] * b.d[j] + a.d[j] * b.d[i];
    return r;
}
/* 1/b: d = -b'/b^2, H = 2 b' b'^T / b^3 - b''/b^2 */
static hdual hinv(hdual b) {
    hdual r; const double i1 = 1.0 / b.v, i2 = i1 * i1, i3 = i2 * i1;
    r.v = i1;
    for (int i = 0; i < DK; ++i) r.d[i] = -b.d[i] * i2;
    for (int i = 0; i < DK; ++i)
        for (int j = 0; j < DK; ++j) r.H[i][j] = 2.0 * b.d[i] * b.d[j] * i3 - b.H[i][j] * i2;
    return r;
}
static hdual hdiv(hdual a, hdual b) { return hmul(a, hinv(b)); }
/* f(a) with f' = f1, f'' = f2: d = f1 a', H = f1 a'' + f2 a' a'^T */
static hdual hchain(hdual a, double f0, double f1, double f2) {
    hdual r; r.v = f0;
    for (int i = 0; i < DK; ++i) r.d[i] = f1 * a.d[i];
    for (int i = 0; i < DK; ++i)
        for (int j = 0; j < DK; ++j) r.H[i][j] = f1 * a.H[i][j] + f2 * a.d[i] * a.d[j];
    return r;
}
static hdual hsin(hdual a) { return hchain(a, sin(a.v), cos(a.v), -sin(a.v)); }
static hdual hcos(hdual a) { return hchain(a, cos(a.v), -sin(a.v), -cos(a.v)); }

/* the accelerations of two_link_dual (examples/ex_model_generate.cpp:36-37) in second-order forward mode */
static void two_link_hdual(const hdual* x, const hdual* u, hdual* acc) {
    const double L = 1.0, m = 1.0, g = 9.81;
    hdual qA = x[0], qB = x[1], dA = x[2], dB = x[3], TA = u[0], TB = u[1];
    hdual cB = hcos(qB), sB = hsin(qB), cA = hcos(qA), cAB = hcos(hadd(qA, qB));
    const double LLm = L * L * m, Lgm = L * g * m;
    hdual dA2 = hmul(dA, dA), dB2 = hmul(dB, dB), dAdB = hmul(dA, dB), cBsB = hmul(cB, sB);
    hdual den = hscale(LLm, hsub(hmul(cB, cB), hc(2.0)));
    hdual nA = hsub(TA, TB);
    nA = hsub(nA, hmul(TB, cB));
    nA = hadd(nA, hscale(LLm, hmul(dA2, sB)));
    nA = hadd(nA, hscale(LLm, hmul(dB2, sB)));
    nA = hsub(nA, hscale(2.0 * Lgm, cA));
    nA = hadd(nA, hscale(LLm, hmul(dA2, cBsB)));
    nA = hadd(nA, hscale(2.0 * LLm, hmul(dAdB, sB)));
    nA = hadd(nA, hscale(Lgm, hmul(cAB, cB)));
    hdual nB = hsub(TA, hscale(3.0, TB));
    nB = hadd(nB, hmul(TA, cB));
    nB = hsub(nB, hscale(2.0, hmul(TB, cB)));
    nB = hadd(nB, hscale(2.0 * Lgm, cAB));
    nB = hadd(nB, hscale(3.0 * LLm, hmul(dA2, sB)));
    nB = hadd(nB, hscale(LLm, hmul(dB2, sB)));
    nB = hsub(nB, hscale(2.0 * Lgm, cA));
    nB = hadd(nB, hscale(2.0 * LLm, hmul(dA2, cBsB)));
    nB = hadd(nB, hscale(LLm, hmul(dB2, cBsB)));
    nB = hsub(nB, hscale(2.0 * Lgm, hmul(cA, cB)));
    nB = hadd(nB, hscale(2.0 * LLm, hmul(dAdB, sB)));
    nB = hadd(nB, hscale(Lgm, hmul(cAB, cB)));
    nB = hadd(nB, hscale(2.0 * LLm, hmul(dAdB, cBsB)));
    acc[0] = hscale(-1.0, hdiv(nA, den));
    acc[1] = hdiv(nB, den);
}

void oracle_two_link_hess(const double* x, const double* u, const double* lam, double* W) {
    hdual xv[4], uv[2], acc[2];
    for (int i = 0; i < 4; ++i) xv[i] = hvar(x[i], i);
    for (int i = 0; i < 2; ++i) uv[i] = hvar(u[i], 4 + i);
    two_link_hdual(xv, uv, acc);
    /* rows 0, 1 of f (qdot) are linear: only the accelerations contribute */
    for (int i = 0; i < DK; ++i)
        for (int j = 0; j < DK; ++j) W[i * DK + j] = lam[2] * acc[0].H[i][j] + lam[3] * acc[1].H[i][j];
}

void oracle_two_link_jac(const double* x, const double* u, double* A, double* B, double* xdot) {
    dual xv[4], uv[2], xd[4];
    for (int i = 0; i < 4; ++i) xv[i] = dvar(x[i], i);
    for (int i = 0; i < 2; ++i) uv[i] = dvar(u[i], 4 + i);
    two_link_dual(xv, uv, xd);
    for (int r = 0; r < 4; ++r) {
        if (xdot) xdot[r] = xd[r].v;
        if (A) for (int c = 0; c < 4; ++c) A[r * 4 + c] = xd[r].d[c];
        if (B) for (int c = 0; c < 2; ++c) B[r * 2 + c] = xd[r].d[4 + c];
    }
}

/* ---------------- 4-DoF exo ----------------
 * xdot = [qd; M(q)^-1 (tau - D qd - G(q))], G_i = g_i sin q_i.  Dense Gauss-Jordan inverse of M (a different
 * factorisation from the device's Cholesky) and the symbolic dM/dq_j of exo_model_gen.h:
 *   d qdd/dq_j = M^-1 (-dM/dq_j qdd - g_j cos q_j e_j),  d qdd/dqd = -M^-1 D,  d qdd/dtau = M^-1. */
static void inv4(const double* M, double* Minv) {
    double a[4][8];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 8; ++c) a[r][c] = (c < 4) ? M[r * 4 + c] : (c - 4 == r ? 1.0 : 0.0);
    for (int k = 0; k < 4; ++k) {
        int piv = k;
        for (int r = k + 1; r < 4; ++r) if (fabs(a[r][k]) > fabs(a[piv][k])) piv = r;
        for (int c = 0; c < 8; ++c) { double t = a[k][c]; a[k][c] = a[piv][c]; a[piv][c] = t; }
        double f = 1.0 / a[k][k];
        for (int c = 0; c < 8; ++c) a[k][c] *= f;
        for (int r = 0; r < 4; ++r) {
            if (r == k) continue;
            double m = a[r][k];
            for (int c = 0; c < 8; ++c) a[r][c] -= m * a[k][c];
        }
    }
    for (int r = 0; r < 4; ++r) for (int c = 0; c < 4; ++c) Minv[r * 4 + c] = a[r][4 + c];
}

void oracle_exo_jac(const double* x, const double* u, double* A, double* B, double* xdot) {
    double M[16], dM[4][16], Minv[16], w[4], qdd[4];
    exo_mass_and_grad(x, M, dM);
    inv4(M, Minv);
    for (int i = 0; i < 4; ++i) w[i] = u[i] - EXO_DAMPING[i] * x[4 + i] - EXO_GRAVITY_GAIN[i] * sin(x[i]);
    for (int r = 0; r < 4; ++r) {
        qdd[r] = 0.0;
        for (int c = 0; c < 4; ++c) qdd[r] += Minv[r * 4 + c] * w[c];
    }
    if (xdot) for (int r = 0; r < 4; ++r) { xdot[r] = x[4 + r]; xdot[4 + r] = qdd[r]; }
    if (A) {
        for (int i = 0; i < 64; ++i) A[i] = 0.0;
        for (int r = 0; r < 4; ++r) A[r * 8 + 4 + r] = 1.0;
        for (int j = 0; j < 4; ++j) {
            double rhs[4];
            for (int r = 0; r < 4; ++r) {
                double t = 0.0;
                for (int c = 0; c < 4; ++c) t += dM[j][r * 4 + c] * qdd[c];
                rhs[r] = -t;
            }
            rhs[j] -= EXO_GRAVITY_GAIN[j] * cos(x[j]);
            for (int r = 0; r < 4; ++r) {
                double t = 0.0;
                for (int c = 0; c < 4; ++c) t += Minv[r * 4 + c] * rhs[c];
                A[(4 + r) * 8 + j] = t;
                A[(4 + r) * 8 + 4 + j] = -Minv[r * 4 + j] * EXO_DAMPING[j];
            }
        }
    }
    if (B) {
        for (int i = 0; i < 32; ++i) B[i] = 0.0;
        for (int r = 0; r < 4; ++r) for (int c = 0; c < 4; ++c) B[(4 + r) * 4 + c] = Minv[r * 4 + c];
    }
}

/* The exo's Lagrangian Hessian block W = sum_r lam_r d^2 f_r / d(x,u)^2 ((nx+nu)^2 = 12 x 12, row-major; round 4,
 * the exact-Hessian SQP on the exo).  Only the accelerations are nonlinear: with acc = M^-1 w, w = tau - D qd - G(q),
 * mu = M^-1 lam_acc and a_j = d acc / dz_j (columns of [Fq | Fqd | Fu]), differentiating M acc = w twice gives
 *   W_ij = sum_k mu_k d^2 w_k / dz_i dz_j - mu^T (d^2 M / dz_i dz_j) acc - mu^T (dM/dz_i) a_j - mu^T (dM/dz_j) a_i,
 * with d^2 w_k / dq_k^2 = g_k sin q_k and the symbolic dM, d^2 M of exo_model_gen.h (nonzero for q1..q3 only). */
void oracle_exo_hess(const double* x, const double* u, const double* lam, double* W) {
    double M[16], dM[4][16], d2M[4][4][16], Minv[16], A[64], B[32], xd[8];
    exo_mass_derivs(x, M, dM, d2M);
    inv4(M, Minv);
    oracle_exo_jac(x, u, A, B, xd);
    const double* acc = xd + 4;
    double mu[4], a[12][4];
    for (int r = 0; r < 4; ++r) {
        mu[r] = 0.0;
        for (int c = 0; c < 4; ++c) mu[r] += Minv[r * 4 + c] * lam[4 + c];
    }
    for (int j = 0; j < 12; ++j)
        for (int r = 0; r < 4; ++r) a[j][r] = j < 8 ? A[(4 + r) * 8 + j] : B[(4 + r) * 4 + (j - 8)];
    /* nu_i = (dM/dq_i) mu (dM symmetric: mu^T dM_i v = nu_i^T v) */
    double nu[4][4];
    for (int i = 0; i < 4; ++i)
        for (int r = 0; r < 4; ++r) {
            nu[i][r] = 0.0;
            for (int c = 0; c < 4; ++c) nu[i][r] += dM[i][r * 4 + c] * mu[c];
        }
    for (int i = 0; i < 12; ++i)
        for (int j = 0; j < 12; ++j) {
            double t = 0.0;
            if (i < 4 && j < 4) {
                if (i == j) t += mu[i] * EXO_GRAVITY_GAIN[i] * sin(x[i]);
                for (int r = 0; r < 4; ++r) {
                    double m = 0.0;
                    for (int c = 0; c < 4; ++c) m += d2M[i][j][r * 4 + c] * acc[c];
                    t -= mu[r] * m;
                }
            }
            if (i < 4)
                for (int r = 0; r < 4; ++r) t -= nu[i][r] * a[j][r];
            if (j < 4)
                for (int r = 0; r < 4; ++r) t -= nu[j][r] * a[i][r];
            W[i * 12 + j] = t;
        }
}

void oracle_exo_mass(const double* q, double* M) {
    double dM[4][16];
    exo_mass_and_grad(q, M, dM);
}

/* Domain of the built-in models' joint angles.  The device evaluates sin / cos of them with a reduced-range routine
 * (mahi-mpc_amd/csrc/fast_trig.h: within 1 ulp of libm for |q| <= 2^20 pi/2) that returns NaN beyond, so the solver
 * reports an iterate with such an angle (a diverging one: 1.6e6 rad) non-finite.  The oracle applies the same domain to
 * the model evaluations, so both report the same status there (tests/test_gpu_trig_domain.py). */
static const double kTrigDomain = 1647099.3291652855;
static int angles_out_of_domain(const double* x) {
    const int nq = t_model == ORACLE_MODEL_EXO_ARM ? 4 : (t_model == ORACLE_MODEL_TWO_LINK_ARM ? 2 : 0);
    for (int i = 0; i < nq; ++i)
        if (!(fabs(x[i]) <= kTrigDomain) && x[i] == x[i]) return 1;   /* NaN propagates by itself */
    return 0;
}
static void model_jac(const double* x, const double* u, double* A, double* B, double* xdot) {
    if (t_model == ORACLE_MODEL_EXO_ARM) oracle_exo_jac(x, u, A, B, xdot);
    else if (t_model == ORACLE_MODEL_USER) {
        double Af[ORACLE_MAX_NX * ORACLE_MAX_NX], Bf[ORACLE_MAX_NX * ORACLE_MAX_NU];
        g_user_jac(x, u, A ? A : Af, B ? B : Bf, xdot);
    } else oracle_two_link_jac(x, u, A, B, xdot);
    if (angles_out_of_domain(x)) {
        for (int r = 0; r < NX; ++r) {
            xdot[r] = NAN;
            if (A) for (int c = 0; c < NX; ++c) A[r * NX + c] = NAN;
            if (B) for (int c = 0; c < NU; ++c) B[r * NU + c] = NAN;
        }
    }
}

/* W = sum_r lam_r d^2 f_r / d(x,u)^2 ((nx+nu)^2, row-major); 0 when the model has no second derivatives */
static oracle_user_hess_fn g_user_hess = NULL;
int oracle_set_user_model_hess(oracle_user_hess_fn hess) {
    g_user_hess = hess;
    return 0;
}
static int model_has_hess(void) {
    if (t_model == ORACLE_MODEL_TWO_LINK_ARM || t_model == ORACLE_MODEL_EXO_ARM) return 1;
    if (t_model == ORACLE_MODEL_USER) return g_user_hess != NULL;
    return 0;
}
static int model_hess(const double* x, const double* u, const double* lam, double* W) {
    if (t_model == ORACLE_MODEL_TWO_LINK_ARM) { oracle_two_link_hess(x, u, lam, W); return 1; }
    if (t_model == ORACLE_MODEL_EXO_ARM) { oracle_exo_hess(x, u, lam, W); return 1; }
    if (t_model == ORACLE_MODEL_USER && g_user_hess) { g_user_hess(x, u, lam, W); return 1; }
    return 0;
}
/* mmpc_opts.hessian (process-wide): ORACLE_HESS_GAUSS_NEWTON or ORACLE_HESS_EXACT */
static int g_hess_mode = ORACLE_HESS_GAUSS_NEWTON;
void oracle_set_hessian(int mode) { g_hess_mode = mode; }
/* EXACT with control bounds: the held controls fixed in the exact QP (1), or such solves keep Gauss-Newton (0) */
static int g_exact_bounded = 1;
void oracle_set_exact_bounded(int on) { g_exact_bounded = on; }
/* Control bounds, primal-dual active set (the 16-lane Riccati kernel, round 3): after each QP solve a held control
 * whose multiplier -- the un-held QP gradient (H0 du + g0)_a at the solution -- points into the box is released as
 * well as a free control whose step crosses a bound held (Hintermueller, Ito & Kunisch 2003); two QP solves at the
 * first iteration, ORACLE_BOUND_PASSES later.  Off: holds are only added (the condensed and lane kernels). */
/* test instrumentation: iterations whose exact-Hessian QP was not positive definite and took the Gauss-Newton step
 * (solve_one and solve_one_riccati), summed over all threads since the last reset */
static long long g_exact_fallbacks = 0;
long long oracle_exact_fallbacks(int reset) {
    long long v;
#pragma omp atomic read
    v = g_exact_fallbacks;
    if (reset) {
#pragma omp atomic write
        g_exact_fallbacks = 0;
    }
    return v;
}
static void count_exact_fallback(void) {
#pragma omp atomic
    g_exact_fallbacks += 1;
}
static int g_bound_release = 0;
void oracle_set_bound_release(int on) { g_bound_release = on; }

void oracle_two_link_xdot(const double* x, const double* u, double* xdot) {
    oracle_two_link_jac(x, u, NULL, NULL, xdot);
}

void oracle_f_lin(int nx, int nu, double h, const double* A, const double* B, const double* x,
                  const double* u, const double* xdot_init, const double* x_init,
                  const double* u_init, double* x_next) {
    /* x_next = x + h (A (x - x*) + B (u - u*) + xdot*)   ModelGenerator.cpp:47-48 */
    for (int r = 0; r < nx; ++r) {
        double s = xdot_init[r];
        for (int c = 0; c < nx; ++c) s += A[r * nx + c] * (x[c] - x_init[c]);
        for (int c = 0; c < nu; ++c) s += B[r * nu + c] * (u[c] - u_init[c]);
        x_next[r] = x[r] + h * s;
    }
}

/* ---------------- NLP pieces ---------------- */
/* linear mode (ModelGenerator.cpp:137-187, ModelControl.cpp:125-136): when non-NULL, lin holds
 * A* (row-major), B*, xdot*, x*, u* and the dynamics are F_lin instead of F. */
static _Thread_local const double* g_lin = NULL;

static void stage_jac(const double* x, const double* u, double* A, double* Bc, double* xd) {
    if (!g_lin) {
        model_jac(x, u, A, Bc, xd);
        return;
    }
    const double *As = g_lin, *Bs = g_lin + NX * NX, *fs = Bs + NX * NU, *xs = fs + NX, *us = xs + NX;
    for (int r = 0; r < NX; ++r) {
        double s = fs[r];
        for (int c = 0; c < NX; ++c) { A[r * NX + c] = As[r * NX + c]; s += As[r * NX + c] * (x[c] - xs[c]); }
        for (int c = 0; c < NU; ++c) { Bc[r * NU + c] = Bs[r * NU + c]; s += Bs[r * NU + c] * (u[c] - us[c]); }
        xd[r] = s;
    }
}

static void euler_step(double h, const double* x, const double* u, double* F, double* Ad, double* Bd) {
    double A[ORACLE_MAX_NX * ORACLE_MAX_NX], Bc[ORACLE_MAX_NX * ORACLE_MAX_NU], xd[ORACLE_MAX_NX];
    stage_jac(x, u, A, Bc, xd);
    for (int r = 0; r < NX; ++r) {
        F[r] = x[r] + h * xd[r];
        if (Ad) for (int c = 0; c < NX; ++c) Ad[r * NX + c] = (r == c ? 1.0 : 0.0) + h * A[r * NX + c];
        if (Bd) for (int c = 0; c < NU; ++c) Bd[r * NU + c] = h * Bc[r * NU + c];
    }
}

/* J and defects of ModelGenerator.cpp:191-222 at the packed V */
void oracle_nlp_eval(int model, int N, double h, const double* V, const double* u_prev,
                     const double* traj, const double* w, double* Jout, double* g) {
    /* nonlinear model; in linear mode solve_one evaluates with g_lin set (same thread, same model) */
    if (!g_lin && set_model(model) != 0) return;
    const double *Q = w, *R = w + NX, *Rm = w + NX + NU;
    double J = 0.0;
    for (int k = 0; k < N; ++k) {
        const double* xk = V + k * ND;
        const double* uk = xk + NX;
        const double* xk1 = V + (k + 1) * ND;
        const double* ukm = (k == 0) ? u_prev : V + (k - 1) * ND + NX;
        double F[ORACLE_MAX_NX];
        euler_step(h, xk, uk, F, NULL, NULL);
        for (int r = 0; r < NX; ++r) {
            if (g) g[k * NX + r] = F[r] - xk1[r];
            double e = F[r] - traj[k * NX + r];
            J += e * Q[r] * e;
        }
        for (int c = 0; c < NU; ++c) {
            double du = uk[c] - ukm[c];
            J += du * R[c] * du + uk[c] * Rm[c] * uk[c];
        }
    }
    if (Jout) *Jout = J;
}

void oracle_reduced_gradient(int model, int N, double h, const double* x0, const double* U,
                             const double* u_prev, const double* traj, const double* w,
                             double* grad) {
    if (set_model(model) != 0) return;
    const double *Q = w, *R = w + NX, *Rm = w + NX + NU;
    double* X = (double*)malloc(sizeof(double) * (N + 1) * NX);
    double* Ad = (double*)malloc(sizeof(double) * N * NX * NX);
    double* Bd = (double*)malloc(sizeof(double) * N * NX * NU);
    memcpy(X, x0, sizeof(double) * NX);
    for (int k = 0; k < N; ++k) euler_step(h, X + k * NX, U + k * NU, X + (k + 1) * NX, Ad + k * NX * NX, Bd + k * NX * NU);
    /* adjoint: lam_{k} = 2Q(x_{k} - r_{k-1}) + A_k^T lam_{k+1}, lam_N = 2Q(x_N - r_{N-1}) */
    double lam[ORACLE_MAX_NX], tmp[ORACLE_MAX_NX];
    for (int r = 0; r < NX; ++r) lam[r] = 2.0 * Q[r] * (X[N * NX + r] - traj[(N - 1) * NX + r]);
    for (int k = N - 1; k >= 0; --k) {
        /* grad wrt u_k: B_k^T lam_{k+1} */
        for (int c = 0; c < NU; ++c) {
            double s = 0.0;
            for (int r = 0; r < NX; ++r) s += Bd[k * NX * NU + r * NU + c] * lam[r];
            double ukm = (k == 0) ? u_prev[c] : U[(k - 1) * NU + c];
            s += 2.0 * R[c] * (U[k * NU + c] - ukm) + 2.0 * Rm[c] * U[k * NU + c];
            if (k + 1 < N) s -= 2.0 * R[c] * (U[(k + 1) * NU + c] - U[k * NU + c]);
            grad[k * NU + c] = s;
        }
        if (k == 0) break;
        for (int c = 0; c < NX; ++c) {
            double s = 0.0;
            for (int r = 0; r < NX; ++r) s += Ad[k * NX * NX + r * NX + c] * lam[r];
            tmp[c] = s + 2.0 * Q[c] * (X[k * NX + c] - traj[(k - 1) * NX + c]);
        }
        memcpy(lam, tmp, sizeof(double) * NX);
    }
    free(X); free(Ad); free(Bd);
}

/* nlp_hess_l (ModelGenerator.cpp:238): stage blocks on (x_k, u_k) of the Hessian of lam_f J + lam_g^T g at V,
 * [N][K][K]; returns -1 when the model has no second derivatives (the Gauss-Newton part alone is not nlp_hess_l) */
int oracle_nlp_hess(int model, int N, double h, const double* V, const double* u_prev, const double* traj,
                    const double* w, double lam_f, const double* lam_g, double* blocks) {
    (void)u_prev;  /* the Delta-u coupling -2 lam_f R is constant */
    if (set_model(model) != 0 || !model_has_hess()) return -1;
    const int K = NX + NU;
    const double *Q = w, *R = w + NX, *Rm = w + NX + NU;
    for (int k = 0; k < N; ++k) {
        const double* xk = V + k * ND;
        const double* uk = xk + NX;
        double A[ORACLE_MAX_NX * ORACLE_MAX_NX], Bc[ORACLE_MAX_NX * ORACLE_MAX_NU], xd[ORACLE_MAX_NX];
        double nu[ORACLE_MAX_NX], W[(ORACLE_MAX_NX + ORACLE_MAX_NU) * (ORACLE_MAX_NX + ORACLE_MAX_NU)];
        model_jac(xk, uk, A, Bc, xd);
        for (int r = 0; r < NX; ++r) {
            const double e = xk[r] + h * xd[r] - traj[k * NX + r];
            nu[r] = h * (2.0 * lam_f * Q[r] * e + (lam_g ? lam_g[k * NX + r] : 0.0));
        }
        model_hess(xk, uk, nu, W);
        double* out = blocks + (size_t)k * K * K;
        for (int i = 0; i < K; ++i)
            for (int j = 0; j < K; ++j) {
                double t = W[i * K + j];
                for (int r = 0; r < NX; ++r) {
                    /* J_F = [I + h A | h B] */
                    const double ji = i < NX ? (r == i ? 1.0 : 0.0) + h * A[r * NX + i] : h * Bc[r * NU + i - NX];
                    const double jj = j < NX ? (r == j ? 1.0 : 0.0) + h * A[r * NX + j] : h * Bc[r * NU + j - NX];
                    t += 2.0 * lam_f * Q[r] * ji * jj;
                }
                if (i == j && i >= NX)
                    t += lam_f * (2.0 * R[i - NX] + 2.0 * Rm[i - NX] + (k + 1 < N ? 2.0 * R[i - NX] : 0.0));
                out[i * K + j] = t;
            }
    }
    return 0;
}

/* ---------------- dense GN-SQP for one instance ---------------- */
typedef struct {
    int N, M;
    double *X, *U, *F, *Ad, *Bd, *c, *d, *e, *G, *H, *g, *du, *dx, *lam, *Xt, *Ut, *Ft, *H0, *g0, *tgt;
    double *Kf, *Wk;  /* Riccati variant: [K_k | kff_k] per stage, exact-Hessian stage blocks W_k */
    double *Hgn, *ggn; /* exact Hessian: the Gauss-Newton QP of the same iteration (fallback when not PD) */
} ws_t;

static void ws_alloc(ws_t* s, int N) {
    s->N = N; s->M = N * NU;
    size_t M = (size_t)s->M;
    s->X = calloc((size_t)(N + 1) * NX, sizeof(double));
    s->U = calloc((size_t)N * NU, sizeof(double));
    s->F = calloc((size_t)N * NX, sizeof(double));
    s->Ad = calloc((size_t)N * NX * NX, sizeof(double));
    s->Bd = calloc((size_t)N * NX * NU, sizeof(double));
    s->c = calloc((size_t)N * NX, sizeof(double));
    s->d = calloc((size_t)(N + 1) * NX, sizeof(double));
    s->e = calloc((size_t)N * NX, sizeof(double));
    s->G = calloc((size_t)N * NX * M, sizeof(double));
    s->H = calloc(M * M, sizeof(double));
    s->g = calloc(M, sizeof(double));
    s->du = calloc(M, sizeof(double));
    s->dx = calloc((size_t)(N + 1) * NX, sizeof(double));
    s->lam = calloc((size_t)(N + 1) * NX, sizeof(double));
    s->Xt = calloc((size_t)(N + 1) * NX, sizeof(double));
    s->Ut = calloc((size_t)N * NU, sizeof(double));
    s->Ft = calloc((size_t)N * NX, sizeof(double));
    s->H0 = calloc(M * M, sizeof(double));
    s->g0 = calloc(M, sizeof(double));
    s->tgt = calloc(M, sizeof(double));
    s->Kf = calloc((size_t)N * NU * (NX + NU + 1), sizeof(double));
    s->Wk = calloc((size_t)N * (NX + NU) * (NX + NU), sizeof(double));
    s->Hgn = calloc(M * M, sizeof(double));
    s->ggn = calloc(M, sizeof(double));
}
static void ws_free(ws_t* s) {
    free(s->X); free(s->U); free(s->F); free(s->Ad); free(s->Bd); free(s->c); free(s->d);
    free(s->e); free(s->G); free(s->H); free(s->g); free(s->du); free(s->dx); free(s->lam);
    free(s->Xt); free(s->Ut); free(s->Ft); free(s->H0); free(s->g0); free(s->tgt);
    free(s->Kf); free(s->Wk); free(s->Hgn); free(s->ggn);
}

/* merit pieces at (X,U): J and sum |c| (F returned) */
static void merit_eval(int N, double h, const double* X, const double* U, const double* u_prev,
                       const double* traj, const double* w, double* F, double* J, double* c1) {
    const double *Q = w, *R = w + NX, *Rm = w + NX + NU;
    double Jv = 0.0, cs = 0.0;
    for (int k = 0; k < N; ++k) {
        euler_step(h, X + k * NX, U + k * NU, F + k * NX, NULL, NULL);
        for (int r = 0; r < NX; ++r) {
            double e = F[k * NX + r] - traj[k * NX + r];
            Jv += e * Q[r] * e;
            cs += fabs(F[k * NX + r] - X[(k + 1) * NX + r]);
        }
        for (int q = 0; q < NU; ++q) {
            double um = (k == 0) ? u_prev[q] : U[(k - 1) * NU + q];
            double du = U[k * NU + q] - um;
            Jv += du * R[q] * du + U[k * NU + q] * Rm[q] * U[k * NU + q];
        }
    }
    *J = Jv; *c1 = cs;
}

static int chol_solve(int M, double* H, double* b /* in: rhs, out: solution */) {
    for (int j = 0; j < M; ++j) {
        double s = H[j * M + j];
        for (int k = 0; k < j; ++k) s -= H[j * M + k] * H[j * M + k];
        if (!(s > 0.0) || !isfinite(s)) return -1;
        double Ljj = sqrt(s);
        H[j * M + j] = Ljj;
        for (int i = j + 1; i < M; ++i) {
            double t = H[i * M + j];
            for (int k = 0; k < j; ++k) t -= H[i * M + k] * H[j * M + k];
            H[i * M + j] = t / Ljj;
        }
    }
    for (int i = 0; i < M; ++i) {
        double t = b[i];
        for (int k = 0; k < i; ++k) t -= H[i * M + k] * b[k];
        b[i] = t / H[i * M + i];
    }
    for (int i = M - 1; i >= 0; --i) {
        double t = b[i];
        for (int k = i + 1; k < M; ++k) t -= H[k * M + i] * b[k];
        b[i] = t / H[i * M + i];
    }
    return 0;
}

/* IPOPT's filter acceptance of a trial (J_t, theta_t = |c_t|_1) w.r.t. the first iterate (J_0, theta_0) -- the
 * filter holds only (theta_max, -inf) then: theta_t <= theta_max = 1e4 max(1, theta_0), and theta_t <= (1 - 1e-5)
 * theta_0 or J_t <= J_0 - 1e-5 theta_0 (gamma_theta = gamma_phi = 1e-5).  J-scale as the merit.
 * That test applies when the first iterate is far from feasible (theta_0 > theta_min = 1e-4 max(1, theta_0): the
 * reference's cold start) or the switching condition of Waechter & Biegler (2006) eq. (19) fails.  A nearly feasible
 * first iterate (a warm start) whose step satisfies alpha (-dJ)^s_phi > delta theta_0^s_theta (s_phi = 2.3,
 * s_theta = 1.1, delta = 1; dJ the directional derivative of J) is an f-type iteration: Armijo alone decides. */
int oracle_first_iter_filter_accepts(double J0, double c0, double Jt, double ct, double dJ, double alpha) {
    if (!(isfinite(Jt) && isfinite(ct))) return 0;
    if (ct > 1e4 * fmax(1.0, c0)) return 0;
    if (c0 <= 1e-4 * fmax(1.0, c0) && dJ < 0.0 && alpha * pow(-dJ, 2.3) > pow(c0, 1.1)) return 0;
    return ct <= (1.0 - 1e-5) * c0 || Jt <= J0 - 1e-5 * c0;
}

/* projection onto [lb, ub] that keeps a NaN a NaN (fmin/fmax would replace it by a bound) */
static double proj(double v, double lb, double ub) { return v < lb ? lb : (v > ub ? ub : v); }

/* exact Hessian, condensed form (solve_one, solve_one_ip): the QP in (dx, du) gains the stage term
 * 1/2 [dx_k; du_k]^T W_k [..] with W_k = h sum_r lam_{k+1,r} d^2 f_r/d(x_k,u_k)^2 (J/2 scale, lam = s->lam); with
 * dx_k = Gamma_k du + d_k (S_k du = [Gamma_k du; du_k]):  H += S_k^T W_k S_k,  g += S_k^T W_k [d_k; 0]
 * (Gamma = s->G, d = s->d). */
static void add_exact_condensed(ws_t* s, double h) {
    const int N = s->N, M = s->M;
    const int K = NX + NU;
    double W[(ORACLE_MAX_NX + ORACLE_MAX_NU) * (ORACLE_MAX_NX + ORACLE_MAX_NU)];
    const double* T = s->G;
    double* WS = (double*)malloc(sizeof(double) * (size_t)K * M);
    for (int k = 0; k < N; ++k) {
        model_hess(s->X + k * NX, s->U + k * NU, s->lam + (k + 1) * NX, W);
        /* WS = W S_k: S_k's x rows are Gamma rows of x_k (none for k = 0), its u rows select du_k */
        for (int i = 0; i < K; ++i)
            for (int a = 0; a < M; ++a) {
                double t = 0.0;
                if (k >= 1)
                    for (int q = 0; q < NX; ++q) t += W[i * K + q] * T[(size_t)((k - 1) * NX + q) * M + a];
                if (a / NU == k) t += W[i * K + NX + a % NU];
                WS[(size_t)i * M + a] = h * t;
            }
        for (int a = 0; a < M; ++a) {
            /* (S^T W S)[a][b] = sum_i S[i][a] WS[i][b] ; (S^T W [d; 0])[a] = sum_i S[i][a] (W [d;0])[i] */
            for (int i = 0; i < K; ++i) {
                double sia;
                if (i < NX) sia = (k >= 1) ? T[(size_t)((k - 1) * NX + i) * M + a] : 0.0;
                else sia = (a == k * NU + (i - NX)) ? 1.0 : 0.0;
                if (sia == 0.0) continue;
                for (int b = 0; b < M; ++b) s->H[a * M + b] += sia * WS[(size_t)i * M + b];
                double wd = 0.0;
                for (int q = 0; q < NX; ++q) wd += W[i * K + q] * s->d[k * NX + q];
                s->g[a] += sia * h * wd;
            }
        }
    }
    free(WS);
}

static int solve_one(ws_t* s, double h, const double* x0, const double* u_prev, const double* traj,
                     const double* w, const double* u_lb, const double* u_ub, int max_iter,
                     double tol_grad, double tol_defect, double* V, int32_t* iters_out,
                     double* kkt_out, double* J_out) {
    const int N = s->N, M = s->M;
    const double *Q = w, *R = w + NX, *Rm = w + NX + NU;
    /* unpack V (ModelGenerator.cpp:86-112); x_0 pinned to the measured state */
    for (int k = 0; k < N; ++k) {
        memcpy(s->X + k * NX, V + k * ND, sizeof(double) * NX);
        memcpy(s->U + k * NU, V + k * ND + NX, sizeof(double) * NU);
    }
    memcpy(s->X + N * NX, V + N * ND, sizeof(double) * NX);
    if (g_init_zero) {  /* MMPC_INIT_ZERO: the reference's first call, V = 0 (ModelControl.cpp:29-50) */
        memset(s->X, 0, sizeof(double) * (N + 1) * NX);
        memset(s->U, 0, sizeof(double) * N * NU);
    }
    memcpy(s->X, x0, sizeof(double) * NX);
    if (g_init_hold)  /* MMPC_INIT_HOLD_X0: the state trajectory starts at the measured state */
        for (int k = 1; k <= N; ++k) memcpy(s->X + k * NX, x0, sizeof(double) * NX);
    /* box constraints on u (ModelControl.cpp:37-50,146-157; |b| >= 1e19 is unbounded, as IPOPT): projected
     * Gauss-Newton SQP -- the iterate starts projected, controls at a bound whose gradient points outward
     * (epsilon-active set, Bertsekas 1982) are held in the QP, trial points are projected onto the box and the
     * stop test uses the projected gradient ||U - P(U - 2g)||_inf. */
    double lbv[ORACLE_MAX_NU], ubv[ORACLE_MAX_NU];
    int has_b = 0;
    for (int q = 0; q < NU; ++q) {
        lbv[q] = (u_lb && u_lb[q] > -1e19) ? u_lb[q] : -INFINITY;
        ubv[q] = (u_ub && u_ub[q] < 1e19) ? u_ub[q] : INFINITY;
        has_b |= (lbv[q] > -INFINITY) || (ubv[q] < INFINITY);
    }
    if (has_b)
        for (int a = 0; a < M; ++a) s->U[a] = proj(s->U[a], lbv[a % NU], ubv[a % NU]);
    double pg_prev = INFINITY;

    int status = ORACLE_MAX_ITER, it = 0;
    double kkt = INFINITY, mu = 0.0;
    for (it = 0; it <= max_iter; ++it) {
        /* (1) stage evaluation: F_k, A_k = I + h df/dx, B_k = h df/du */
        for (int k = 0; k < N; ++k)
            euler_step(h, s->X + k * NX, s->U + k * NU, s->F + k * NX, s->Ad + k * NX * NX, s->Bd + k * NX * NU);
        double cmax = 0.0;
        for (int i = 0; i < N * NX; ++i) {
            s->c[i] = s->F[i] - s->X[NX + i];
            if (fabs(s->c[i]) > cmax || s->c[i] != s->c[i]) cmax = fabs(s->c[i]);
        }
        /* (2) d_0 = 0, d_{k+1} = A_k d_k + c_k ; e_k = F_k + A_k d_k - r_k */
        memset(s->d, 0, sizeof(double) * NX);
        for (int k = 0; k < N; ++k) {
            for (int r = 0; r < NX; ++r) {
                double ad = 0.0;
                for (int q = 0; q < NX; ++q) ad += s->Ad[k * NX * NX + r * NX + q] * s->d[k * NX + q];
                s->d[(k + 1) * NX + r] = ad + s->c[k * NX + r];
                s->e[k * NX + r] = s->F[k * NX + r] + ad - traj[k * NX + r];
            }
        }
        /* (3) dense Gamma: rows = x_{k+1} (k<N), cols = u_j (j<=k) */
        memset(s->G, 0, sizeof(double) * (size_t)N * NX * M);
        for (int j = 0; j < N; ++j) {
            double col[ORACLE_MAX_NX][ORACLE_MAX_NU], nxt[ORACLE_MAX_NX][ORACLE_MAX_NU];
            for (int r = 0; r < NX; ++r) for (int q = 0; q < NU; ++q) col[r][q] = s->Bd[j * NX * NU + r * NU + q];
            for (int k = j; k < N; ++k) {
                if (k > j) {
                    for (int r = 0; r < NX; ++r) for (int q = 0; q < NU; ++q) {
                        double t = 0.0;
                        for (int p = 0; p < NX; ++p) t += s->Ad[k * NX * NX + r * NX + p] * col[p][q];
                        nxt[r][q] = t;
                    }
                    memcpy(col, nxt, sizeof col);
                }
                for (int r = 0; r < NX; ++r) for (int q = 0; q < NU; ++q)
                    s->G[(size_t)(k * NX + r) * M + j * NU + q] = col[r][q];
            }
        }
        /* (4) H = G^T Qb G + D^T Rb D + Rmb ; g = G^T Qb e + D^T Rb (D u - u~) + Rmb u */
        for (int a = 0; a < M; ++a) {
            for (int b = 0; b <= a; ++b) {
                double t = 0.0;
                for (int i = 0; i < N * NX; ++i) t += s->G[(size_t)i * M + a] * Q[i % NX] * s->G[(size_t)i * M + b];
                s->H[a * M + b] = t;
                s->H[b * M + a] = t;
            }
            double t = 0.0;
            for (int i = 0; i < N * NX; ++i) t += s->G[(size_t)i * M + a] * Q[i % NX] * s->e[i];
            s->g[a] = t;
        }
        for (int k = 0; k < N; ++k) {
            for (int q = 0; q < NU; ++q) {
                int a = k * NU + q;
                double um = (k == 0) ? u_prev[q] : s->U[(k - 1) * NU + q];
                s->H[a * M + a] += R[q] + Rm[q];
                s->g[a] += R[q] * (s->U[a] - um) + Rm[q] * s->U[a];
                if (k + 1 < N) {
                    s->H[a * M + a] += R[q];
                    s->H[a * M + a + NU] -= R[q];
                    s->H[(a + NU) * M + a] -= R[q];
                    s->g[a] -= R[q] * (s->U[a + NU] - s->U[a]);
                }
            }
        }
        double gmax = 0.0;
        if (!has_b) {
            for (int a = 0; a < M; ++a) { double t = fabs(2.0 * s->g[a]); if (t > gmax || t != t) gmax = t; }
        } else {
            /* epsilon-active set (Bertsekas 1982) from the previous iteration's projected gradient: the
             * Riccati kernels decide a stage's set inside the backward sweep that computes this iteration's
             * gradient.  A held control is fixed at its bound in the QP (du_a = bound - u_a). */
            const double eps = fmin(ORACLE_BOUND_EPS, pg_prev);
            for (int a = 0; a < M; ++a) {
                const double u = s->U[a], lb = lbv[a % NU], ub = ubv[a % NU];
                double t = fabs(u - proj(u - 2.0 * s->g[a], lb, ub));
                if (t > gmax || t != t) gmax = t;
                s->tgt[a] = (u <= lb + eps && s->g[a] > 0.0) ? lb : (u >= ub - eps && s->g[a] < 0.0) ? ub : NAN;
            }
            pg_prev = gmax;
        }
        kkt = gmax > cmax ? gmax : cmax;
        if (!isfinite(kkt)) { status = ORACLE_NONFINITE; break; }
        if (gmax <= tol_grad && cmax <= tol_defect) { status = ORACLE_CONVERGED; break; }
        if (it == max_iter) { status = ORACLE_MAX_ITER; break; }

        /* (5) adjoint for the penalty weight: lam_N = Q e_{N-1}; lam_k = Q e_{k-1} + A_k^T lam_{k+1} */
        for (int r = 0; r < NX; ++r) s->lam[N * NX + r] = Q[r] * s->e[(N - 1) * NX + r];
        double lmax = 0.0;
        for (int r = 0; r < NX; ++r) if (fabs(s->lam[N * NX + r]) > lmax) lmax = fabs(s->lam[N * NX + r]);
        for (int k = N - 1; k >= 1; --k) {
            for (int r = 0; r < NX; ++r) {
                double t = Q[r] * s->e[(k - 1) * NX + r];
                for (int p = 0; p < NX; ++p) t += s->Ad[k * NX * NX + p * NX + r] * s->lam[(k + 1) * NX + p];
                s->lam[k * NX + r] = t;
                if (fabs(t) > lmax) lmax = fabs(t);
            }
        }

        /* (6) step: Cholesky of H, du = -H^-1 g; dx_0 = 0, dx_{k+1} = A dx + B du + c.
         * With bounds: the equality-constrained QP with du_a = tgt_a - u_a for the held controls; a free control
         * whose step leaves the box is then held at the bound it crosses and the QP solved again (at most
         * ORACLE_BOUND_PASSES solves; the projected line search absorbs what is left). */
        int fact_fail = 0;
        /* exact Hessian (ORACLE_HESS_EXACT): the QP in (dx, du) gains the stage term 1/2 [dx_k; du_k]^T W_k [..]
         * with W_k = h sum_r lam_{k+1,r} d^2 f_r/d(x_k,u_k)^2 (J/2 scale, lam of step 5); condensed with
         * dx_k = Gamma_k du + d_k (S_k du = [Gamma_k du; du_k]):  H += S_k^T W_k S_k,  g += S_k^T W_k [d_k; 0].
         * The stop test above used the true reduced gradient; W only changes the step.  With control bounds the
         * held controls are fixed in this exact QP as in the Gauss-Newton one (g_exact_bounded). */
        const int use_exact = g_hess_mode == ORACLE_HESS_EXACT && (!has_b || g_exact_bounded) && !g_lin &&
                              model_has_hess();
        if (use_exact) {
            memcpy(s->Hgn, s->H, sizeof(double) * M * M);
            memcpy(s->ggn, s->g, sizeof(double) * M);
            add_exact_condensed(s, h);
        }
        if (has_b) { memcpy(s->H0, s->H, sizeof(double) * M * M); memcpy(s->g0, s->g, sizeof(double) * M); }
        int gn_fallback = 0;
        for (int pass = 0;; ++pass) {
            if (has_b) {
                if (pass) memcpy(s->H, s->H0, sizeof(double) * M * M);
                for (int a = 0; a < M; ++a) s->g[a] = s->g0[a];
                for (int a = 0; a < M; ++a) {
                    if (s->tgt[a] != s->tgt[a]) continue;
                    const double da = s->tgt[a] - s->U[a];
                    for (int b = 0; b < M; ++b) {
                        s->g[b] += s->H0[b * M + a] * da;
                        s->H[a * M + b] = s->H[b * M + a] = 0.0;
                    }
                }
                for (int a = 0; a < M; ++a)
                    if (s->tgt[a] == s->tgt[a]) { s->H[a * M + a] = 1.0; s->g[a] = s->U[a] - s->tgt[a]; }
            }
            for (int a = 0; a < M; ++a) s->du[a] = -s->g[a];
            if (chol_solve(M, s->H, s->du) != 0) {
                if (!use_exact || gn_fallback) { fact_fail = 1; break; }
                /* exact KKT matrix not positive definite: this iteration takes the Gauss-Newton step */
                gn_fallback = 1;
                count_exact_fallback();
                if (has_b) {   /* the same pass again on the Gauss-Newton QP */
                    memcpy(s->H0, s->Hgn, sizeof(double) * M * M);
                    memcpy(s->g0, s->ggn, sizeof(double) * M);
                    memcpy(s->H, s->Hgn, sizeof(double) * M * M);
                    --pass;
                    continue;
                }
                memcpy(s->H, s->Hgn, sizeof(double) * M * M);
                for (int a = 0; a < M; ++a) s->du[a] = -s->ggn[a];
                if (chol_solve(M, s->H, s->du) != 0) { fact_fail = 1; break; }
            }
            if (!has_b || pass + 1 >= ((g_bound_release && it == 0) ? 2 : ORACLE_BOUND_PASSES)) break;
            int added = 0;
            for (int a = 0; a < M; ++a) {
                if (s->tgt[a] == s->tgt[a]) {
                    if (g_bound_release) {   /* the hold's multiplier: release it when it points into the box */
                        double r = s->g0[a];
                        for (int b = 0; b < M; ++b) r += s->H0[a * M + b] * s->du[b];
                        if ((s->tgt[a] == lbv[a % NU] && r < 0.0) || (s->tgt[a] == ubv[a % NU] && r > 0.0)) {
                            s->tgt[a] = NAN;
                            added = 1;
                        }
                    }
                    continue;
                }
                const double t = s->U[a] + s->du[a];
                if (t < lbv[a % NU]) { s->tgt[a] = lbv[a % NU]; added = 1; }
                else if (t > ubv[a % NU]) { s->tgt[a] = ubv[a % NU]; added = 1; }
            }
            if (!added) break;
        }
        if (fact_fail) { status = ORACLE_FACTORIZATION_FAILED; break; }
        memset(s->dx, 0, sizeof(double) * NX);
        for (int k = 0; k < N; ++k)
            for (int r = 0; r < NX; ++r) {
                double t = s->c[k * NX + r];
                for (int q = 0; q < NX; ++q) t += s->Ad[k * NX * NX + r * NX + q] * s->dx[k * NX + q];
                for (int q = 0; q < NU; ++q) t += s->Bd[k * NX * NU + r * NU + q] * s->du[k * NU + q];
                s->dx[(k + 1) * NX + r] = t;
            }

        /* (7) l1-merit Armijo backtracking: phi = J + mu sum|c| */
        double mu_new = 4.0 * lmax + 1.0;
        if (mu_new > mu) mu = mu_new;
        double J0 = 0.0, c1 = 0.0, dJ = 0.0;
        for (int k = 0; k < N; ++k) {
            double qe[ORACLE_MAX_NX];
            for (int r = 0; r < NX; ++r) {
                qe[r] = 2.0 * Q[r] * (s->F[k * NX + r] - traj[k * NX + r]);
                J0 += 0.5 * qe[r] * (s->F[k * NX + r] - traj[k * NX + r]);
                c1 += fabs(s->c[k * NX + r]);
            }
            for (int r = 0; r < NX; ++r) {
                double ax = 0.0, bu = 0.0;
                for (int q = 0; q < NX; ++q) ax += s->Ad[k * NX * NX + r * NX + q] * s->dx[k * NX + q];
                for (int q = 0; q < NU; ++q) bu += s->Bd[k * NX * NU + r * NU + q] * s->du[k * NU + q];
                dJ += qe[r] * (ax + bu);
            }
            for (int q = 0; q < NU; ++q) {
                double um = (k == 0) ? u_prev[q] : s->U[(k - 1) * NU + q];
                double dum = (k == 0) ? 0.0 : s->du[(k - 1) * NU + q];
                double dif = s->U[k * NU + q] - um;
                J0 += dif * R[q] * dif + s->U[k * NU + q] * Rm[q] * s->U[k * NU + q];
                dJ += 2.0 * R[q] * dif * (s->du[k * NU + q] - dum) + 2.0 * Rm[q] * s->U[k * NU + q] * s->du[k * NU + q];
            }
        }
        double phi0 = J0 + mu * c1;
        double dphi = dJ - mu * c1;
        double alpha = 1.0;
        int accepted = 0;
        for (int ls = 0; ls < 30; ++ls) {
            for (int i = 0; i < (N + 1) * NX; ++i) s->Xt[i] = s->X[i] + alpha * s->dx[i];
            for (int i = 0; i < M; ++i) s->Ut[i] = s->U[i] + alpha * s->du[i];
            if (has_b)  /* projected trial point */
                for (int i = 0; i < M; ++i) s->Ut[i] = proj(s->Ut[i], lbv[i % NU], ubv[i % NU]);
            double Jt, ct;
            merit_eval(N, h, s->Xt, s->Ut, u_prev, traj, w, s->Ft, &Jt, &ct);
            double phit = Jt + mu * ct;
            /* noise-aware Armijo (same rule as the HIP kernel): an unresolvable decrease is taken whole,
             * and the test allows 1e-13 |phi| of roundoff in the merit sum */
            double noise = 1.0 + fabs(phi0);
            if (dphi >= -1e-11 * noise || phit <= phi0 + 1e-4 * alpha * dphi + 1e-13 * noise) { accepted = 1; break; }
            /* first iteration: IPOPT's filter acceptance (Waechter & Biegler 2006, eqs. (18)-(21)) -- its filter then
             * holds only theta_max = 1e4 max(1, theta_0), the cold start is far from feasible (no switching), so a
             * trial is taken when it reduces the constraint violation or the objective sufficiently */
            if (it == 0 && oracle_first_iter_filter_accepts(J0, c1, Jt, ct, dJ, alpha)) { accepted = 1; break; }
            alpha *= 0.5;
        }
        if (!accepted) { status = ORACLE_LINESEARCH_FAILED; break; }
        memcpy(s->X, s->Xt, sizeof(double) * (N + 1) * NX);
        memcpy(s->U, s->Ut, sizeof(double) * M);
    }
    /* pack V */
    for (int k = 0; k < N; ++k) {
        memcpy(V + k * ND, s->X + k * NX, sizeof(double) * NX);
        memcpy(V + k * ND + NX, s->U + k * NU, sizeof(double) * NU);
    }
    memcpy(V + N * ND, s->X + N * NX, sizeof(double) * NX);
    if (J_out) {
        double J;
        oracle_nlp_eval(t_model, N, h, V, u_prev, traj, w, &J, NULL);
        *J_out = J;
    }
    *iters_out = it;
    *kkt_out = kkt;
    return status;
}

/* ---------------- the same SQP with a Riccati KKT solve (ORACLE_KKT_RICCATI) ----------------
 * The HIP kernels solve each QP by a Riccati recursion on the augmented state s_k = [dx_k; du_{k-1}] (NS = nx + nu;
 * du_{k-1} carries the Delta-u weight of ModelGenerator.cpp:216-221) instead of condensing.  This restates that
 * formulation on the CPU -- stage evaluation, propagated defects d, adjoint lam and reduced gradient (stop test),
 * exact-Hessian stage blocks, backward Riccati sweep, forward step, l1-merit line search -- so that the CPU
 * baseline of bench.py runs the algorithm the GPU runs (cpu_baseline.riccati).  Same NLP, iterates and stop test
 * as solve_one (the QP solution is identical up to roundoff); unbounded nonlinear solves only.  O(N (nx+nu)^3)
 * per iteration against solve_one's O((N nu)^3). */
static int g_kkt_mode = ORACLE_KKT_DENSE;
void oracle_set_kkt(int mode) { g_kkt_mode = mode; }

/* Cholesky of the nu x nu stage matrix Hw (lower factor in place); -1 if not positive definite */
static int small_chol(int n, double* Hw) {
    for (int j = 0; j < n; ++j) {
        double sd = Hw[j * n + j];
        for (int q = 0; q < j; ++q) sd -= Hw[j * n + q] * Hw[j * n + q];
        if (!(sd > 0.0) || !isfinite(sd)) return -1;
        const double l = sqrt(sd);
        Hw[j * n + j] = l;
        for (int i = j + 1; i < n; ++i) {
            double t = Hw[i * n + j];
            for (int q = 0; q < j; ++q) t -= Hw[i * n + q] * Hw[j * n + q];
            Hw[i * n + j] = t / l;
        }
    }
    return 0;
}
/* x = Hw^-1 b with the factor of small_chol */
static void small_chol_solve(int n, const double* L, const double* b, double* x) {
    double y[ORACLE_MAX_NU];
    for (int i = 0; i < n; ++i) {
        double t = b[i];
        for (int q = 0; q < i; ++q) t -= L[i * n + q] * y[q];
        y[i] = t / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double t = y[i];
        for (int q = i + 1; q < n; ++q) t -= L[q * n + i] * x[q];
        x[i] = t / L[i * n + i];
    }
}

/* backward Riccati sweep of the QP at the current iterate (J/2 scale): value function 1/2 s^T P s + p^T s of
 * s_k = [dx_k; du_{k-1}], P_N = blkdiag(Q, 0), p_N = [Q (x_N - r_{N-1}); 0]; per stage k
 *   Q_uu = [B;I]^T P [B;I] + R + Rm (+ W_uu),   Q_us = [G^T A (+ W_ux) | -R],  G = P_xx B + P_xu,
 *   q_u  = B^T (P_xx c + p_x) + P_ux c + p_u + R (u_k - u_{k-1}) + Rm u_k,
 *   [K_k | kff_k] = -Q_uu^-1 [Q_us | q_u],
 *   P_k = blkdiag(A^T P_xx A + Q (+ W_xx), R) - Q_us^T Q_uu^-1 Q_us,
 *   p_k = [A^T (P_xx c + p_x) + Q (x_k - r_{k-1}); -R (u_k - u_{k-1})] - Q_us^T Q_uu^-1 q_u.
 * useW: add the exact-Hessian blocks s->Wk.  Returns -1 when a Q_uu is not positive definite. */
static int riccati_backward(ws_t* s, const double* traj, const double* w, const double* u_prev, int useW) {
    const int N = s->N, NS = NX + NU, K = NX + NU;
    const double *Q = w, *R = w + NX, *Rm = w + NX + NU;
    double P[(ORACLE_MAX_NX + ORACLE_MAX_NU) * (ORACLE_MAX_NX + ORACLE_MAX_NU)], p[ORACLE_MAX_NX + ORACLE_MAX_NU];
    double Pn[(ORACLE_MAX_NX + ORACLE_MAX_NU) * (ORACLE_MAX_NX + ORACLE_MAX_NU)], pn[ORACLE_MAX_NX + ORACLE_MAX_NU];
    for (int i = 0; i < NS * NS; ++i) P[i] = 0.0;
    for (int r = 0; r < NX; ++r) {
        P[r * NS + r] = Q[r];
        p[r] = Q[r] * (s->X[N * NX + r] - traj[(N - 1) * NX + r]);
    }
    for (int c = 0; c < NU; ++c) p[NX + c] = 0.0;
    for (int k = N - 1; k >= 0; --k) {
        const double *A = s->Ad + (size_t)k * NX * NX, *Bm = s->Bd + (size_t)k * NX * NU, *cc = s->c + k * NX;
        const double* u = s->U + k * NU;
        const double* um = (k == 0) ? u_prev : s->U + (k - 1) * NU;
        const double* Wk = s->Wk + (size_t)k * K * K;
        double G[ORACLE_MAX_NX * ORACLE_MAX_NU], mv[ORACLE_MAX_NX], Hw[ORACLE_MAX_NU * ORACLE_MAX_NU];
        double Y[ORACLE_MAX_NU * (ORACLE_MAX_NX + ORACLE_MAX_NU + 1)];   /* [Q_us | q_u], NU x (NS + 1) */
        for (int r = 0; r < NX; ++r) {
            for (int c = 0; c < NU; ++c) {
                double t = P[r * NS + NX + c];
                for (int q = 0; q < NX; ++q) t += P[r * NS + q] * Bm[q * NU + c];
                G[r * NU + c] = t;
            }
            double t = p[r];
            for (int q = 0; q < NX; ++q) t += P[r * NS + q] * cc[q];
            mv[r] = t;
        }
        for (int a = 0; a < NU; ++a) {
            for (int b = 0; b < NU; ++b) {
                double t = P[(NX + a) * NS + NX + b];
                for (int q = 0; q < NX; ++q) t += Bm[q * NU + a] * G[q * NU + b] + P[(NX + a) * NS + q] * Bm[q * NU + b];
                if (a == b) t += R[a] + Rm[a];
                if (useW) t += Wk[(NX + a) * K + NX + b];
                Hw[a * NU + b] = t;
            }
            double* y = Y + a * (NS + 1);
            for (int j = 0; j < NX; ++j) {   /* (G^T A)[a][j] (+ W_ux) */
                double t = 0.0;
                for (int q = 0; q < NX; ++q) t += G[q * NU + a] * A[q * NX + j];
                if (useW) t += Wk[(NX + a) * K + j];
                y[j] = t;
            }
            for (int c = 0; c < NU; ++c) y[NX + c] = (a == c) ? -R[a] : 0.0;
            double t = p[NX + a] + R[a] * (u[a] - um[a]) + Rm[a] * u[a];
            for (int q = 0; q < NX; ++q) t += Bm[q * NU + a] * mv[q] + P[(NX + a) * NS + q] * cc[q];
            y[NS] = t;
        }
        if (small_chol(NU, Hw) != 0) return -1;
        double* Kk = s->Kf + (size_t)k * NU * (NS + 1);   /* row a: K_k[a][0..NS), kff_k[a] */
        for (int j = 0; j <= NS; ++j) {
            double col[ORACLE_MAX_NU], sol[ORACLE_MAX_NU];
            for (int a = 0; a < NU; ++a) col[a] = Y[a * (NS + 1) + j];
            small_chol_solve(NU, Hw, col, sol);
            for (int a = 0; a < NU; ++a) Kk[a * (NS + 1) + j] = -sol[a];
        }
        if (k == 0) break;
        /* P_k, p_k before the Schur complement */
        for (int i = 0; i < NS * NS; ++i) Pn[i] = 0.0;
        for (int i = 0; i < NX; ++i) {
            for (int j = 0; j < NX; ++j) {
                double t = 0.0;
                for (int q = 0; q < NX; ++q) {
                    double pa = 0.0;
                    for (int r = 0; r < NX; ++r) pa += P[q * NS + r] * A[r * NX + j];
                    t += A[q * NX + i] * pa;
                }
                if (i == j) t += Q[i];
                if (useW) t += Wk[i * K + j];
                Pn[i * NS + j] = t;
            }
            double t = Q[i] * (s->X[k * NX + i] - traj[(k - 1) * NX + i]);
            for (int q = 0; q < NX; ++q) t += A[q * NX + i] * mv[q];
            pn[i] = t;
        }
        for (int c = 0; c < NU; ++c) {
            Pn[(NX + c) * NS + NX + c] = R[c];
            pn[NX + c] = -R[c] * (u[c] - um[c]);
        }
        /* - Q_us^T Q_uu^-1 [Q_us | q_u] = + Q_us^T [K | kff] */
        for (int i = 0; i < NS; ++i) {
            for (int j = 0; j < NS; ++j) {
                double t = Pn[i * NS + j];
                for (int a = 0; a < NU; ++a) t += Y[a * (NS + 1) + i] * Kk[a * (NS + 1) + j];
                P[i * NS + j] = t;
            }
            double t = pn[i];
            for (int a = 0; a < NU; ++a) t += Y[a * (NS + 1) + i] * Kk[a * (NS + 1) + NS];
            p[i] = t;
        }
        for (int i = 0; i < NS; ++i)   /* symmetric by construction up to roundoff: keep it exactly symmetric */
            for (int j = i + 1; j < NS; ++j) P[j * NS + i] = P[i * NS + j] = 0.5 * (P[i * NS + j] + P[j * NS + i]);
    }
    return 0;
}

static int solve_one_riccati(ws_t* s, double h, const double* x0, const double* u_prev, const double* traj,
                             const double* w, int max_iter, double tol_grad, double tol_defect, double* V,
                             int32_t* iters_out, double* kkt_out, double* J_out) {
    const int N = s->N, M = s->M, K = NX + NU, NS = NX + NU;
    const double *Q = w, *R = w + NX, *Rm = w + NX + NU;
    for (int k = 0; k < N; ++k) {
        memcpy(s->X + k * NX, V + k * ND, sizeof(double) * NX);
        memcpy(s->U + k * NU, V + k * ND + NX, sizeof(double) * NU);
    }
    memcpy(s->X + N * NX, V + N * ND, sizeof(double) * NX);
    if (g_init_zero) {
        memset(s->X, 0, sizeof(double) * (N + 1) * NX);
        memset(s->U, 0, sizeof(double) * N * NU);
    }
    memcpy(s->X, x0, sizeof(double) * NX);
    if (g_init_hold)
        for (int k = 1; k <= N; ++k) memcpy(s->X + k * NX, x0, sizeof(double) * NX);
    const int use_exact = g_hess_mode == ORACLE_HESS_EXACT && !g_lin && model_has_hess();
    int status = ORACLE_MAX_ITER, it = 0;
    double kkt = INFINITY, mu = 0.0;
    for (it = 0; it <= max_iter; ++it) {
        double cmax = 0.0;
        for (int k = 0; k < N; ++k)
            euler_step(h, s->X + k * NX, s->U + k * NU, s->F + k * NX, s->Ad + (size_t)k * NX * NX,
                       s->Bd + (size_t)k * NX * NU);
        for (int i = 0; i < N * NX; ++i) {
            s->c[i] = s->F[i] - s->X[NX + i];
            if (fabs(s->c[i]) > cmax || s->c[i] != s->c[i]) cmax = fabs(s->c[i]);
        }
        /* propagated defects d and the adjoint of the condensed objective (J/2 scale) */
        memset(s->d, 0, sizeof(double) * NX);
        for (int k = 0; k < N; ++k)
            for (int r = 0; r < NX; ++r) {
                double t = s->c[k * NX + r];
                for (int q = 0; q < NX; ++q) t += s->Ad[(size_t)k * NX * NX + r * NX + q] * s->d[k * NX + q];
                s->d[(k + 1) * NX + r] = t;
            }
        double lmax = 0.0;
        for (int r = 0; r < NX; ++r) {
            s->lam[N * NX + r] = Q[r] * (s->d[N * NX + r] + s->X[N * NX + r] - traj[(N - 1) * NX + r]);
            if (fabs(s->lam[N * NX + r]) > lmax) lmax = fabs(s->lam[N * NX + r]);
        }
        for (int k = N - 1; k >= 1; --k)
            for (int r = 0; r < NX; ++r) {
                double t = Q[r] * (s->d[k * NX + r] + s->X[k * NX + r] - traj[(k - 1) * NX + r]);
                for (int q = 0; q < NX; ++q) t += s->Ad[(size_t)k * NX * NX + q * NX + r] * s->lam[(k + 1) * NX + q];
                s->lam[k * NX + r] = t;
                if (fabs(t) > lmax) lmax = fabs(t);
            }
        double gmax = 0.0;
        for (int k = 0; k < N; ++k)
            for (int c = 0; c < NU; ++c) {
                double g = 0.0;
                for (int q = 0; q < NX; ++q) g += s->Bd[(size_t)k * NX * NU + q * NU + c] * s->lam[(k + 1) * NX + q];
                const double uk = s->U[k * NU + c], um = (k == 0) ? u_prev[c] : s->U[(k - 1) * NU + c];
                g += R[c] * (uk - um) + Rm[c] * uk;
                if (k + 1 < N) g -= R[c] * (s->U[(k + 1) * NU + c] - uk);
                const double t = fabs(2.0 * g);
                if (t > gmax || t != t) gmax = t;
            }
        kkt = gmax > cmax ? gmax : cmax;
        if (!isfinite(kkt)) { status = ORACLE_NONFINITE; break; }
        if (gmax <= tol_grad && cmax <= tol_defect) { status = ORACLE_CONVERGED; break; }
        if (it == max_iter) { status = ORACLE_MAX_ITER; break; }
        if (use_exact)   /* W_k = h sum_r lam_{k+1,r} d^2 f_r/d(x_k,u_k)^2 */
            for (int k = 0; k < N; ++k) {
                double* Wk = s->Wk + (size_t)k * K * K;
                model_hess(s->X + k * NX, s->U + k * NU, s->lam + (k + 1) * NX, Wk);
                for (int i = 0; i < K * K; ++i) Wk[i] *= h;
            }
        int rc = riccati_backward(s, traj, w, u_prev, use_exact);
        if (rc != 0 && use_exact) {   /* not PD: Gauss-Newton step */
            count_exact_fallback();
            rc = riccati_backward(s, traj, w, u_prev, 0);
        }
        if (rc != 0) { status = ORACLE_FACTORIZATION_FAILED; break; }
        /* forward: du_k = K_k [dx_k; du_{k-1}] + kff_k, dx_{k+1} = A dx_k + B du_k + c_k */
        memset(s->dx, 0, sizeof(double) * NX);
        for (int k = 0; k < N; ++k) {
            const double* Kk = s->Kf + (size_t)k * NU * (NS + 1);
            for (int a = 0; a < NU; ++a) {
                double t = Kk[a * (NS + 1) + NS];
                for (int q = 0; q < NX; ++q) t += Kk[a * (NS + 1) + q] * s->dx[k * NX + q];
                if (k > 0)
                    for (int c = 0; c < NU; ++c) t += Kk[a * (NS + 1) + NX + c] * s->du[(k - 1) * NU + c];
                s->du[k * NU + a] = t;
            }
            for (int r = 0; r < NX; ++r) {
                double t = s->c[k * NX + r];
                for (int q = 0; q < NX; ++q) t += s->Ad[(size_t)k * NX * NX + r * NX + q] * s->dx[k * NX + q];
                for (int q = 0; q < NU; ++q) t += s->Bd[(size_t)k * NX * NU + r * NU + q] * s->du[k * NU + q];
                s->dx[(k + 1) * NX + r] = t;
            }
        }
        /* l1-merit Armijo line search, as solve_one */
        double mu_new = 4.0 * lmax + 1.0;
        if (mu_new > mu) mu = mu_new;
        double J0 = 0.0, c1 = 0.0, dJ = 0.0;
        for (int k = 0; k < N; ++k) {
            for (int r = 0; r < NX; ++r) {
                const double e = s->F[k * NX + r] - traj[k * NX + r];
                J0 += e * Q[r] * e;
                c1 += fabs(s->c[k * NX + r]);
                double ad = s->dx[(k + 1) * NX + r] - s->c[k * NX + r];   /* A dx_k + B du_k */
                dJ += 2.0 * Q[r] * e * ad;
            }
            for (int q = 0; q < NU; ++q) {
                const double um = (k == 0) ? u_prev[q] : s->U[(k - 1) * NU + q];
                const double dum = (k == 0) ? 0.0 : s->du[(k - 1) * NU + q];
                const double uk = s->U[k * NU + q], dif = uk - um;
                J0 += dif * R[q] * dif + uk * Rm[q] * uk;
                dJ += 2.0 * R[q] * dif * (s->du[k * NU + q] - dum) + 2.0 * Rm[q] * uk * s->du[k * NU + q];
            }
        }
        const double phi0 = J0 + mu * c1, dphi = dJ - mu * c1;
        double alpha = 1.0;
        int accepted = 0;
        for (int ls = 0; ls < 30; ++ls) {
            for (int i = 0; i < (N + 1) * NX; ++i) s->Xt[i] = s->X[i] + alpha * s->dx[i];
            for (int i = 0; i < M; ++i) s->Ut[i] = s->U[i] + alpha * s->du[i];
            double Jt, ct;
            merit_eval(N, h, s->Xt, s->Ut, u_prev, traj, w, s->Ft, &Jt, &ct);
            const double phit = Jt + mu * ct, noise = 1.0 + fabs(phi0);
            if (dphi >= -1e-11 * noise || phit <= phi0 + 1e-4 * alpha * dphi + 1e-13 * noise) { accepted = 1; break; }
            if (it == 0 && oracle_first_iter_filter_accepts(J0, c1, Jt, ct, dJ, alpha)) { accepted = 1; break; }
            alpha *= 0.5;
        }
        if (!accepted) { status = ORACLE_LINESEARCH_FAILED; break; }
        memcpy(s->X, s->Xt, sizeof(double) * (N + 1) * NX);
        memcpy(s->U, s->Ut, sizeof(double) * M);
    }
    for (int k = 0; k < N; ++k) {
        memcpy(V + k * ND, s->X + k * NX, sizeof(double) * NX);
        memcpy(V + k * ND + NX, s->U + k * NU, sizeof(double) * NU);
    }
    memcpy(V + N * ND, s->X + N * NX, sizeof(double) * NX);
    if (J_out) {
        double J;
        oracle_nlp_eval(t_model, N, h, V, u_prev, traj, w, &J, NULL);
        *J_out = J;
    }
    *iters_out = it;
    *kkt_out = kkt;
    return status;
}

/* ---------------- state bounds: primal-dual interior point (IPOPT-style) on the same GN model ----------------
 * The reference hands x_min/x_max to IPOPT as lbx/ubx of x_1..x_N (ModelControl.cpp:37-50,146-157) -- IPOPT is a
 * primal-dual barrier method (Waechter & Biegler 2006).  With finite state bounds the build runs the same kind of
 * method on its Gauss-Newton model, for the state AND control bounds of the instance (the projected method of
 * solve_one covers control-only bounds):
 *   f = J/2 (the H, g of solve_one), barrier problem  min f - mu sum log s,  s = y - l | u - y  (finite bounds);
 *   step: (H + Sigma) on the multiple-shooting variables, Sigma = z_l/s_l + z_u/s_u, gradient g - mu/s_l + mu/s_u,
 *         condensed: Hc = H + Sigma_U + G^T Sigma_X G, gc = g + b_U + G^T (b_X + Sigma_X d);
 *   dz_l = mu/s_l - z_l - (z_l/s_l) dy,  dz_u = mu/s_u - z_u + (z_u/s_u) dy;
 *   fraction to the boundary tau = 0.99 for the primal (alpha_max) and dual (alpha_z) steps;
 *   l1-merit Armijo backtracking from alpha_max on  J - 2 mu sum log s + nu |c|_1  (J-scale, as solve_one);
 *   z safeguard  z in [mu / (1e10 s), 1e10 mu / s]  (IPOPT kappa_Sigma);
 *   KKT error E_mu = max(|g + G^T(z_ux - z_lx) + z_uu - z_lu|, |c|, |s z - mu|); the barrier parameter is
 *   updated after the step when E_mu <= 10 mu:  mu <- max(tol_c/20, min(0.2 mu, mu^1.5))  (IPOPT monotone rule,
 *   lagged one iteration so that the Riccati kernels can fuse the test into their backward sweep);
 *   start: mu = 0.1, z = 1, y pushed 1e-2 max(1, |bound|) (at most 1e-2 of the box) inside its bounds;
 *   stop: 2|reduced Lagrangian gradient| <= tol_grad, |c| <= tol_defect, 2 max s z <= IP_TOL_COMPL (J-scale). */
#define IP_MU0 0.1
#define IP_KAPPA_EPS 10.0
#define IP_KAPPA_MU 0.2
#define IP_THETA_MU 1.5
#define IP_PUSH 1e-2
#define IP_KAPPA_SIGMA 1e10
/* complementarity tolerance (J-scale, 2 max s z; IPOPT's default compl_inf_tol is 1e-4) and a constant fraction
 * to the boundary tau = 0.99 (IPOPT: max(0.99, 1 - mu), which near the solution lets a slack collapse by a factor
 * mu in one step): together they keep Sigma = z/s near z^2/mu_final ~ 1e12 -- the Riccati kernels' Schur
 * complements lose positive definiteness to cancellation once Sigma reaches ~1e15 */
#define IP_TOL_COMPL 1e-8
#define IP_TAU 0.99

/* barrier-parameter rule of solve_one_ip: 0 = IPOPT's monotone rule (shipped), 1 = Mehrotra predictor-corrector
 * (round 5 experiment: an affine predictor solve, sigma = (mu_aff / mu)^3, a corrector solve with the second-order
 * term on the same factor) */
static int g_ip_rule = 0;
void oracle_set_ip_rule(int rule) { g_ip_rule = rule; }

/* solve with the Cholesky factor chol_solve left in the lower triangle of H */
static void chol_resolve(int M, const double* L, double* b) {
    for (int i = 0; i < M; ++i) {
        double t = b[i];
        for (int k = 0; k < i; ++k) t -= L[i * M + k] * b[k];
        b[i] = t / L[i * M + i];
    }
    for (int i = M - 1; i >= 0; --i) {
        double t = b[i];
        for (int k = i + 1; k < M; ++k) t -= L[k * M + i] * b[k];
        b[i] = t / L[i * M + i];
    }
}

static double ip_push(double y, double l, double u) {
    const double pl = (l > -INFINITY) ? fmin(IP_PUSH * fmax(1.0, fabs(l)), (u < INFINITY) ? IP_PUSH * (u - l) : INFINITY) : 0.0;
    const double pu = (u < INFINITY) ? fmin(IP_PUSH * fmax(1.0, fabs(u)), (l > -INFINITY) ? IP_PUSH * (u - l) : INFINITY) : 0.0;
    if (l > -INFINITY && y < l + pl) y = l + pl;
    if (u < INFINITY && y > u - pu) y = u - pu;
    return y;
}

static int solve_one_ip(ws_t* s, double h, const double* x0, const double* u_prev, const double* traj,
                        const double* w, const double* u_lb, const double* u_ub, const double* x_lb,
                        const double* x_ub, int max_iter, double tol_grad, double tol_defect, double* V,
                        int32_t* iters_out, double* kkt_out, double* J_out) {
    const int N = s->N, M = s->M, S = N * NX;
    const double *Q = w, *R = w + NX, *Rm = w + NX + NU;
    double lx[ORACLE_MAX_NX], ux[ORACLE_MAX_NX], lu[ORACLE_MAX_NU], uu[ORACLE_MAX_NU];
    for (int r = 0; r < NX; ++r) {
        lx[r] = (x_lb && x_lb[r] > -1e19) ? x_lb[r] : -INFINITY;
        ux[r] = (x_ub && x_ub[r] < 1e19) ? x_ub[r] : INFINITY;
    }
    for (int q = 0; q < NU; ++q) {
        lu[q] = (u_lb && u_lb[q] > -1e19) ? u_lb[q] : -INFINITY;
        uu[q] = (u_ub && u_ub[q] < 1e19) ? u_ub[q] : INFINITY;
    }
    /* y = (X_1..X_N | U): bounds, duals, Sigma, barrier gradient b, steps */
    const int NY = S + M;
    double* yl = calloc((size_t)NY, sizeof(double));
    double* yu = calloc((size_t)NY, sizeof(double));
    double* zl = calloc((size_t)NY, sizeof(double));
    double* zu = calloc((size_t)NY, sizeof(double));
    double* sg = calloc((size_t)NY, sizeof(double));
    double* bb = calloc((size_t)NY, sizeof(double));
    double* zg = calloc((size_t)NY, sizeof(double));
    double* dy = calloc((size_t)NY, sizeof(double));
    double* tv = calloc((size_t)S, sizeof(double));
    for (int i = 0; i < S; ++i) { yl[i] = lx[i % NX]; yu[i] = ux[i % NX]; }
    for (int a = 0; a < M; ++a) { yl[S + a] = lu[a % NU]; yu[S + a] = uu[a % NU]; }
#define YV(i) ((i) < S ? s->X[NX + (i)] : s->U[(i) - S])
    for (int k = 0; k < N; ++k) {
        memcpy(s->X + k * NX, V + k * ND, sizeof(double) * NX);
        memcpy(s->U + k * NU, V + k * ND + NX, sizeof(double) * NU);
    }
    memcpy(s->X + N * NX, V + N * ND, sizeof(double) * NX);
    if (g_init_zero) {  /* MMPC_INIT_ZERO: the reference's first call, V = 0 (ModelControl.cpp:29-50) */
        memset(s->X, 0, sizeof(double) * (N + 1) * NX);
        memset(s->U, 0, sizeof(double) * N * NU);
    }
    memcpy(s->X, x0, sizeof(double) * NX);
    if (g_init_hold)  /* MMPC_INIT_HOLD_X0: the state trajectory starts at the measured state */
        for (int k = 1; k <= N; ++k) memcpy(s->X + k * NX, x0, sizeof(double) * NX);
    for (int i = 0; i < NY; ++i) {
        double* p = (i < S) ? &s->X[NX + i] : &s->U[i - S];
        *p = ip_push(*p, yl[i], yu[i]);
        zl[i] = (yl[i] > -INFINITY) ? 1.0 : 0.0;
        zu[i] = (yu[i] < INFINITY) ? 1.0 : 0.0;
    }
    double mu_b = IP_MU0;  /* barrier parameter (f-scale) */
    int status = ORACLE_MAX_ITER, it = 0;
    double kkt = INFINITY, nu_pen = 0.0;
    for (it = 0; it <= max_iter; ++it) {
        for (int k = 0; k < N; ++k)
            euler_step(h, s->X + k * NX, s->U + k * NU, s->F + k * NX, s->Ad + k * NX * NX, s->Bd + k * NX * NU);
        double cmax = 0.0;
        for (int i = 0; i < S; ++i) {
            s->c[i] = s->F[i] - s->X[NX + i];
            if (fabs(s->c[i]) > cmax || s->c[i] != s->c[i]) cmax = fabs(s->c[i]);
        }
        memset(s->d, 0, sizeof(double) * NX);
        for (int k = 0; k < N; ++k)
            for (int r = 0; r < NX; ++r) {
                double ad = 0.0;
                for (int q = 0; q < NX; ++q) ad += s->Ad[k * NX * NX + r * NX + q] * s->d[k * NX + q];
                s->d[(k + 1) * NX + r] = ad + s->c[k * NX + r];
                s->e[k * NX + r] = s->F[k * NX + r] + ad - traj[k * NX + r];
            }
        memset(s->G, 0, sizeof(double) * (size_t)S * M);
        for (int j = 0; j < N; ++j) {
            double col[ORACLE_MAX_NX][ORACLE_MAX_NU], nxt[ORACLE_MAX_NX][ORACLE_MAX_NU];
            for (int r = 0; r < NX; ++r) for (int q = 0; q < NU; ++q) col[r][q] = s->Bd[j * NX * NU + r * NU + q];
            for (int k = j; k < N; ++k) {
                if (k > j) {
                    for (int r = 0; r < NX; ++r) for (int q = 0; q < NU; ++q) {
                        double t = 0.0;
                        for (int p2 = 0; p2 < NX; ++p2) t += s->Ad[k * NX * NX + r * NX + p2] * col[p2][q];
                        nxt[r][q] = t;
                    }
                    memcpy(col, nxt, sizeof col);
                }
                for (int r = 0; r < NX; ++r) for (int q = 0; q < NU; ++q)
                    s->G[(size_t)(k * NX + r) * M + j * NU + q] = col[r][q];
            }
        }
        for (int a = 0; a < M; ++a) {
            for (int b = 0; b <= a; ++b) {
                double t = 0.0;
                for (int i = 0; i < S; ++i) t += s->G[(size_t)i * M + a] * Q[i % NX] * s->G[(size_t)i * M + b];
                s->H[a * M + b] = t;
                s->H[b * M + a] = t;
            }
            double t = 0.0;
            for (int i = 0; i < S; ++i) t += s->G[(size_t)i * M + a] * Q[i % NX] * s->e[i];
            s->g[a] = t;
        }
        for (int k = 0; k < N; ++k)
            for (int q = 0; q < NU; ++q) {
                int a = k * NU + q;
                double um = (k == 0) ? u_prev[q] : s->U[(k - 1) * NU + q];
                s->H[a * M + a] += R[q] + Rm[q];
                s->g[a] += R[q] * (s->U[a] - um) + Rm[q] * s->U[a];
                if (k + 1 < N) {
                    s->H[a * M + a] += R[q];
                    s->H[a * M + a + NU] -= R[q];
                    s->H[(a + NU) * M + a] -= R[q];
                    s->g[a] -= R[q] * (s->U[a + NU] - s->U[a]);
                }
            }
        /* barrier pieces at y: Sigma, b = -mu/s_l + mu/s_u, z_u - z_l, complementarity */
        double cmpl0 = 0.0, cmplmu = 0.0, logsum = 0.0;
        for (int i = 0; i < NY; ++i) {
            const double y = YV(i);
            sg[i] = 0.0; bb[i] = 0.0; zg[i] = 0.0;
            if (yl[i] > -INFINITY) {
                const double sl = y - yl[i];
                sg[i] += zl[i] / sl; bb[i] -= mu_b / sl; zg[i] -= zl[i];
                cmpl0 = fmax(cmpl0, fabs(sl * zl[i])); cmplmu = fmax(cmplmu, fabs(sl * zl[i] - mu_b));
                logsum += log(sl);
            }
            if (yu[i] < INFINITY) {
                const double su = yu[i] - y;
                sg[i] += zu[i] / su; bb[i] += mu_b / su; zg[i] += zu[i];
                cmpl0 = fmax(cmpl0, fabs(su * zu[i])); cmplmu = fmax(cmplmu, fabs(su * zu[i] - mu_b));
                logsum += log(su);
            }
        }
        /* reduced Lagrangian gradient gz = g + G^T zg_X + zg_U */
        double gzmax = 0.0;
        for (int a = 0; a < M; ++a) {
            double t = s->g[a] + zg[S + a];
            for (int i = 0; i < S; ++i) t += s->G[(size_t)i * M + a] * zg[i];
            if (fabs(t) > gzmax || t != t) gzmax = fabs(t);
        }
        kkt = fmax(fmax(2.0 * gzmax, cmax), 2.0 * cmpl0);
        if (!isfinite(kkt)) { status = ORACLE_NONFINITE; break; }
        if (2.0 * gzmax <= tol_grad && cmax <= tol_defect && 2.0 * cmpl0 <= IP_TOL_COMPL) { status = ORACLE_CONVERGED; break; }
        if (it == max_iter) { status = ORACLE_MAX_ITER; break; }
        const double e_mu = fmax(fmax(gzmax, cmax), cmplmu);
        const double mu_next = (e_mu <= IP_KAPPA_EPS * mu_b)
                                   ? fmax(IP_TOL_COMPL / 20.0, fmin(IP_KAPPA_MU * mu_b, pow(mu_b, IP_THETA_MU)))
                                   : mu_b;
        /* adjoint of the barrier problem's Lagrangian (the merit's penalty weight, as solve_one, and the multipliers of
         * the exact Hessian): lam_k = Q e_{k-1} + A_k^T lam_{k+1} + (z_u - z_l) of x_k -- the kernels' adjoint
         * (sqp_lane.h / sqp_group.h XB; round 6: the bound duals' term, which the reduced gradient gz above carries
         * as G^T zg_X, was left out here before) */
        for (int r = 0; r < NX; ++r) s->lam[N * NX + r] = Q[r] * s->e[(N - 1) * NX + r] + zg[(N - 1) * NX + r];
        double lmax = 0.0;
        for (int r = 0; r < NX; ++r) if (fabs(s->lam[N * NX + r]) > lmax) lmax = fabs(s->lam[N * NX + r]);
        for (int k = N - 1; k >= 1; --k)
            for (int r = 0; r < NX; ++r) {
                double t = Q[r] * s->e[(k - 1) * NX + r];
                for (int p2 = 0; p2 < NX; ++p2) t += s->Ad[k * NX * NX + p2 * NX + r] * s->lam[(k + 1) * NX + p2];
                t += zg[(k - 1) * NX + r];
                s->lam[k * NX + r] = t;
                if (fabs(t) > lmax) lmax = fabs(t);
            }
        /* condensed barrier Newton step: Hc = H + Sigma_U + G^T Sigma_X G, gc = g + b_U + G^T (b_X + Sigma_X d) */
        for (int a = 0; a < M; ++a) {
            for (int b = 0; b <= a; ++b) {
                double t = 0.0;
                for (int i = 0; i < S; ++i) t += s->G[(size_t)i * M + a] * sg[i] * s->G[(size_t)i * M + b];
                s->H[a * M + b] += t;
                if (b != a) s->H[b * M + a] += t;
            }
            s->H[a * M + a] += sg[S + a];
        }
        /* exact Hessian (ORACLE_HESS_EXACT; IPOPT's default with the barrier, ModelGenerator.cpp:232,238): the
         * barrier Newton matrix gains the condensed stage terms S_k^T W_k S_k (lam: the adjoint above); when the
         * result is not positive definite this iteration takes the Gauss-Newton barrier step (the kernels redo
         * their Riccati sweep without W: a stage H_ww not positive definite <=> the condensed matrix is not) */
        if (g_hess_mode == ORACLE_HESS_EXACT && !g_lin && model_has_hess()) {
            memcpy(s->Hgn, s->H, sizeof(double) * M * M);
            memcpy(s->ggn, s->g, sizeof(double) * M);
            add_exact_condensed(s, h);
            memcpy(s->H0, s->H, sizeof(double) * M * M);
            for (int a = 0; a < M; ++a) s->g0[a] = 0.0;
            if (chol_solve(M, s->H0, s->g0) != 0) {   /* not positive definite: the Gauss-Newton step */
                count_exact_fallback();
                memcpy(s->H, s->Hgn, sizeof(double) * M * M);
                memcpy(s->g, s->ggn, sizeof(double) * M);
            }
        }
        /* rhs of the step for the barrier gradient bv (b of the monotone rule; the corrected b of Mehrotra's),
         * solved with the factor of Hc (factored by the first call), expanded to dx and dy */
        int fact_done = 0;
        #define IP_SOLVE(bv)                                                                                        \
            do {                                                                                                    \
                for (int i = 0; i < S; ++i) tv[i] = (bv)[i] + sg[i] * s->d[NX + i];                                 \
                for (int a = 0; a < M; ++a) {                                                                       \
                    double t = s->g[a] + (bv)[S + a];                                                               \
                    for (int i = 0; i < S; ++i) t += s->G[(size_t)i * M + a] * tv[i];                              \
                    s->du[a] = -t;                                                                                  \
                }                                                                                                   \
                if (!fact_done) {                                                                                   \
                    if (chol_solve(M, s->H, s->du) != 0) { fact_done = -1; break; }                                 \
                    fact_done = 1;                                                                                  \
                } else {                                                                                            \
                    chol_resolve(M, s->H, s->du);                                                                   \
                }                                                                                                   \
                memset(s->dx, 0, sizeof(double) * NX);                                                              \
                for (int k = 0; k < N; ++k)                                                                         \
                    for (int r = 0; r < NX; ++r) {                                                                  \
                        double t = s->c[k * NX + r];                                                                \
                        for (int q = 0; q < NX; ++q) t += s->Ad[k * NX * NX + r * NX + q] * s->dx[k * NX + q];      \
                        for (int q = 0; q < NU; ++q) t += s->Bd[k * NX * NU + r * NU + q] * s->du[k * NU + q];      \
                        s->dx[(k + 1) * NX + r] = t;                                                                \
                    }                                                                                               \
                for (int i = 0; i < S; ++i) dy[i] = s->dx[NX + i];                                                  \
                for (int a = 0; a < M; ++a) dy[S + a] = s->du[a];                                                   \
            } while (0)
        /* Mehrotra: the target mu and the corrected barrier gradient replace mu_b and bb of this iteration */
        double* ccl = NULL;   /* corrector terms of the dual steps: mu_t - ds_aff dz_aff per lower / upper bound */
        double* ccu = NULL;
        if (g_ip_rule == 1 || g_ip_rule == 2) {
            double* b0 = calloc((size_t)NY, sizeof(double));
            IP_SOLVE(b0);   /* affine predictor: mu = 0 */
            if (fact_done < 0) { free(b0); status = ORACLE_FACTORIZATION_FAILED; break; }
            double ap = 1.0, ad = 1.0, sz = 0.0;
            int m = 0;
            for (int i = 0; i < NY; ++i) {
                const double y = YV(i);
                if (yl[i] > -INFINITY) {
                    const double sl = y - yl[i], dz = -zl[i] - zl[i] / sl * dy[i];
                    if (dy[i] < 0.0) ap = fmin(ap, -sl / dy[i]);
                    if (dz < 0.0) ad = fmin(ad, -zl[i] / dz);
                    sz += sl * zl[i];
                    ++m;
                }
                if (yu[i] < INFINITY) {
                    const double su = yu[i] - y, dz = -zu[i] + zu[i] / su * dy[i];
                    if (dy[i] > 0.0) ap = fmin(ap, su / dy[i]);
                    if (dz < 0.0) ad = fmin(ad, -zu[i] / dz);
                    sz += su * zu[i];
                    ++m;
                }
            }
            double saff = 0.0;
            ccl = calloc((size_t)NY, sizeof(double));
            ccu = calloc((size_t)NY, sizeof(double));
            for (int i = 0; i < NY; ++i) {
                const double y = YV(i);
                if (yl[i] > -INFINITY) {
                    const double sl = y - yl[i], dz = -zl[i] - zl[i] / sl * dy[i];
                    saff += (sl + ap * dy[i]) * (zl[i] + ad * dz);
                    ccl[i] = -dy[i] * dz;
                }
                if (yu[i] < INFINITY) {
                    const double su = yu[i] - y, dz = -zu[i] + zu[i] / su * dy[i];
                    saff += (su - ap * dy[i]) * (zu[i] + ad * dz);
                    ccu[i] = dy[i] * dz;   /* -(ds_u)(dz_u), ds_u = -dy */
                }
            }
            const double muc = m ? sz / m : 0.0, mua = m ? saff / m : 0.0;
            const double sig = muc > 0.0 ? pow(mua / muc, 3.0) : 0.0;
            mu_b = fmax(IP_TOL_COMPL / 20.0, fmin(sig * muc, IP_MU0));
            for (int i = 0; i < NY; ++i) {
                const double y = YV(i);
                bb[i] = 0.0;
                if (g_ip_rule == 2) ccl[i] = ccu[i] = 0.0;   /* probing only: no second-order correction */
                if (yl[i] > -INFINITY) { ccl[i] += mu_b; bb[i] -= ccl[i] / (y - yl[i]); }
                if (yu[i] < INFINITY) { ccu[i] += mu_b; bb[i] += ccu[i] / (yu[i] - y); }
            }
            free(b0);
        }
        IP_SOLVE(bb);
        #undef IP_SOLVE
        if (fact_done < 0) { status = ORACLE_FACTORIZATION_FAILED; break; }
        /* fraction to the boundary: primal alpha_max, dual alpha_z */
        const double tau = IP_TAU;
        double amax = 1.0, az = 1.0, dbar = 0.0;
        for (int i = 0; i < NY; ++i) {
            const double y = YV(i);
            double bmu = 0.0;   /* barrier gradient at mu_b (the merit's), = bb for the monotone rule */
            if (yl[i] > -INFINITY) {
                const double sl = y - yl[i];
                if (dy[i] < 0.0) amax = fmin(amax, -tau * sl / dy[i]);
                const double dz = (ccl ? ccl[i] : mu_b) / sl - zl[i] - zl[i] / sl * dy[i];
                if (dz < 0.0) az = fmin(az, -tau * zl[i] / dz);
                bmu -= mu_b / sl;
            }
            if (yu[i] < INFINITY) {
                const double su = yu[i] - y;
                if (dy[i] > 0.0) amax = fmin(amax, tau * su / dy[i]);
                const double dz = (ccu ? ccu[i] : mu_b) / su - zu[i] + zu[i] / su * dy[i];
                if (dz < 0.0) az = fmin(az, -tau * zu[i] / dz);
                bmu += mu_b / su;
            }
            dbar += 2.0 * bmu * dy[i];  /* J-scale directional derivative of -2 mu sum log s */
        }
        /* l1-merit Armijo backtracking from alpha_max on J - 2 mu sum log s + nu |c|_1 */
        double nu_new = 4.0 * lmax + 1.0;
        if (nu_new > nu_pen) nu_pen = nu_new;
        double J0 = 0.0, c1 = 0.0, dJ = 0.0;
        for (int k = 0; k < N; ++k) {
            double qe[ORACLE_MAX_NX];
            for (int r = 0; r < NX; ++r) {
                qe[r] = 2.0 * Q[r] * (s->F[k * NX + r] - traj[k * NX + r]);
                J0 += 0.5 * qe[r] * (s->F[k * NX + r] - traj[k * NX + r]);
                c1 += fabs(s->c[k * NX + r]);
            }
            for (int r = 0; r < NX; ++r) {
                double ax = 0.0, bu = 0.0;
                for (int q = 0; q < NX; ++q) ax += s->Ad[k * NX * NX + r * NX + q] * s->dx[k * NX + q];
                for (int q = 0; q < NU; ++q) bu += s->Bd[k * NX * NU + r * NU + q] * s->du[k * NU + q];
                dJ += qe[r] * (ax + bu);
            }
            for (int q = 0; q < NU; ++q) {
                double um = (k == 0) ? u_prev[q] : s->U[(k - 1) * NU + q];
                double dum = (k == 0) ? 0.0 : s->du[(k - 1) * NU + q];
                double dif = s->U[k * NU + q] - um;
                J0 += dif * R[q] * dif + s->U[k * NU + q] * Rm[q] * s->U[k * NU + q];
                dJ += 2.0 * R[q] * dif * (s->du[k * NU + q] - dum) + 2.0 * Rm[q] * s->U[k * NU + q] * s->du[k * NU + q];
            }
        }
        const double phi0 = J0 - 2.0 * mu_b * logsum + nu_pen * c1;
        const double dphi = dJ + dbar - nu_pen * c1;
        double alpha = amax;
        int accepted = 0;
        for (int ls = 0; ls < 30; ++ls) {
            for (int i = 0; i < (N + 1) * NX; ++i) s->Xt[i] = s->X[i] + alpha * s->dx[i];
            for (int i = 0; i < M; ++i) s->Ut[i] = s->U[i] + alpha * s->du[i];
            double Jt, ct, lt = 0.0;
            merit_eval(N, h, s->Xt, s->Ut, u_prev, traj, w, s->Ft, &Jt, &ct);
            for (int i = 0; i < NY; ++i) {
                const double y = (i < S) ? s->Xt[NX + i] : s->Ut[i - S];
                if (yl[i] > -INFINITY) lt += log(y - yl[i]);
                if (yu[i] < INFINITY) lt += log(yu[i] - y);
            }
            const double phit = Jt - 2.0 * mu_b * lt + nu_pen * ct;
            const double noise = 1.0 + fabs(phi0);
            if (dphi >= -1e-11 * noise || phit <= phi0 + 1e-4 * alpha * dphi + 1e-13 * noise) { accepted = 1; break; }
            alpha *= 0.5;
        }
        if (!accepted) { free(ccl); free(ccu); status = ORACLE_LINESEARCH_FAILED; break; }
        /* duals: z + alpha_z dz (dz at the old point), then the kappa_Sigma safeguard at the new point */
        for (int i = 0; i < NY; ++i) {
            const double y = YV(i);
            if (yl[i] > -INFINITY)
                zl[i] += az * ((ccl ? ccl[i] : mu_b) / (y - yl[i]) - zl[i] - zl[i] / (y - yl[i]) * dy[i]);
            if (yu[i] < INFINITY)
                zu[i] += az * ((ccu ? ccu[i] : mu_b) / (yu[i] - y) - zu[i] + zu[i] / (yu[i] - y) * dy[i]);
        }
        free(ccl);
        free(ccu);
        memcpy(s->X, s->Xt, sizeof(double) * (N + 1) * NX);
        memcpy(s->U, s->Ut, sizeof(double) * M);
        for (int i = 0; i < NY; ++i) {
            const double y = YV(i);
            if (yl[i] > -INFINITY) {
                const double sl = y - yl[i];
                zl[i] = fmax(fmin(zl[i], IP_KAPPA_SIGMA * mu_b / sl), mu_b / (IP_KAPPA_SIGMA * sl));
            }
            if (yu[i] < INFINITY) {
                const double su = yu[i] - y;
                zu[i] = fmax(fmin(zu[i], IP_KAPPA_SIGMA * mu_b / su), mu_b / (IP_KAPPA_SIGMA * su));
            }
        }
        if (g_ip_rule == 0) mu_b = mu_next;
    }
#undef YV
    for (int k = 0; k < N; ++k) {
        memcpy(V + k * ND, s->X + k * NX, sizeof(double) * NX);
        memcpy(V + k * ND + NX, s->U + k * NU, sizeof(double) * NU);
    }
    memcpy(V + N * ND, s->X + N * NX, sizeof(double) * NX);
    if (J_out) {
        double J;
        oracle_nlp_eval(t_model, N, h, V, u_prev, traj, w, &J, NULL);
        *J_out = J;
    }
    free(yl); free(yu); free(zl); free(zu); free(sg); free(bb); free(zg); free(dy); free(tv);
    *iters_out = it;
    *kkt_out = kkt;
    return status;
}

int oracle_solve_batch(int model, int is_linear, int N, double h, int64_t B, const double* x0,
                       const double* u_prev, const double* traj, const double* weights,
                       int64_t w_stride, const double* u_lb, const double* u_ub, int max_iter,
                       double tol_grad, double tol_defect, double* V, int32_t* status,
                       int32_t* iters, double* kkt, double* Jout, int nthreads) {
    return oracle_solve_batch_xb(model, is_linear, N, h, B, x0, u_prev, traj, weights, w_stride, u_lb, u_ub, NULL,
                                 NULL, max_iter, tol_grad, tol_defect, V, status, iters, kkt, Jout, nthreads);
}

int oracle_solve_batch_xb(int model, int is_linear, int N, double h, int64_t B, const double* x0,
                          const double* u_prev, const double* traj, const double* weights, int64_t w_stride,
                          const double* u_lb, const double* u_ub, const double* x_lb, const double* x_ub,
                          int max_iter, double tol_grad, double tol_defect, double* V, int32_t* status,
                          int32_t* iters, double* kkt, double* Jout, int nthreads) {
    if (set_model(model) != 0 || N < 1 || B < 0) return -1;
    int x_bounded = 0;
    for (int r = 0; r < NX; ++r) x_bounded |= (x_lb && x_lb[r] > -1e19) || (x_ub && x_ub[r] < 1e19);
    const int NV = NX * (N + 1) + NU * N;
    int u_b = 0;   /* finite control bounds (the Riccati variant covers unbounded solves only) */
    for (int c = 0; c < NU; ++c) u_b |= (u_lb && u_lb[c] > -1e19) || (u_ub && u_ub[c] < 1e19);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel
    {
        set_model(model);
        ws_t s;
        ws_alloc(&s, N);
#pragma omp for schedule(dynamic, 4)
        for (int64_t b = 0; b < B; ++b) {
            int32_t it;
            double kk, J;
            double lin[ORACLE_MAX_NX * ORACLE_MAX_NX + ORACLE_MAX_NX * ORACLE_MAX_NU + 2 * ORACLE_MAX_NX + ORACLE_MAX_NU];
            if (is_linear) {
                /* A*, B*, xdot* at (state, control) = (x0, u_prev), ModelControl.cpp:125-136 */
                model_jac(x0 + b * NX, u_prev + b * NU, lin, lin + NX * NX, lin + NX * NX + NX * NU);
                memcpy(lin + NX * NX + NX * NU + NX, x0 + b * NX, sizeof(double) * NX);
                memcpy(lin + NX * NX + NX * NU + 2 * NX, u_prev + b * NU, sizeof(double) * NU);
                g_lin = lin;
            } else {
                g_lin = NULL;
            }
            if (x_bounded)
                status[b] = solve_one_ip(&s, h, x0 + b * NX, u_prev + b * NU, traj + b * (int64_t)N * NX,
                                         weights + b * w_stride, u_lb, u_ub, x_lb, x_ub, max_iter, tol_grad,
                                         tol_defect, V + b * NV, &it, &kk, &J);
            else if (g_kkt_mode == ORACLE_KKT_RICCATI && !is_linear && !u_b)
                status[b] = solve_one_riccati(&s, h, x0 + b * NX, u_prev + b * NU, traj + b * (int64_t)N * NX,
                                              weights + b * w_stride, max_iter, tol_grad, tol_defect, V + b * NV,
                                              &it, &kk, &J);
            else
                status[b] = solve_one(&s, h, x0 + b * NX, u_prev + b * NU, traj + b * (int64_t)N * NX,
                                      weights + b * w_stride, u_lb, u_ub, max_iter, tol_grad, tol_defect,
                                      V + b * NV, &it, &kk, &J);
            iters[b] = it;
            kkt[b] = kk;
            if (Jout) Jout[b] = J;
            g_lin = NULL;
        }
        ws_free(&s);
    }
    return 0;
}

/* ---------------- synthetic instances (cfg#2) ---------------- */
static uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double unit_draw(uint64_t seed, int64_t index, int j) {
    uint64_t v = splitmix64(seed ^ splitmix64((uint64_t)index * 16ull + (uint64_t)j));
    return (double)(v >> 11) * 0x1.0p-53;
}

/* lo + span * u with the product rounded separately (never fused), so that the C, HIP and Python
 * generators produce bit-identical instances. */
__attribute__((optimize("-ffp-contract=off"))) static double affine_draw(double lo, double span, double u) {
    volatile double p = span * u;
    return lo + p;
}

__attribute__((optimize("-ffp-contract=off")))
void oracle_synth_two_link(uint64_t seed, int64_t first, int64_t B, int N, double h,
                           double* x0, double* u_prev, double* traj) {
    const double PI = 3.14159265358979323846;
    for (int64_t b = 0; b < B; ++b) {
        int64_t gi = first + b;
        x0[b * 4 + 0] = affine_draw(-PI / 4, PI / 2, unit_draw(seed, gi, 0));
        x0[b * 4 + 1] = affine_draw(-PI / 4, PI / 2, unit_draw(seed, gi, 1));
        x0[b * 4 + 2] = affine_draw(-1.0, 2.0, unit_draw(seed, gi, 2));
        x0[b * 4 + 3] = affine_draw(-1.0, 2.0, unit_draw(seed, gi, 3));
        u_prev[b * 2 + 0] = affine_draw(-5.0, 10.0, unit_draw(seed, gi, 4));
        u_prev[b * 2 + 1] = affine_draw(-5.0, 10.0, unit_draw(seed, gi, 5));
        double a = affine_draw(0.5, 0.5, unit_draw(seed, gi, 6));
        double f = affine_draw(0.25, 0.75, unit_draw(seed, gi, 7));
        double ph = affine_draw(0.0, 2.0 * PI, unit_draw(seed, gi, 8));
        for (int k = 0; k < N; ++k) {
            double arg = 2.0 * PI * f * (k * h) + ph;
            double sv = a * sin(arg), cv = 2.0 * PI * f * a * cos(arg);
            double* r = traj + (b * N + k) * 4;
            r[0] = sv; r[1] = -sv; r[2] = cv; r[3] = -cv;
        }
    }
}

/* cfg#3 instances: q, qd ~ U[-0.5, 0.5], tau_prev ~ U[-1, 1], per joint a ~ U[0.1, 0.4],
 * f ~ U[0.25, 1] Hz, phase ~ U[0, 2 pi]; r_k = [a sin(2 pi f t_k + phase); 2 pi f a cos(.)], t_k = k h.
 * Same recipe as the device generator (mmpc.hip synth_exo_kernel). */
static double unit_draw_exo(uint64_t seed, int64_t index, int j) {
    uint64_t v = splitmix64((seed + 0x3C6EF372FE94F82Aull) ^ splitmix64((uint64_t)index * 32ull + (uint64_t)j));
    return (double)(v >> 11) * 0x1.0p-53;
}

__attribute__((optimize("-ffp-contract=off")))
void oracle_synth_exo(uint64_t seed, int64_t first, int64_t B, int N, double h, double* x0, double* u_prev,
                      double* traj) {
    const double PI = 3.14159265358979323846;
    for (int64_t b = 0; b < B; ++b) {
        int64_t gi = first + b;
        double a[4], f[4], ph[4];
        for (int j = 0; j < 4; ++j) {
            x0[b * 8 + j] = affine_draw(-0.5, 1.0, unit_draw_exo(seed, gi, j));
            x0[b * 8 + 4 + j] = affine_draw(-0.5, 1.0, unit_draw_exo(seed, gi, 4 + j));
            u_prev[b * 4 + j] = affine_draw(-1.0, 2.0, unit_draw_exo(seed, gi, 8 + j));
            a[j] = affine_draw(0.1, 0.3, unit_draw_exo(seed, gi, 12 + j));
            f[j] = affine_draw(0.25, 0.75, unit_draw_exo(seed, gi, 16 + j));
            ph[j] = affine_draw(0.0, 2.0 * PI, unit_draw_exo(seed, gi, 20 + j));
        }
        for (int k = 0; k < N; ++k) {
            double* r = traj + (b * N + k) * 8;
            for (int j = 0; j < 4; ++j) {
                double arg = 2.0 * PI * f[j] * (k * h) + ph[j];
                r[j] = a[j] * sin(arg);
                r[4 + j] = 2.0 * PI * f[j] * a[j] * cos(arg);
            }
        }
    }
}
