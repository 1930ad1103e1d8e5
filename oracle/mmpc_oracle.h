/*
 * mmpc_oracle.h -- CPU fp64 restatement of the mahi-mpc NLP and of the
 * Gauss-Newton SQP that the HIP path runs.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker / CPU baseline.  The product path (mahi-mpc_amd/) never links it.
 *
 * Parity status: the reference solve (CasADi @ fadc864 + IPOPT 3.14.3) cannot
 * be built or run here, so the full solve is pinned by
 *   - the reference's own known-answer material (lin_test.m:31-50, lin_test.m:22-28,
 *     old/Models/DoublePendulumModel.hpp closed-form Jacobian, src/nlp_codegen.cpp:41-62)
 *     restated as fixtures in tests/golden/, and
 *   - independent scipy solves of the identical NLP (tests/golden/make_golden.py).
 * See DESIGN.md "Oracle".
 */
#ifndef MMPC_ORACLE_H
#define MMPC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_MODEL_TWO_LINK_ARM = 0, ORACLE_MODEL_EXO_ARM = 1, ORACLE_MODEL_USER = 2 };
#define ORACLE_MAX_NX 16
#define ORACLE_MAX_NU 16

/* Dynamics of a model generated from SX expressions (mahi::mpc::ModelGenerator): continuous Jacobians
 * A = df/dx (nx x nx), B = df/du (nx x nu) ROW-major and xdot.  The tests register the host build of the
 * generated <name>_model.h (oracle/user_model_host.cpp), whose expressions are pinned against an independent
 * sympy restatement of the same model (tests/test_sx_models.py). */
typedef void (*oracle_user_jac_fn)(const double* x, const double* u, double* A, double* B, double* xdot);
int oracle_set_user_model(int nx, int nu, oracle_user_jac_fn jac);
/* second derivatives of the same generated model: W = sum_r lam[r] d^2 f_r / d(x,u)^2, (nx+nu)^2 row-major
 * (NULL: the model has none and every solve uses the Gauss-Newton Hessian) */
typedef void (*oracle_user_hess_fn)(const double* x, const double* u, const double* lam, double* W);
int oracle_set_user_model_hess(oracle_user_hess_fn hess);

/* Hessian of the SQP subproblem (mmpc_opts.hessian, process-wide for the following solves):
 * GAUSS_NEWTON = J_F^T Q J_F + R terms only; EXACT = the Lagrangian Hessian (CasADi nlp_hess_l,
 * ModelGenerator.cpp:238; IPOPT's default, ModelControl.cpp:54-59): adds, per stage, h sum_r lam_{k+1,r}
 * d^2 f_r/d(x_k,u_k)^2 with lam the adjoint of the QP at the current iterate.  EXACT applies to unbounded,
 * nonlinear solves of models with second derivatives (2-link arm, generated models); an iteration whose
 * exact KKT matrix is not positive definite on the null space falls back to Gauss-Newton. */
enum { ORACLE_HESS_GAUSS_NEWTON = 0, ORACLE_HESS_EXACT = 1 };
void oracle_set_hessian(int mode);
/* EXACT with control bounds (projected SQP): 1 (default) = the held controls are fixed in the exact QP as in the
 * Gauss-Newton one (the kernels' bounded exact-Hessian path); 0 = bounded solves keep the Gauss-Newton Hessian */
void oracle_set_exact_bounded(int on);
/* control bounds: release holds whose QP multiplier points into the box (the 16-lane Riccati kernel's rule) */
void oracle_set_bound_release(int on);
/* W = sum_r lam[r] d^2 f_r/d(x,u)^2 of the 2-link arm (6x6 row-major, x then u; lam[4]) */
void oracle_two_link_hess(const double* x, const double* u, const double* lam, double* W);

/* per-instance status, same numbering as include/mmpc.h */
enum {
    ORACLE_CONVERGED = 0,
    ORACLE_MAX_ITER = 1,
    ORACLE_LINESEARCH_FAILED = 2,
    ORACLE_NONFINITE = 3,
    ORACLE_FACTORIZATION_FAILED = 4,
    ORACLE_BOUNDS_VIOLATED = 5  /* reserved: u bounds are enforced (projected GN-SQP), never reported */
};
/* epsilon of the epsilon-active set of the bound-constrained solve: min(ORACLE_BOUND_EPS, previous ||pg||) */
#define ORACLE_BOUND_EPS 1e-6
/* QP solves per SQP iteration with bounds: the first, plus re-solves after holding crossed bounds */
#define ORACLE_BOUND_PASSES 4

/* x_dot = f(x,u) of the 2-link arm, examples/ex_model_generate.cpp:24-43 */
void oracle_two_link_xdot(const double* x, const double* u, double* xdot);
/* continuous Jacobians A = df/dx (4x4), B = df/du (4x2), ROW-major, plus xdot */
void oracle_two_link_jac(const double* x, const double* u, double* A, double* B, double* xdot);
/* 4-DoF exo (build-defined parameters, tests/golden/exo_params.json):
 * A = df/dx (8x8), B = df/du (8x4) row-major, xdot; and the mass matrix M(q) (4x4 row-major) */
void oracle_exo_jac(const double* x, const double* u, double* A, double* B, double* xdot);
void oracle_exo_mass(const double* q, double* M);
/* W = sum_r lam_r d^2 f_r / d(x,u)^2 of the exo (12 x 12 row-major; lam: [nx]) */
void oracle_exo_hess(const double* x, const double* u, const double* lam, double* W);
/* linearised Euler step F_lin, ModelGenerator.cpp:47-48 (A,B row-major here) */
void oracle_f_lin(int nx, int nu, double h, const double* A, const double* B, const double* x,
                  const double* u, const double* xdot_init, const double* x_init,
                  const double* u_init, double* x_next);

/* NLP value: J (ModelGenerator.cpp:208-222) and defects g (ModelGenerator.cpp:206)
 * at the decision vector V (layout ModelGenerator.cpp:61-112). */
void oracle_nlp_eval(int model, int N, double h, const double* V, const double* u_prev,
                     const double* traj, const double* weights, double* J, double* g);
/* gradient of the single-shooting objective w.r.t. U (x rolled out from x0),
 * exact via the adjoint; used as an independent stationarity certificate. */
void oracle_reduced_gradient(int model, int N, double h, const double* x0, const double* U,
                             const double* u_prev, const double* traj, const double* weights,
                             double* grad);

/* nlp_hess_l (ModelGenerator.cpp:238): the (x_k, u_k) stage blocks [N][K][K] (K = nx+nu, row-major) of the Hessian
 * of lam_f J + lam_g^T g at V (lam_g [N*nx], g order; may be NULL); d^2/du_k du_{k-1} = -2 lam_f R is constant.
 * Returns -1 for a model without second derivatives. */
int oracle_nlp_hess(int model, int N, double h, const double* V, const double* u_prev, const double* traj,
                    const double* weights, double lam_f, const double* lam_g, double* blocks);

/* Batched GN-SQP solve (the algorithm of DESIGN.md "Solver"), OpenMP over instances.
 * Layouts are instance-major:  x0[B][nx], u_prev[B][nu], traj[B][N*nx],
 * weights[w_stride==0 ? 1 : B][nx+2nu] = (Q | R | Rm), V[B][NV] (warm start in,
 * solution out; V[b][0:nx] is overwritten by x0 as the reference pins x_0 by
 * bounds, ModelControl.cpp:144-145).  u_lb/u_ub may be NULL (unbounded).  is_linear selects
 * F_lin with A*, B*, xdot* taken at (x0, u_prev) (ModelControl.cpp:125-136). */
int oracle_solve_batch(int model, int is_linear, int N, double h, int64_t B, const double* x0,
                       const double* u_prev, const double* traj, const double* weights,
                       int64_t w_stride, const double* u_lb, const double* u_ub, int max_iter,
                       double tol_grad, double tol_defect, double* V, int32_t* status,
                       int32_t* iters, double* kkt, double* Jout, int nthreads);

/* as oracle_solve_batch, plus state bounds x_lb/x_ub [nx] on x_1..x_N (ModelControl.cpp:37-50; NULL or
 * |b| >= 1e19 = unbounded).  Any finite state bound selects the primal-dual interior-point variant
 * (solve_one_ip), which then also handles the control bounds. */
int oracle_solve_batch_xb(int model, int is_linear, int N, double h, int64_t B, const double* x0,
                          const double* u_prev, const double* traj, const double* weights, int64_t w_stride,
                          const double* u_lb, const double* u_ub, const double* x_lb, const double* x_ub,
                          int max_iter, double tol_grad, double tol_defect, double* V, int32_t* status,
                          int32_t* iters, double* kkt, double* Jout, int nthreads);

/* the first SQP iteration's line-search acceptance (IPOPT's filter with theta_min and the switching condition,
 * Waechter & Biegler 2006 eqs. (18)-(21)); 1 = accept.  The kernels run the same rule (sqp_wave.h). */
int oracle_first_iter_filter_accepts(double J0, double c0, double Jt, double ct, double dJ, double alpha);

/* KKT solve of the following unbounded nonlinear solves (process-wide): ORACLE_KKT_DENSE (explicit condensing +
 * Cholesky, the default) or ORACLE_KKT_RICCATI (the Riccati recursion the HIP kernels run, same iterates) */
enum { ORACLE_KKT_DENSE = 0, ORACLE_KKT_RICCATI = 1 };
void oracle_set_kkt(int mode);
/* barrier rule of the interior-point solve: 0 monotone (shipped), 1 Mehrotra predictor-corrector (experiment) */
void oracle_set_ip_rule(int rule);
/* test instrumentation: exact-Hessian iterations that fell back to the Gauss-Newton step since the last reset */
long long oracle_exact_fallbacks(int reset);

/* mmpc_opts.init_states for the following solves (process-wide): 0 = V as given, 1 = x_1..x_N start at x_0,
 * 2 = V taken as zero (MMPC_INIT_ZERO) */
void oracle_set_init_states(int mode);

/* counter-based synthetic cfg#2 instances: splitmix64(seed, index) */
void oracle_synth_two_link(uint64_t seed, int64_t first_index, int64_t B, int N, double h,
                           double* x0, double* u_prev, double* traj);
/* counter-based synthetic cfg#3 (exo) instances */
void oracle_synth_exo(uint64_t seed, int64_t first_index, int64_t B, int N, double h, double* x0,
                      double* u_prev, double* traj);

#ifdef __cplusplus
}
#endif
#endif
