/*
 * mmpc.h -- C-ABI of the MI355X-native batched nonlinear-MPC solve path.
 *
 * This is the drop-in boundary for mahi-mpc's hot path.  Each entry point names
 * the reference interface it replaces (paths relative to the mahi-mpc tree):
 *
 *   mmpc_create / mmpc_create_from_json
 *       replaces ModelControl::load_model  (src/Mahi/Mpc/ModelControl.cpp:21-73):
 *       reads the <name>.json written by ModelGenerator::save_param_file
 *       (src/Mahi/Mpc/ModelGenerator.cpp:261-270; schema ModelParameters.cpp:37-72)
 *       instead of dlopen'ing the CasADi-generated <name>.so via nlpsol(...).
 *   mmpc_solve_batch / mmpc_solve_batch_host
 *       replaces `m_solver_result = m_solver(m_solver_args);`
 *       (src/Mahi/Mpc/ModelControl.cpp:159) -- the IPOPT call over the CasADi NLP
 *       evaluators -- for B independent instances at once, including the
 *       per-step linearisation of ModelControl.cpp:125-135 in linear mode.
 *   mmpc_linearize_batch
 *       replaces the CasADi externals <name>_get_A / _get_B / _get_x_dot_init
 *       (ModelGenerator.cpp:51-53, loaded at ModelControl.cpp:70-72; used by the
 *       examples' plant model, examples/model_control_example.cpp:81-82).
 *       A and B are returned COLUMN-major, as CasADi DM -> std::vector does.
 *   mmpc_nlp_eval_batch
 *       replaces the nlp_f / nlp_g evaluators of the generated <name>.so
 *       (ModelGenerator.cpp:206-222, generated at :238).
 *
 * Conventions.
 *   - All sizes are int64_t, all arithmetic fp64.
 *   - Layouts are instance-major ("array of instances"), reference order inside:
 *       x0[B][nx], u_prev[B][nu], traj[B][N][nx]   (traj row k = target of F(x_k,u_k),
 *       ModelGenerator.cpp:207-211), weights = (Q[nx] | R[nu] | Rm[nu]) shared
 *       (weights_stride 0) or per instance (weights_stride = nx+2nu),
 *       V[B][NV] with V = [x0,u0,x1,u1,...,x_{N-1},u_{N-1},x_N] (ModelGenerator.cpp:61-112).
 *   - V_inout is the primal warm start on entry (the reference keeps the previous
 *     solution as x0 for the next call, ModelControl.cpp:160-161; first call = zeros,
 *     ModelControl.cpp:29-50) and the solution on exit.  V[b][0:nx] is pinned to x0[b]
 *     as the reference pins x_0 through lbx = ubx = state (ModelControl.cpp:144-145).
 *   - mmpc_solve_batch takes DEVICE pointers and is stream-ordered on `stream`
 *     (a hipStream_t; NULL = default stream) and never synchronises.  The condensed
 *     solver never allocates; the Riccati solver uses a per-handle device workspace
 *     that grows (synchronously) when a larger B arrives -- call
 *     mmpc_reserve_workspace first to keep solves allocation-free (hipGraph capture).
 *     mmpc_solve_batch_host takes host pointers and is synchronous.
 *   - Functions return MMPC_OK (0) or a negative mmpc_result and never throw.
 *     Non-convergence is NOT an API error: it is reported per instance in
 *     status[] (the reference silently uses non-converged IPOPT output,
 *     ModelControl.cpp:159-163; callers here can see it).
 *   - A handle may be used from several threads only on distinct streams and only
 *     for the device-pointer entry points of the condensed solver (the Riccati
 *     workspace is per handle: use one handle per concurrent stream); the _host
 *     entry points serialise on an internal mutex.
 */
#ifndef MMPC_H
#define MMPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMPC_ABI_VERSION 6

typedef struct mmpc_handle mmpc_handle;

/* API result codes (return values) */
enum mmpc_result {
    MMPC_OK = 0,
    MMPC_ERR_INVALID_ARG = -1,
    MMPC_ERR_IO = -2,
    MMPC_ERR_PARSE = -3,
    MMPC_ERR_UNSUPPORTED = -4,
    MMPC_ERR_HIP = -5,
    MMPC_ERR_NO_DEVICE = -6
};

/* per-instance solver status (status[] outputs) */
enum mmpc_status {
    MMPC_STATUS_CONVERGED = 0,            /* ||grad||_inf <= tol_grad and ||g||_inf <= tol_defect */
    MMPC_STATUS_MAX_ITER = 1,             /* opts.max_iter SQP iterations without convergence */
    MMPC_STATUS_LINESEARCH_FAILED = 2,    /* no sufficient merit decrease after 30 halvings */
    MMPC_STATUS_NONFINITE = 3,            /* NaN/Inf in the iterate or the KKT residual */
    MMPC_STATUS_FACTORIZATION_FAILED = 4, /* condensed Hessian not positive definite */
    MMPC_STATUS_BOUNDS_VIOLATED = 5       /* reserved (ABI 1 reported violated u bounds); u bounds are
                                             now enforced and this status is never produced */
};

/* built-in dynamics (device code; see DESIGN.md "Models") */
enum mmpc_model_id {
    MMPC_MODEL_TWO_LINK_ARM = 0, /* examples/ex_model_generate.cpp:24-43, nx=4 nu=2 */
    MMPC_MODEL_EXO_ARM = 1,      /* 4-DoF exo, nx=8 nu=4: M(q) of src/inverseTest.cpp:59-74 with the
                                    build-defined parameters of tests/golden/exo_params.json */
    MMPC_MODEL_USER = 2          /* dynamics given as SX expressions to mahi::mpc::ModelGenerator
                                    (ModelGenerator.hpp:23; examples/ex_model_generate.cpp:36-43), compiled by
                                    compile_model() into the model's own <name>.so, which exports this same
                                    C-ABI for that one model (the JSON's dll_filepath, ModelGenerator.cpp:255) */
};

/* KKT solve of each SQP iteration (both solve the same Gauss-Newton QP exactly) */
enum mmpc_kkt_solver {
    MMPC_KKT_AUTO = 0,      /* by shape and batch: 2-link arm -- CONDENSED for N*nu <= 64 and
                               B <= 2560, RICCATI_GROUP up to B*N = 1e6, else RICCATI; exo -- RICCATI_GROUP
                               for B <= 4096 when two workgroups fit a CU's LDS, else RICCATI */
    MMPC_KKT_CONDENSED = 1, /* one wavefront per instance, condensed Hessian row per lane (N*nu <= 64) */
    MMPC_KKT_RICCATI = 2,   /* one lane per instance, Riccati recursion, any N (needs a workspace).  Unbounded
                               nonlinear solves of models with nx+nu < 16 hand instances still unconverged after
                               iteration 4 (or once at most 8 lanes of their wave are left) to a 16-lane resume
                               launch on the same stream that continues the same iterates; with
                               factor_fp32 that tail runs the fp64 factor; bounded solves hand over by the wave
                               rule alone (4 lanes), with their duals and barrier parameter (state bounds) or the
                               lane kernel's active-set rule (control bounds).  Policy: opts.tail_* (ABI 6) */
    MMPC_KKT_RICCATI_GROUP = 3 /* 16 lanes per instance: stage-parallel model evaluations and line search,
                                  serial Riccati sweeps from LDS (stage data of 4 instances <= 160 KB LDS) */
};

/* how a solve starts from V_inout (the converged KKT point does not depend on it) */
enum mmpc_init_states {
    MMPC_INIT_AS_GIVEN = 0, /* the reference: V as given (first call zeros, ModelControl.cpp:29-50; later the
                               previous solution, :160-161), x_0 pinned to the measured state */
    MMPC_INIT_HOLD_X0 = 1,  /* x_1..x_N start at the measured state x_0 (controls as given): a consistent-ish
                               state trajectory for cold starts, fewer SQP iterations */
    MMPC_INIT_ZERO = 2      /* the reference's first call, V = 0 with x_0 pinned (ModelControl.cpp:29-50), without
                               reading V_inout: a cold start needs no zeroed input (same iterates as AS_GIVEN on a
                               zero V) */
};

/* Hessian of each SQP subproblem.  The reference's IPOPT uses the exact Lagrangian Hessian by default
 * (hessian_approximation = exact; opts at ModelControl.cpp:54-59, nlp_hess_l generated at ModelGenerator.cpp:238).
 * Both choices converge to the same KKT point; they differ in the path and the iteration count. */
enum mmpc_hessian {
    MMPC_HESSIAN_AUTO = 0,         /* EXACT where supported and the model enables it by default (the built-in 2-link
                                      arm and SX-generated models; the exo keeps Gauss-Newton, whose small-residual
                                      fits converge in 3-5 iterations), else GAUSS_NEWTON */
    MMPC_HESSIAN_GAUSS_NEWTON = 1, /* J_F^T Q J_F + R terms: positive semidefinite, linear convergence for large
                                      tracking residuals */
    MMPC_HESSIAN_EXACT = 2         /* + h sum_r lam_{k+1,r} d^2 f_r/d(x_k,u_k)^2 per stage (lam: the QP adjoint);
                                      an iteration whose KKT matrix is not positive definite on the null space takes
                                      the Gauss-Newton step.  Supported: nonlinear solves of models with second
                                      derivatives (the built-in 2-link arm and exo, SX-generated models) on the
                                      RICCATI_GROUP solver (nx+nu < 16) and the RICCATI (lane) solver with its fp64
                                      factor, unbounded or with control bounds (the held controls are fixed in the
                                      exact QP; AUTO keeps Gauss-Newton for bounded solves); AUTO keeps Gauss-Newton
                                      for the exo and on the lane solver.  State bounds, linear mode, the fp32
                                      factor and any other solve return MMPC_ERR_UNSUPPORTED */
};

typedef struct mmpc_opts {
    int32_t max_iter;   /* SQP iteration cap. default 200 (the reference IPOPT option, ModelControl.cpp:55) */
    int32_t device;     /* HIP device ordinal; -1 = the calling thread's current device. default -1 */
    double tol_grad;    /* ||grad_u J_reduced||_inf stop tolerance. default 1e-8 */
    double tol_defect;  /* ||g||_inf stop tolerance. default 1e-10 */
    int32_t kkt_solver; /* enum mmpc_kkt_solver. default MMPC_KKT_AUTO */
    int32_t factor_fp32; /* 1: Riccati factor/solve in fp32, residuals/merit/iterates in fp64 (SURVEY 8d
                            cfg#5; each SQP iteration refines the fp32 step). Riccati solver only. default 0 */
    int32_t init_states; /* enum mmpc_init_states. default MMPC_INIT_AS_GIVEN */
    int32_t hessian;     /* enum mmpc_hessian. default MMPC_HESSIAN_AUTO (ABI 4) */
    /* Iteration-tail hand-over of the RICCATI (lane) solver (ABI 6; -1 = the default policy; the
     * environment variables MMPC_TAIL_CAP / MMPC_TAIL_WAVE / MMPC_TAIL_ROUNDS, read at mmpc_create, override them for
     * tests and A/B runs).  An instance still unconverged at the stop test of iteration tail_cap, or from iteration 2
     * on once at most tail_wave_max lanes of its 64-instance wave are still iterating, continues in a 16-lane resume
     * launch on the same stream, from the same iterate with the same algorithm.  The two kernels round differently,
     * so an instance's bits (and, within the stop test's roundoff, its iteration count) depend on whether it was
     * handed over -- which the wave rule decides by its wave-mates: the same instance solved alone (B = 1, the
     * calc_u case), inside another batch or in another shard of a multi-device solve agrees to 1e-10 relative in V*
     * (tests/test_gpu_tail.py), not bit for bit.  tail_cap = 0 turns the hand-over off: results then depend only on
     * the instance's own data. */
    int32_t tail_cap;      /* -1: 4 for unbounded solves, none (the wave rule alone) for bounded ones; 0: off */
    int32_t tail_wave_max; /* -1: 8 lanes (unbounded), 4 (bounded); 0: no wave rule; <= 64 */
    int32_t tail_rounds;   /* resume slots in rounds of up to 4 one-wave workgroups per CU; -1: 4 */
} mmpc_opts;

typedef struct mmpc_model_info {
    char name[128];
    int32_t model_id;           /* enum mmpc_model_id */
    int32_t num_x, num_u;       /* nx, nu */
    int32_t num_shooting_nodes; /* N */
    int32_t num_v;              /* NV = nx(N+1) + nu N */
    int32_t num_g;              /* NG = nx N */
    int32_t is_linear;
    double step_size;           /* h [s] */
    int64_t timespan_us;        /* h N in microseconds, as serialised */
    int64_t step_size_us;
    double u_min[16], u_max[16], x_min[16], x_max[16]; /* first nu / nx entries valid */
} mmpc_model_info;

int mmpc_abi_version(void);
void mmpc_default_opts(mmpc_opts* opts);

/* load <name>.json (ModelParameters schema); opts may be NULL (defaults) */
int mmpc_create(const char* model_json_path, const mmpc_opts* opts, mmpc_handle** out);
int mmpc_create_from_json(const char* json_text, const mmpc_opts* opts, mmpc_handle** out);
int mmpc_destroy(mmpc_handle* h);
int mmpc_get_model_info(const mmpc_handle* h, mmpc_model_info* info);
int mmpc_set_opts(mmpc_handle* h, const mmpc_opts* opts);
/* State bounds x_lb <= x_k <= x_ub for k = 1..N ([nx] host arrays, NULL = unbounded; |b| >= 1e19 is infinite),
 * the lbx/ubx IPOPT receives for the states (ModelControl.cpp:37-50,146-157).  A handle starts with the JSON's
 * x_min/x_max (ModelParameters.cpp:66-69: +-10e30 -> +-inf).  Finite state bounds make the solves run the
 * primal-dual interior-point variant (IPOPT-style barrier on the same Gauss-Newton model), which
 * then also handles u_lb/u_ub; it needs a Riccati solver (AUTO never picks CONDENSED for it). */
int mmpc_set_state_bounds(mmpc_handle* h, const double* x_lb, const double* x_ub);
int mmpc_get_state_bounds(const mmpc_handle* h, double* x_lb, double* x_ub);

/* Pre-allocate the Riccati solvers' device workspace for batches up to B (so that later
 * stream-ordered solves allocate nothing; the workspace grows on demand otherwise; it includes the iteration-tail
 * hand-over list).  *bytes (may be NULL) receives the workspace size. */
int mmpc_reserve_workspace(mmpc_handle* h, int64_t B, uint64_t* bytes);

/* The KKT solver (enum mmpc_kkt_solver) a solve of B instances runs under the handle's options:
 * opts.kkt_solver, or what MMPC_KKT_AUTO picks for this model, horizon and B. */
int mmpc_resolve_kkt_solver(const mmpc_handle* h, int64_t B, int32_t* solver);

/* The Hessian (MMPC_HESSIAN_GAUSS_NEWTON or MMPC_HESSIAN_EXACT) a solve of B instances runs under the handle's
 * options; u_bounded = whether the solve passes control bounds (AUTO resolves control-bounded solves to
 * Gauss-Newton; an explicit EXACT is honoured with control bounds on RICCATI_GROUP and RICCATI).
 * MMPC_ERR_UNSUPPORTED when opts.hessian = EXACT cannot be honoured (CONDENSED, fp32 factor); state bounds: yes. */
int mmpc_resolve_hessian(const mmpc_handle* h, int64_t B, int32_t u_bounded, int32_t* hessian);

/* Batched SQP solve, DEVICE pointers, stream-ordered.  u_lb/u_ub: device [nu] or NULL
 * (unbounded; |bound| >= 1e19 is unbounded as in IPOPT).  Finite bounds are enforced (the lbx/ubx
 * of ModelControl.cpp:146-157): projected Gauss-Newton SQP, every returned u_k inside [u_lb, u_ub],
 * kkt_res = max(||U - P(U - grad)||_inf, ||g||_inf).  status/iters/kkt_res: device
 * [B] outputs, each may be NULL. */
int mmpc_solve_batch(mmpc_handle* h, int64_t B, const double* x0, const double* u_prev,
                     const double* traj, const double* weights, int64_t weights_stride,
                     const double* u_lb, const double* u_ub, double* V_inout, int32_t* status,
                     int32_t* iters, double* kkt_res, void* stream);

/* mmpc_solve_batch that also writes u_0* [B][nu] -- the control calc_u returns, V[b][nx:nx+nu]
 * (ModelControl.cpp:174-190) -- to u0_out (NULL = not written).  u0_out, status and iters may point into
 * memory from mmpc_host_alloc: the kernel then stores the per-tick results straight into host memory and they
 * are on the host when the stream's work completes (no copy kernel, no D2H; a controller loop reads them after
 * synchronising the stream).  Since ABI 5. */
int mmpc_solve_batch_u0(mmpc_handle* h, int64_t B, const double* x0, const double* u_prev,
                        const double* traj, const double* weights, int64_t weights_stride,
                        const double* u_lb, const double* u_ub, double* V_inout, int32_t* status,
                        int32_t* iters, double* kkt_res, double* u0_out, void* stream);

/* Pinned host memory mapped into every device's address space at the same address (hipHostMalloc mapped |
 * portable | coherent), for the outputs of mmpc_solve_batch_u0.  bytes = 0 gives *out = NULL.  Since ABI 5. */
int mmpc_host_alloc(uint64_t bytes, void** out);
int mmpc_host_free(void* p);

/* Same contract with HOST pointers; synchronous (H2D, solve, D2H on an internal stream). */
int mmpc_solve_batch_host(mmpc_handle* h, int64_t B, const double* x0, const double* u_prev,
                          const double* traj, const double* weights, int64_t weights_stride,
                          const double* u_lb, const double* u_ub, double* V_inout, int32_t* status,
                          int32_t* iters, double* kkt_res);

/* Continuous-time linearisation at (x[b], u[b]): A = df/dx [nx*nx], B = df/du [nx*nu]
 * column-major, xdot = f(x,u) [nx].  DEVICE pointers; any output may be NULL. */
int mmpc_linearize_batch(mmpc_handle* h, int64_t B, const double* x, const double* u,
                         double* A_colmajor, double* B_colmajor, double* xdot, void* stream);
int mmpc_linearize_batch_host(mmpc_handle* h, int64_t B, const double* x, const double* u,
                              double* A_colmajor, double* B_colmajor, double* xdot);

/* NLP value at V: J (ModelGenerator.cpp:208-222) and max |g| (g of :206).  DEVICE pointers. */
int mmpc_nlp_eval_batch(mmpc_handle* h, int64_t B, const double* V, const double* u_prev,
                        const double* traj, const double* weights, int64_t weights_stride,
                        double* J, double* defect_inf, void* stream);

/* nlp_grad_f / nlp_jac_g of the reference's generated NLP (ModelGenerator.cpp:238; CasADi generate_dependencies)
 * at V: J [B], dJ/dV [B][NV] (V layout) and the nonzero Jacobian blocks of the defects g_k = F(x_k,u_k) - x_{k+1},
 * [dg_k/dx_k | dg_k/du_k] = [I + h df/dx | h df/du] as [B][N][nx][nx+nu] row-major (dg_k/dx_{k+1} = -I).
 * DEVICE pointers; any output may be NULL. */
int mmpc_nlp_derivs_batch(mmpc_handle* h, int64_t B, const double* V, const double* u_prev,
                          const double* traj, const double* weights, int64_t weights_stride,
                          double* J, double* grad, double* jac_blocks, void* stream);

/* nlp_hess_l of the reference's generated NLP (ModelGenerator.cpp:238; CasADi generate_dependencies): the Hessian of
 * the Lagrangian lam_f J + lam_g^T g at V.  Output: the nonzero stage blocks on (x_k, u_k), [B][N][K][K] row-major
 * (K = nx + nu, symmetric); the remaining nonzeros are constant, d^2 L / du_k du_{k-1} = -2 lam_f R, and x_N enters
 * L linearly.  lam_g: DEVICE [B][N*nx] (g order, ModelGenerator.cpp:206) or NULL (zeros).  Needs second derivatives
 * of the dynamics (built-in 2-link arm, SX-generated models; linear mode always): MMPC_ERR_UNSUPPORTED otherwise. */
int mmpc_nlp_hess_batch(mmpc_handle* h, int64_t B, const double* V, const double* u_prev,
                        const double* traj, const double* weights, int64_t weights_stride, double lam_f,
                        const double* lam_g, double* hess_blocks, void* stream);

/* Synthetic instances: cfg#2 recipe for the 2-link arm, cfg#3 recipe for the exo;
 * counter-based splitmix64(seed, first_index + b), so shards generate identical instances
 * whatever the GPU count.  DEVICE pointers. */
int mmpc_synth_batch(mmpc_handle* h, uint64_t seed, int64_t first_index, int64_t B, double* x0,
                     double* u_prev, double* traj, void* stream);

/* ---- one process, several devices (the reference's per-instance worker loop of
 *      ModelControl.cpp:75-112, batched and sharded) ----
 * Contiguous split of B instances over n shards: shard i = [floor(i B / n), floor((i+1) B / n)) (first, count);
 * the same partition as the multi-process path (mmpc/dist.py shard_strong).  Pure arithmetic, no device. */
int mmpc_shard(int64_t B, int32_t n, int32_t i, int64_t* first, int64_t* count);

typedef struct mmpc_multi mmpc_multi;
/* One handle per listed device ordinal (each with its own stream, workspace and staging; a device may be listed
 * more than once: its shards then run on concurrent streams).  opts.device is ignored. */
int mmpc_multi_create(const char* model_json_path, const mmpc_opts* opts, const int32_t* devices, int32_t n_devices,
                      mmpc_multi** out);
int mmpc_multi_destroy(mmpc_multi* m);
int mmpc_multi_num_devices(const mmpc_multi* m, int32_t* n);
/* the handle of shard g (to reserve workspace, set state bounds or options device by device) */
int mmpc_multi_handle(mmpc_multi* m, int32_t g, mmpc_handle** h);
/* mmpc_solve_batch_host contract for the whole batch: shard g = mmpc_shard(B, n_devices, g) is solved on device g
 * (H2D, solve, D2H on that device's stream, all devices concurrently) straight from/into the caller's arrays;
 * synchronous.  Results equal a single-device solve of each shard bit for bit; against a single-device solve of the
 * whole batch they are bit for bit except where the RICCATI solver's iteration-tail hand-over decides differently
 * for a different wave composition (opts.tail_cap: 1e-10 relative in V*, tests/test_gpu_multi.py). */
int mmpc_multi_solve_batch_host(mmpc_multi* m, int64_t B, const double* x0, const double* u_prev,
                                const double* traj, const double* weights, int64_t weights_stride,
                                const double* u_lb, const double* u_ub, double* V_inout, int32_t* status,
                                int32_t* iters, double* kkt_res);

/* The same solve through RCCL (SURVEY.md 8e's single-process design; replaces the per-tick m_solver call of
 * ModelControl.cpp:159 for a batch resident on one GPU): DEVICE pointers on the multi handle's FIRST device; shard g
 * (mmpc_shard) of every input goes to device g by ncclSend/ncclRecv, shared weights and u_lb/u_ub (device [nu] or
 * NULL) by ncclBroadcast, every device solves its shard, and V / status / iters / kkt_res come back to the first
 * device by ncclSend/ncclRecv (ncclCommInitAll over the listed devices at the first call).  The devices must be
 * distinct (RCCL refuses a device listed twice: MMPC_ERR_UNSUPPORTED); RCCL is loaded with dlopen at the first call
 * (MMPC_ERR_UNSUPPORTED when librccl is absent).  `stream` (hipStream_t on the first device, NULL = the null
 * stream): the call's first RCCL operation is ordered after the work already queued there, and work queued there
 * later sees the results.  Per-instance weights (weights_stride >= nx + 2 nu) need (B - 1) weights_stride + nx + 2 nu
 * doubles.  Every RCCL operation's result is checked; after an error every stream of the call is drained before the
 * call returns.  Synchronous; results as mmpc_multi_solve_batch_host's.  `stream` must belong to the first device
 * (MMPC_ERR_INVALID_ARG otherwise). */
int mmpc_multi_solve_batch_rccl(mmpc_multi* m, int64_t B, const double* x0, const double* u_prev,
                                const double* traj, const double* weights, int64_t weights_stride,
                                const double* u_lb, const double* u_ub, double* V_inout, int32_t* status,
                                int32_t* iters, double* kkt_res, void* stream);
/* the version of the RCCL library the call above loads (ncclGetVersion, e.g. 22606), MMPC_ERR_UNSUPPORTED if none */
int mmpc_rccl_version(int32_t* version);

const char* mmpc_status_string(int32_t status);
/* thread-local description of the last API error on this thread ("" if none) */
const char* mmpc_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MMPC_H */
