// sqp_wave.h -- fused Gauss-Newton SQP, one 64-lane wavefront per MPC instance.
//
// Replaces the IPOPT call `m_solver(m_solver_args)` of src/Mahi/Mpc/ModelControl.cpp:159
// for the NLP built by src/Mahi/Mpc/ModelGenerator.cpp:23-233 (see DESIGN.md "Solver").
// Valid for NX == 4 and M = N*NU <= 64 (the condensed Hessian has one row per lane).
//
// Per SQP iteration, all inside one workgroup of 64 lanes (no HBM traffic after the
// initial load; everything lives in LDS and VGPRs):
//   1. stage evaluation, lane k < N: F_k = x_k + h f(x_k,u_k), A_k = I + h f_x, B_k = h f_u
//      (forward-mode duals), defects c_k = F_k - x_{k+1}                (ModelGenerator.cpp:33-34, :206)
//   2. forward d_{k+1} = A_k d_k + c_k and e_k = F_k + A_k d_k - r_k    (quad-DPP, no LDS round trip)
//   3. adjoint lam_k = Q e_{k-1} + A_k^T lam_{k+1}; gradient g = B^T lam + R/Rm terms; stop test
//   4. Lyapunov P_i = Q + A_i^T P_{i+1} A_i, Z_i = B_i^T P_{i+1}         (16 lanes, LDS)
//   5. condensed Hessian H = Gamma^T Q Gamma + D^T R D + Rm, one row per lane, built by two
//      O(N) recursions per row (no Gamma is ever formed):
//         H_ij = Z_i Phi_{i+1,j+1} B_j (j <= i),   H_ij = (Z_j Phi_{j+1,i+1} B_i)^T (j > i)
//   6. Gauss-Jordan on [H | -g] with the row in registers; pivot rows are broadcast with
//      v_readlane and the active window is shifted left each step, so the pivot column
//      is always register 0 (runtime loop, static register indices)
//   7. dx_0 = 0, dx_{k+1} = A_k dx_k + B_k du_k + c_k                     (quad-DPP)
//   8. l1-merit Armijo backtracking, trial stages evaluated in parallel
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "models.h"

#ifndef MMPC_WAVES_PER_SIMD
#define MMPC_WAVES_PER_SIMD 2
#endif

namespace mmpc {

struct SolveParams {
    int64_t B;
    int N;
    int max_iter;
    double h;
    double tol_grad;
    double tol_defect;
    int is_linear;
    const double* x0;
    const double* u_prev;
    const double* traj;
    const double* weights;
    int64_t w_stride;
    const double* u_lb;
    const double* u_ub;
    // state bounds of x_1..x_N (ModelControl.cpp:37-50) BY VALUE (nx <= 16): a solve captures the bounds of its
    // launch, so mmpc_set_state_bounds between stream-ordered solves never changes one already in flight
    int x_bounded;  // any finite state bound: the interior-point variant
    double x_lb[16];
    double x_ub[16];
    double* V;
    int32_t* status;
    int32_t* iters;
    double* kkt;
    // u_0* [B][nu] (the control ModelControl::calc_u returns, ModelControl.cpp:174-190) or nullptr; may be
    // host-mapped pinned memory (mmpc_host_alloc): the result then reaches the host without a copy
    double* u0_out;
    double* trace;  // debug: [B][max_iter+1][8] per-iteration diagnostics, or nullptr
    int init_hold;  // mmpc_opts.init_states == MMPC_INIT_HOLD_X0: x_1..x_N start at x_0 (controls as given)
    int init_zero;  // mmpc_opts.init_states == MMPC_INIT_ZERO: V is not read, the iterate starts at 0 (x_0 pinned)
    // iteration-tail hand-over, lane kernel -> 16-lane kernel (DESIGN.md 4b "tail hand-over"): at the stop test of
    // iteration tail_cap an unconverged lane-kernel instance claims a slot of the list (atomic on tail_count) and
    // stops with its iterate written back; a 16-lane resume launch over the list continues it from there, with the
    // same iteration count and l1-merit weight.  Instances beyond tail_slots keep iterating in the lane kernel.
    int tail_cap;          // 0: no hand-over
    int tail_wave_max;     // also hand over at iterations >= 2 when at most this many lanes of the wave are left
    int tail_slots;        // capacity of the list
    int32_t* tail_count;   // [1] claims (may exceed tail_slots)
    int32_t* tail_idx;     // [tail_slots] instance; in a 16-lane launch, non-null = resume launch over the list
    int32_t* tail_it;      // [tail_slots] iteration whose stop test failed
    double* tail_mu;       // [tail_slots] l1-merit penalty weight
    double* tail_mub;      // [tail_slots] barrier parameter (state bounds) / previous projected gradient (control bounds)
    int no_release;        // 16-lane BOUNDED: holds are only added, kBoundPasses QP solves (the lane kernel's rule)
    // state-bounded resume: the duals z_l, z_u stay in the handing-over lane launch's workspace (stage-major
    // [64-instance block][stage][field][lane]); the resume launch's own workspace lies after it
    const double* tail_lws;
    int64_t tail_lws_block;  // doubles per 64-instance block
    int tail_lws_ss;         // doubles per stage (x 64 lanes)
    int tail_lws_zl;         // field offset of z_l; z_u follows at + nx + nu
    int gpw;               // 16-lane kernel: instance groups per wave of this launch (kGroupsPerWave, or fewer)
    // 16-lane kernel, launches whose grid is resident at once (DESIGN.md 4c "resident finish"): waves count themselves
    // out here when they finish and stay resident, sleeping, while other waves of the launch still run; the last one
    // resets it to 0.  nullptr: waves exit as they finish
    int32_t* exit_count;
};
// instance status while handed over (never returned: the resume launch overwrites it)
constexpr int ST_HANDED_OVER = 6;

enum {
    ST_CONVERGED = 0,
    ST_MAX_ITER = 1,
    ST_LS_FAILED = 2,
    ST_NONFINITE = 3,
    ST_FACT_FAILED = 4,
    ST_BOUNDS = 5  // reserved: u bounds are enforced, never reported
};

// ---------------- box constraints on u (ModelControl.cpp:37-50,146-157), projected GN-SQP ----------------
// Same rule as oracle/mmpc_oracle.c solve_one: controls within eps = min(kBoundEps, previous projected
// gradient) of a bound with the gradient pointing outward are held at that bound in the QP (Bertsekas'
// epsilon-active set), a free control whose step crosses a bound is held there and the QP solved again (at
// most kBoundPasses solves per iteration), trial points are projected, and the stop test uses
// ||U - P(U - 2g)||_inf.  Kernels take a BOUNDED template flag so that the unbounded code is unchanged.
constexpr double kBoundEps = 1e-6;
constexpr int kBoundPasses = 4;
__device__ __forceinline__ double proj(double v, double lb, double ub) { return v < lb ? lb : (v > ub ? ub : v); }

// First SQP iteration: IPOPT's filter acceptance (Waechter & Biegler 2006, eqs. (18)-(21); oracle
// first_iter_filter_accepts).  Its filter then holds only theta_max = 1e4 max(1, theta_0).  When the iterate is far
// from feasible (theta_0 > theta_min = 1e-4 max(1, theta_0), the cold start) or the switching condition (19) fails,
// a trial (J_t, theta_t = |c_t|_1) is taken when theta_t <= theta_max and theta_t <= (1 - 1e-5) theta_0 or
// J_t <= J_0 - 1e-5 theta_0.  A nearly feasible first iterate (a warm start) whose step satisfies the switching
// condition alpha (-dJ)^s_phi > theta_0^s_theta (s_phi = 2.3, s_theta = 1.1, delta = 1) is an f-type iteration:
// the Armijo test alone decides it, as every later iteration.
__device__ __forceinline__ bool first_iter_filter_accepts(double J0, double c0, double Jt, double ct, double dJ,
                                                          double alpha) {
    if (!(isfinite(Jt) && isfinite(ct))) return false;
    if (ct > 1e4 * fmax(1.0, c0)) return false;
    if (c0 <= 1e-4 * fmax(1.0, c0) && dJ < 0.0 && alpha * pow(-dJ, 2.3) > pow(c0, 1.1)) return false;
    return ct <= (1.0 - 1e-5) * c0 || Jt <= J0 - 1e-5 * c0;
}
// bound values of |b| >= 1e19 are infinite (IPOPT's convention); NaN marks a free control in hold fields
template <int NU, bool BOUNDED>
__device__ __forceinline__ void load_bounds(const SolveParams& p, double* lbv, double* ubv) {
#pragma unroll
    for (int c = 0; c < NU; ++c) {
        lbv[c] = -INFINITY;
        ubv[c] = INFINITY;
        if (BOUNDED) {
            if (p.u_lb && p.u_lb[c] > -1e19) lbv[c] = p.u_lb[c];
            if (p.u_ub && p.u_ub[c] < 1e19) ubv[c] = p.u_ub[c];
        }
    }
}

// ---------------- state bounds: primal-dual interior point (oracle/mmpc_oracle.c solve_one_ip) ----------------
// With finite state bounds the Riccati kernels run the XB variant: barrier problem min f - mu sum log s on f = J/2
// for the state AND control bounds, Sigma = z_l/s_l + z_u/s_u and b = -mu/s_l + mu/s_u added to the Riccati
// stage blocks, fraction-to-the-boundary steps, l1 merit with the barrier term, mu updated (lagged) when
// E_mu <= 10 mu.  The constants are IPOPT's defaults (mu_init, kappa_eps, kappa_mu, theta_mu, bound_push,
// kappa_Sigma).
constexpr double kIpMu0 = 0.1, kIpKappaEps = 10.0, kIpKappaMu = 0.2, kIpThetaMu = 1.5, kIpPush = 1e-2,
                 kIpKappaSigma = 1e10;
// complementarity tolerance 2 max s z (J-scale), barrier floor kIpTolCompl / 20 and a constant fraction to the
// boundary (oracle IP_TOL_COMPL, IP_TAU): keep Sigma = z/s where the Riccati Schur complements stay positive
// definite (IPOPT: compl_inf_tol 1e-4, tau = max(0.99, 1 - mu))
constexpr double kIpTolCompl = 1e-8, kIpTau = 0.99;
// y pushed inside [l, u] (IPOPT bound_push / bound_frac): by 1e-2 max(1, |bound|), at most 1e-2 of the box
__device__ __forceinline__ double ip_push(double y, double l, double u) {
    const double pl = (l > -INFINITY) ? fmin(kIpPush * fmax(1.0, fabs(l)), (u < INFINITY) ? kIpPush * (u - l) : INFINITY) : 0.0;
    const double pu = (u < INFINITY) ? fmin(kIpPush * fmax(1.0, fabs(u)), (l > -INFINITY) ? kIpPush * (u - l) : INFINITY) : 0.0;
    if (l > -INFINITY && y < l + pl) y = l + pl;
    if (u < INFINITY && y > u - pu) y = u - pu;
    return y;
}
// bounds of y = (x_{k+1} [nx] | u_k [nu]) of a stage: |b| >= 1e19 is infinite
template <int NX, int NU>
__device__ __forceinline__ void load_ip_bounds(const SolveParams& p, double* yl, double* yu) {
#pragma unroll
    for (int j = 0; j < NX + NU; ++j) {
        const double* lo = j < NX ? (p.x_bounded ? p.x_lb : nullptr) : p.u_lb;
        const double* hi = j < NX ? (p.x_bounded ? p.x_ub : nullptr) : p.u_ub;
        const int i = j < NX ? j : j - NX;
        yl[j] = (lo && lo[i] > -1e19) ? lo[i] : -INFINITY;
        yu[j] = (hi && hi[i] < 1e19) ? hi[i] : INFINITY;
    }
}
// barrier pieces of one bounded variable (oracle solve_one_ip): Sigma, b, zu - zl, complementarity, log slacks
__device__ __forceinline__ void ip_terms(double y, double l, double u, double zl, double zu, double mub, double& sg,
                                         double& bb, double& zg, double& c0, double& cmu, double& lg) {
    sg = 0.0;
    bb = 0.0;
    zg = 0.0;
    if (l > -INFINITY) {
        const double sl = y - l;
        sg += zl / sl;
        bb -= mub / sl;
        zg -= zl;
        c0 = fmax(c0, fabs(sl * zl));
        cmu = fmax(cmu, fabs(sl * zl - mub));
        lg += log(sl);
    }
    if (u < INFINITY) {
        const double su = u - y;
        sg += zu / su;
        bb += mub / su;
        zg += zu;
        c0 = fmax(c0, fabs(su * zu));
        cmu = fmax(cmu, fabs(su * zu - mub));
        lg += log(su);
    }
}
// fraction to the boundary (tau) of a primal step dy and of the dual steps it implies; dbar += 2 b dy (J-scale)
__device__ __forceinline__ void ip_step_limits(double y, double dy, double l, double u, double zl, double zu,
                                               double mub, double tau, double bb, double& amax, double& az,
                                               double& dbar) {
    if (l > -INFINITY) {
        const double sl = y - l;
        if (dy < 0.0) amax = fmin(amax, -tau * sl / dy);
        const double dz = mub / sl - zl - zl / sl * dy;
        if (dz < 0.0) az = fmin(az, -tau * zl / dz);
    }
    if (u < INFINITY) {
        const double su = u - y;
        if (dy > 0.0) amax = fmin(amax, tau * su / dy);
        const double dz = mub / su - zu + zu / su * dy;
        if (dz < 0.0) az = fmin(az, -tau * zu / dz);
    }
    dbar = fma(2.0 * bb, dy, dbar);
}
// dual update z + alpha_z dz (dz at the old point), then the kappa_Sigma safeguard at the new point y + alpha dy
__device__ __forceinline__ void ip_update(double y, double dy, double l, double u, double& zl, double& zu, double mub,
                                          double alpha, double az, double& ynew) {
    ynew = fma(alpha, dy, y);
    if (l > -INFINITY) {
        const double sl = y - l;
        zl += az * (mub / sl - zl - zl / sl * dy);
        const double sn = ynew - l;
        zl = fmax(fmin(zl, kIpKappaSigma * mub / sn), mub / (kIpKappaSigma * sn));
    }
    if (u < INFINITY) {
        const double su = u - y;
        zu += az * (mub / su - zu + zu / su * dy);
        const double sn = u - ynew;
        zu = fmax(fmin(zu, kIpKappaSigma * mub / sn), mub / (kIpKappaSigma * sn));
    }
}
__device__ __forceinline__ double ip_log_slacks(double y, double l, double u) {
    double lg = 0.0;
    if (l > -INFINITY) lg += log(y - l);
    if (u < INFINITY) lg += log(u - y);
    return lg;
}

// ---------------- wave helpers ----------------
// Pin a value at this point of the instruction stream.  Without it the optimiser sinks the
// unrolled H-build / Gauss-Jordan arithmetic to its final uses and keeps every broadcast
// operand alive until then (measured: 2.7 KB/lane of scratch spills); with it the kernel
// fits 3 waves/SIMD with no spills.
#define MMPC_PIN(x) asm volatile("" : "+v"(x))
__device__ __forceinline__ double readlane_d(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

// DPP move of a double (both halves), all lanes active
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// broadcast lane Q of each quad to the whole quad (DPP quad_perm [Q,Q,Q,Q])
template <int Q>
__device__ __forceinline__ double quad_bcast(double v) {
    return dpp_d<Q | (Q << 2) | (Q << 4) | (Q << 6)>(v);
}
// rotate within each 16-lane row by 4*S lanes (DPP row_ror:4S); the source lane is queried at run time
// with the same instruction, so nothing depends on the rotation direction
template <int S>
__device__ __forceinline__ double row_rot4(double v) {
    return dpp_d<0x120 + 4 * S>(v);
}
template <int S>
__device__ __forceinline__ int row_rot4_src(int lane) {
    return __builtin_amdgcn_mov_dpp(lane, 0x120 + 4 * S, 0xF, 0xF, false);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

// reciprocal to ~1 ulp: hardware estimate + two Newton steps
__device__ __forceinline__ double rcp_nr(double a) {
    double r = __builtin_amdgcn_rcp(a);
    double e = fma(-a, r, 1.0);
    r = fma(r, e, r);
    e = fma(-a, r, 1.0);
    return fma(r, e, r);
}

// ---------------- diagnostic phase timing (separate build, -DMMPC_PHASE_TIMING) ----------------
// s_memtime stamps between phases, accumulated per wave and added to a device table at exit.
// Only the diagnostic library libmmpc_timing.so is built with it; its run time is not quoted.
// slots 16..16+4095 (round 6): each wave's wall-clock duration (s_memrealtime ticks) at 16 + blockIdx.x (one wave
// per block in the lane and 16-lane kernels), and at 16 + 4096 + blockIdx.x its shader cycles (s_memtime) over the
// same extent; read by mmpc_debug_phase_table
// and, for the first 1024 waves, the ten phase sums of lanes 0, 16, 32, 48 (the first lanes of the 16-lane kernel's
// four instance groups) at 16 + 2 * 4096 + 40 * blockIdx.x + 10 * (lane / 16)
// and (-DMMPC_PHASE_STAGES) the s_memtime stamp after each stage of the last Riccati sweep of each group of the first
// 1024 waves at kPhaseStageLog + 128 * blockIdx.x + 32 * group + stage (stages < 32)
constexpr int kPhaseWaveLog = 4096;
constexpr int kPhaseWavePhases = 1024;
constexpr int kPhaseStageLog = 16 + 2 * kPhaseWaveLog + 40 * kPhaseWavePhases;
// slots 0..15 are accumulated by atomics into kPhaseSpread copies (one per 256-byte line, copy = blockIdx.x % 64) at
// kPhaseSpreadBase and folded on the host (phase_table_read): 16 atomics of every wave on ONE line serialise in one L2
// channel and stalled the memory operations of the waves still running (round 6)
constexpr int kPhaseSpread = 64;
constexpr int kPhaseSpreadBase = kPhaseStageLog + 128 * kPhaseWavePhases;
constexpr int kPhaseSlots = kPhaseSpreadBase + 32 * kPhaseSpread;
__device__ unsigned long long g_mmpc_phase_cycles[kPhaseSlots];
// this translation unit's table (static: device variables are per code object without -fgpu-rdc), spread copies
// folded into slots 0..15, the first n slots to out
static inline hipError_t phase_table_read(unsigned long long* out, int n, bool reset) {
    static unsigned long long full[kPhaseSlots];
    hipError_t e = hipMemcpyFromSymbol(full, HIP_SYMBOL(g_mmpc_phase_cycles), sizeof(full));
    if (e != hipSuccess) return e;
    for (int c = 0; c < kPhaseSpread; ++c)
        for (int q = 0; q < 16; ++q) {
            const unsigned long long v = full[kPhaseSpreadBase + 32 * c + q];
            full[q] = (q >= 10 && q <= 12) ? (v > full[q] ? v : full[q]) : full[q] + v;
        }
    for (int i = 0; i < n; ++i) out[i] = full[i];
    if (reset) {
        static const unsigned long long z[kPhaseSlots] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_mmpc_phase_cycles), z, sizeof(z));
    }
    return e;
}
#ifdef MMPC_PHASE_TIMING
// Slots 10-14 (round 6): the wave's wall-clock extent from s_memrealtime (100 MHz) -- 10: latest end, 11: ~earliest
// start (atomicMax of the complement), 12: longest wave, 13: sum of wave durations, 14: sum of shader cycles (s_memtime)
// over the same extents, so that cycles / duration gives the clock the waves ran at.
#define MMPC_PHASE_DECL                                                                            \
    unsigned long long ph_acc[10] = {0}, ph_t = __builtin_amdgcn_s_memtime(), ph_m0 = ph_t,        \
                       ph_r0 = __builtin_amdgcn_s_memrealtime();
#define MMPC_PHASE(i)                                        \
    do {                                                     \
        __builtin_amdgcn_sched_barrier(0);                   \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        ph_acc[i] += t_ - ph_t;                              \
        ph_t = t_;                                           \
        __builtin_amdgcn_sched_barrier(0);                   \
    } while (0)
#define MMPC_PHASE_FLUSH                                                                   \
    if (lane0 == 0) {                                                                      \
        const unsigned long long r1_ = __builtin_amdgcn_s_memrealtime(),                   \
                                 m1_ = __builtin_amdgcn_s_memtime();                       \
        unsigned long long* const pc_ = g_mmpc_phase_cycles + kPhaseSpreadBase + 32 * (blockIdx.x % kPhaseSpread); \
        for (int q_ = 0; q_ < 10; ++q_) atomicAdd(&pc_[q_], ph_acc[q_]);                   \
        atomicMax(&pc_[10], r1_);                                                          \
        atomicMax(&pc_[11], ~ph_r0);                                                       \
        atomicMax(&pc_[12], r1_ - ph_r0);                                                  \
        atomicAdd(&pc_[13], r1_ - ph_r0);                                                  \
        atomicAdd(&pc_[14], m1_ - ph_m0);                                                  \
        atomicAdd(&pc_[15], 1ull);                                                         \
        if (blockIdx.x < kPhaseWaveLog) {                                                  \
            g_mmpc_phase_cycles[16 + blockIdx.x] = r1_ - ph_r0;                            \
            g_mmpc_phase_cycles[16 + kPhaseWaveLog + blockIdx.x] = m1_ - ph_m0;            \
        }                                                                                  \
    }                                                                                      \
    if ((lane0 & 15) == 0 && blockIdx.x < kPhaseWavePhases) {                              \
        for (int q_ = 0; q_ < 10; ++q_)                                                    \
            g_mmpc_phase_cycles[16 + 2 * kPhaseWaveLog + 40 * blockIdx.x + 10 * (lane0 >> 4) + q_] = ph_acc[q_]; \
    }
#else
#define MMPC_PHASE_DECL
#define MMPC_PHASE(i)
#define MMPC_PHASE_FLUSH
#endif

// ---------------- the kernel ----------------
template <class Model, int NMAX, bool BOUNDED = false>
__global__ __launch_bounds__(64, MMPC_WAVES_PER_SIMD) void sqp_wave_kernel(SolveParams p) {
    constexpr int NX = Model::NX, NU = Model::NU, ND = NX + NU;
    constexpr int MMAX = NMAX * NU;
    static_assert(NX == 4, "quad-DPP recursions assume NX == 4");
    static_assert(MMAX <= 64, "one Hessian row per lane");

    __shared__ __attribute__((aligned(16))) double sX[(NMAX + 1) * NX];
    __shared__ __attribute__((aligned(16))) double sU[NMAX * NU];
    __shared__ __attribute__((aligned(16))) double sF[NMAX * NX];
    __shared__ __attribute__((aligned(16))) double sA[NMAX * NX * NX];
    __shared__ __attribute__((aligned(16))) double sB[NMAX * NX * NU];
    __shared__ __attribute__((aligned(16))) double sZ[NMAX * NU * NX];
    __shared__ __attribute__((aligned(16))) double sC[NMAX * NX];
    __shared__ __attribute__((aligned(16))) double sE[NMAX * NX];
    __shared__ __attribute__((aligned(16))) double sR[NMAX * NX];
    __shared__ __attribute__((aligned(16))) double sLam[(NMAX + 1) * NX];
    __shared__ __attribute__((aligned(16))) double sDX[(NMAX + 1) * NX];
    __shared__ __attribute__((aligned(16))) double sDU[MMAX];
    __shared__ __attribute__((aligned(16))) double sPiv[66];
    __shared__ __attribute__((aligned(16))) double sDiag[64];
    __shared__ __attribute__((aligned(16))) double sW[NX + 2 * NU];
    __shared__ __attribute__((aligned(16))) double sLin[NX * NX + NX * NU + NX];
    __shared__ __attribute__((aligned(16))) double sUp[NU];

    const int lane0 = threadIdx.x;
    const int lane = lane0;
    MMPC_PHASE_DECL
    const int64_t inst = blockIdx.x;
    const int N = p.N;
    const int M = N * NU;
    const int NV = NX * (N + 1) + NU * N;
    const double hstep = p.h;

    double lbv[NU], ubv[NU];
    load_bounds<NU, BOUNDED>(p, lbv, ubv);
    // bounds of the control a Hessian-row lane owns (input lane % NU)
    double lb_row = lbv[0], ub_row = ubv[0];
#pragma unroll
    for (int c = 1; c < NU; ++c) {
        lb_row = (lane % NU == c) ? lbv[c] : lb_row;
        ub_row = (lane % NU == c) ? ubv[c] : ub_row;
    }
    // ---- load the instance (the only HBM reads of the solve) ----
    const double* w = p.weights + inst * p.w_stride;
    if (lane < NX + 2 * NU) sW[lane] = w[lane];
    const double* trj = p.traj + inst * (int64_t)N * NX;
    for (int i = lane; i < N * NX; i += 64) sR[i] = trj[i];
    const double* Vin = p.V + inst * (int64_t)NV;
    for (int i = lane; i < NV; i += 64) {
        const int k = i / ND, r = i - k * ND;
        const double v = p.init_zero ? 0.0 : Vin[i];
        const double xv = (p.init_hold && r < NX) ? p.x0[inst * NX + r] : v;  // state entries only
        if (k < N) {
            if (r < NX) sX[k * NX + r] = xv;
            else sU[k * NU + r - NX] = v;
        } else {
            sX[N * NX + r] = xv;
        }
    }
    // stages >= N are structurally zero in the static-NMAX loops below
    for (int i = N * NX * NX + lane; i < NMAX * NX * NX; i += 64) sA[i] = 0.0;
    for (int i = N * NX * NU + lane; i < NMAX * NX * NU; i += 64) sB[i] = 0.0;
    for (int i = N * NX + lane; i < NMAX * NX; i += 64) sE[i] = 0.0;
    __syncthreads();
    if (lane < NX) sX[lane] = p.x0[inst * NX + lane];  // x_0 pinned (ModelControl.cpp:144-145)
    if (lane < NU) sUp[lane] = p.u_prev[inst * NU + lane];
    __syncthreads();
    if (BOUNDED) {  // the iterate starts projected onto the box
        if (lane < M) sU[lane] = proj(sU[lane], lb_row, ub_row);
        __syncthreads();
    }
    double up[NU];
#pragma unroll
    for (int c = 0; c < NU; ++c) up[c] = sUp[c];

    // linear mode: A*, B*, xdot* at (state, control) once per solve (ModelControl.cpp:125-135)
    if (p.is_linear) {
        if (lane == 0) {
            double x[NX], xd[NX], fx[NX * NX], fu[NX * NU];
#pragma unroll
            for (int i = 0; i < NX; ++i) x[i] = sX[i];
            model_eval_jac<Model>(x, up, xd, fx, fu);
#pragma unroll
            for (int i = 0; i < NX * NX; ++i) sLin[i] = fx[i];
#pragma unroll
            for (int i = 0; i < NX * NU; ++i) sLin[NX * NX + i] = fu[i];
#pragma unroll
            for (int i = 0; i < NX; ++i) sLin[NX * NX + NX * NU + i] = xd[i];
        }
        __syncthreads();
    }

    int status = ST_MAX_ITER;
    int it = 0;
    double kkt = 0.0, mu = 0.0, pg_prev = INFINITY;
    MMPC_PHASE(0);

    for (it = 0; it <= p.max_iter; ++it) {
        // Re-derive the lane id opaquely each iteration: otherwise LICM hoists every lane-dependent
        // compare mask and LDS address of the unrolled phases out of this loop (hundreds of SGPR
        // pairs -> spills).  Recomputing them costs a few SALU/VALU ops per iteration.
        int lane = lane0;
        asm volatile("" : "+v"(lane));
        const int qa = lane & 3;  // quad lane = state row index for the vector recursions
        // ---- 1. stage evaluation ----
        double cmax = 0.0;
        bool nonfinite = false;
        if (lane < N) {
            const int k = lane;
            double x[NX], u[NU], xd[NX], fx[NX * NX], fu[NX * NU];
#pragma unroll
            for (int i = 0; i < NX; ++i) x[i] = sX[k * NX + i];
#pragma unroll
            for (int i = 0; i < NU; ++i) u[i] = sU[k * NU + i];
            if (!p.is_linear) {
#ifndef MMPC_DBG_NO_JAC
                model_eval_jac<Model>(x, u, xd, fx, fu);
#else
                for (int i = 0; i < NX; ++i) { xd[i] = x[i] * u[0]; for (int q = 0; q < NX; ++q) fx[i*NX+q] = x[q]*x[i]; for (int q = 0; q < NU; ++q) fu[i*NU+q] = u[q]*x[i]; }
#endif
            } else {
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    double s = sLin[NX * NX + NX * NU + r];
#pragma unroll
                    for (int c = 0; c < NX; ++c) {
                        fx[r * NX + c] = sLin[r * NX + c];
                        s = fma(fx[r * NX + c], x[c] - sX[c], s);
                    }
#pragma unroll
                    for (int c = 0; c < NU; ++c) {
                        fu[r * NU + c] = sLin[NX * NX + r * NU + c];
                        s = fma(fu[r * NU + c], u[c] - up[c], s);
                    }
                    xd[r] = s;
                }
            }
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                const double F = fma(hstep, xd[r], x[r]);
                sF[k * NX + r] = F;
                const double c = F - sX[(k + 1) * NX + r];
                sC[k * NX + r] = c;
                cmax = fmax(cmax, fabs(c));
                nonfinite |= !isfinite(c);
#pragma unroll
                for (int q = 0; q < NX; ++q)
                    sA[k * NX * NX + r * NX + q] = (r == q ? 1.0 : 0.0) + hstep * fx[r * NX + q];
#pragma unroll
                for (int q = 0; q < NU; ++q) sB[k * NX * NU + r * NU + q] = hstep * fu[r * NU + q];
            }
        }
        __syncthreads();
        cmax = wave_max(cmax);
        MMPC_PHASE(1);

        const double Qa = sW[qa];
        // ---- 2. forward d / e (all quads redundant, quad 0 stores) ----
        {
            double d = 0.0;  // d_0 = x0 - x_0 = 0 (x_0 is pinned)
            // operands of step k+1 are loaded while step k computes (the recursion is latency-bound)
            double2 a01 = reinterpret_cast<const double2*>(sA + qa * NX)[0];
            double2 a23 = reinterpret_cast<const double2*>(sA + qa * NX)[1];
            double fr = sF[qa] - sR[qa], cc = sC[qa];
            for (int k = 0; k < N; ++k) {
                const int kn = (k + 1 < N) ? k + 1 : k;
                const double2 na01 = reinterpret_cast<const double2*>(sA + kn * NX * NX + qa * NX)[0];
                const double2 na23 = reinterpret_cast<const double2*>(sA + kn * NX * NX + qa * NX)[1];
                const double nfr = sF[kn * NX + qa] - sR[kn * NX + qa], ncc = sC[kn * NX + qa];
                const double d0 = quad_bcast<0>(d), d1 = quad_bcast<1>(d), d2 = quad_bcast<2>(d),
                             d3 = quad_bcast<3>(d);
                const double ad = fma(a01.x, d0, a01.y * d1) + fma(a23.x, d2, a23.y * d3);
                if (lane < NX) sE[k * NX + qa] = fr + ad;
                d = ad + cc;
                a01 = na01;
                a23 = na23;
                fr = nfr;
                cc = ncc;
            }
        }
        __syncthreads();
        MMPC_PHASE(2);

        // Steps 3-7 run once, or (bounded) again after holding controls whose step crosses a bound.
        bool done = false;
        double lmax = 0.0;
        double tgt = NAN;  // bounded: the bound this lane's control (Hessian row) is held at, NaN = free
        const double beps = BOUNDED ? fmin(kBoundEps, pg_prev) : 0.0;
        double* trc = p.trace ? p.trace + (inst * (p.max_iter + 1) + it) * 8 : nullptr;
        for (int pass = 0;; ++pass) {
            // ---- 3+4+5a. one backward sweep over the stages, j = NMAX-1 .. 0 ----
            //   lanes 0..15  (row 0): P_{j+1}[pa][pb] -> P_j = Q + A_j^T P_{j+1} A_j, Z_{j-1} = B_{j-1}^T P_j
            //                         (rows of P/T via quad_perm, columns via row_ror:4/8/12)
            //   lanes 16..19 (quad 4): adjoint lam_j = Q e_{j-1} + A_j^T lam_{j+1}
            //   all lanes           : lower half of the condensed Hessian row (stage si, input sr),
            //                         t_j = t_{j+1} A_{j+1} + d_j Z_j[sr],  H_ij = t_j B_j   (d_j = [j == si])
            // The serial P / lam chains are latency-bound; the Hessian row work fills their gaps.  Stages
            // >= N are structurally zero (A = B = e = 0), so P_j = Q and lam_j = 0 there.  Z_j goes through
            // LDS (lanes 0..7 write, every lane reads its row one step later; same-wave LDS order).
            const int si = lane / NU, sr = lane - (lane / NU) * NU;  // Hessian row lane = (stage si, input sr)
            const bool row_valid = lane < M;
            double hrow[MMAX];
            const double Rr = sW[NX + sr], Rmr = sW[NX + NU + sr];
            const double dterm = Rr * ((si + 1 < N) ? 2.0 : 1.0) + Rmr;
            double wdiag[NU], woff[NU];
#pragma unroll
            for (int c = 0; c < NU; ++c) {
                wdiag[c] = (c == sr) ? dterm : 0.0;
                woff[c] = (c == sr) ? -Rr : 0.0;
            }
            {
                const int pa = (lane >> 2) & 3, pb = lane & 3;
                // row index of the value each lane receives from row_ror:4s (s = 1,2,3)
                const int c1 = (row_rot4_src<1>(lane) >> 2) & 3;
                const int c2 = (row_rot4_src<2>(lane) >> 2) & 3;
                const int c3 = (row_rot4_src<3>(lane) >> 2) & 3;
                const bool lam_lane = (lane >> 2) == 4;
                const bool z_lane = lane < 16 && pa < NU;
                const int zr = pa < NU ? pa : NU - 1;
                const double pq = (pa == pb) ? sW[pa] : 0.0;
                double P = pq;                                   // P_NMAX = Q
                double lam = Qa * sE[(NMAX - 1) * NX + qa];      // lam_NMAX (e_j = 0 for j >= N)
                if (lam_lane) sLam[NMAX * NX + qa] = lam;
                lmax = lam_lane ? fabs(lam) : 0.0;
                {   // Z_{NMAX-1} = B^T Q
                    const double* Bi = sB + (NMAX - 1) * NX * NU;
                    const double P1 = row_rot4<1>(P), P2 = row_rot4<2>(P), P3 = row_rot4<3>(P);
                    const double z = fma(Bi[c3 * NU + zr], P3, fma(Bi[c2 * NU + zr], P2,
                                         fma(Bi[c1 * NU + zr], P1, Bi[pa * NU + zr] * P)));
                    if (z_lane) sZ[(NMAX - 1) * NU * NX + pa * NX + pb] = z;
                }
                double t[NX] = {0.0, 0.0, 0.0, 0.0};
                double dprev = 0.0;  // d_{j+1}
#pragma unroll
                for (int j = NMAX - 1; j >= 0; --j) {
                    int jj = j;
                    asm volatile("" : "+s"(jj));
                    const double dj = (si == jj) ? 1.0 : 0.0;
                    // (a) Hessian row, lower part
                    {
                        const double2* zp = reinterpret_cast<const double2*>(sZ + j * NU * NX + sr * NX);
                        const double2 z01 = zp[0], z23 = zp[1];
                        const double zz[NX] = {z01.x, z01.y, z23.x, z23.y};
                        if (j < NMAX - 1) {
                            const double* A1 = sA + (j + 1) * NX * NX;
                            double tn[NX];
#pragma unroll
                            for (int q = 0; q < NX; ++q)
                                tn[q] = fma(dj, zz[q], fma(t[3], A1[3 * NX + q], fma(t[2], A1[2 * NX + q],
                                                           fma(t[1], A1[1 * NX + q], t[0] * A1[0 * NX + q]))));
#pragma unroll
                            for (int q = 0; q < NX; ++q) t[q] = tn[q];
                        } else {
#pragma unroll
                            for (int q = 0; q < NX; ++q) t[q] = dj * zz[q];
                        }
                        const double* Bj = sB + j * NX * NU;
#pragma unroll
                        for (int c = 0; c < NU; ++c) {
                            const double base = fma(dprev, woff[c], dj * wdiag[c]);
                            hrow[j * NU + c] = fma(t[3], Bj[3 * NU + c],
                                                   fma(t[2], Bj[2 * NU + c], fma(t[1], Bj[1 * NU + c], fma(t[0], Bj[0 * NU + c], base))));
                            MMPC_PIN(hrow[j * NU + c]);
                        }
#pragma unroll
                        for (int q = 0; q < NX; ++q) MMPC_PIN(t[q]);
                        dprev = dj;
                    }
                    // (b) P_j = Q + A_j^T (P_{j+1} A_j), lam_j
                    {
                        const double* Ai = sA + j * NX * NX;
                        double aT[4];
#pragma unroll
                        for (int c = 0; c < 4; ++c) aT[c] = Ai[c * NX + pb];  // column pb (= qa) of A_j
                        const double r0 = quad_bcast<0>(P), r1 = quad_bcast<1>(P), r2 = quad_bcast<2>(P), r3 = quad_bcast<3>(P);
                        const double T = fma(r0, aT[0], r1 * aT[1]) + fma(r2, aT[2], r3 * aT[3]);
                        const double T1 = row_rot4<1>(T), T2 = row_rot4<2>(T), T3 = row_rot4<3>(T);
                        P = pq + (fma(Ai[pa * NX + pa], T, Ai[c1 * NX + pa] * T1) +
                                  fma(Ai[c2 * NX + pa], T2, Ai[c3 * NX + pa] * T3));
                        if (j >= 1) {
                            const double l0 = quad_bcast<0>(lam), l1 = quad_bcast<1>(lam), l2 = quad_bcast<2>(lam),
                                         l3 = quad_bcast<3>(lam);
                            lam = fma(Qa, sE[(j - 1) * NX + qa], fma(aT[0], l0, aT[1] * l1) + fma(aT[2], l2, aT[3] * l3));
                            if (lam_lane) {
                                sLam[j * NX + qa] = lam;
                                lmax = fmax(lmax, fabs(lam));
                            }
                        }
                    }
                    // (c) Z_{j-1} = B_{j-1}^T P_j for the next step's Hessian rows
                    if (j >= 1) {
                        const double* Bi = sB + (j - 1) * NX * NU;
                        const double P1 = row_rot4<1>(P), P2 = row_rot4<2>(P), P3 = row_rot4<3>(P);
                        const double z = fma(Bi[c3 * NU + zr], P3, fma(Bi[c2 * NU + zr], P2,
                                             fma(Bi[c1 * NU + zr], P1, Bi[pa * NU + zr] * P)));
                        if (z_lane) sZ[(j - 1) * NU * NX + pa * NX + pb] = z;
                    }
                }
            }
            __syncthreads();
            MMPC_PHASE(4);
            double g = 0.0;
            if (row_valid) {
                const double* ln = sLam + (si + 1) * NX;
#pragma unroll
                for (int q = 0; q < NX; ++q) g = fma(sB[si * NX * NU + q * NU + sr], ln[q], g);
                const double ui = sU[si * NU + sr];
                const double um = (si == 0) ? sUp[sr] : sU[(si - 1) * NU + sr];
                g = fma(Rr, ui - um, fma(Rmr, ui, g));
                if (si + 1 < N) g -= Rr * (sU[(si + 1) * NU + sr] - ui);
                nonfinite |= !isfinite(g);
            }
            double gmax;
            if (!BOUNDED) {
                gmax = wave_max(fabs(2.0 * g));
            } else {  // projected gradient; hold rule (pass 0), later passes keep their holds
                const double ur = row_valid ? sU[lane] : 0.0;
                gmax = wave_max(row_valid ? fabs(ur - proj(ur - 2.0 * g, lb_row, ub_row)) : 0.0);
                if (pass == 0)
                    tgt = !row_valid                                ? NAN
                          : (ur <= lb_row + beps && g > 0.0)   ? lb_row
                          : (ur >= ub_row - beps && g < 0.0)   ? ub_row
                                                               : NAN;
            }
            if (pass == 0) {
                kkt = fmax(gmax, cmax);
                if (trc && lane == 0) {
                    trc[0] = gmax;
                    trc[1] = cmax;
                }
                if (__any(nonfinite) || !isfinite(kkt)) {
                    status = ST_NONFINITE;
                    done = true;
                    break;
                }
                if (gmax <= p.tol_grad && cmax <= p.tol_defect) {
                    status = ST_CONVERGED;
                    done = true;
                    break;
                }
                if (it == p.max_iter) {
                    status = ST_MAX_ITER;
                    done = true;
                    break;
                }
                if (BOUNDED) pg_prev = gmax;
            }
            MMPC_PHASE(3);

            // ---- 5b. condensed Hessian, upper part (j > si): w_j = A_j v_{j-1},  H_ij = Z_j w_j,
            //      v_j = w_j + d_j b (w_j == 0 for j <= si).  The lower and upper parts never overlap, so they
            //      simply add (no selects).  The D^T R D + Rm band (ModelGenerator.cpp:216-221) rides on the
            //      same indicators: diagonal at d_j, sub/super diagonals at d_{j+1} (lower) and d_{j-1} (upper).
            {
                double bcol[NX];
#pragma unroll
                for (int q = 0; q < NX; ++q) bcol[q] = row_valid ? sB[si * NX * NU + q * NU + sr] : 0.0;
                double v[NX] = {0.0, 0.0, 0.0, 0.0};
                double dprev = 0.0;  // d_{j-1}
#pragma unroll
                for (int j = 0; j < NMAX; ++j) {
                    int jj = j;
                    asm volatile("" : "+s"(jj));
                    const double dj = (si == jj) ? 1.0 : 0.0;
                    const double* Aj = sA + j * NX * NX;
                    double w[NX];
#pragma unroll
                    for (int q = 0; q < NX; ++q)
                        w[q] = fma(Aj[q * NX + 3], v[3], fma(Aj[q * NX + 2], v[2], fma(Aj[q * NX + 1], v[1], Aj[q * NX + 0] * v[0])));
                    const double* Zj = sZ + j * NU * NX;
#pragma unroll
                    for (int c = 0; c < NU; ++c) {
                        hrow[j * NU + c] = fma(Zj[c * NX + 3], w[3],
                                               fma(Zj[c * NX + 2], w[2], fma(Zj[c * NX + 1], w[1],
                                                   fma(Zj[c * NX + 0], w[0], fma(dprev, woff[c], hrow[j * NU + c])))));
                        MMPC_PIN(hrow[j * NU + c]);
                    }
#pragma unroll
                    for (int q = 0; q < NX; ++q) {
                        v[q] = fma(dj, bcol[q], w[q]);
                        MMPC_PIN(v[q]);
                    }
                    dprev = dj;
                }
            }
            MMPC_PHASE(5);
            // ---- 6. Gauss-Jordan on [H | -g] ----
            // The trailing block stays symmetric under elimination, so the pivot ROW entries a_kj (j > k)
            // equal the pivot COLUMN entries a_jk that lane j holds in register k: one ds_write_b64 per step
            // publishes the pivot row, and every update is an FMA with a broadcast LDS operand.  The row is
            // written at an offset that makes every pair (k+1+2q, k+2+2q) 16-byte aligned (ds_read_b128), and
            // the reads run two 8-value chunks ahead of the FMAs (LDS latency hidden inside the wave).
            double rhs = row_valid ? -g : 0.0;
            if (BOUNDED) {  // held rows: du_a = target - u_a fixed, the free rows' QP takes its coupling to the rhs
                const bool held = tgt == tgt;
                const double dl = held ? tgt - sU[lane] : 0.0;
                const uint64_t hm = __ballot(held);
                if (hm) {
                    double t = 0.0;
#pragma unroll
                    for (int j = 0; j < MMAX; ++j) t = fma(hrow[j], readlane_d(dl, j), t);
                    rhs = held ? dl : rhs - t;
#pragma unroll
                    for (int j = 0; j < MMAX; ++j)
                        if (held || ((hm >> j) & 1)) hrow[j] = (j == lane) ? 1.0 : 0.0;
                }
            }
            bool fact_bad = false;
#pragma unroll
            for (int k = 0; k < MMAX; ++k) {
                if (k < M) {
                    constexpr int CH = 8;
                    double* piv = sPiv + (((k & 1) ^ 1));  // (k+1+off) even -> aligned pairs
                    const double col = hrow[k];
                    piv[lane] = col;
                    __builtin_amdgcn_wave_barrier();
                    int ko = k;  // opaque copy: keeps the lane == k compare inside this step (no SGPR-mask hoisting)
                    asm volatile("" : "+s"(ko));
                    const double akk = reinterpret_cast<const double2*>(sPiv)[(((k & 1) ^ 1) + k - 1) >> 1].y;
                    const int NCH = (MMAX - 1 - k + CH - 1) / CH;
                    const double2* piv2 = reinterpret_cast<const double2*>(sPiv);  // 16-B aligned pairs
                    const int off = (k & 1) ^ 1;
                    double preA[CH], preB[CH];
#pragma unroll
                    for (int q = 0; q < CH; q += 2) {
                        const int j0 = k + 1 + q, j1 = k + 1 + CH + q;
                        if (j0 < MMAX) {
                            const double2 v = piv2[(off + j0) >> 1];
                            preA[q] = v.x;
                            preA[q + 1] = v.y;
                        }
                        if (j1 < MMAX) {
                            const double2 v = piv2[(off + j1) >> 1];
                            preB[q] = v.x;
                            preB[q + 1] = v.y;
                        }
                    }
                    fact_bad |= !(akk > 0.0) || !isfinite(akk);
                    const double inv = rcp_nr(akk);
                    const double mlt = (lane == ko) ? 0.0 : col * inv;
                    if (lane == 0) sDiag[k] = akk;
                    rhs = fma(-mlt, readlane_d(rhs, k), rhs);
#pragma unroll
                    for (int c = 0; c < NCH; ++c) {
                        double cur[CH];
#pragma unroll
                        for (int q = 0; q < CH; ++q) cur[q] = (c & 1) ? preB[q] : preA[q];
#pragma unroll
                        for (int q = 0; q < CH; q += 2) {
                            const int jn = k + 1 + (c + 2) * CH + q;  // refill the buffer just consumed
                            if (c + 2 < NCH && jn < MMAX) {
                                const double2 v = piv2[(off + jn) >> 1];
                                if (c & 1) {
                                    preB[q] = v.x;
                                    preB[q + 1] = v.y;
                                } else {
                                    preA[q] = v.x;
                                    preA[q + 1] = v.y;
                                }
                            }
                        }
#pragma unroll
                        for (int q = 0; q < CH; ++q) {
                            const int j = k + 1 + c * CH + q;
                            if (j < MMAX) hrow[j] = fma(-mlt, cur[q], hrow[j]);
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
            if (fact_bad) {
                status = ST_FACT_FAILED;
                done = true;
                break;
            }
            __syncthreads();
            const double du = row_valid ? rhs / sDiag[lane] : 0.0;
            if (row_valid) sDU[lane] = du;
            __syncthreads();
            MMPC_PHASE(6);

            // ---- 7. dx forward ----
            {
                double dx = 0.0;
                if (lane < NX) sDX[qa] = 0.0;
                auto ld = [&](int k, double2& a01, double2& a23, double2& b01, double& cc, double2& du01) {
                    a01 = reinterpret_cast<const double2*>(sA + k * NX * NX + qa * NX)[0];
                    a23 = reinterpret_cast<const double2*>(sA + k * NX * NX + qa * NX)[1];
                    b01 = reinterpret_cast<const double2*>(sB + k * NX * NU + qa * NU)[0];
                    cc = sC[k * NX + qa];
                    du01 = reinterpret_cast<const double2*>(sDU + k * NU)[0];
                };
                static_assert(NU == 2, "dx recursion packs the two controls of a stage");
                double2 a01, a23, b01, du01;
                double cc;
                ld(0, a01, a23, b01, cc, du01);
                for (int k = 0; k < N; ++k) {
                    double2 na01, na23, nb01, ndu01;
                    double ncc;
                    ld((k + 1 < N) ? k + 1 : k, na01, na23, nb01, ncc, ndu01);
                    const double x0v = quad_bcast<0>(dx), x1v = quad_bcast<1>(dx), x2v = quad_bcast<2>(dx),
                                 x3v = quad_bcast<3>(dx);
                    const double bu = fma(b01.x, du01.x, fma(b01.y, du01.y, cc));
                    const double dn = (fma(a01.x, x0v, a01.y * x1v) + fma(a23.x, x2v, a23.y * x3v)) + bu;
                    if (lane < NX) sDX[(k + 1) * NX + qa] = dn;
                    dx = dn;
                    a01 = na01;
                    a23 = na23;
                    b01 = nb01;
                    cc = ncc;
                    du01 = ndu01;
                }
            }
            __syncthreads();
            MMPC_PHASE(7);
            bool resolve = false;
            if (BOUNDED && pass + 1 < kBoundPasses) {  // a free control whose step crosses a bound: hold it, solve again
                bool add = false;
                if (row_valid && tgt != tgt) {
                    const double t = sU[lane] + sDU[lane];
                    if (t < lb_row || t > ub_row) {
                        tgt = t < lb_row ? lb_row : ub_row;
                        add = true;
                    }
                }
                resolve = __any(add);
            }
            if (!BOUNDED || !resolve || pass + 1 >= kBoundPasses) break;
        }  // pass
        if (done) break;

        // ---- 8. l1-merit Armijo line search ----
        mu = fmax(mu, 4.0 * wave_max(lmax) + 1.0);
        double J0 = 0.0, c1 = 0.0, dJ = 0.0;
        if (lane < N) {
            const int k = lane;
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                const double er = sF[k * NX + r] - sR[k * NX + r];
                const double qe = 2.0 * sW[r] * er;
                J0 = fma(0.5 * qe, er, J0);
                c1 += fabs(sC[k * NX + r]);
                double ad = 0.0;
#pragma unroll
                for (int q = 0; q < NX; ++q) ad = fma(sA[k * NX * NX + r * NX + q], sDX[k * NX + q], ad);
#pragma unroll
                for (int q = 0; q < NU; ++q) ad = fma(sB[k * NX * NU + r * NU + q], sDU[k * NU + q], ad);
                dJ = fma(qe, ad, dJ);
            }
#pragma unroll
            for (int c = 0; c < NU; ++c) {
                const double um = (k == 0) ? up[c] : sU[(k - 1) * NU + c];
                const double dum = (k == 0) ? 0.0 : sDU[(k - 1) * NU + c];
                const double uk = sU[k * NU + c], duk = sDU[k * NU + c];
                const double dif = uk - um;
                const double Rr = sW[NX + c], Rmr = sW[NX + NU + c];
                J0 = fma(dif * Rr, dif, fma(uk * Rmr, uk, J0));
                dJ = fma(2.0 * Rr * dif, duk - dum, fma(2.0 * Rmr * uk, duk, dJ));
            }
        }
        J0 = wave_sum(J0);
        c1 = wave_sum(c1);
        dJ = wave_sum(dJ);
        const double phi0 = fma(mu, c1, J0);
        const double dphi = dJ - mu * c1;
        double alpha = 1.0;
        bool accepted = false;
        for (int ls = 0; ls < 30; ++ls) {
            double Jt = 0.0, ct = 0.0;
            if (lane < N) {
                const int k = lane;
                double x[NX], u[NU], xd[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) x[i] = fma(alpha, sDX[k * NX + i], sX[k * NX + i]);
#pragma unroll
                for (int i = 0; i < NU; ++i) {
                    u[i] = fma(alpha, sDU[k * NU + i], sU[k * NU + i]);
                    if (BOUNDED) u[i] = proj(u[i], lbv[i], ubv[i]);  // projected trial point
                }
                if (!p.is_linear) {
                    model_eval<Model>(x, u, xd);
                } else {
#pragma unroll
                    for (int r = 0; r < NX; ++r) {
                        double s = sLin[NX * NX + NX * NU + r];
#pragma unroll
                        for (int c = 0; c < NX; ++c) s = fma(sLin[r * NX + c], x[c] - sX[c], s);
#pragma unroll
                        for (int c = 0; c < NU; ++c) s = fma(sLin[NX * NX + r * NU + c], u[c] - up[c], s);
                        xd[r] = s;
                    }
                }
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    const double F = fma(hstep, xd[r], x[r]);
                    const double er = F - sR[k * NX + r];
                    Jt = fma(er * sW[r], er, Jt);
                    ct += fabs(F - fma(alpha, sDX[(k + 1) * NX + r], sX[(k + 1) * NX + r]));
                }
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    double um = (k == 0) ? up[c] : fma(alpha, sDU[(k - 1) * NU + c], sU[(k - 1) * NU + c]);
                    if (BOUNDED && k > 0) um = proj(um, lbv[c], ubv[c]);
                    const double dif = u[c] - um;
                    Jt = fma(dif * sW[NX + c], dif, fma(u[c] * sW[NX + NU + c], u[c], Jt));
                }
            }
            Jt = wave_sum(Jt);
            ct = wave_sum(ct);
            const double phit = fma(mu, ct, Jt);
            // Noise-aware Armijo: a decrease below ~1e-11 |phi| cannot be resolved by the fp64 merit
            // (it is a sum of ~200 terms), so such a step is taken whole, and the test allows 1e-13 |phi|
            // of roundoff.  Without this the test compares noise and alpha collapses.
            const double noise = 1.0 + fabs(phi0);
            if (dphi >= -1e-11 * noise || phit <= phi0 + 1e-4 * alpha * dphi + 1e-13 * noise ||
                (it == 0 && first_iter_filter_accepts(J0, c1, Jt, ct, dJ, alpha))) {
                accepted = true;
                break;
            }
            alpha *= 0.5;
        }
        if (trc && lane == 0) {
            trc[2] = alpha;
            trc[3] = dphi;
            trc[4] = phi0;
            trc[5] = mu;
            trc[6] = wave_max(0.0);
            trc[7] = accepted ? 1.0 : 0.0;
        }
        if (trc) {
            const double dumax = wave_max(lane < M ? fabs(sDU[lane]) : 0.0);
            if (lane == 0) trc[6] = dumax;
        }
        if (!accepted) {
            status = ST_LS_FAILED;
            break;
        }
        for (int i = NX + lane; i < (N + 1) * NX; i += 64) sX[i] = fma(alpha, sDX[i], sX[i]);
        if (lane < M) {
            const double un = fma(alpha, sDU[lane], sU[lane]);
            sU[lane] = BOUNDED ? proj(un, lb_row, ub_row) : un;
        }
        __syncthreads();
        MMPC_PHASE(8);
    }
    MMPC_PHASE(3);

    // ---- write back V (reference layout) ----
    __syncthreads();
    double* Vout = p.V + inst * (int64_t)NV;
    for (int i = lane; i < NV; i += 64) {
        const int k = i / ND, r = i - k * ND;
        double v;
        if (k < N) v = (r < NX) ? sX[k * NX + r] : sU[k * NU + r - NX];
        else v = sX[N * NX + r];
        Vout[i] = v;
    }
    if (p.u0_out && lane < NU) p.u0_out[inst * NU + lane] = sU[lane];
    if (lane == 0) {
        if (p.status) p.status[inst] = status;
        if (p.iters) p.iters[inst] = it;
        if (p.kkt) p.kkt[inst] = kkt;
    }
    MMPC_PHASE(9);
    MMPC_PHASE_FLUSH
}

}  // namespace mmpc
