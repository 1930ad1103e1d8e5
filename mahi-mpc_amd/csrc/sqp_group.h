// sqp_group.h -- batched GN-SQP with a Riccati KKT solve, SIXTEEN LANES PER INSTANCE (four instances per wave).
//
// The condensed kernel (sqp_wave.h) spends O(N^2 nu^2 nx + (N nu)^3) flops per SQP iteration (288 kflop at
// cfg#2); a Riccati recursion solves the same GN QP exactly in O(N (nx+nu)^3) (~15 kflop at
// cfg#2).  The lane-per-instance Riccati kernel (sqp_lane.h) cannot fill the GPU at cfg#2's B = 4096 (64 waves),
// so here one instance owns a 16-lane DPP row and the work splits by its shape:
//   * stage-parallel (all 16 lanes, stage k on lane k mod 16): model + Jacobian evaluations, defects, merit
//     terms, line-search trial evaluations, iterate updates, loads and stores;
//   * O(N) recursions (one lane per instance): defect propagation d, adjoint + reduced gradient + Riccati
//     backward sweep, forward step sweep -- reading the stage blocks the other lanes left in LDS.
// Group reductions (J, |c|_1, max|c|, merit) are 16-lane butterflies; the NLP, merit, line search and stop test
// are those of sqp_wave.h / sqp_lane.h / oracle.  B = 4096 gives 1024 waves = one per SIMD.
//
// LDS per instance (fp64): x_k, u_k, F_k, c_k, hFq_k, hFqd_k, hFu_k, d_k, dx_k, du_k (cross-lane data); the
// targets stay in HBM (read-only) and the gains K_k in a per-instance HBM workspace (serial lane only).
#pragma once
#include <type_traits>

#include "models.h"
#include "sqp_lane.h"
#include "sqp_wave.h"

namespace mmpc {

#ifndef MMPC_GROUP_BOUNDED_PAIRS
#define MMPC_GROUP_BOUNDED_PAIRS 0
#endif
#ifndef MMPC_GROUP_XB_PAIRS
#define MMPC_GROUP_XB_PAIRS 1
#endif
// A/B switch (round 6, diagnostic builds): the W_k and [K_k | kff_k] records go to the HBM workspace with
// non-temporal stores (no L2 allocation) instead of plain ones
#ifndef MMPC_GROUP_EXIT_HOLD   // resident finish of the 16-lane kernel; 0: waves exit as they finish
#define MMPC_GROUP_EXIT_HOLD 0
#endif
#ifndef MMPC_GROUP_WZERO_ONCE   // W_k's structural zeros stored once per launch (w_struct_zero)
#define MMPC_GROUP_WZERO_ONCE 1
#endif
#ifndef MMPC_GROUP_WB_COALESCED   // A/B switch: V written back 16 consecutive doubles per store instruction
#define MMPC_GROUP_WB_COALESCED 0
#endif
#ifndef MMPC_GROUP_NT_STORES
#define MMPC_GROUP_NT_STORES 0
#endif
template <class T>
__device__ __forceinline__ void ws_store(T* p, T v) {
    if constexpr (MMPC_GROUP_NT_STORES) __builtin_nontemporal_store(v, p);
    else *p = v;
}
// Entries of W_k's x rows that Model::eval_hess always leaves 0 (structural zeros): a launch stores them in its first
// W pass only (MMPC_GROUP_WZERO_ONCE, round 6).  2-link arm (two_link_fast.h eval_hess: q_A enters only through
// gravity, the torques linearly): row 0 is zero in columns 2..5, rows 2 and 3 in columns 0, 4 and 5.
template <class Model>
__device__ constexpr bool w_struct_zero(int, int) { return false; }
template <>
__device__ constexpr bool w_struct_zero<TwoLinkArm>(int r, int j) { return (r == 0 && j >= 2) || (r >= 2 && (j == 0 || j >= 4)); }
constexpr int kGroupLanes = 16;
constexpr int kGroupsPerWave = 4;

// LDS doubles per instance.  The hold targets (bounded solves) and the linear-mode block are only allocated
// when used: at cfg#2 that keeps a 4-instance workgroup at 39.0 KB (bounded: 39.75 KB), so 4 workgroups (one per
// SIMD) fit a CU's 160 KB.  nq = kinematic rows of the model (sqp_lane.h a_mul); the stage blocks are h da/dq,
// h da/dz, h da/du.  xb (the interior-point variant) adds nothing here since round 5: its per-stage z_l, z_u, Sigma,
// b, z_u - z_l live in the HBM workspace (group_ws_doubles) -- in LDS they made 67.8 KB per workgroup at cfg#2, two
// workgroups per CU, half the SIMDs idle and a 4096-instance batch in two rounds.
// The d recursion prefetches two stages ahead without a clamp (d_recursion_dist): its reads of stages N and N + 1 of
// sC, sFq and sFqd land in the arrays that follow each of them.  When the arrays after sFqd (sFu, sR, ...) are
// shorter than sFqd's overreach of 2 (nx - nq)^2 doubles (exo shapes at N = 1), a tail pad of that size keeps the read
// inside the instance's own block, never in the next group's block or past the end of the dynamic LDS; otherwise no
// pad (round 4 always padded: the control-bounded cfg#2 layout was then 40,960 B per workgroup).  The prefetched
// values are never used.
__host__ __device__ constexpr int group_lds_doubles(int nx, int nu, int nq, int N, bool bounded = true,
                                                   bool linear = true, bool xb = false) {
    return N * (3 * nx + (nx - nq) * (nq + (nx - nq) + nu) + 2 * nu) + 3 * (N + 1) * nx + (bounded ? N * nu : 0) +
           (linear ? (nx - nq) * (nq + (nx - nq) + nu) + nx : 0) +
           (N * ((nx - nq) * nu + nx) >= 2 * (nx - nq) * (nx - nq) ? 0 : 2 * (nx - nq) * (nx - nq));
}
// exact Hessian (EXACT): per stage the x rows of W_k = h sum_s lam_{k+1,NQ+s} d^2 acc_s/d(x,u)^2 (nx x (nx+nu))
// and its u-u block (nu x nu), written stage-parallel and read by the lane-distributed Riccati sweep
__host__ __device__ constexpr int group_hess_doubles(int nx, int nu) { return nx * (nx + nu) + nu * nu; }
// HBM workspace doubles per instance: K_k | kff_k per stage, then the W_k blocks per stage, then (control-bounded
// solves only) the un-held rows [H_wx | -R | H_ww | h_w] of each stage QP, for the multipliers of the held controls.
// The kernel strides instances by its own variant's size (unbounded solves: 1020 instead of 1560 doubles at cfg#2);
// the host reserves the bounded size, the largest.
// xb (the interior-point variant, never with `bounded`): the per-stage z_l, z_u, Sigma, b, z_u - z_l of
// (x_{k+1} | u_k) after the W blocks, in place of the bounded solves' rows.
__host__ __device__ constexpr int group_ws_doubles(int nx, int nu, int N, bool bounded = true, bool xb = false) {
    return N * nu * (nx + nu + 1) + N * group_hess_doubles(nx, nu) + (bounded ? N * nu * (nx + 2 * nu + 1) : 0) +
           (xb ? 5 * N * (nx + nu) : 0);
}

struct GroupWork {
    double* ws;
};

__device__ __forceinline__ double group_sum(double v) {
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double group_min(double v) {
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double group_max(double v) {
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double group_bcast(double v, int base) { return __shfl(v, base); }
__device__ __forceinline__ int group_bcast_i(int v, int base) { return __shfl(v, base); }

// Lane L of every 16-lane row (= one instance group) to the whole row: one v_mov_b64_dpp row_newbcast:L
// (gfx950 DPP64).  Measured on MI355X (tools/ubench/f64_latency.hip): a dependent FMA through it costs
// 17 cycles against 11 for a plain dependent FMA and ~80 through __shfl (ds_bpermute) or an LDS round trip,
// so the lane-distributed Riccati sweep below exchanges data with it.
template <int L>
__device__ __forceinline__ double row_bcast(double v) {
    static_assert(L >= 0 && L < 16, "row lane");
    // bound_ctrl with full row/bank masks: every lane is written, so the old value is dead (no copy)
    return __builtin_amdgcn_update_dpp(v, v, 0x150 + L, 0xf, 0xf, true);
}
// compile-time loop: f(std::integral_constant<int, I>) for I = B .. E-1 (row_bcast needs a constant lane)
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(static_cast<F&&>(f));
    }
}

// xd = f(x, u); with jac also the acceleration partials (unscaled).  Linear mode (ModelGenerator.cpp:47-48):
// F_lin with the acceleration Jacobians lFq, lFqd, lFu and xdot lxd taken at (lxs, lus).
template <class Model>
__device__ __forceinline__ void group_model(bool lin, const double* lFq, const double* lFqd, const double* lFu,
                                            const double* lxd, const double* lxs, const double* lus, const double* x,
                                            const double* u, double* xd, double* Fq, double* Fqd, double* Fu,
                                            bool jac) {
    constexpr int NQ = Model::NQ, NU = Model::NU, NA = Model::NX - NQ;
    if (!lin) {
        if (jac) {
            Model::eval_acc_jac(x, u, xd + NQ, Fq, Fqd, Fu);
#pragma unroll
            for (int i = 0; i < NQ; ++i) xd[i] = x[NQ + i];
        } else {
            Model::eval(x, u, xd);
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i) xd[i] = lxd[i] + (x[NQ + i] - lxs[NQ + i]);
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        double t = lxd[NQ + i];
#pragma unroll
        for (int s = 0; s < (NQ > NA ? NQ : NA); ++s) {
            if (s < NA) t = fma(lFqd[i * NA + s], x[NQ + s] - lxs[NQ + s], t);
            if (s < NQ) t = fma(lFq[i * NQ + s], x[s] - lxs[s], t);
        }
#pragma unroll
        for (int c = 0; c < NU; ++c) t = fma(lFu[i * NU + c], u[c] - lus[c], t);
        xd[NQ + i] = t;
    }
    if (jac) {
#pragma unroll
        for (int i = 0; i < NA * NQ; ++i) Fq[i] = lFq[i];
#pragma unroll
        for (int i = 0; i < NA * NA; ++i) Fqd[i] = lFqd[i];
#pragma unroll
        for (int i = 0; i < NA * NU; ++i) Fu[i] = lFu[i];
    }
}

// XB: state bounds (oracle solve_one_ip), the primal-dual interior-point variant for state AND control bounds;
// BOUNDED: control bounds only (projected GN-SQP).  At most one of them.
// EXACT: exact Hessian of the Lagrangian (mmpc_opts.hessian; oracle ORACLE_HESS_EXACT) -- solves of models with
// second derivatives on the lane-distributed path: unbounded, control-bounded (held controls fixed in the exact QP)
// and, round 6, state-bounded (W_k joins the barrier-augmented stage blocks; oracle solve_one_ip with the exact
// Hessian).
template <class Model, bool BOUNDED = false, bool XB = false, bool EXACT = false>
__global__ __launch_bounds__(64) void sqp_group_kernel(SolveParams p, GroupWork gw) {
    static_assert(!(BOUNDED && XB), "the interior-point variant handles the control bounds itself");
    constexpr int NX = Model::NX, NU = Model::NU, NQ = Model::NQ, NA = NX - NQ, NS = NX + NU, ND = NX + NU;
    constexpr int SQ = NA * NQ > 0 ? NA * NQ : 1;  // extent of the h da/dq block (empty for NQ = 0)
    constexpr int FQ = NA * NQ, FD = NA * NA, FU = NA * NU;  // stage block sizes (sqp_lane.h a_mul)
    static_assert(NQ >= 0 && NA >= NQ, "x = [q; z] with qdot = z[0:NQ]");
    constexpr int G = kGroupLanes;
    extern __shared__ double shm[];
    const int gl = threadIdx.x & (G - 1);
    const int gi = threadIdx.x / G;
    [[maybe_unused]] const int lane0 = threadIdx.x;
    MMPC_PHASE_DECL
#ifdef MMPC_GROUP_SLEEP_EXIT
    const unsigned long long sl_t0 = __builtin_amdgcn_s_memrealtime();
#endif
#if MMPC_GROUP_EXIT_HOLD
    const unsigned long long fin_t0 = __builtin_amdgcn_s_memrealtime();   // resident finish: this wave's start
#endif
    const int gbase = gi * G;  // first lane of this instance's group
    // slot of this group in the launch: the instance itself, or (resume launch, p.tail_idx) an entry of the lane
    // kernel's hand-over list
    const int64_t slot = (int64_t)blockIdx.x * p.gpw + gi;
    const bool resume = p.tail_idx != nullptr;
    const bool valid = gi < p.gpw && slot < (resume ? (int64_t)min(*p.tail_count, p.tail_slots) : p.B);
    // a group past the end of the batch (the last wave of a B not divisible by 4) leaves at once: no group reads
    // another group's lanes (row_bcast and the group reductions stay inside the 16-lane row) or LDS block, so
    // nothing else in the wave needs it, and it issues no memory access at all (round 4 had those groups run on
    // aliased to instance 0 and masked by `done`, which made every store's masking a correctness condition)
    if (!valid) return;
    const int64_t inst = resume ? (int64_t)p.tail_idx[slot] : slot;
    const int64_t ii = inst;
    const int N = p.N;
    const int NV = NX * (N + 1) + NU * N;
    const double h = p.h;

    // ---- LDS views of this instance ----
    double* const sX = shm + gi * group_lds_doubles(NX, NU, NQ, N, BOUNDED, p.is_linear != 0, XB);  // [N+1][NX]
    double* const sDX = sX + (N + 1) * NX;                         // [N+1][NX]
    double* const sD = sDX + (N + 1) * NX;                         // [N+1][NX]
    double* const sU = sD + (N + 1) * NX;                          // [N][NU]
    double* const sDU = sU + N * NU;                               // [N][NU]
    double* const sF = sDU + N * NU;                               // [N][NX]
    double* const sC = sF + N * NX;                                // [N][NX]
    double* const sFq = sC + N * NX;                               // [N][NA*NQ]   h da/dq
    double* const sFqd = sFq + N * FQ;                             // [N][NA*NA]   h da/dz
    double* const sFu = sFqd + N * FD;                             // [N][NA*NU]   h da/du
    double* const sR = sFu + N * FU;                               // [N][NX]      targets r_k
    double* const sHold = sR + N * NX;                             // [N][NU]      bound a control is held at
    double* const sLin = sHold + (BOUNDED ? N * NU : 0);           // linear mode: Fq | Fqd | Fu | xdot
    constexpr int NY = NX + NU;
    double* const wK = gw.ws + slot * (int64_t)group_ws_doubles(NX, NU, N, BOUNDED, XB);  // [N][NU][NS+1]
    constexpr int KZ = NX + NU, HW = group_hess_doubles(NX, NU);
    double* const wH = wK + N * NU * (NS + 1);  // EXACT: [N][HW] = W_k x rows [NX][KZ] | W_k uu block [NU][NU]
    constexpr int NR = NS + NU + 1;             // BOUNDED: [N][NU][NR] = un-held [H_wx | -R | H_ww | h_w] rows
    double* const wRel = wH + N * HW;
    bool w_zeros_stored = false;   // W_k's structural zeros are in the workspace (this launch's first W pass stored them)
    // interior point (XB): per stage k, y = (x_{k+1} | u_k) [NY]: duals z_l, z_u, Sigma, b, z_u - z_l -- in the HBM
    // workspace after the W blocks (group_lds_doubles); the stage-parallel phases write them, the serial sweeps read
    // them on other lanes after a workgroup fence
    double* const sZl = wRel;  // [N][NY]
    double* const sZu = sZl + N * NY;
    double* const sSg = sZu + N * NY;
    double* const sBb = sSg + N * NY;
    double* const sZg = sBb + N * NY;
    const double* const trg = p.traj + ii * (int64_t)N * NX;

    const double* w = p.weights + ii * p.w_stride;
    double Q[NX], R[NU], Rm[NU], up[NU];
#pragma unroll
    for (int r = 0; r < NX; ++r) Q[r] = w[r];
#pragma unroll
    for (int c = 0; c < NU; ++c) {
        R[c] = w[NX + c];
        Rm[c] = w[NX + NU + c];
        up[c] = p.u_prev[ii * NU + c];
    }
    double lbv[NU], ubv[NU];
    load_bounds<NU, BOUNDED>(p, lbv, ubv);
    // ---- lane-distributed Riccati (DIST): lane r of the group owns row r of the augmented value function
    //      P~ (NS x NS) and of every per-row quantity; small per-stage quantities are computed redundantly on
    //      all lanes; rows are exchanged with row_bcast.  Control bounds (BOUNDED) run the same
    //      sweeps with the held controls of the projected SQP folded into the per-stage quantities; state bounds
    //      (XB) add the barrier terms and use the Cholesky (Y^T Y) form of the stage update.  Models with
    //      nx + nu >= 16 keep the one-lane sweep below. ----
    constexpr bool DIST = (NS < G);
    // control-affine model: the u-u block of the exact-Hessian W_k is zero -- neither stored, loaded nor added
    constexpr bool CAFF = IsControlAffine<Model>::value;
    static_assert(!EXACT || (DIST && HasHess<Model>::value), "exact Hessian: lane-distributed path, model eval_hess");
    const int r = gl;
    const bool lx = r < NX, lu = r >= NX && r < NS, la = r >= NQ && r < NX;
    const int rx = lx ? r : 0;                        // x row of this lane (clamped for address arithmetic)
    const int ru = lu ? r - NX : 0;                   // u row
    const int ta = la ? r - NQ : 0;                   // row of the a-blocks (hFq, hFqd, hFu) of an a-lane
    const double Qr = lx ? w[rx] : 0.0;               // Q of this lane's x row
    // lane-role masks as blend factors: the DIST loops blend loaded values with FMAs instead of selects (a select
    // of an LDS load becomes a branch or a pointer select)
    const double lqd = r < NQ ? 1.0 : 0.0, lad = la ? 1.0 : 0.0;
    // x-lane factor for the sweeps' per-stage masking: one FP64 multiply where a 64-bit select is two cndmasks (the
    // masked values are finite sums of this instance's own data, so 0 * v == 0)
    const double lxf = lx ? 1.0 : 0.0;
    const int rq = r < NQ ? r : 0;                    // q column of a q-lane (clamped)
    const double Rr = lu ? w[NX + ru] : 0.0;          // R of this lane's u row
    double dgx[NS];                                    // XB: this x-lane's diagonal entry of P~ (barrier Sigma)
#pragma unroll
    for (int j = 0; j < NS; ++j) dgx[j] = (lx && j == r) ? 1.0 : 0.0;
    double lbr = -INFINITY, ubr = INFINITY;            // bounds of this u-lane's control (BOUNDED)
#pragma unroll
    for (int c = 0; c < NU; ++c)
        if (lu && ru == c) {
            lbr = lbv[c];
            ubr = ubv[c];
        }
    double hq[NQ > 0 ? NQ : 1], hrow[NX], qoh[NX], rdg[NU];
#pragma unroll
    for (int z = 0; z < NQ; ++z) hq[z] = (r == NQ + z) ? h : 0.0;   // column r of A holds h in row z (kinematics)
#pragma unroll
    for (int j = 0; j < NX; ++j) {
        hrow[j] = (r < NQ && j == NQ + r) ? h : 0.0;  // row r of A of a q-lane (besides the identity)
        qoh[j] = (j == r) ? Qr : 0.0;
    }
#pragma unroll
    for (int c = 0; c < NU; ++c) rdg[c] = (r == NX + c) ? R[c] : 0.0;
    // ---- load: V (reference layout) -> LDS, x_0 pinned (ModelControl.cpp:144-145) ----
    {
        const double* Vin = p.V + ii * (int64_t)NV;
        for (int k = gl; k <= N; k += G) {
#pragma unroll
            for (int r = 0; r < NX; ++r)
                sX[k * NX + r] = (k == 0 || p.init_hold) ? p.x0[ii * NX + r] : (p.init_zero ? 0.0 : Vin[k * ND + r]);
            if (k < N) {
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    const double v = p.init_zero ? 0.0 : Vin[k * ND + NX + c];
                    sU[k * NU + c] = BOUNDED ? proj(v, lbv[c], ubv[c]) : v;
                }
#pragma unroll
                for (int r = 0; r < NX; ++r) sR[k * NX + r] = trg[k * NX + r];
            }
        }
    }
    const double* const tr = sR;
    double yl[XB ? NY : 1], yu[XB ? NY : 1];
    double mub = (XB && resume) ? p.tail_mub[slot] : kIpMu0;  // barrier parameter (f = J/2 scale)
    if constexpr (XB) {
        load_ip_bounds<NX, NU>(p, yl, yu);
        __builtin_amdgcn_wave_barrier();
        if (resume) {   // the handed-over duals, from the lane launch's workspace (the iterate is interior already)
            const double* const lz = p.tail_lws + (inst >> 6) * p.tail_lws_block + (inst & 63);
            for (int k = gl; k < N; k += G) {
#pragma unroll
                for (int j = 0; j < NY; ++j) {
                    sZl[k * NY + j] = lz[((int64_t)k * p.tail_lws_ss + p.tail_lws_zl + j) * 64];
                    sZu[k * NY + j] = lz[((int64_t)k * p.tail_lws_ss + p.tail_lws_zl + NY + j) * 64];
                }
            }
        } else {
            // y pushed into the interior, z = 1 on finite bounds (oracle solve_one_ip)
            for (int k = gl; k < N; k += G) {
#pragma unroll
                for (int j = 0; j < NY; ++j) {
                    double& y = j < NX ? sX[(k + 1) * NX + j] : sU[k * NU + j - NX];
                    y = ip_push(y, yl[j], yu[j]);
                    sZl[k * NY + j] = yl[j] > -INFINITY ? 1.0 : 0.0;
                    sZu[k * NY + j] = yu[j] < INFINITY ? 1.0 : 0.0;
                }
            }
        }
    }
    // linear mode: acceleration Jacobians and xdot at (x_0, u_prev) (ModelControl.cpp:125-135), in LDS (keeps
    // 20-64 VGPRs free for the serial Riccati sweep); the linearisation point x_0 is sX[0..NX) (pinned)
    const bool lin = p.is_linear != 0;
    double* const lFq = sLin;
    double* const lFqd = lFq + FQ;
    double* const lFu = lFqd + FD;
    double* const lxd = lFu + FU;
    const double* const lxs = sX;
    if (lin && gl == 0) {
        double acc[NA], x[NX], Fq[SQ], Fqd[FD], Fu[FU];
#pragma unroll
        for (int r = 0; r < NX; ++r) x[r] = p.x0[ii * NX + r];
        Model::eval_acc_jac(x, up, acc, Fq, Fqd, Fu);
#pragma unroll
        for (int i = 0; i < FQ; ++i) lFq[i] = Fq[i];
#pragma unroll
        for (int i = 0; i < FD; ++i) lFqd[i] = Fqd[i];
#pragma unroll
        for (int i = 0; i < FU; ++i) lFu[i] = Fu[i];
#pragma unroll
        for (int i = 0; i < NQ; ++i) lxd[i] = x[NQ + i];
#pragma unroll
        for (int i = 0; i < NA; ++i) lxd[NQ + i] = acc[i];
    }
    __builtin_amdgcn_wave_barrier();
    int status = ST_MAX_ITER;
    int it = 0;
    double kkt = 0.0, mu = resume ? p.tail_mu[slot] : 0.0, pg_prev = (BOUNDED && resume) ? p.tail_mub[slot] : INFINITY;
    bool done = !valid;
    // FUSE_FWD: the line search's alpha = 1 trial evaluates the model with its Jacobian and writes everything phase A
    // computes at that point (F_k, c_k, the stage blocks; J, |c|_1, max|c|); when the full step is accepted (every
    // cfg#2 iteration, tools/alpha_stats.py) the next iteration skips phase A.  The trial point fma(1, d, v) is the
    // update's iterate and the sums run in phase A's order, so the values are phase A's bit for bit.  The old stage
    // blocks are dead once the directional derivative is formed; a rejected full step recomputes them in phase A.
    // XB (round 5): the first trial is at alpha = alpha_max (fraction to the boundary) and the update's y is the same
    // fma(alpha, dy, y) (ip_update), so the fused evaluation is again phase A's; the barrier terms (ip_terms) of phase
    // A still run every iteration, after the dual update.
    constexpr bool FUSE_FWD = true;
    bool fwd_ready = false;
    double J0n = 0.0, c1n = 0.0, cmaxn = 0.0;
    int nfn = 0;
    MMPC_PHASE(0);
    for (it = resume ? p.tail_it[slot] : 0; !done; ++it) {
        MMPC_PHASE(8);
        __builtin_amdgcn_wave_barrier();
        // ---- A. stage-parallel: F_k, A_k/B_k blocks, defects, merit value ----
        double J0 = J0n, c1 = c1n, cmax = cmaxn;
        int nonfinite = nfn;
        const bool evalA = !(FUSE_FWD && fwd_ready);
        if (evalA) {
            J0 = 0.0;
            c1 = 0.0;
            cmax = 0.0;
            nonfinite = 0;
            for (int k = gl; k < N; k += G) {
                double x[NX], u[NU], xd[NX], Fq[SQ], Fqd[FD], Fu[FU];
#pragma unroll
                for (int r = 0; r < NX; ++r) x[r] = sX[k * NX + r];
#pragma unroll
                for (int c = 0; c < NU; ++c) u[c] = sU[k * NU + c];
                group_model<Model>(lin, lFq, lFqd, lFu, lxd, lxs, up, x, u, xd, Fq, Fqd, Fu, true);
#pragma unroll
                for (int i = 0; i < FQ; ++i) sFq[k * FQ + i] = h * Fq[i];
#pragma unroll
                for (int i = 0; i < FD; ++i) sFqd[k * FD + i] = h * Fqd[i];
#pragma unroll
                for (int i = 0; i < FU; ++i) sFu[k * FU + i] = h * Fu[i];
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    const double F = fma(h, xd[r], x[r]);
                    sF[k * NX + r] = F;
                    const double c = F - sX[(k + 1) * NX + r];
                    sC[k * NX + r] = c;
                    cmax = fmax(cmax, fabs(c));
                    c1 += fabs(c);
                    nonfinite |= !isfinite(c);
                    const double e = F - tr[k * NX + r];
                    J0 = fma(e * Q[r], e, J0);
                }
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    const double um = (k == 0) ? up[c] : sU[(k - 1) * NU + c];
                    const double dif = u[c] - um;
                    J0 = fma(dif * R[c], dif, fma(u[c] * Rm[c], u[c], J0));
                }
            }
        }
        double lsum = 0.0, cmpl0 = 0.0, cmplmu = 0.0;  // interior point: sum log s, max |s z|, max |s z - mu|
        if constexpr (XB) {
            for (int k = gl; k < N; k += G) {
#pragma unroll
                for (int j = 0; j < NY; ++j) {
                    const double y = j < NX ? sX[(k + 1) * NX + j] : sU[k * NU + j - NX];
                    double sg, bb, zg;
                    ip_terms(y, yl[j], yu[j], sZl[k * NY + j], sZu[k * NY + j], mub, sg, bb, zg, cmpl0, cmplmu, lsum);
                    sSg[k * NY + j] = sg;
                    sBb[k * NY + j] = bb;
                    sZg[k * NY + j] = zg;
                }
            }
            lsum = group_sum(lsum);
            cmpl0 = group_max(cmpl0);
            cmplmu = group_max(cmplmu);
            nonfinite |= !isfinite(lsum);
            // Sigma, b, z_u - z_l of every stage (HBM workspace) visible to the other lanes' serial sweeps
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
        if (evalA) {
            J0 = group_sum(J0);
            c1 = group_sum(c1);
            cmax = group_max(cmax);
        }
        fwd_ready = false;
        __builtin_amdgcn_wave_barrier();
        MMPC_PHASE(1);

        // ---- B. one lane: d recursion, then adjoint + gradient + Riccati backward sweep (the 6x6 / 12x12
        //      Riccati step of one stage is too small to pay for lane-parallel exchanges: measured slower) ----
        double gmax = 0.0, lmax = 0.0;
        int fact_ok = 1;
        const double beps = BOUNDED ? fmin(kBoundEps, pg_prev) : 0.0;
        // backward sweep of QP solve `pass` (gradient and stop-test quantities are the same in every pass)
        auto backward = [&](int pass) {
            // P~ (symmetric, upper triangle used) and p~ on s = [dx_k; du_{k-1}]; P~_N = blkdiag(Q, 0)
            double P[NS][NS], pv[NS], lam[NX], unext[NU];
#define Ps(i, j) ((i) <= (j) ? P[(i)][(j)] : P[(j)][(i)])
#pragma unroll
            for (int a = 0; a < NS; ++a) {
                pv[a] = 0.0;
#pragma unroll
                for (int b = a; b < NS; ++b) P[a][b] = (a == b && a < NX) ? Q[a] : 0.0;
            }
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                const double eb = sX[N * NX + r] - tr[(N - 1) * NX + r];  // x_N - r_{N-1}
                pv[r] = Q[r] * eb;
                lam[r] = Q[r] * (sD[N * NX + r] + eb);  // lam_N = Q e_{N-1}
                if constexpr (XB) {  // barrier at x_N: Sigma, b in the value function, z_u - z_l in the adjoint
                    P[r][r] += sSg[(N - 1) * NY + r];
                    pv[r] += sBb[(N - 1) * NY + r];
                    lam[r] += sZg[(N - 1) * NY + r];
                }
                lmax = fmax(lmax, fabs(lam[r]));
            }
#pragma unroll
            for (int c = 0; c < NU; ++c) unext[c] = 0.0;
            for (int k = N - 1; k >= 0; --k) {
                const double* hFq = sFq + k * FQ;
                const double* hFqd = sFqd + k * FD;
                double hFu[FU], x[NX], u[NU], um[NU], cc[NX], tg[NU];
#pragma unroll
                for (int i = 0; i < FU; ++i) hFu[i] = sFu[k * FU + i];
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    x[r] = sX[k * NX + r];
                    cc[r] = sC[k * NX + r];
                }
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    u[c] = sU[k * NU + c];
                    um[c] = (k == 0) ? up[c] : sU[(k - 1) * NU + c];
                }
                // reduced gradient g_k = B_k^T lam_{k+1} + R/Rm terms
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    double g = 0.0;
#pragma unroll
                    for (int s = 0; s < NA; ++s) g = fma(hFu[s * NU + c], lam[NQ + s], g);
                    g = fma(R[c], u[c] - um[c], fma(Rm[c], u[c], g));
                    if (k + 1 < N) g -= R[c] * (unext[c] - u[c]);
                    if (XB) g += sZg[k * NY + NX + c];  // reduced Lagrangian gradient
                    if (!BOUNDED) {
                        gmax = fmax(gmax, fabs(2.0 * g));
                    } else {  // projected gradient; hold rule (pass 0) or the holds of the previous solve
                        gmax = fmax(gmax, fabs(u[c] - proj(u[c] - 2.0 * g, lbv[c], ubv[c])));
                        if (pass == 0) {
                            tg[c] = (u[c] <= lbv[c] + beps && g > 0.0)   ? lbv[c]
                                    : (u[c] >= ubv[c] - beps && g < 0.0) ? ubv[c]
                                                                          : NAN;
                            sHold[k * NU + c] = tg[c];
                        } else {
                            tg[c] = sHold[k * NU + c];
                        }
                    }
                    nonfinite |= !isfinite(g);
                    unext[c] = u[c];
                }
                // adjoint lam_k = Q e_{k-1} + A_k^T lam_{k+1},  e_{k-1} = d_k + x_k - r_{k-1}
                if (k >= 1) {
                    double ln[NX];
                    at_mul<NQ, NA, double>(h, hFq, hFqd, lam, ln);
#pragma unroll
                    for (int r = 0; r < NX; ++r) {
                        lam[r] = fma(Q[r], sD[k * NX + r] + x[r] - tr[(k - 1) * NX + r], ln[r]);
                        if (XB) lam[r] += sZg[(k - 1) * NY + r];
                        lmax = fmax(lmax, fabs(lam[r]));
                    }
                }
                // Riccati step (sqp_lane.h): G = P_xx B + P_xu, H_ww, h_w, Y = L^-1 [H_wx | -R | h_w]
                double Gm[NX][NU];
#pragma unroll
                for (int r = 0; r < NX; ++r)
#pragma unroll
                    for (int c = 0; c < NU; ++c) {
                        double t = Ps(r, NX + c);
#pragma unroll
                        for (int s = 0; s < NA; ++s) t = fma(Ps(r, NQ + s), hFu[s * NU + c], t);
                        Gm[r][c] = t;
                    }
                double mv[NX];
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    double t = pv[r];
#pragma unroll
                    for (int q = 0; q < NX; ++q) t = fma(Ps(r, q), cc[q], t);
                    mv[r] = t;
                }
                double Hww[NU][NU], Y[NU][NS + 1];
#pragma unroll
                for (int a = 0; a < NU; ++a) {
#pragma unroll
                    for (int b = a; b < NU; ++b) {
                        double t = Ps(NX + a, NX + b);
#pragma unroll
                        for (int s = 0; s < NA; ++s)
                            t = fma(hFu[s * NU + a], Gm[NQ + s][b], fma(Ps(NQ + s, NX + a), hFu[s * NU + b], t));
                        if (a == b) t += R[a] + Rm[a];
                        if (XB && a == b) t += sSg[k * NY + NX + a];
                        Hww[a][b] = t;
                    }
                    double t = fma(R[a], u[a] - um[a], fma(Rm[a], u[a], pv[NX + a]));
                    if (XB) t += sBb[k * NY + NX + a];
#pragma unroll
                    for (int s = 0; s < NA; ++s) t = fma(hFu[s * NU + a], mv[NQ + s], t);
#pragma unroll
                    for (int r = 0; r < NX; ++r) t = fma(Ps(r, NX + a), cc[r], t);
                    Y[a][NS] = t;
                    double ga[NX];
#pragma unroll
                    for (int r = 0; r < NX; ++r) ga[r] = Gm[r][a];
                    at_mul<NQ, NA, double>(h, hFq, hFqd, ga, &Y[a][0]);
#pragma unroll
                    for (int c = 0; c < NU; ++c) Y[a][NX + c] = (a == c) ? -R[a] : 0.0;
                }
                // held controls (bounded): w_A = target - u fixed in the stage QP, as sqp_lane.h
                double pex[NS];
                if (BOUNDED) {
                    bool hd[NU], any = false;
                    double dl[NU];
#pragma unroll
                    for (int j = 0; j < NS; ++j) pex[j] = 0.0;
#pragma unroll
                    for (int a = 0; a < NU; ++a) {
                        hd[a] = tg[a] == tg[a];
                        dl[a] = hd[a] ? tg[a] - u[a] : 0.0;
                        any |= hd[a];
                    }
                    if (any) {
#pragma unroll
                        for (int a = 0; a < NU; ++a)
#pragma unroll
                            for (int j = 0; j < NS; ++j) pex[j] = fma(Y[a][j], dl[a], pex[j]);
#pragma unroll
                        for (int b = 0; b < NU; ++b) {
                            double t = Y[b][NS];
#pragma unroll
                            for (int a = 0; a < NU; ++a) t = fma(Hww[a < b ? a : b][a < b ? b : a], dl[a], t);
                            Y[b][NS] = hd[b] ? -dl[b] : t;
                        }
#pragma unroll
                        for (int a = 0; a < NU; ++a) {
#pragma unroll
                            for (int b = a; b < NU; ++b)
                                if (hd[a] || hd[b]) Hww[a][b] = (a == b) ? 1.0 : 0.0;
                            if (hd[a])
#pragma unroll
                                for (int j = 0; j < NS; ++j) Y[a][j] = 0.0;
                        }
                    }
                }
                // P~_k x block A^T P_xx A + Q and p~_k x part A^T mv + Q (x_k - r_{k-1}), before P is overwritten
                double Pn[NX][NX], pn[NS];
                if (k >= 1) {
#pragma unroll
                    for (int b = 0; b < NX; ++b) {
                        double row[NX], tcol[NX];
#pragma unroll
                        for (int r = 0; r < NX; ++r) {
                            double t;
                            if (b < NQ) {
                                t = Ps(r, b);
#pragma unroll
                                for (int s = 0; s < NA; ++s) t = fma(hFq[s * NQ + b], Ps(r, NQ + s), t);
                            } else {
                                t = (b - NQ < NQ) ? fma(h, Ps(r, b - NQ), Ps(r, b)) : Ps(r, b);
#pragma unroll
                                for (int s = 0; s < NA; ++s) t = fma(hFqd[s * NA + b - NQ], Ps(r, NQ + s), t);
                            }
                            tcol[r] = t;
                        }
                        at_mul<NQ, NA, double>(h, hFq, hFqd, tcol, row);
#pragma unroll
                        for (int a = 0; a <= b; ++a)
                            Pn[a][b] = row[a] + ((a == b) ? Q[a] + (XB ? sSg[(k - 1) * NY + a] : 0.0) : 0.0);
                    }
                    double t[NX];
                    at_mul<NQ, NA, double>(h, hFq, hFqd, mv, t);
#pragma unroll
                    for (int q = 0; q < NX; ++q) {
                        pn[q] = fma(Q[q], x[q] - tr[(k - 1) * NX + q], t[q]);
                        if (XB) pn[q] += sBb[(k - 1) * NY + q];
                    }
#pragma unroll
                    for (int c = 0; c < NU; ++c) pn[NX + c] = -R[c] * (u[c] - um[c]);
                }
                // [K_k | kff_k] = -H_ww^-1 [H_wx | -R | h_w] (into wK) and Y with Y^T Y = Z^T H_ww^-1 Z for the
                // update of P~ and p~.  nu = 2: explicit inverse (one reciprocal; no square roots -- the serial
                // sweep is latency-bound); otherwise Cholesky, Y = L^-1 Z.
                double Kt[NU][NS + 1];
                if constexpr (NU == 2 && !XB) {  // XB: Cholesky (Y^T Y stays PSD with the large barrier Sigma)
                    const double det = fma(Hww[0][0], Hww[1][1], -Hww[0][1] * Hww[0][1]);
                    fact_ok &= (Hww[0][0] > 0.0) && (det > 0.0) && isfinite(det);
                    const double idet = rcp_nr(det);  // two Newton steps: ~1 ulp, off the division's long chain
                    const double i00 = Hww[1][1] * idet, i11 = Hww[0][0] * idet, i01 = -Hww[0][1] * idet;
#pragma unroll
                    for (int j = 0; j <= NS; ++j) {
                        Kt[0][j] = fma(i00, Y[0][j], i01 * Y[1][j]);
                        Kt[1][j] = fma(i01, Y[0][j], i11 * Y[1][j]);
                    }
                } else {
                    double Ld[NU][NU], il[NU];
#pragma unroll
                    for (int a = 0; a < NU; ++a) {
                        double sd = Hww[a][a];
#pragma unroll
                        for (int q = 0; q < a; ++q) sd = fma(-Ld[a][q], Ld[a][q], sd);
                        fact_ok &= (sd > 0.0) && isfinite(sd);
                        // 1/sqrt by v_rsq + two Newton steps (no square root and division on the serial chain)
                        const double sp = fmax(sd, 1e-300);
                        double r = __builtin_amdgcn_rsq(sp);
                        r = r * fma(-0.5 * sp * r, r, 1.5);
                        r = r * fma(-0.5 * sp * r, r, 1.5);
                        Ld[a][a] = sp * r;
                        il[a] = r;
#pragma unroll
                        for (int b = a + 1; b < NU; ++b) {
                            double t = Hww[a][b];
#pragma unroll
                            for (int q = 0; q < a; ++q) t = fma(-Ld[b][q], Ld[a][q], t);
                            Ld[b][a] = t * il[a];
                        }
                    }
#pragma unroll
                    for (int a = 0; a < NU; ++a)
#pragma unroll
                        for (int j = 0; j <= NS; ++j) {
                            double t = Y[a][j];
#pragma unroll
                            for (int q = 0; q < a; ++q) t = fma(-Ld[a][q], Y[q][j], t);
                            Y[a][j] = t * il[a];
                        }
#pragma unroll
                    for (int a = NU - 1; a >= 0; --a)
#pragma unroll
                        for (int j = 0; j <= NS; ++j) {
                            double t = Y[a][j];
#pragma unroll
                            for (int q = a + 1; q < NU; ++q) t = fma(-Ld[q][a], Kt[q][j], t);
                            Kt[a][j] = t * il[a];
                        }
                }
#pragma unroll
                for (int a = 0; a < NU; ++a)
#pragma unroll
                    for (int j = 0; j <= NS; ++j) wK[(k * NU + a) * (NS + 1) + j] = -Kt[a][j];
                if (k == 0) break;
                // P~_k = blkdiag(A^T P_xx A + Q, R) - Z^T H_ww^-1 Z, p~_k = pn - Z^T H_ww^-1 h_w:
                // nu = 2 as Y^T Kt (Y = Z, Kt = H_ww^-1 Z), Cholesky as Y^T Y (Y = L^-1 Z)
                const double(&YB)[NU][NS + 1] = (NU == 2 && !XB) ? Kt : Y;
#pragma unroll
                for (int a = 0; a < NS; ++a) {
                    double t = pn[a];
#pragma unroll
                    for (int q = 0; q < NU; ++q) t = fma(-Y[q][a], YB[q][NS], t);
                    if (BOUNDED) t += pex[a];
                    pv[a] = t;
#pragma unroll
                    for (int b = a; b < NS; ++b) {
                        double v = (b < NX) ? Pn[a][b] : ((a == b) ? R[a - NX] : 0.0);
#pragma unroll
                        for (int q = 0; q < NU; ++q) v = fma(-Y[q][a], YB[q][b], v);
                        P[a][b] = v;
                    }
                }
            }
#undef Ps
        };
        // ---- C. one lane: step sweep du = K s + kff, dx, directional derivative ----
        double dJ = 0.0;
        bool resolve = false;
        auto step_sweep = [&](int pass) {
            dJ = 0.0;
            double dx[NX], dup[NU], um[NU];
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                dx[r] = 0.0;
                sDX[r] = 0.0;
            }
#pragma unroll
            for (int c = 0; c < NU; ++c) {
                dup[c] = 0.0;
                um[c] = up[c];
            }
            // software pipeline: K_{k+1} (HBM) and the LDS operands of step k+1 are loaded during step k
            constexpr int NK = NU * (NS + 1);
            double nK[NK], nFq[SQ], nFqd[FD], nFu[FU], nF[NX], nc[NX], nr[NX], nu_[NU];
#define GROUP_LOAD_STEP(k_)                                                                        \
        do {                                                                                           \
            const int kk_ = (k_);                                                                      \
            _Pragma("unroll") for (int i_ = 0; i_ < NK; ++i_) nK[i_] = wK[kk_ * NK + i_];              \
            _Pragma("unroll") for (int i_ = 0; i_ < FQ; ++i_) nFq[i_] = sFq[kk_ * FQ + i_];             \
            _Pragma("unroll") for (int i_ = 0; i_ < FD; ++i_) nFqd[i_] = sFqd[kk_ * FD + i_];           \
            _Pragma("unroll") for (int i_ = 0; i_ < FU; ++i_) nFu[i_] = sFu[kk_ * FU + i_];             \
            _Pragma("unroll") for (int r_ = 0; r_ < NX; ++r_) {                                        \
            nF[r_] = sF[kk_ * NX + r_];                                                            \
            nc[r_] = sC[kk_ * NX + r_];                                                            \
            nr[r_] = sR[kk_ * NX + r_];                                                            \
            }                                                                                          \
            _Pragma("unroll") for (int c_ = 0; c_ < NU; ++c_) nu_[c_] = sU[kk_ * NU + c_];             \
        } while (0)
            GROUP_LOAD_STEP(0);
            // unrolled by two so that the prefetch buffers are renamed instead of copied (2-link only: the exo
            // step spills when unrolled)
            constexpr int kStepUnroll = NX <= 4 ? 2 : 1;
#pragma unroll kStepUnroll
            for (int k = 0; k < N; ++k) {
                double K[NK], hFq[SQ], hFqd[FD], hFu[FU], Fk[NX], ck[NX], rk[NX], uk[NU];
#pragma unroll
                for (int i = 0; i < NK; ++i) K[i] = nK[i];
#pragma unroll
                for (int i = 0; i < FQ; ++i) hFq[i] = nFq[i];
#pragma unroll
                for (int i = 0; i < FD; ++i) hFqd[i] = nFqd[i];
#pragma unroll
                for (int i = 0; i < FU; ++i) hFu[i] = nFu[i];
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    Fk[r] = nF[r];
                    ck[r] = nc[r];
                    rk[r] = nr[r];
                }
#pragma unroll
                for (int c = 0; c < NU; ++c) uk[c] = nu_[c];
                if (k + 1 < N) GROUP_LOAD_STEP(k + 1);
                double du[NU];
#pragma unroll
                for (int a = 0; a < NU; ++a) {
                    double t = K[a * (NS + 1) + NS];
#pragma unroll
                    for (int q = 0; q < NX; ++q) t = fma(K[a * (NS + 1) + q], dx[q], t);
#pragma unroll
                    for (int c = 0; c < NU; ++c) t = fma(K[a * (NS + 1) + NX + c], dup[c], t);
                    du[a] = t;
                    sDU[k * NU + a] = t;
                }
                if (BOUNDED && pass + 1 < kBoundPasses) {  // a free control whose step crosses a bound: hold it
#pragma unroll
                    for (int a = 0; a < NU; ++a) {
                        const double hv = sHold[k * NU + a], t = uk[a] + du[a];
                        if (hv != hv && (t < lbv[a] || t > ubv[a])) {
                            sHold[k * NU + a] = t < lbv[a] ? lbv[a] : ubv[a];
                            resolve = true;
                        }
                    }
                }
                double ad[NX];
                a_mul<NQ, NA, double>(h, hFq, hFqd, dx, ad);
#pragma unroll
                for (int s = 0; s < NA; ++s)
#pragma unroll
                    for (int c = 0; c < NU; ++c) ad[NQ + s] = fma(hFu[s * NU + c], du[c], ad[NQ + s]);
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    const double qe = 2.0 * Q[r] * (Fk[r] - rk[r]);
                    dJ = fma(qe, ad[r], dJ);
                    dx[r] = ad[r] + ck[r];
                    sDX[(k + 1) * NX + r] = dx[r];
                }
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    const double dif = uk[c] - um[c];
                    dJ = fma(2.0 * R[c] * dif, du[c] - dup[c], fma(2.0 * Rm[c] * uk[c], du[c], dJ));
                    um[c] = uk[c];
                    dup[c] = du[c];
                }
            }
#undef GROUP_LOAD_STEP
        };
        // ---- DIST: the same recursions with row r of every quantity on lane r of the group ----
        // column r of A (x-lanes): own row (identity) + h in row z for r = NQ + z + acol[t] in row NQ + t, where
        // acol = hFq[:, r] (q-lanes) or hFqd[:, r - NQ] (a-lanes); so (A^T v)[r] = colA(v_r, vb) with vb = all v.
        auto colA = [&](double own, const double* acol, const double* vb) {
            double t = lxf * own;
#pragma unroll
            for (int z = 0; z < NQ; ++z) t = fma(hq[z], vb[z], t);
#pragma unroll
            for (int s2 = 0; s2 < NA; ++s2) t = fma(acol[s2], vb[NQ + s2], t);
            return t;
        };
        // row r of [A - I | B] (x-lanes) at stage k: q-lanes h e_{NQ+r}, a-lanes [hFq, hFqd | hFu] row r - NQ
        // (loads are unconditional from clamped rows and then selected: a conditional LDS load becomes a branch)
        // (the asm pins keep the selects on values: select(load, hrow[j]) otherwise becomes a flat load through a
        // selected LDS-or-scratch pointer)
        auto load_arow = [&](int k, double* arow, double* brow) {
#pragma unroll
            for (int s2 = 0; s2 < NQ; ++s2) arow[s2] = fma(lad, sFq[k * FQ + ta * NQ + s2], hrow[s2]);
#pragma unroll
            for (int s2 = 0; s2 < NA; ++s2) arow[NQ + s2] = fma(lad, sFqd[k * FD + ta * NA + s2], hrow[NQ + s2]);
#pragma unroll
            for (int c = 0; c < NU; ++c) brow[c] = lad * sFu[k * FU + ta * NU + c];
        };
        // d_{k+1} = A_k d_k + c_k (d_0 = 0): lane r holds d_k[r]
        // The recursions below are latency-bound (a few FMAs per stage on the dependency chain): every stage's
        // LDS operands are loaded one stage ahead and the dot products split into two partial sums.
        auto d_recursion_dist = [&]() {
            double dr = 0.0;
            if (lx) sD[rx] = 0.0;
            // stage operands as loaded (the blend with the lane-role factors happens at the use, so the wait for a
            // load sits a full stage after its issue): two buffers, each refilled two stages ahead
            struct Op {
                double q[NQ > 0 ? NQ : 1], d[NA], c;
            };
            auto fetch = [&](int k, Op& o) {
#pragma unroll
                for (int s2 = 0; s2 < NQ; ++s2) o.q[s2] = sFq[k * FQ + ta * NQ + s2];
#pragma unroll
                for (int s2 = 0; s2 < NA; ++s2) o.d[s2] = sFqd[k * FD + ta * NA + s2];
                o.c = sC[k * NX + rx];
            };
            auto stage = [&](int k, Op& o) {
                double db[NX], arow[NX];
#pragma unroll
                for (int s2 = 0; s2 < NQ; ++s2) arow[s2] = fma(lad, o.q[s2], hrow[s2]);
#pragma unroll
                for (int s2 = 0; s2 < NA; ++s2) arow[NQ + s2] = fma(lad, o.d[s2], hrow[NQ + s2]);
                const double cr = o.c;
                // unconditional and unclamped (static wait counts; the address is a strength-reduced increment): past
                // the last stage the loads read the next arrays of this instance's LDS block (sFq -> sFqd -> sFu,
                // sC -> sFq), values never used
                fetch(k + 2, o);
                sfor<0, NX>([&](auto I) { db[I] = row_bcast<I>(dr); });
                double t0 = dr + cr, t1 = 0.0;
#pragma unroll
                for (int j = 0; j < NX; ++j) {
                    if (j & 1) t1 = fma(arow[j], db[j], t1);
                    else t0 = fma(arow[j], db[j], t0);
                }
                // no lane-role mask on the chain: only the x-lanes' d is broadcast or stored, and the other lanes'
                // finite leftovers (a sum of c_k[0]) are never read
                dr = t0 + t1;
                if (lx) sD[(k + 1) * NX + rx] = dr;
            };
            Op o0, o1;
            fetch(0, o0);
            fetch(N > 1 ? 1 : 0, o1);
            int k = 0;
            for (; k + 1 < N; k += 2) {
                stage(k, o0);
                stage(k + 1, o1);
            }
            if (k < N) stage(k, o0);
        };
        // adjoint + reduced gradient + Riccati backward sweep; lane r: row r of P~ (Prow) and p~ (pvr), lam[r]
        // column r of the a-rows of A at stage k: hFq[:, r] (q-lanes), hFqd[:, r - NQ] (a-lanes), 0 otherwise
        auto load_acol = [&](int k, double* acol) {
#pragma unroll
            for (int t2 = 0; t2 < NA; ++t2) {
                double v = lad * sFqd[k * FD + t2 * NA + ta];
                if constexpr (NQ > 0) v = fma(lqd, sFq[k * FQ + t2 * NQ + rq], v);
                acol[t2] = v;
            }
        };
        // adjoint lam_k = Q e_{k-1} + A_k^T lam_{k+1} (lam_N = Q e_{N-1}, e_{k-1} = d_k + x_k - r_{k-1}), lane r holds
        // lam[r] (x-lanes) and writes it over d_k in sD (d_k is read one stage earlier); then, stage-parallel, the
        // reduced gradient g_k = B_k^T lam_{k+1} + R (u_k - u_{k-1}) + Rm u_k - R (u_{k+1} - u_k) from the stored
        // lam (the serial sweep carries only the lam chain: the gradient's loads and arithmetic were a quarter of
        // its instructions).  gmax, lmax are per-lane maxima (reduced by the caller).
        // Runs before the stop test, so a converged wave skips the Riccati sweep.
        auto adjoint_dist = [&]() {
            double lamr;
            {
                const double eb = lx ? sX[N * NX + rx] - tr[(N - 1) * NX + rx] : 0.0;   // x_N - r_{N-1}
                lamr = Qr * (sD[N * NX + rx] + eb);
                if constexpr (XB) lamr += lxf * sZg[(N - 1) * NY + rx];   // z_u - z_l of x_N's bounds
                lmax = fmax(lmax, fabs(lamr));
                if (lx) sD[N * NX + rx] = lamr;   // lam_k replaces d_k (read one stage earlier)
            }
            // stage operands as loaded, two buffers refilled two stages ahead (d_k is read before stage k writes lam_k
            // over it): column r of A's a-rows and the pieces of Q (d_k + x_k - r_{k-1})[r], combined at the use
            struct Op {
                double fd[NA], fq[NA], xk, trm, dk, zg;
            };
            auto fetch = [&](int k, Op& o) {   // k >= 1
#pragma unroll
                for (int t2 = 0; t2 < NA; ++t2) {
                    o.fd[t2] = sFqd[k * FD + t2 * NA + ta];
                    if constexpr (NQ > 0) o.fq[t2] = sFq[k * FQ + t2 * NQ + rq];
                }
                o.xk = sX[k * NX + rx];
                o.trm = tr[(k - 1) * NX + rx];
                o.dk = sD[k * NX + rx];
                if constexpr (XB) o.zg = sZg[(k - 1) * NY + rx];   // z_u - z_l of x_k's bounds (masked by lxf)
            };
            // stage k >= 1: lam_k from lam_{k+1}; then refill o with stage k - 2 (k >= 3)
            auto stage = [&](int k, Op& o) {
                double acol[NA];
#pragma unroll
                for (int t2 = 0; t2 < NA; ++t2) {
                    double v = lad * o.fd[t2];
                    if constexpr (NQ > 0) v = fma(lqd, o.fq[t2], v);
                    acol[t2] = v;
                }
                double qe = Qr * (o.dk + (o.xk - o.trm));
                if constexpr (XB) qe += o.zg;
                fetch(k >= 3 ? k - 2 : 1, o);   // unconditional: static wait counts
                double lamb[NX];
                sfor<0, NX>([&](auto I) { lamb[I] = row_bcast<I>(lamr); });
                // (A^T lam)[r] + Q e_{k-1}[r], two partial sums
                // unmasked chain: a lane without an x row has Qr = 0, acol = 0 and hq = 0, so it carries 0 (XB: a finite
                // sum of another row's z gaps) -- never broadcast or stored, and masked out of lmax
                double t0 = lamr + qe, t1 = 0.0;
#pragma unroll
                for (int z = 0; z < NQ; ++z) t1 = fma(hq[z], lamb[z], t1);
#pragma unroll
                for (int s2 = 0; s2 < NA; ++s2) {
                    if (s2 & 1) t1 = fma(acol[s2], lamb[NQ + s2], t1);
                    else t0 = fma(acol[s2], lamb[NQ + s2], t0);
                }
                lamr = t0 + t1;
                lmax = fmax(lmax, fabs(lxf * lamr));
                if (lx) sD[k * NX + rx] = lamr;
            };
            if (N >= 2) {
                Op o0, o1;
                fetch(N - 1, o0);
                fetch(N >= 3 ? N - 2 : 1, o1);
                int k = N - 1;
                for (; k >= 2; k -= 2) {
                    stage(k, o0);
                    stage(k - 1, o1);
                }
                if (k == 1) stage(1, o0);
            }
            // the lam rows of the other lanes of this wave must be visible to the gradient pass
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            for (int k = gl; k < N; k += G) {
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    double g = 0.0;
#pragma unroll
                    for (int s2 = 0; s2 < NA; ++s2) g = fma(sFu[k * FU + s2 * NU + c], sD[(k + 1) * NX + NQ + s2], g);
                    const double uk = sU[k * NU + c], um = k == 0 ? up[c] : sU[(k - 1) * NU + c];
                    g = fma(R[c], uk - um, fma(Rm[c], uk, g));
                    if (k < N - 1) g -= R[c] * (sU[(k + 1) * NU + c] - uk);
                    if constexpr (XB) g += sZg[k * NY + NX + c];   // reduced Lagrangian gradient
                    if constexpr (!BOUNDED) {
                        gmax = fmax(gmax, fabs(2.0 * g));
                    } else {   // projected gradient; epsilon-active holds of the first QP solve (oracle solve_one)
                        gmax = fmax(gmax, fabs(uk - proj(uk - 2.0 * g, lbv[c], ubv[c])));
                        sHold[k * NU + c] = (uk <= lbv[c] + beps && g > 0.0)   ? lbv[c]
                                            : (uk >= ubv[c] - beps && g < 0.0) ? ubv[c]
                                                                                : NAN;
                    }
                    nonfinite |= !isfinite(g);
                }
            }
        };
        auto backward_dist = [&](bool useW) {
            if constexpr (BOUNDED) {   // the hold targets (sHold) the gradient pass stored on every lane of this wave
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            double Prow[NS], pvr;
            const double lxm = lx ? 1.0 : 0.0;
            // W_k row rx and uu block from the workspace, loaded one stage ahead into one buffer.  (Round 2 used two
            // buffers two stages ahead; once the control-affine sweep dropped the uu block, the second buffer's
            // registers cost more than the load latency it hid: 0.1875 -> 0.1808 ms with one buffer)
            struct Wb {
                double r[KZ], u[NU * NU];
            };
            Wb w0;
            auto load_w = [&](int k, Wb& b) {
#pragma unroll
                for (int j = 0; j < KZ; ++j) b.r[j] = wH[k * HW + rx * KZ + j];   // row rx; masked at its uses
                if constexpr (!CAFF) {
#pragma unroll
                    for (int j = 0; j < NU * NU; ++j) b.u[j] = wH[k * HW + NX * KZ + j];
                }
            };
            if (EXACT && useW) {
                load_w(N - 1, w0);
            }
#pragma unroll
            for (int j = 0; j < NS; ++j) Prow[j] = j < NX ? qoh[j] : 0.0;   // P~_N = blkdiag(Q, 0)
            pvr = Qr * (lx ? sX[N * NX + rx] - tr[(N - 1) * NX + rx] : 0.0);   // Q (x_N - r_{N-1})
            if constexpr (XB) {   // barrier at x_N: Sigma on the diagonal, b in p~
                const double sgN = sSg[(N - 1) * NY + rx], bbN = sBb[(N - 1) * NY + rx];
#pragma unroll
                for (int j = 0; j < NX; ++j) Prow[j] = fma(dgx[j], sgN, Prow[j]);
                pvr = fma(lxm, bbN, pvr);
            }
            // (the sweep is issue-bound: its LDS operands are read in place; a prefetch buffer spills to AGPRs)
            // stage k; LAST = (k == 0), peeled so that the stages k >= 1 carry no k == 0 selects or branches
            auto stage = [&](int k, auto last_c, Wb& wb) {
                constexpr bool LAST = decltype(last_c)::value;
#if defined(MMPC_PHASE_TIMING) && defined(MMPC_PHASE_STAGES)
                if (gl == 0 && blockIdx.x < kPhaseWavePhases && k < 32)
                    g_mmpc_phase_cycles[kPhaseStageLog + 128 * blockIdx.x + 32 * gi + k] = __builtin_amdgcn_s_memtime();
#endif
                double hFq[SQ], hFqd[FD], hFu[FU], cc[NX], u[NU], um[NU], acol[NA];
#pragma unroll
                for (int i = 0; i < FQ; ++i) hFq[i] = sFq[k * FQ + i];
#pragma unroll
                for (int i = 0; i < FD; ++i) hFqd[i] = sFqd[k * FD + i];
#pragma unroll
                for (int i = 0; i < FU; ++i) hFu[i] = sFu[k * FU + i];
#pragma unroll
                for (int q = 0; q < NX; ++q) cc[q] = sC[k * NX + q];
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    u[c] = sU[k * NU + c];
                    um[c] = LAST ? up[c] : sU[(k - 1) * NU + c];
                }
                load_acol(k, acol);
                // XB: the barrier pieces of this stage (u_k) and of x_k (stage k-1), loaded with the stage operands:
                // read at their uses, deep in the stage, their HBM latency was exposed
                double xsgu[XB ? NU : 1], xbbu[XB ? NU : 1], xsgx = 0.0, xbbx = 0.0;
                if constexpr (XB) {
#pragma unroll
                    for (int a = 0; a < NU; ++a) {
                        xsgu[a] = sSg[k * NY + NX + a];
                        xbbu[a] = sBb[k * NY + NX + a];
                    }
                    if constexpr (!LAST) {
                        xsgx = sSg[(k - 1) * NY + rx];
                        xbbx = sBb[(k - 1) * NY + rx];
                    }
                }
                double exr = 0.0, duu = 0.0;
                if constexpr (!LAST) {
                    const double xk = sX[k * NX + rx], trm = tr[(k - 1) * NX + rx];
                    exr = xk - trm;   // non-x lanes: finite leftovers of the clamped row, masked by lxm in pn
                    duu = sU[k * NU + ru] - sU[(k - 1) * NU + ru];
                }
                double wr[KZ], wu[NU * NU];
                if constexpr (EXACT) {
#pragma unroll
                    for (int j = 0; j < KZ; ++j) wr[j] = useW ? wb.r[j] : 0.0;
#pragma unroll
                    for (int j = 0; j < NU * NU; ++j) wu[j] = (useW && !CAFF) ? wb.u[j] : 0.0;
                    if (!LAST && useW) load_w(k - 1, wb);
                }
                // T = P~ [B; I] (row r), mv = P~_x. c + p~ (row r)
                double T[NU], mv = pvr;
#pragma unroll
                for (int b = 0; b < NU; ++b) {
                    double t = Prow[NX + b];
#pragma unroll
                    for (int s2 = 0; s2 < NA; ++s2) t = fma(Prow[NQ + s2], hFu[s2 * NU + b], t);
                    T[b] = t;
                }
#pragma unroll
                for (int q = 0; q < NX; ++q) mv = fma(Prow[q], cc[q], mv);
                double Tb[NS][NU], mvb[NS];
                sfor<0, NS>([&](auto I) {
#pragma unroll
                    for (int b = 0; b < NU; ++b) Tb[I][b] = row_bcast<I>(T[b]);
                    mvb[I] = row_bcast<I>(mv);
                });
                // H_ww = B^T P_xx B + B^T P_xu + P_ux B + P_uu + R + Rm, h_w (redundant)
                double Hww[NU][NU], hw[NU];
#pragma unroll
                for (int a = 0; a < NU; ++a) {
#pragma unroll
                    for (int b = a; b < NU; ++b) {
                        double t = Tb[NX + a][b];
#pragma unroll
                        for (int s2 = 0; s2 < NA; ++s2) t = fma(hFu[s2 * NU + a], Tb[NQ + s2][b], t);
                        if (a == b) t += R[a] + Rm[a];
                        if constexpr (EXACT && !CAFF) t += wu[a * NU + b];
                        if constexpr (XB) {
                            if (a == b) t += xsgu[a];   // barrier Sigma of u_k
                        }
                        Hww[a][b] = t;
                        Hww[b][a] = t;
                    }
                    double t = fma(R[a], u[a] - um[a], fma(Rm[a], u[a], mvb[NX + a]));
#pragma unroll
                    for (int s2 = 0; s2 < NA; ++s2) t = fma(hFu[s2 * NU + a], mvb[NQ + s2], t);
                    if constexpr (XB) t += xbbu[a];   // barrier gradient b of u_k
                    hw[a] = t;
                }
                // column r of Y = [H_wx | -R | .]: x-lanes (A^T T)[r], u-lanes -R e_{r-NX}
                double Ycol[NU];
#pragma unroll
                for (int a = 0; a < NU; ++a) {
                    double tb[NX];
#pragma unroll
                    for (int q = 0; q < NX; ++q) tb[q] = Tb[q][a];
                    Ycol[a] = colA(T[a], acol, tb) - rdg[a];
                    if constexpr (EXACT) Ycol[a] = fma(lxm, wr[NX + a], Ycol[a]);   // H_wx[a][r] += W_ux[a][r] (x-lanes)
                }
                // BOUNDED: the un-held stage rows [H_wx | -R | H_ww | h_w] (lane j < NS: column j; lanes NS.. the H_ww
                // columns and h_w, the idle lanes duplicating h_w) -- the step sweep forms the multiplier of a held
                // control from them (primal-dual active set: release a hold whose multiplier points into the box)
                if constexpr (BOUNDED) {
#pragma unroll
                    for (int c0 = 0; c0 < NR; c0 += G) {   // column c0 + r; lanes past the row rewrite its last entry
                        const int col = c0 + r < NR ? c0 + r : NR - 1;
#pragma unroll
                        for (int a = 0; a < NU; ++a) {
                            double v = hw[a];
#pragma unroll
                            for (int b = 0; b < NU; ++b)
                                if (col == NS + b) v = Hww[a][b];
                            wRel[(k * NU + a) * NR + col] = col < NS ? Ycol[a] : v;
                        }
                    }
                }
                // held controls (BOUNDED, sHold of this QP solve): du_a = target - u_a fixed in the stage QP, as the
                // one-lane sweep -- p~ gains [H_wx | -R]^T delta, h_w the coupling H_ww delta, the held rows and
                // columns of H_ww become the identity and the held rows of [H_wx | -R] zero, so that K_a = 0 and
                // kff_a = delta_a exactly; Rk: the -R columns of the u-lanes with the held rows removed
                double pexr = 0.0, Rk[NU];
#pragma unroll
                for (int c = 0; c < NU; ++c) Rk[c] = R[c];
                if constexpr (BOUNDED) {
                    bool hd[NU];
                    double dl[NU], hw2[NU];
#pragma unroll
                    for (int a = 0; a < NU; ++a) {
                        const double tg = sHold[k * NU + a];
                        hd[a] = tg == tg;
                        dl[a] = hd[a] ? tg - u[a] : 0.0;
                        pexr = fma(Ycol[a], dl[a], pexr);
                    }
#pragma unroll
                    for (int b = 0; b < NU; ++b) {
                        double t = hw[b];
#pragma unroll
                        for (int a = 0; a < NU; ++a) t = fma(Hww[a][b], dl[a], t);
                        hw2[b] = hd[b] ? -dl[b] : t;
                    }
#pragma unroll
                    for (int a = 0; a < NU; ++a) {
                        hw[a] = hw2[a];
#pragma unroll
                        for (int b = 0; b < NU; ++b)
                            if (hd[a] || hd[b]) Hww[a][b] = (a == b) ? 1.0 : 0.0;
                        if (hd[a]) {
                            Ycol[a] = 0.0;
                            Rk[a] = 0.0;
                        }
                    }
                }
                // Kcol = H_ww^-1 Ycol (this lane's column of K~), kff = H_ww^-1 h_w (redundant)
                double Kcol[NU], kff[NU], Ku[NU][NU];
                // XB: Cholesky H_ww = L L^T, Ytil = L^-1 Ycol (this lane's column of L^-1 [H_wx | -R]), htil = L^-1 h_w;
                // the update P~ -= Ytil^T Ytil stays positive semidefinite under the barrier's large Sigma
                double Ytil[NU], htil[NU];
                if constexpr (XB) {
                    double Ld[NU][NU], il[NU];
#pragma unroll
                    for (int a = 0; a < NU; ++a) {
                        double sd = Hww[a][a];
#pragma unroll
                        for (int q = 0; q < a; ++q) sd = fma(-Ld[a][q], Ld[a][q], sd);
                        fact_ok &= (sd > 0.0) && isfinite(sd);
                        const double sp = fmax(sd, 1e-300);
                        double rr = __builtin_amdgcn_rsq(sp);
                        rr = rr * fma(-0.5 * sp * rr, rr, 1.5);
                        rr = rr * fma(-0.5 * sp * rr, rr, 1.5);
                        Ld[a][a] = sp * rr;
                        il[a] = rr;
#pragma unroll
                        for (int b = a + 1; b < NU; ++b) {
                            double t = Hww[a][b];
#pragma unroll
                            for (int q = 0; q < a; ++q) t = fma(-Ld[b][q], Ld[a][q], t);
                            Ld[b][a] = t * il[a];
                        }
                    }
#pragma unroll
                    for (int a = 0; a < NU; ++a) {   // forward substitutions
                        double t = Ycol[a], th = hw[a];
#pragma unroll
                        for (int q = 0; q < a; ++q) {
                            t = fma(-Ld[a][q], Ytil[q], t);
                            th = fma(-Ld[a][q], htil[q], th);
                        }
                        Ytil[a] = t * il[a];
                        htil[a] = th * il[a];
                    }
#pragma unroll
                    for (int a = NU - 1; a >= 0; --a) {   // back substitutions: K~ column, kff
                        double t = Ytil[a], th = htil[a];
#pragma unroll
                        for (int q = a + 1; q < NU; ++q) {
                            t = fma(-Ld[q][a], Kcol[q], t);
                            th = fma(-Ld[q][a], kff[q], th);
                        }
                        Kcol[a] = t * il[a];
                        kff[a] = th * il[a];
                    }
                } else if constexpr (NU == 2) {
                    const double det = fma(Hww[0][0], Hww[1][1], -Hww[0][1] * Hww[0][1]);
                    fact_ok &= (Hww[0][0] > 0.0) && (det > 0.0) && isfinite(det);
                    const double idet = rcp_nr(det);
                    const double i00 = Hww[1][1] * idet, i11 = Hww[0][0] * idet, i01 = -Hww[0][1] * idet;
                    Kcol[0] = fma(i00, Ycol[0], i01 * Ycol[1]);
                    Kcol[1] = fma(i01, Ycol[0], i11 * Ycol[1]);
                    kff[0] = fma(i00, hw[0], i01 * hw[1]);
                    kff[1] = fma(i01, hw[0], i11 * hw[1]);
                    Ku[0][0] = -i00 * Rk[0];
                    Ku[0][1] = -i01 * Rk[1];
                    Ku[1][0] = -i01 * Rk[0];
                    Ku[1][1] = -i11 * Rk[1];
                } else {   // Cholesky H_ww = L L^T (rsq + Newton), solves with L and L^T
                    double Ld[NU][NU], il[NU];
#pragma unroll
                    for (int a = 0; a < NU; ++a) {
                        double sd = Hww[a][a];
#pragma unroll
                        for (int q = 0; q < a; ++q) sd = fma(-Ld[a][q], Ld[a][q], sd);
                        fact_ok &= (sd > 0.0) && isfinite(sd);
                        const double sp = fmax(sd, 1e-300);
                        double rr = __builtin_amdgcn_rsq(sp);
                        rr = rr * fma(-0.5 * sp * rr, rr, 1.5);
                        rr = rr * fma(-0.5 * sp * rr, rr, 1.5);
                        Ld[a][a] = sp * rr;
                        il[a] = rr;
#pragma unroll
                        for (int b = a + 1; b < NU; ++b) {
                            double t = Hww[a][b];
#pragma unroll
                            for (int q = 0; q < a; ++q) t = fma(-Ld[b][q], Ld[a][q], t);
                            Ld[b][a] = t * il[a];
                        }
                    }
                    auto chol_solve = [&](const double* rhs, double* out) {
                        double y[NU];
#pragma unroll
                        for (int a = 0; a < NU; ++a) {
                            double t = rhs[a];
#pragma unroll
                            for (int q = 0; q < a; ++q) t = fma(-Ld[a][q], y[q], t);
                            y[a] = t * il[a];
                        }
#pragma unroll
                        for (int a = NU - 1; a >= 0; --a) {
                            double t = y[a];
#pragma unroll
                            for (int q = a + 1; q < NU; ++q) t = fma(-Ld[q][a], out[q], t);
                            out[a] = t * il[a];
                        }
                    };
                    chol_solve(Ycol, Kcol);
                    chol_solve(hw, kff);
#pragma unroll
                    for (int c = 0; c < NU; ++c) {   // column NX + c of K~: H_ww^-1 (-R_c e_c)
                        double e[NU], o[NU];
#pragma unroll
                        for (int a = 0; a < NU; ++a) e[a] = (a == c) ? -Rk[c] : 0.0;
                        chol_solve(e, o);
#pragma unroll
                        for (int a = 0; a < NU; ++a) Ku[a][c] = o[a];
                    }
                }
                // [K_k | kff_k] = -[K~ | kff~] (lane j < NS stores column j, lanes >= NS the feed-forward column: kff
                // is computed redundantly, bit-identical on every lane of the group, so the duplicate stores of the
                // idle lanes write the same value -- no exec-mask branch in the sweep)
                {
                    const int col = r < NS ? r : NS;
#pragma unroll
                    for (int a = 0; a < NU; ++a) ws_store(&wK[(k * NU + a) * (NS + 1) + col], -(r < NS ? Kcol[a] : kff[a]));
                }
                if constexpr (LAST) return;
                // A^T P_xx A (row r) from the broadcast P_xx, p~_x = A^T mv + Q (x_k - r_{k-1})
                double Pb[NX][NX];
                sfor<0, NX>([&](auto I) {
#pragma unroll
                    for (int j = I; j < NX; ++j) {
                        Pb[I][j] = row_bcast<I>(Prow[j]);
                        Pb[j][I] = Pb[I][j];
                    }
                });
                double Ur[NX], Pn[NX];
#pragma unroll
                for (int j = 0; j < NX; ++j) {
                    double pc[NX];
#pragma unroll
                    for (int q = 0; q < NX; ++q) pc[q] = Pb[q][j];
                    Ur[j] = colA(Prow[j], acol, pc);
                }
                at_mul<NQ, NA, double>(h, hFq, hFqd, Ur, Pn);
                // x-lanes A^T mv + Q (x_k - r_{k-1}), u-lanes -R (u_k - u_{k-1}), idle lanes 0 -- blended with the
                // lane-role factor (Rr = 0 off the u-lanes) instead of a branch
                double pn = fma(-Rr, duu, lxm * fma(Qr, exr, colA(mv, acol, mvb)));
                double sgk = 0.0;   // XB: barrier Sigma and b of x_k (stage k-1's y)
                if constexpr (XB) {
                    sgk = xsgx;
                    pn = fma(lxm, xbbx, pn);
                }
                if constexpr (XB) {   // P~_k = blkdiag(A^T P_xx A + Q + Sigma, R) - Ytil^T Ytil, p~_k = pn - Ytil^T htil
                    double Yb[NU][NS];
                    sfor<0, NS>([&](auto I) {
#pragma unroll
                        for (int a = 0; a < NU; ++a) Yb[a][I] = row_bcast<I>(Ytil[a]);
                    });
#pragma unroll
                    for (int j = 0; j < NS; ++j) {
                        double v = j < NX ? fma(dgx[j], sgk, Pn[j] + qoh[j]) : rdg[j - NX];
                        if constexpr (EXACT) {
                            if (j < NX) v = fma(lxm, wr[j], v);   // + W_xx row r (round 6: the exact Hessian under bounds)
                        }
#pragma unroll
                        for (int a = 0; a < NU; ++a) v = fma(-Ytil[a], Yb[a][j], v);
                        Prow[j] = v;
                    }
                    double pv2 = pn;
#pragma unroll
                    for (int a = 0; a < NU; ++a) pv2 = fma(-Ytil[a], htil[a], pv2);
                    pvr = pv2;
                    return;
                }
                // K~ columns of the other lanes
                double Kb[NU][NX];
                sfor<0, NX>([&](auto I) {
#pragma unroll
                    for (int a = 0; a < NU; ++a) Kb[a][I] = row_bcast<I>(Kcol[a]);
                });
                // P~_k = blkdiag(A^T P_xx A + Q, R) - Y^T K~, p~_k = pn - Y^T kff (row r)
#pragma unroll
                for (int j = 0; j < NS; ++j) {
                    double v = j < NX ? Pn[j] + qoh[j] : rdg[j - NX];
                    if constexpr (EXACT) {
                        if (j < NX) v = fma(lxm, wr[j], v);   // W_xx row r (x-lanes; the mask folded into the add)
                    }
#pragma unroll
                    for (int a = 0; a < NU; ++a) v = fma(-Ycol[a], j < NX ? Kb[a][j] : Ku[a][j - NX], v);
                    Prow[j] = v;
                }
                double pv2 = pn;
#pragma unroll
                for (int a = 0; a < NU; ++a) pv2 = fma(-Ycol[a], kff[a], pv2);
                if constexpr (BOUNDED) pv2 += pexr;
                pvr = pv2;
            };
            // inner stages N-1 .. 1 by unconditional pairs (an odd count peels stage N-1 in front), as the step sweep;
            // the control-bounded sweep one stage per trip (its hold logic and relaxation rows fill the registers: two
            // stages in flight spilled to scratch inside the loop)
            using F_ = std::false_type;
            if constexpr ((BOUNDED && !MMPC_GROUP_BOUNDED_PAIRS) || (XB && (EXACT || !MMPC_GROUP_XB_PAIRS))) {
                for (int k = N - 1; k >= 1; --k) stage(k, F_{}, w0);
                stage(0, std::true_type{}, w0);
            } else if ((N - 1) & 1) {
                stage(N - 1, F_{}, w0);
                for (int k = N - 2; k >= 2; k -= 2) {
                    stage(k, F_{}, w0);
                    stage(k - 1, F_{}, w0);
                }
                stage(0, std::true_type{}, w0);
            } else {
                for (int k = N - 1; k >= 2; k -= 2) {
                    stage(k, F_{}, w0);
                    stage(k - 1, F_{}, w0);
                }
                stage(0, std::true_type{}, w0);
            }
        };
        if constexpr (DIST) {
            d_recursion_dist();
            adjoint_dist();
            lmax = group_max(lmax);
            gmax = group_max(gmax);
        } else if (gl == 0) {
            {
                double d[NX];
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    d[r] = 0.0;
                    sD[r] = 0.0;
                }
                // the operands of step k+1 are loaded during step k (the recursion is latency-bound)
                double aq[SQ], ad[FD], ac[NX];
#pragma unroll
                for (int i = 0; i < FQ; ++i) aq[i] = sFq[i];
#pragma unroll
                for (int i = 0; i < FD; ++i) ad[i] = sFqd[i];
#pragma unroll
                for (int r = 0; r < NX; ++r) ac[r] = sC[r];
                constexpr int kDUnroll = NX <= 4 ? 2 : 1;
#pragma unroll kDUnroll
                for (int k = 0; k < N; ++k) {
                    double fq[SQ], fd[FD], cc[NX], dn[NX];
#pragma unroll
                    for (int i = 0; i < FQ; ++i) fq[i] = aq[i];
#pragma unroll
                    for (int i = 0; i < FD; ++i) fd[i] = ad[i];
#pragma unroll
                    for (int r = 0; r < NX; ++r) cc[r] = ac[r];
                    const int kn = k + 1 < N ? k + 1 : k;
#pragma unroll
                    for (int i = 0; i < FQ; ++i) aq[i] = sFq[kn * FQ + i];
#pragma unroll
                    for (int i = 0; i < FD; ++i) ad[i] = sFqd[kn * FD + i];
#pragma unroll
                    for (int r = 0; r < NX; ++r) ac[r] = sC[kn * NX + r];
                    a_mul<NQ, NA, double>(h, fq, fd, d, dn);
#pragma unroll
                    for (int r = 0; r < NX; ++r) {
                        d[r] = dn[r] + cc[r];
                        sD[(k + 1) * NX + r] = d[r];
                    }
                }
            }
            backward(0);
        }
        if constexpr (!DIST) {
            gmax = group_bcast(gmax, gbase);
            lmax = group_bcast(lmax, gbase);
            fact_ok = group_bcast_i(fact_ok, gbase);
        }
        MMPC_PHASE(2);
        nonfinite = (group_max((double)nonfinite) != 0.0);
        kkt = fmax(gmax, cmax);
        if (XB) kkt = fmax(kkt, 2.0 * cmpl0);  // J-scale complementarity
        double* trc = p.trace && valid ? p.trace + (inst * (p.max_iter + 1) + it) * 8 : nullptr;
        if (trc && gl == 0) {
            trc[0] = gmax;
            trc[1] = cmax;
            trc[2] = J0;
            trc[3] = c1;
            trc[7] = lmax;
        }
        if (nonfinite || !isfinite(kkt)) {
            status = ST_NONFINITE;
            break;
        }
        if (gmax <= p.tol_grad && cmax <= p.tol_defect && (!XB || 2.0 * cmpl0 <= kIpTolCompl)) {
            status = ST_CONVERGED;
            break;
        }
        if (it == p.max_iter) {
            status = ST_MAX_ITER;
            break;
        }
        MMPC_PHASE(9);
        if constexpr (EXACT) {
            // stage-parallel: W_k = h sum_s lam_{k+1,NQ+s} d^2 acc_s/d(x_k,u_k)^2 (lam from the adjoint, in sD)
            __builtin_amdgcn_wave_barrier();
            for (int k = gl; k < N; k += G) {
                double x[NX], u[NU], la[NA], W[KZ * KZ];
#pragma unroll
                for (int r2 = 0; r2 < NX; ++r2) x[r2] = sX[k * NX + r2];
#pragma unroll
                for (int c = 0; c < NU; ++c) u[c] = sU[k * NU + c];
#pragma unroll
                for (int s2 = 0; s2 < NA; ++s2) la[s2] = h * sD[(k + 1) * NX + NQ + s2];
                Model::eval_hess(x, u, la, W);
                double* const dst = wH + k * HW;
#pragma unroll
                for (int r2 = 0; r2 < NX; ++r2)
#pragma unroll
                    for (int j = 0; j < KZ; ++j)
                        if (!(MMPC_GROUP_WZERO_ONCE && w_struct_zero<Model>(r2, j)) || !w_zeros_stored)
                            ws_store(&dst[r2 * KZ + j], W[r2 * KZ + j]);
                if constexpr (!CAFF) {
#pragma unroll
                    for (int a = 0; a < NU; ++a)
#pragma unroll
                        for (int b = 0; b < NU; ++b) ws_store(&dst[NX * KZ + a * NU + b], W[(NX + a) * KZ + NX + b]);
                }
            }
            w_zeros_stored = true;
            MMPC_PHASE(9);   // (timing build: "check" = the stop test and this W pass up to its fence)
            // the stores of the other lanes of this wave must be visible to the sweep's loads
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#ifdef MMPC_PHASE_FENCE_IN_LOAD
            MMPC_PHASE(0);   // (diagnostic: the fence's wait for the W stores, accumulated with the load phase)
#endif
        }
        // exact Hessian in this iteration's QP solves (false after a Gauss-Newton fallback)
        bool use_w = EXACT;
        if constexpr (DIST) {   // Riccati sweep (fact_ok is uniform over the group)
            backward_dist(use_w);
            // exact KKT matrix not positive definite on the null space: this iteration takes the Gauss-Newton step
            // (oracle solve_one: Cholesky of the exact condensed Hessian fails -> Gauss-Newton)
            if (EXACT && !fact_ok) {
                fact_ok = 1;
                use_w = false;
                backward_dist(false);
            }
        }
        if (!fact_ok) {
            status = ST_FACT_FAILED;
            break;
        }
        if (BOUNDED) pg_prev = gmax;
        // barrier update for the next iteration (IPOPT monotone rule, lagged; oracle solve_one_ip)
        const double mub_next = (XB && fmax(fmax(0.5 * gmax, cmax), cmplmu) <= kIpKappaEps * mub)
                                    ? fmax(kIpTolCompl / 20.0, fmin(kIpKappaMu * mub, pow(mub, kIpThetaMu)))
                                    : mub;

        MMPC_PHASE(3);
        if constexpr (DIST) {
            // step sweep: lane r holds s_k[r], s = [dx_k; du_{k-1}]; u-lanes du_k = K_k s_k + kff_k (row r - NX of
            // K from the workspace), x-lanes dx_{k+1} = A dx + B du + c.  A dx_k + B du_k goes to sD[k+1] (d is
            // dead after the backward sweep) for the directional derivative below.
            // check: a free control whose step crosses a bound is held there (sHold) and the QP solved again (BOUNDED)
            auto step_dist = [&](bool check) {
                // K_k columns were stored by the other lanes of this wave in the backward sweep
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                double sr = 0.0;
                if (lx) sDX[rx] = 0.0;
                constexpr int NK = NS + 1;
                const double* const Kp = wK + ru * NK;   // row ru of K_k | kff_k at Kp + k NU NK
                // operands double-buffered two stages ahead (manual unroll by two, so the buffers are renamed, not
                // copied): the K row from the HBM/L2 workspace, row r of [A - I | B] and c_k[r] from LDS
                struct Ops {
                    double K[NK], a[NX], b[NU], c, Rw[BOUNDED ? NR : 1];
                };
                const double* const Rp = wRel + ru * NR;   // BOUNDED: un-held row ru at Rp + k NU NR
                auto fetch = [&](int k, Ops& o) {
#pragma unroll
                    for (int j = 0; j < NK; ++j) o.K[j] = Kp[k * NU * NK + j];
                    load_arow(k, o.a, o.b);
                    o.c = sC[k * NX + rx];
                    if constexpr (BOUNDED) {
#pragma unroll
                        for (int j = 0; j < NR; ++j) o.Rw[j] = Rp[k * NU * NR + j];
                    }
                };
                auto stage = [&](int k, Ops& o) {
                    double sb[NS];
                    sfor<0, NS>([&](auto I) { sb[I] = row_bcast<I>(sr); });
                    double du0 = o.K[NS], du1 = 0.0;
#pragma unroll
                    for (int j = 0; j < NS; ++j) {
                        if (j & 1) du1 = fma(o.K[j], sb[j], du1);
                        else du0 = fma(o.K[j], sb[j], du0);
                    }
                    const double du = du0 + du1;
                    double ad = sr;
#pragma unroll
                    for (int j = 0; j < NX; ++j) ad = fma(o.a[j], sb[j], ad);
                    double dub[NU];
                    sfor<0, NU>([&](auto I) { dub[I] = row_bcast<NX + I>(du); });
#pragma unroll
                    for (int c = 0; c < NU; ++c) ad = fma(o.b[c], dub[c], ad);
                    const double dxn = ad + o.c;
                    if (lx) {
                        sDX[(k + 1) * NX + rx] = dxn;
                        sD[(k + 1) * NX + rx] = ad;
                    }
                    if (lu) sDU[k * NU + ru] = du;
                    if constexpr (BOUNDED) {
                        if (check && lu) {
                            const double hv = sHold[k * NU + ru], t = sU[k * NU + ru] + du;
                            if (hv != hv) {   // free: hold it where its step crosses a bound
                                if (t < lbr || t > ubr) {
                                    sHold[k * NU + ru] = t < lbr ? lbr : ubr;
                                    resolve = true;
                                }
                            } else if (!p.no_release) {   // held: release it when its multiplier H_ww du + [H_wx | -R] s + h_w points inward
                                double m = o.Rw[NR - 1];
#pragma unroll
                                for (int j = 0; j < NS; ++j) m = fma(o.Rw[j], sb[j], m);
#pragma unroll
                                for (int b = 0; b < NU; ++b) m = fma(o.Rw[NS + b], dub[b], m);
                                if ((hv == lbr && m < 0.0) || (hv == ubr && m > 0.0)) {
                                    sHold[k * NU + ru] = NAN;
                                    resolve = true;
                                }
                            }
                        }
                    }
                    sr = lx ? dxn : (lu ? du : 0.0);
                    fetch(k + 3 < N ? k + 3 : N - 1, o);   // unconditional: static wait counts
                };
                // three buffers, refilled three stages ahead: the K rows come from L2/MALL (the workspace of a
                // 512-instance XCD exceeds its 4 MB L2) and one stage of the sweep (~300 cycles) did not cover that
                // latency -- with two buffers every stage waited for the loads issued one stage earlier
                Ops o0, o1, o2;
                fetch(0, o0);
                fetch(N > 1 ? 1 : 0, o1);
                fetch(N > 2 ? 2 : 0, o2);
                // all three stages of the unrolled body unconditional (N mod 3 stages peeled in front, the buffers
                // rotate roles): the loop top then has the same outstanding loads on every path, so the wait before
                // stage k's operands is vmcnt(#loads of stages k+1, k+2), not vmcnt(0)
                if (N % 3 == 1) {
                    stage(0, o0);
                    for (int k = 1; k < N; k += 3) {
                        stage(k, o1);
                        stage(k + 1, o2);
                        stage(k + 2, o0);
                    }
                } else if (N % 3 == 2) {
                    stage(0, o0);
                    stage(1, o1);
                    for (int k = 2; k < N; k += 3) {
                        stage(k, o2);
                        stage(k + 1, o0);
                        stage(k + 2, o1);
                    }
                } else {
                    for (int k = 0; k < N; k += 3) {
                        stage(k, o0);
                        stage(k + 1, o1);
                        stage(k + 2, o2);
                    }
                }
            };
            for (int pass = 0;; ++pass) {
                if (pass > 0) {   // BOUNDED: controls held after the previous step -- solve the QP again
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    backward_dist(use_w);
                    if (EXACT && use_w && !fact_ok) {   // the held exact QP not positive definite: Gauss-Newton
                        fact_ok = 1;
                        use_w = false;
                        backward_dist(false);
                    }
                    if (!fact_ok) break;
                }
                resolve = false;
                // QP solves of this iteration: two at the first (the cold start's active set moves most there, and a
                // wave pays its slowest instance's solves), kBoundPasses later (oracle bound_release)
                const int passes = (it == 0 && !p.no_release) ? 2 : kBoundPasses;
                step_dist(BOUNDED && pass + 1 < passes);
                if constexpr (!BOUNDED) {
                    break;
                } else {
                    resolve = group_max(resolve ? 1.0 : 0.0) != 0.0;
                    if (!resolve || pass + 1 >= passes) break;
                }
            }
            __builtin_amdgcn_wave_barrier();
            // directional derivative of J along (dx, du), stage-parallel:
            // sum_k 2Q(F_k - r_k).(A dx_k + B du_k) + 2R(u_k - u_{k-1})(du_k - du_{k-1}) + 2Rm u_k du_k
            double dj = 0.0;
            for (int k = gl; k < N; k += G) {
#pragma unroll
                for (int q = 0; q < NX; ++q) dj = fma(2.0 * Q[q] * (sF[k * NX + q] - tr[k * NX + q]), sD[(k + 1) * NX + q], dj);
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    const double uk = sU[k * NU + c], duk = sDU[k * NU + c];
                    const double um = (k == 0) ? up[c] : sU[(k - 1) * NU + c];
                    const double dum = (k == 0) ? 0.0 : sDU[(k - 1) * NU + c];
                    dj = fma(2.0 * R[c] * (uk - um), duk - dum, fma(2.0 * Rm[c] * uk, duk, dj));
                }
            }
            dJ = group_sum(dj);
        } else {
            if (gl == 0) {
                for (int pass = 0;; ++pass) {
                    if (pass > 0) backward(pass);
                    if (!fact_ok) break;
                    resolve = false;
                    step_sweep(pass);
                    if (!BOUNDED || !resolve || pass + 1 >= kBoundPasses) break;
                }
            }
            fact_ok = group_bcast_i(fact_ok, gbase);
            dJ = group_bcast(dJ, gbase);
        }
        if (!fact_ok) {
            status = ST_FACT_FAILED;
            break;
        }
        __builtin_amdgcn_wave_barrier();
        MMPC_PHASE(4);
        // interior point: fraction to the boundary (primal alpha_max, dual alpha_z), barrier directional derivative
        double amax = 1.0, az = 1.0, dbar = 0.0;
        if constexpr (XB) {
            const double tau = kIpTau;
            for (int k = gl; k < N; k += G) {
#pragma unroll
                for (int j = 0; j < NY; ++j) {
                    const double y = j < NX ? sX[(k + 1) * NX + j] : sU[k * NU + j - NX];
                    const double dy = j < NX ? sDX[(k + 1) * NX + j] : sDU[k * NU + j - NX];
                    ip_step_limits(y, dy, yl[j], yu[j], sZl[k * NY + j], sZu[k * NY + j], mub, tau, sBb[k * NY + j],
                                   amax, az, dbar);
                }
            }
            amax = group_min(amax);
            az = group_min(az);
            dbar = group_sum(dbar);
        }

        // ---- D. stage-parallel l1-merit Armijo line search (noise-aware, as sqp_wave.h), update ----
        mu = fmax(mu, 4.0 * lmax + 1.0);
        const double phi0 = XB ? fma(mu, c1, fma(-2.0 * mub, lsum, J0)) : fma(mu, c1, J0);
        const double dphi = XB ? dJ + dbar - mu * c1 : dJ - mu * c1;
        double alpha = amax;
        bool accepted = false;
        // the alpha = 1 trial with the Jacobian (FUSE_FWD): ctm, nft are phase A's max|c| and nonfinite flag there
        double ctm = 0.0;
        int nft = 0;
        auto trial = [&](auto jac_c, double& Jt, double& ct, double& lt) {
            constexpr bool JAC = decltype(jac_c)::value;
            for (int k = gl; k < N; k += G) {
                double x[NX], u[NU], xd[NX];
#pragma unroll
                for (int r = 0; r < NX; ++r) x[r] = fma(alpha, sDX[k * NX + r], sX[k * NX + r]);
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    u[c] = fma(alpha, sDU[k * NU + c], sU[k * NU + c]);
                    if (BOUNDED) u[c] = proj(u[c], lbv[c], ubv[c]);  // projected trial point
                }
                if constexpr (JAC) {   // = phase A at the trial point (stored for the next iteration)
                    double Fq[SQ], Fqd[FD], Fu[FU];
                    group_model<Model>(lin, lFq, lFqd, lFu, lxd, lxs, up, x, u, xd, Fq, Fqd, Fu, true);
#pragma unroll
                    for (int i = 0; i < FQ; ++i) sFq[k * FQ + i] = h * Fq[i];
#pragma unroll
                    for (int i = 0; i < FD; ++i) sFqd[k * FD + i] = h * Fqd[i];
#pragma unroll
                    for (int i = 0; i < FU; ++i) sFu[k * FU + i] = h * Fu[i];
#pragma unroll
                    for (int r = 0; r < NX; ++r) {
                        const double F = fma(h, xd[r], x[r]);
                        sF[k * NX + r] = F;
                        const double c = F - fma(alpha, sDX[(k + 1) * NX + r], sX[(k + 1) * NX + r]);
                        sC[k * NX + r] = c;
                        ctm = fmax(ctm, fabs(c));
                        ct += fabs(c);
                        nft |= !isfinite(c);
                        const double er = F - tr[k * NX + r];
                        Jt = fma(er * Q[r], er, Jt);
                    }
                } else {
                    group_model<Model>(lin, lFq, lFqd, lFu, lxd, lxs, up, x, u, xd, nullptr, nullptr, nullptr, false);
#pragma unroll
                    for (int r = 0; r < NX; ++r) {
                        const double F = fma(h, xd[r], x[r]);
                        const double er = F - tr[k * NX + r];
                        Jt = fma(er * Q[r], er, Jt);
                        ct += fabs(F - fma(alpha, sDX[(k + 1) * NX + r], sX[(k + 1) * NX + r]));
                    }
                }
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    double um = (k == 0) ? up[c] : fma(alpha, sDU[(k - 1) * NU + c], sU[(k - 1) * NU + c]);
                    if (BOUNDED && k > 0) um = proj(um, lbv[c], ubv[c]);
                    const double dif = u[c] - um;
                    Jt = fma(dif * R[c], dif, fma(u[c] * Rm[c], u[c], Jt));
                }
                if constexpr (XB) {
#pragma unroll
                    for (int j = 0; j < NY; ++j) {
                        const double y = j < NX ? fma(alpha, sDX[(k + 1) * NX + j], sX[(k + 1) * NX + j]) : u[j - NX];
                        lt += ip_log_slacks(y, yl[j], yu[j]);
                    }
                }
            }
        };
        bool jac_trial = false;
        for (int ls = 0; ls < 30; ++ls) {
            double Jt = 0.0, ct = 0.0, lt = 0.0;
            jac_trial = FUSE_FWD && ls == 0;   // alpha = amax (1 without state bounds)
            if (jac_trial) trial(std::true_type{}, Jt, ct, lt);
            else trial(std::false_type{}, Jt, ct, lt);
            Jt = group_sum(Jt);
            ct = group_sum(ct);
            if (XB) lt = group_sum(lt);
            const double phit = XB ? fma(mu, ct, fma(-2.0 * mub, lt, Jt)) : fma(mu, ct, Jt);
            const double noise = 1.0 + fabs(phi0);
            if (dphi >= -1e-11 * noise || phit <= phi0 + 1e-4 * alpha * dphi + 1e-13 * noise ||
                (!XB && it == 0 && first_iter_filter_accepts(J0, c1, Jt, ct, dJ, alpha))) {
                accepted = true;
                if (FUSE_FWD && jac_trial) {   // the next iteration starts after phase A
                    fwd_ready = true;
                    J0n = Jt;
                    c1n = ct;
                    cmaxn = group_max(ctm);
                    nfn = nft;
                }
                break;
            }
            alpha *= 0.5;
        }
        if (trc && gl == 0) {
            trc[4] = XB ? amax : dJ;
            trc[5] = alpha;
            trc[6] = XB ? mub : mu;
            if (XB) trc[3] = cmpl0;
        }
        MMPC_PHASE(5);
        if (!accepted) {
            status = ST_LS_FAILED;
            break;
        }
        __builtin_amdgcn_wave_barrier();
        if constexpr (XB) {  // y and the duals of stage k's (x_{k+1} | u_k), as oracle solve_one_ip
            for (int k = gl; k < N; k += G) {
#pragma unroll
                for (int j = 0; j < NY; ++j) {
                    double& y = j < NX ? sX[(k + 1) * NX + j] : sU[k * NU + j - NX];
                    const double dy = j < NX ? sDX[(k + 1) * NX + j] : sDU[k * NU + j - NX];
                    double zl = sZl[k * NY + j], zu = sZu[k * NY + j], yn;
                    ip_update(y, dy, yl[j], yu[j], zl, zu, mub, alpha, az, yn);
                    y = yn;
                    sZl[k * NY + j] = zl;
                    sZu[k * NY + j] = zu;
                }
            }
            mub = mub_next;
        } else {
            for (int k = gl; k <= N; k += G) {
                if (k > 0) {
#pragma unroll
                    for (int r = 0; r < NX; ++r) sX[k * NX + r] = fma(alpha, sDX[k * NX + r], sX[k * NX + r]);
                }
                if (k < N) {
#pragma unroll
                    for (int c = 0; c < NU; ++c) {
                        const double un = fma(alpha, sDU[k * NU + c], sU[k * NU + c]);
                        sU[k * NU + c] = BOUNDED ? proj(un, lbv[c], ubv[c]) : un;
                    }
                }
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    MMPC_PHASE(6);
    if (!valid) return;
    // ---- write back V (reference layout), stage-parallel ----
    double* Vout = p.V + inst * (int64_t)NV;
#if MMPC_GROUP_WB_COALESCED
    // V element e on lane e mod 16: each store instruction writes 16 consecutive doubles of the instance's row
    for (int e = gl; e < NV; e += G) {
        const int k = e / ND, r = e - k * ND;
        Vout[e] = r < NX ? sX[k * NX + r] : sU[k * NU + r - NX];
    }
    if (false)
#endif
    for (int k = gl; k <= N; k += G) {
#pragma unroll
        for (int r = 0; r < NX; ++r) Vout[k * ND + r] = sX[k * NX + r];
        if (k < N) {
#pragma unroll
            for (int c = 0; c < NU; ++c) Vout[k * ND + NX + c] = sU[k * NU + c];
        }
    }
    if (p.u0_out && gl < NU) p.u0_out[inst * NU + gl] = sU[gl];
    if (gl == 0) {
        if (p.status) p.status[inst] = status;
        if (p.iters) p.iters[inst] = it;
        if (p.kkt) p.kkt[inst] = kkt;
    }
    MMPC_PHASE(7);
    MMPC_PHASE_FLUSH
#ifdef MMPC_GROUP_SLEEP_EXIT
    // diagnostic A/B (lib_var builds only): a finished wave sleeps MMPC_GROUP_SLEEP_EXIT % of its own duration before
    // it exits (s_memrealtime, no memory traffic), so the chip stays occupied while the waves of the last iteration run
    {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const unsigned long long until = t1 + (t1 - sl_t0) * MMPC_GROUP_SLEEP_EXIT / 100;
#ifdef MMPC_GROUP_SPIN_EXIT   // ... busy with FP64 FMAs instead of sleeping (the power draw of a running wave)
        double sp = (double)threadIdx.x;
        while (__builtin_amdgcn_s_memrealtime() < until) {
            for (int i = 0; i < 64; ++i) sp = fma(sp, 0.999, 1e-3);
            asm volatile("" : "+v"(sp));
        }
#else
        while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(32);
#endif
    }
#endif
#if MMPC_GROUP_EXIT_HOLD
    // resident finish: a wave that finishes while other waves of the launch still run stays resident,
    // sleeping, until at most 1/32 of the launch's waves are still running (or, a bound, half its own duration has
    // passed).  Waves that ran on a chip whose other waves had left ran their last iteration up to ~1.5x slower
    // (cfg#2 at tol 1e-5, profiles/r06/sleep).  One atomic per wave; the wave that finishes last resets the counter
    // for the next launch; polls every ~2 us (s_sleep, no traffic in between).
    if (!resume && p.exit_count) {
        int done_before = 0;
        if (threadIdx.x == 0) done_before = atomicAdd(p.exit_count, 1);
        done_before = __builtin_amdgcn_readfirstlane(done_before);   // lane 0 (group 0 of a wave is always valid)
        const int waves = (int)gridDim.x;
        if (done_before + 1 >= waves) {
            if (threadIdx.x == 0) __hip_atomic_store(p.exit_count, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            const unsigned long long until = t1 + (t1 - fin_t0) / 2;
            const int leave = waves - max(1, waves / 32);   // finished count at which the waiting waves leave
            while (__builtin_amdgcn_s_memrealtime() < until) {
                __builtin_amdgcn_s_sleep(64);
                const int n = __hip_atomic_load(p.exit_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (n == 0 || n >= leave) break;   // 0: the last wave has reset it
            }
        }
    }
#endif
}

}  // namespace mmpc
