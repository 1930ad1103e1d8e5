// sqp_lane.h -- batched GN-SQP with a Riccati KKT solve, ONE INSTANCE PER LANE.
//
// The wave kernel (sqp_wave.h) condenses the QP into an (N nu)x(N nu) Hessian held one row per lane,
// which caps N nu at 64.  The exo configurations (SURVEY.md 8d cfg#3-#5: nx=8, nu=4, N=50, B=65536)
// have N nu = 200: a condensed Hessian would be 320 KB per instance (2x the LDS of a CU) and
// 9.3 MFLOP per iteration.  The same QP is solved exactly by a Riccati recursion on the augmented
// state s_k = [dx_k; du_{k-1}] (the du_{k-1} block carries the Delta-u weight R of
// ModelGenerator.cpp:216-221) in ~0.25 MFLOP per iteration, and at B = 65536 one instance per lane
// already fills every SIMD of the MI355X (1024 waves), so lanes never exchange data.
//
// Per SQP iteration, per lane (all fp64; the NLP, merit, line search and stopping test are those of
// sqp_wave.h and oracle/mmpc_oracle.c):
//   (1) forward  : F_k, A_k = I + h f_x, B_k = h f_u, defects c_k, d_{k+1} = A_k d_k + c_k, merit J, |c|_1
//   (2) backward : adjoint lam_k and reduced gradient g_k (stopping test), Riccati
//                  H_ww = B^T G + P_ux B + P_uu + R + Rm,  G = P_xx B + P_xu,  H_wx = G^T A,
//                  H_xx = A^T P_xx A,  K_k = -H_ww^-1 [H_wx | -R],  P_k = blkdiag(H_xx, R) - ...
//   (3) forward  : du_k = K_k s_k + kff_k, dx_{k+1} = A_k dx_k + B_k du_k + c_k, directional derivative
//   (4) l1-merit Armijo line search (value-only model evaluations)
// A_k, B_k are recomputed in (2) and (3) instead of stored: one Jacobian evaluation costs ~1k FMA
// while storing them would add 2x768 B of HBM traffic per stage and lane (DESIGN.md "Riccati path").
// Per-lane state lives in a structure-of-arrays workspace in HBM ([wave block][element][lane]), so every
// wave access is one contiguous 512-byte line.
#pragma once
#include <limits>
#include "models.h"
#include "sqp_wave.h"

// A/B switches of the fp32-factor instantiations (diagnostic builds only; defaults are the shipped choice)
#ifndef MMPC_LANE_YLO32
#define MMPC_LANE_YLO32 1
#endif
#ifndef MMPC_LANE_JACH32
#define MMPC_LANE_JACH32 1
#endif
#ifndef MMPC_LANE_LB32
#define MMPC_LANE_LB32 1
#endif
#ifndef MMPC_LANE_XB_BATCHED
#define MMPC_LANE_XB_BATCHED 1
#endif
#ifndef MMPC_LANE_FWD32
#define MMPC_LANE_FWD32 1
#endif
#ifndef MMPC_LANE_WPE32
#define MMPC_LANE_WPE32 1
#endif
#ifndef MMPC_LANE_C_RECOMPUTE   // step sweep: c_k from its own model evaluation instead of the stored C (round 6)
#define MMPC_LANE_C_RECOMPUTE 1
#endif
#ifndef MMPC_LANE_C_NOSTORE   // no C record: the backward sweep recomputes c_k too (requires MMPC_LANE_C_RECOMPUTE)
#define MMPC_LANE_C_NOSTORE 1
#endif
#ifndef MMPC_LANE_LAZY_DXU   // unbounded solves: DX / DU stored in the first iteration only (regenerated on demand)
#define MMPC_LANE_LAZY_DXU 1
#endif
#ifndef MMPC_LANE_KPACK   // gain record with H_ww^-1 instead of K_u (kgain_idx; not for control-bounded solves)
#define MMPC_LANE_KPACK 1
#endif
#ifndef MMPC_LANE_LS_HANDOVER   // a rejected full step after the first iteration is handed to the resume launch
#define MMPC_LANE_LS_HANDOVER 1
#endif
#ifndef MMPC_LANE_XTRA_K
#define MMPC_LANE_XTRA_K 0
#endif
#ifndef MMPC_LANE_XB_EARLY
#define MMPC_LANE_XB_EARLY 1
#endif
#ifndef MMPC_LANE_XB_EARLY_STEP
#define MMPC_LANE_XB_EARLY_STEP MMPC_LANE_XB_EARLY
#endif

namespace mmpc {

// Workspace layout, stage-major: [64-instance block][stage k = 0..N+1][field][lane].  All fields of
// stage k sit at compile-time offsets from one wave-uniform base, so an access is base(k) + const in
// scalar registers plus the lane offset in one VGPR (an [element][lane] layout hoists one 64-bit
// per-lane pointer per (field, element) and spills).  Stage N holds x_N, d_N, dx_N; stages N+1.. hold
// the linear-mode data (one stage for the built-in models); the stage(s) after it are per-lane scratch for
// the Riccati step (W = P_xx A).  A field block longer than a stage simply runs on into the next stage.
// xb: the interior-point variant's per-stage z_l, z_u, Sigma, b, z_u - z_l of (x_{k+1} | u_k) replace the hold field
__host__ __device__ constexpr int lane_stage_stride(int nx, int nu, bool xb = false) {
    return 5 * nx + 2 * nu + nu * (nx + nu + 1) + (xb ? 5 * (nx + nu) : 2 * nu + nx);
}
// field offset of the interior-point duals z_l (z_u follows at + nx + nu) in a stage (StageFields<.., true>::ZL)
__host__ __device__ constexpr int lane_zl_offset(int nx, int nu) { return 5 * nx + 2 * nu + nu * (nx + nu + 1); }
// linear-mode block: h-free Jacobian blocks da/dq (na x nq), da/dz (na x na), da/du (na x nu), xdot*, x*, u*
__host__ __device__ constexpr int lane_lin_doubles(int nx, int nu, int nq) {
    return (nx - nq) * (nq + (nx - nq) + nu) + 2 * nx + nu;
}
__host__ __device__ constexpr int lane_lin_stages(int nx, int nu, int nq, bool xb = false) {
    return (lane_lin_doubles(nx, nu, nq) + lane_stage_stride(nx, nu, xb) - 1) / lane_stage_stride(nx, nu, xb);
}
__host__ __device__ constexpr bool lane_w_in_lds(int nx, int nu, int nq);
__host__ __device__ constexpr int lane_scratch_stages(int nx, int nu, int nq, bool xb = false) {
    return lane_w_in_lds(nx, nu, nq) ? 0 : (nx * nx + lane_stage_stride(nx, nu, xb) - 1) / lane_stage_stride(nx, nu, xb);
}
__host__ __device__ constexpr int lane_ws_doubles(int nx, int nu, int nq, int N, bool xb = false) {
    return (N + 1 + lane_lin_stages(nx, nu, nq, xb) + lane_scratch_stages(nx, nu, nq, xb)) *
           lane_stage_stride(nx, nu, xb);
}
template <int NX, int NU, bool XB = false>
struct StageFields {
    static constexpr int NS = NX + NU;
    static constexpr int X = 0;             // x_k
    static constexpr int U = X + NX;        // u_k
    static constexpr int R = U + NU;        // r_k (target of F(x_k, u_k))
    static constexpr int C = R + NX;        // defect c_k = F_k - x_{k+1}
    static constexpr int D = C + NX;        // d_k (defect propagation)
    static constexpr int DX = D + NX;       // dx_k
    static constexpr int DU = DX + NX;      // du_k
    static constexpr int K = DU + NU;       // kff_k (nu, fp64) then K_k (nu x (nx+nu), factor type)
    static constexpr int HOLD = K + NU * (NS + 1);  // bounded solves: bound u_k is held at, NaN = free
    // unbounded solves: the second iterate buffer (x_k, u_k) -- the step sweep writes the full-step point there and an
    // accepted full step swaps the buffers instead of running the update pass (sqp_lane_kernel SWAP)
    static constexpr int X1 = HOLD + NU, U1 = X1 + NX;
    // interior point (XB, no hold field): y = (x_{k+1} | u_k) duals, Sigma, b, z_u - z_l
    static constexpr int NY = NX + NU;
    static constexpr int ZL = HOLD, ZU = ZL + NY, SG = ZU + NY, BB = SG + NY, ZG = BB + NY;
    static constexpr int SS = XB ? ZG + NY : U1 + NU;
    static_assert(SS == lane_stage_stride(NX, NU, XB), "layout");
    static_assert(ZL == lane_zl_offset(NX, NU), "layout of the duals (state-bounded tail hand-over)");
};

struct LaneWork {
    double* ws;  // ceil(B/64) blocks of lane_ws_doubles(nx, nu, N) x 64 doubles
};

// packed upper-triangle index of (i, j), i <= j, of an n x n symmetric matrix
__host__ __device__ constexpr int sym_idx(int n, int i, int j) {
    return i <= j ? i * n - i * (i - 1) / 2 + (j - i) : j * n - j * (j - 1) / 2 + (i - j);
}

// Gain record [K_k] after kff_k (round 6, KPACK): K_x row-major [NU][NX], then H_ww^-1 packed (sym_idx): K_u =
// -H_ww^-1 (-R) = H_ww^-1 diag(R), so the step sweep forms K_u du_{k-1} as H_ww^-1 (R o du_{k-1}) from 10 stored
// values instead of 16 (exo).  Not for control-bounded solves (held rows change K_u).  Otherwise [NU][NX + NU].
template <int NX, int NU, bool KPACK>
__host__ __device__ constexpr int kgain_idx(int a, int j) {
    return !KPACK    ? a * (NX + NU) + j
           : j < NX ? a * NX + j
                    : NU * NX + sym_idx(NU, a < j - NX ? a : j - NX, a < j - NX ? j - NX : a);
}
template <int NX, int NU, bool KPACK>
__host__ __device__ constexpr int kgain_count() { return KPACK ? NU * NX + NU * (NU + 1) / 2 : NU * (NX + NU); }

// The P~_xu / P~_uu entries of the packed P~ are dead once G, H_ww, h_w and Y of a Riccati step are formed: their
// slots hold the rows NQ..NX-1 of W = P_xx A (NA x NX) while P~_xx is rebuilt in place (sqp_lane_kernel, "W in
// LDS").  i-th such slot in packed order; lane_w_in_lds: whether W's a-rows fit.
__host__ __device__ constexpr int lane_dead_slot(int nx, int nu, int i) {
    const int ns = nx + nu;
    for (int a = 0; a < ns; ++a)
        for (int b = (a > nx ? a : nx); b < ns; ++b) {
            if (i == 0) return sym_idx(ns, a, b);
            --i;
        }
    return -1;
}
__host__ __device__ constexpr bool lane_w_in_lds(int nx, int nu, int nq) {
    return (nx - nq) * nx <= nx * nu + nu * (nu + 1) / 2;
}

// Products with the discrete stage matrices of a model with NQ kinematic rows (x = [q; z], qdot_i = z_i for
// i < NQ, zdot = a(x, u) with NA = NX - NQ >= NQ rows; second-order models have NA = NQ, a general first-order
// model NQ = 0):
//   A = I + h f_x = [[I, h [I 0]], [hFq, I + hFqd]],   B = h f_u = [[0], [hFu]]
// where hFq = h da/dq (NA x NQ), hFqd = h da/dz (NA x NA), hFu = h da/du (NA x NU), all row-major.  For
// NA = NQ the FMA order is that of the second-order-only version (same instructions, same rounding).
template <int NQ, int NA, class T>
MMPC_HD void a_mul(T h, const T* hFq, const T* hFqd, const T* v, T* out) {
    constexpr int NM = NQ > NA ? NQ : NA;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        T t = v[NQ + i];
#pragma unroll
        for (int s = 0; s < NM; ++s) {
            if (s < NA) t = fma(hFqd[i * NA + s], v[NQ + s], t);
            if (s < NQ) t = fma(hFq[i * NQ + s], v[s], t);
        }
        out[NQ + i] = t;
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i) out[i] = fma(h, v[NQ + i], v[i]);
}
template <int NQ, int NA, class T>
MMPC_HD void at_mul(T h, const T* hFq, const T* hFqd, const T* v, T* out) {
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        T tq = a < NQ ? v[a] : T(0), td = a < NQ ? fma(h, v[a], v[NQ + a]) : v[NQ + a];
#pragma unroll
        for (int s = 0; s < NA; ++s) {
            if (a < NQ) tq = fma(hFq[s * NQ + a], v[NQ + s], tq);
            td = fma(hFqd[s * NA + a], v[NQ + s], td);
        }
        if (a < NQ) out[a] = tq;
        out[NQ + a] = td;
    }
}

// A v (+ B w) from the directional derivative jv = da/d(x, u) . (v, w): [v_q + h v_z[0:NQ]; v_z + h jv]
template <int NQ, int NA>
MMPC_HD void jvp_step(double h, const double* v, const double* jv, double* out) {
#pragma unroll
    for (int i = 0; i < NQ; ++i) out[i] = fma(h, v[NQ + i], v[i]);
#pragma unroll
    for (int i = 0; i < NA; ++i) out[NQ + i] = fma(h, jv[i], v[NQ + i]);
}

// Per-lane pointer to stage k of the workspace, opaque to the optimiser: every access of a stage loop is
// derived from it (offset folded into the instruction or one add), so nothing is hoisted out of the loop.
// Without it LICM materialises one 64-bit offset per (field, element) before the loop and spills them.
// The pointer is typed global (address space 1): an opaque generic pointer compiles to flat_load/flat_store,
// whose every use waits for vmcnt(0) AND lgkmcnt(0) (flat operations complete out of order), i.e. drains the
// next stage's prefetches and all LDS traffic at each workspace access.
template <class T>
using gmem = __attribute__((address_space(1))) T;
__device__ __forceinline__ gmem<double>* stage_ptr(double* wsb, int64_t k, int SS, int lane) {
    gmem<double>* q = (gmem<double>*)(wsb + k * SS * 64 + lane);
    asm volatile("" : "+v"(q));
    return q;
}

// FT: arithmetic type of the Riccati factor/solve (double, or float for SURVEY.md 8d cfg#5: the backward
// recursion, P in LDS, the gains K and the W scratch in fp32; model evaluations, defects, adjoint, gradient,
// merit and iterates stay fp64, so every SQP iteration refines the fp32 step against fp64 residuals).
// XB: state bounds, the primal-dual interior-point variant (oracle solve_one_ip; see sqp_group.h)
// EXACT: the exact Lagrangian Hessian (IPOPT's default, CasADi nlp_hess_l at ModelGenerator.cpp:238; oracle
// solve_one_riccati / solve_one with ORACLE_HESS_EXACT): the backward step of stage k adds W_k = h sum_s
// lam_{k+1,NQ+s} d^2 acc_s / d(x_k,u_k)^2 (Model::eval_hess at the iterate, lam the adjoint of this sweep) to H_ww,
// H_wx and the x block of P~_k; a sweep whose H_ww is not positive definite is redone without W (the Gauss-Newton
// step).  With control bounds (BOUNDED, round 5) the held controls are fixed in the exact stage QPs exactly as in
// the Gauss-Newton ones (the hold rule acts on H_ww, H_wx, h_w after W is added).  With state bounds (XB, round 6:
// IPOPT's exact Hessian under the barrier) W_k joins the barrier-augmented stage blocks (Sigma, b) -- the adjoint
// that weights it carries the bound duals -- and a sweep whose H_ww is not positive definite is redone without W.
template <class Model, class FT = double, bool BOUNDED = false, bool XB = false, bool EXACT = false>
// one wave per SIMD by design (P~ in LDS, ~40 KB per wave): telling the scheduler so lets it schedule for latency
// rather than for a second wave's registers (cfg#3: 12.06 -> 11.94 ms).  The fp32-factor variant's P~ takes 20 KB, so
// 8 waves fit a CU's LDS: MMPC_LANE_WPE32 = 2 (A/B builds) asks for 2 waves per SIMD there (256 registers)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(std::is_same<FT, float>::value ? MMPC_LANE_WPE32 : 1,
                                                                    std::is_same<FT, float>::value ? MMPC_LANE_WPE32
                                                                                                   : 1))) void
sqp_lane_kernel(SolveParams p,
                                                                                                 LaneWork lw) {
    static_assert(!(BOUNDED && XB), "the interior-point variant handles the control bounds itself");
    static_assert(!EXACT || (HasHess<Model>::value && std::is_same<FT, double>::value),
                  "exact Hessian: fp64 solves of models with second derivatives");
    constexpr int NX = Model::NX, NU = Model::NU, NQ = Model::NQ, NA = NX - NQ, NS = NX + NU, ND = NX + NU;
    constexpr int SQ = NA * NQ > 0 ? NA * NQ : 1;  // extent of the h da/dq block (empty for NQ = 0)
    static_assert(NQ >= 0 && NA >= NQ, "x = [q; z] with qdot = z[0:NQ]");
    const int64_t inst = blockIdx.x * (int64_t)64 + threadIdx.x;
    [[maybe_unused]] const int lane0 = threadIdx.x;  // used by the phase-timing build
    MMPC_PHASE_DECL
    // Riccati matrix P~ (packed upper, NS(NS+1)/2 doubles per lane) lives in LDS, lane-interleaved
    // (conflict-free): holding it in registers next to the stage blocks and the factor spills to scratch.
    __shared__ FT sP[NS * (NS + 1) / 2][64];
    if (inst >= p.B) return;  // lanes never exchange data
    FT* __restrict__ Pl = &sP[0][threadIdx.x];
#define PS(i, j) Pl[sym_idx(NS, (i), (j)) * 64]
    const int N = p.N;
    const int NV = NX * (N + 1) + NU * N;
    const double h = p.h;
    using SF = StageFields<NX, NU, XB>;
    constexpr int NY = NX + NU;
    constexpr int SS = SF::SS;
    const int lane = threadIdx.x;
    double* const wsb = lw.ws + (int64_t)blockIdx.x * ((int64_t)lane_ws_doubles(NX, NU, NQ, N, XB) * 64);  // wave-uniform
    const int kScratch = N + 1 + lane_lin_stages(NX, NU, NQ, XB);  // first stage of the W = P_xx A scratch
    constexpr bool WLDS = lane_w_in_lds(NX, NU, NQ);  // W's a-rows in the dead P~ slots, no HBM scratch
#define ST(k, f, e) wsb[((int64_t)(k) * SS + (f) + (e)) * 64 + lane]  // one-off accesses
#define SK(dk, f, e) sk[((dk) * SS + (f) + (e)) * 64]                   // stage k + dk inside a stage loop
    // SWAP (unbounded): the iterate (x_k, u_k) lives in one of two field pairs; FX/FU name the current one, FXo/FUo
    // the other, which the step sweep fills with the full-step point (x_k + dx_k, u_k + du_k) -- an accepted full step
    // (99.7 % of the cfg#3 iterations) swaps the names instead of running the update pass over the workspace
    constexpr bool SWAP = !BOUNDED && !XB;
    constexpr bool KPACK = !BOUNDED && MMPC_LANE_KPACK;   // gain record layout (kgain_idx)
    // lazy step records (DX / DU, below): unbounded solves; not with the exact Hessian, whose kernel ran 11.19 -> 11.74 ms
    // with them (cfg#3 exact, the regeneration's registers: profiles/r06/kpack/abx)
    constexpr bool LAZY = SWAP && !EXACT && MMPC_LANE_LAZY_DXU;
    constexpr int KN = kgain_count<NX, NU, KPACK>();
    int FX = SF::X, FU = SF::U, FXo = SWAP ? SF::X1 : SF::X, FUo = SWAP ? SF::U1 : SF::U;

    const double* w = p.weights + inst * p.w_stride;
    double Q[NX], R[NU], Rm[NU], up[NU];
#pragma unroll
    for (int r = 0; r < NX; ++r) Q[r] = w[r];
#pragma unroll
    for (int c = 0; c < NU; ++c) {
        R[c] = w[NX + c];
        Rm[c] = w[NX + NU + c];
        up[c] = p.u_prev[inst * NU + c];
    }
    double lbv[NU], ubv[NU];
    load_bounds<NU, BOUNDED>(p, lbv, ubv);
    // ---- load: V (reference layout) -> SoA X/U, x_0 pinned (ModelControl.cpp:144-145), targets ----
    // Every copy below loads LB stages into registers before storing them: the workspace stores may alias the input
    // pointers, so a load-store-load order would wait out one memory round trip per element (the load and
    // write-back phases took 9.5 % of the cfg#3 kernel that way).
    constexpr int LB = (std::is_same<FT, double>::value || MMPC_LANE_LB32) ? 5 : 1;
    {
        const double* Vin = p.V + inst * (int64_t)NV;
        double x0v[NX];
#pragma unroll
        for (int r = 0; r < NX; ++r) x0v[r] = p.x0[inst * NX + r];
        for (int k0 = 0; k0 < N; k0 += LB) {
            double v[LB][ND];
#pragma unroll
            for (int j = 0; j < LB; ++j) {   // one uniform branch per stage, not per element
                if (!p.init_zero && k0 + j < N) {
#pragma unroll
                    for (int e = 0; e < ND; ++e) v[j][e] = Vin[(k0 + j) * ND + e];
                } else {
#pragma unroll
                    for (int e = 0; e < ND; ++e) v[j][e] = 0.0;
                }
            }
#pragma unroll
            for (int j = 0; j < LB; ++j) {
                const int k = k0 + j;
                if (k < N) {
#pragma unroll
                    for (int r = 0; r < NX; ++r) ST(k, FX, r) = (k == 0 || p.init_hold) ? x0v[r] : v[j][r];
#pragma unroll
                    for (int c = 0; c < NU; ++c) ST(k, FU, c) = BOUNDED ? proj(v[j][NX + c], lbv[c], ubv[c]) : v[j][NX + c];
                }
            }
        }
#pragma unroll
        for (int r = 0; r < NX; ++r)
            ST(N, FX, r) = p.init_hold ? p.x0[inst * NX + r] : (p.init_zero ? 0.0 : Vin[N * ND + r]);
        if constexpr (SWAP) {   // x_0 (pinned) in both iterate buffers: the step sweep writes stages 1..N of the other
#pragma unroll
            for (int r = 0; r < NX; ++r) ST(0, FXo, r) = p.x0[inst * NX + r];
        }
        const double* tr = p.traj + inst * (int64_t)N * NX;
        for (int k0 = 0; k0 < N; k0 += LB) {
            double t[LB][NX];
#pragma unroll
            for (int j = 0; j < LB; ++j) {
                const int kj = k0 + j < N ? k0 + j : N - 1;   // past the end: stage N-1 again, not stored
#pragma unroll
                for (int r = 0; r < NX; ++r) t[j][r] = tr[kj * NX + r];
            }
#pragma unroll
            for (int j = 0; j < LB; ++j)
                if (k0 + j < N)
#pragma unroll
                    for (int r = 0; r < NX; ++r) ST(k0 + j, SF::R, r) = t[j][r];
        }
    }
    double yl[XB ? NY : 1], yu[XB ? NY : 1];
    double mub = kIpMu0;  // barrier parameter (f = J/2 scale)
    if constexpr (XB) {  // y pushed into the interior, z = 1 on finite bounds (oracle solve_one_ip)
        load_ip_bounds<NX, NU>(p, yl, yu);
        for (int k = 0; k < N; ++k) {
#pragma unroll
            for (int j = 0; j < NY; ++j) {
                double& y = j < NX ? ST(k + 1, FX, j) : ST(k, FU, j - NX);
                y = ip_push(y, yl[j], yu[j]);
                ST(k, SF::ZL, j) = yl[j] > -INFINITY ? 1.0 : 0.0;
                ST(k, SF::ZU, j) = yu[j] < INFINITY ? 1.0 : 0.0;
            }
        }
    }
    // linear mode: acceleration Jacobians and xdot at (state, control) = (x_0, u_prev), ModelControl.cpp:125-135
    const bool lin = p.is_linear != 0;
    constexpr int LFQ = 0, LFQD = NA * NQ, LFU = LFQD + NA * NA, LXD = LFU + NA * NU, LXS = LXD + NX,
                  LUS = LXS + NX;
    static_assert(LUS + NU == lane_lin_doubles(NX, NU, NQ), "linear-mode block layout");
    if (lin) {
        double x[NX], acc[NA], Fq[SQ], Fqd[NA * NA], Fu[NA * NU];
#pragma unroll
        for (int r = 0; r < NX; ++r) x[r] = ST(0, FX, r);
        Model::eval_acc_jac(x, up, acc, Fq, Fqd, Fu);
#pragma unroll
        for (int t = 0; t < NA * NQ; ++t) ST(N + 1, LFQ, t) = Fq[t];
#pragma unroll
        for (int t = 0; t < NA * NA; ++t) ST(N + 1, LFQD, t) = Fqd[t];
#pragma unroll
        for (int t = 0; t < NA * NU; ++t) ST(N + 1, LFU, t) = Fu[t];
#pragma unroll
        for (int t = 0; t < NQ; ++t) ST(N + 1, LXD, t) = x[NQ + t];
#pragma unroll
        for (int t = 0; t < NA; ++t) ST(N + 1, LXD, NQ + t) = acc[t];
#pragma unroll
        for (int t = 0; t < NX; ++t) ST(N + 1, LXS, t) = x[t];
#pragma unroll
        for (int t = 0; t < NU; ++t) ST(N + 1, LUS, t) = up[t];
    }
    // Stage model: xd = f(x, u) and (jac) the SCALED blocks hFq, hFqd, hFu of A_k, B_k.
    // Linear mode: F_lin of ModelGenerator.cpp:47-48 with the stored A*, B*, xdot*.
#define STAGE_EVAL(x, u, xd, hFq, hFqd, hFu, jac)                                                        \
    do {                                                                                                 \
        if (!lin) {                                                                                      \
            if (jac && JACH) {   /* blocks come scaled: no pass below */                                   \
                model_acc_jac_h<Model>(x, u, h, xd + NQ, hFq, hFqd, hFu);                                \
                _Pragma("unroll") for (int i_ = 0; i_ < NQ; ++i_) xd[i_] = x[NQ + i_];                   \
            } else if (jac) {                                                                            \
                Model::eval_acc_jac(x, u, xd + NQ, hFq, hFqd, hFu);                                      \
                _Pragma("unroll") for (int i_ = 0; i_ < NQ; ++i_) xd[i_] = x[NQ + i_];                   \
            } else {                                                                                     \
                Model::eval(x, u, xd);                                                                   \
            }                                                                                            \
        } else {                                                                                         \
            gmem<double>* const lp_ = stage_ptr(wsb, N + 1, SS, lane);                                         \
            double dx_[NX], du_[NU];                                                                     \
            _Pragma("unroll") for (int i_ = 0; i_ < NX; ++i_) dx_[i_] = x[i_] - lp_[((LXS) + (i_)) * 64];        \
            _Pragma("unroll") for (int i_ = 0; i_ < NU; ++i_) du_[i_] = u[i_] - lp_[((LUS) + (i_)) * 64];        \
            _Pragma("unroll") for (int i_ = 0; i_ < NQ; ++i_) xd[i_] = lp_[((LXD) + (i_)) * 64] + dx_[NQ + i_];  \
            _Pragma("unroll") for (int i_ = 0; i_ < NA; ++i_) {                                          \
                double t_ = lp_[((LXD) + (NQ + i_)) * 64];                                                       \
                _Pragma("unroll") for (int s_ = 0; s_ < (NQ > NA ? NQ : NA); ++s_) {                      \
                    if (s_ < NA) {                                                                       \
                        const double fd_ = lp_[((LFQD) + (i_ * NA + s_)) * 64];                          \
                        if (jac) hFqd[i_ * NA + s_] = fd_;                                               \
                        t_ = fma(fd_, dx_[NQ + s_], t_);                                                 \
                    }                                                                                    \
                    if (s_ < NQ) {                                                                       \
                        const double fq_ = lp_[((LFQ) + (i_ * NQ + s_)) * 64];                           \
                        if (jac) hFq[i_ * NQ + s_] = fq_;                                                \
                        t_ = fma(fq_, dx_[s_], t_);                                                      \
                    }                                                                                    \
                }                                                                                        \
                _Pragma("unroll") for (int c_ = 0; c_ < NU; ++c_) {                                      \
                    const double fu_ = lp_[((LFU) + (i_ * NU + c_)) * 64];                                       \
                    if (jac) hFu[i_ * NU + c_] = fu_;                                                    \
                    t_ = fma(fu_, du_[c_], t_);                                                          \
                }                                                                                        \
                xd[NQ + i_] = t_;                                                                        \
            }                                                                                            \
        }                                                                                                \
        if (jac && (lin || !JACH)) {                                                                             \
            _Pragma("unroll") for (int i_ = 0; i_ < NA * NQ; ++i_) hFq[i_] *= h;                         \
            _Pragma("unroll") for (int i_ = 0; i_ < NA * NA; ++i_) hFqd[i_] *= h;                        \
            _Pragma("unroll") for (int i_ = 0; i_ < NA * NU; ++i_) hFu[i_] *= h;                         \
        }                                                                                                \
    } while (0)

    int status = ST_MAX_ITER;
    int it = 0;
    double kkt = 0.0, mu = 0.0, pg_prev = INFINITY;
    constexpr bool FUSE_TRIAL = !BOUNDED && !XB;  // the alpha = 1 trial is evaluated inside the step sweep
    // the forward and step sweeps need only A d and A dx + B du: a model with a directional derivative (ExoArm)
    // evaluates that instead of the Jacobian blocks (linear mode keeps its stored blocks)
    constexpr bool JVP = HasJvp<Model>::value;
    constexpr bool F64 = std::is_same<FT, double>::value;
    // first row q of Y = L^-1 [H_wx | -R] that can be nonzero in column j (the -R block is lower triangular)
    auto ylo = [](int j) constexpr { return (j < NX || !(F64 || MMPC_LANE_YLO32)) ? 0 : j - NX; };
    constexpr bool JACH = HasJacH<Model>::value && (F64 || MMPC_LANE_JACH32);
    // FUSE_FWD: the step sweep evaluates the alpha = 1 trial point with its Jacobian and forms there
    // everything pass (1) of the next iteration computes at that point (defects, d, J, |c|_1, max|c|), so when the
    // full step is accepted (99.7 % of the cfg#3 iterations, every one after the first: tools/alpha_stats.py) the
    // next iteration starts at (2).  This saves the value-only trial evaluation and pass (1)'s sweep (cfg#3:
    // 11.63 -> 11.20 ms).  The fp32-factor build (cfg#5) spilled more with it in round 2 (10.05 -> 11.77 ms); with
    // the directional derivative instead of the trial Jacobian (round 4) it gains there too (7.70 -> 7.34 ms,
    // profiles/r04/ab_fwd).  fwd_ready: C and D of the workspace hold the accepted iterate's values.
    constexpr bool FUSE_FWD = FUSE_TRIAL && (std::is_same<FT, double>::value || MMPC_LANE_FWD32);
    bool fwd_ready = false;
    double J0n = 0.0, c1n = 0.0, cmaxn = 0.0;
    bool nfn = false;
    bool lean_off = false;   // a hand-over of this instance found the list full: no lean sweeps, no further claims
    MMPC_PHASE(0);
    #pragma unroll 1
    for (it = 0; it <= p.max_iter; ++it) {
        // ---- (1) forward: F, defects, d_{k+1} = A_k d_k + c_k, merit value ----
        double J0 = J0n, c1 = c1n, cmax = cmaxn;
        double lsum = 0.0, cmpl0 = 0.0, cmplmu = 0.0;  // interior point: sum log s, max |s z|, max |s z - mu|
        bool nonfinite = nfn;
        if (!(FUSE_FWD && fwd_ready)) {
            J0 = 0.0;
            c1 = 0.0;
            cmax = 0.0;
            nonfinite = false;
            // software pipeline: the model inputs of stage k+1 are loaded during stage k (one wave per SIMD
            // has no other wave to hide HBM latency behind); the other loads of a stage are issued before
            // its model evaluation, which covers them
            double d[NX], xk[NX], um[NU], un[NU];
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                d[r] = 0.0;
                xk[r] = ST(0, FX, r);
            }
#pragma unroll
            for (int c = 0; c < NU; ++c) {
                um[c] = up[c];
                un[c] = ST(0, FU, c);
            }
            #pragma unroll 1
            for (int k = 0; k < N; ++k) {
                gmem<double>* const sk = stage_ptr(wsb, k, SS, lane);
                double u[NU], xn[NX], rk[NX], xd[NX], hFq[SQ], hFqd[NA * NA], hFu[NA * NU];
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    u[c] = un[c];
                    un[c] = SK(1, FU, c);  // stage N's U slot exists (unused) when k = N-1
                }
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    xn[r] = SK(1, FX, r);
                    rk[r] = SK(0, SF::R, r);
                }
                // XB: this stage's duals, loaded before the model evaluation (their latency hides behind it)
                constexpr int XF = (XB && MMPC_LANE_XB_EARLY) ? NY : 1;
                double zlf[XF], zuf[XF];
                if constexpr (XB && MMPC_LANE_XB_EARLY) {
#pragma unroll
                    for (int j = 0; j < NY; ++j) {
                        zlf[j] = SK(0, SF::ZL, j);
                        zuf[j] = SK(0, SF::ZU, j);
                    }
                }
                double dn[NX];   // A_k d_k
                if (JVP && !lin) {
                    double zu[NU], jv[NA];
#pragma unroll
                    for (int c = 0; c < NU; ++c) zu[c] = 0.0;
                    model_jvp<Model>(xk, u, d, zu, xd, jv);
                    jvp_step<NQ, NA>(h, d, jv, dn);
                } else {
                    STAGE_EVAL(xk, u, xd, hFq, hFqd, hFu, true);
                    a_mul<NQ, NA>(h, hFq, hFqd, d, dn);
                }
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    const double F = fma(h, xd[r], xk[r]);
                    const double c = F - xn[r];
                    if constexpr (!MMPC_LANE_C_NOSTORE) SK(0, SF::C, r) = c;
                    cmax = fmax(cmax, fabs(c));
                    c1 += fabs(c);
                    nonfinite |= !isfinite(c);
                    const double e = F - rk[r];
                    J0 = fma(e * Q[r], e, J0);
                    d[r] = dn[r] + c;
                    SK(1, SF::D, r) = d[r];
                    xk[r] = xn[r];
                }
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    const double dif = u[c] - um[c];
                    J0 = fma(dif * R[c], dif, fma(u[c] * Rm[c], u[c], J0));
                    um[c] = u[c];
                }
                if constexpr (XB) {  // barrier pieces of (x_{k+1} | u_k); xk now holds x_{k+1}
#pragma unroll
                    for (int j = 0; j < NY; ++j) {
                        double sg, bb, zg;
                        double zl, zu;
                        if constexpr (MMPC_LANE_XB_EARLY) {
                            zl = zlf[j];
                            zu = zuf[j];
                        } else {
                            zl = SK(0, SF::ZL, j);
                            zu = SK(0, SF::ZU, j);
                        }
                        ip_terms(j < NX ? xk[j] : u[j - NX], yl[j], yu[j], zl, zu, mub, sg, bb, zg, cmpl0, cmplmu, lsum);
                        SK(0, SF::SG, j) = sg;
                        SK(0, SF::BB, j) = bb;
                        SK(0, SF::ZG, j) = zg;
                    }
                }
            }
            nonfinite |= !isfinite(lsum);
        }

        MMPC_PHASE(1);
        // (2)+(3) run once, or (bounded) again after holding controls whose step crosses a bound
        double gmax = 0.0, lmax = 0.0, dJ = 0.0;
        double mub_next = mub, amax = 1.0, az = 1.0, dbar = 0.0;  // interior point (XB)
        bool fact_ok = true, done = false;
        // lazy step records (round 6): an unbounded solve's step sweep stores dx_k / du_k (DX / DU) only in the first
        // iteration; later the full step is nearly always taken (cfg#3: every instance-iteration after the first,
        // profiles/r03/alpha_stats_cfg3_v1.json), and a lane whose full step is rejected regenerates them (same
        // expressions, same bits) before its first shorter trial
        const bool wdxu = !LAZY || it == 0;
        bool have_dxu = wdxu;
        fwd_ready = false;
        const double beps = BOUNDED ? fmin(kBoundEps, pg_prev) : 0.0;
        double Jt1 = 0.0, ct1 = 0.0, cmt1 = 0.0;
        bool nft1 = false;
        // diagnostic trace [B][max_iter+1][8] = (||2g||, ||c||, J, |c|_1, dJ, alpha, mu, ||lam||)
        double* trc = p.trace ? p.trace + (inst * (p.max_iter + 1) + it) * 8 : nullptr;
        // ---- (2') lean sweep (round 6): when every lane of the wave leaves at this iteration's stop test -- it converges,
        // or it is handed over to the resume launch (the rule of the stop test below: `it` and the number of lanes still
        // iterating, both known before the sweep; the lanes that converge at this test are counted here too, so the
        // count is an upper bound of the stop test's), or the iteration limit is reached -- the backward sweep forms only
        // the adjoint, the reduced gradient and the stop test: the Riccati step's gains would never be read (the resume
        // launch solves its own QP).  Same expressions and order as sweep (2), so gmax / lmax / nonfinite are its values
        // bit for bit.  An instance whose hand-over finds the list full (lean_off) continues into the full sweep below,
        // which recomputes them.  At cfg#3 this is the wave's last backward sweep (iteration 4: every unconverged lane
        // is handed over at the cap).
        if (!lean_off && it >= 1 &&
            (it == p.max_iter || (p.tail_cap > 0 && (it >= p.tail_cap || (it >= 2 && p.tail_wave_max > 0 &&
                                                                           __popcll(__ballot(1)) <= p.tail_wave_max))))) {
            double lam[NX], unext[NU], xpf[NX], upf[NU];
#pragma unroll
            for (int r = 0; r < NX; ++r) {
                const double eb = ST(N, FX, r) - ST(N - 1, SF::R, r);  // x_N - r_{N-1}
                lam[r] = Q[r] * (ST(N, SF::D, r) + eb);                // lam_N = Q e_{N-1}
                if constexpr (XB) lam[r] += ST(N - 1, SF::ZG, r);
                lmax = fmax(lmax, fabs(lam[r]));
                xpf[r] = ST(N - 1, FX, r);
            }
#pragma unroll
            for (int c = 0; c < NU; ++c) {
                unext[c] = 0.0;
                upf[c] = ST(N - 1, FU, c);
            }
            #pragma unroll 1
            for (int k = N - 1; k >= 0; --k) {
                gmem<double>* const sk = stage_ptr(wsb, k, SS, lane);
                double x[NX], u[NU], um[NU], dk[NX], rkm[NX], xd[NX], hFq[SQ], hFqd[NA * NA], hFu[NA * NU];
                double zgu[XB ? NU : 1], zgx[XB ? NX : 1];
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    x[r] = xpf[r];
                    dk[r] = SK(0, SF::D, r);
                }
#pragma unroll
                for (int c = 0; c < NU; ++c) u[c] = upf[c];
                if (k >= 1) {
#pragma unroll
                    for (int r = 0; r < NX; ++r) {
                        rkm[r] = SK(-1, SF::R, r);
                        xpf[r] = SK(-1, FX, r);
                    }
#pragma unroll
                    for (int c = 0; c < NU; ++c) um[c] = SK(-1, FU, c);
                } else {
#pragma unroll
                    for (int r = 0; r < NX; ++r) rkm[r] = 0.0;
#pragma unroll
                    for (int c = 0; c < NU; ++c) um[c] = up[c];
                }
#pragma unroll
                for (int c = 0; c < NU; ++c) upf[c] = um[c];
                if constexpr (XB) {
#pragma unroll
                    for (int c = 0; c < NU; ++c) zgu[c] = SK(0, SF::ZG, NX + c);
                    if (k >= 1) {
#pragma unroll
                        for (int r = 0; r < NX; ++r) zgx[r] = SK(-1, SF::ZG, r);
                    }
                }
                STAGE_EVAL(x, u, xd, hFq, hFqd, hFu, true);
#pragma unroll
                for (int c = 0; c < NU; ++c) {   // reduced gradient, as sweep (2)
                    double g = 0.0;
#pragma unroll
                    for (int s = 0; s < NA; ++s) g = fma(hFu[s * NU + c], lam[NQ + s], g);
                    g = fma(R[c], u[c] - um[c], fma(Rm[c], u[c], g));
                    if (k + 1 < N) g -= R[c] * (unext[c] - u[c]);
                    if constexpr (XB) g += zgu[c];
                    if (!BOUNDED) gmax = fmax(gmax, fabs(2.0 * g));
                    else gmax = fmax(gmax, fabs(u[c] - proj(u[c] - 2.0 * g, lbv[c], ubv[c])));
                    nonfinite |= !isfinite(g);
                    unext[c] = u[c];
                }
                if (k >= 1) {   // adjoint, as sweep (2)
                    double ln[NX];
                    at_mul<NQ, NA>(h, hFq, hFqd, lam, ln);
#pragma unroll
                    for (int r = 0; r < NX; ++r) {
                        lam[r] = fma(Q[r], dk[r] + x[r] - rkm[r], ln[r]);
                        if constexpr (XB) lam[r] += zgx[r];
                        lmax = fmax(lmax, fabs(lam[r]));
                    }
                }
            }
            kkt = fmax(gmax, cmax);
            if (XB) kkt = fmax(kkt, 2.0 * cmpl0);
            if (trc) {
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
            const int slot = atomicAdd(p.tail_count, 1);   // the hand-over of the stop test below
            if (slot < p.tail_slots) {
                p.tail_idx[slot] = (int32_t)inst;
                p.tail_it[slot] = it;
                p.tail_mu[slot] = mu;
                if constexpr (XB) p.tail_mub[slot] = mub;
                if constexpr (BOUNDED) p.tail_mub[slot] = pg_prev;
                status = ST_HANDED_OVER;
                break;
            }
            lean_off = true;   // list full: the overflow path (the full sweep and the rest of this iteration)
            gmax = 0.0;
            lmax = 0.0;
        }
        // exact-Hessian blocks in this iteration's sweeps; false after a sweep's exact QP was not positive definite:
        // that sweep is redone and, with control bounds, every later QP solve of the iteration stays Gauss-Newton
        // (oracle solve_one: gn_fallback)
        bool useW = EXACT;
        #pragma unroll 1
        for (int pass = 0;; ++pass) {
            bool resolve = false;
            #pragma unroll 1
            for (;;) {
            gmax = 0.0;
            lmax = 0.0;
            fact_ok = true;
            // ---- (2) backward: adjoint + reduced gradient (stopping test) and the Riccati recursion ----
            // Value function V_k(s) = s^T P s + 2 p^T s on s = [dx_k; du_{k-1}] (no 1/2: J has none,
            // ModelGenerator.cpp:208-222); (P, pv) hold P~_{k+1} = P_{k+1} + blkdiag(Q, 0) on entry to step k.
            {
                double pv[NS], lam[NX], unext[NU];
#pragma unroll
                for (int a = 0; a < NS; ++a) {
                    pv[a] = 0.0;
#pragma unroll
                    for (int b = a; b < NS; ++b) PS(a, b) = (FT)((a == b && a < NX) ? Q[a] : 0.0);
                }
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    const double eb = ST(N, FX, r) - ST(N - 1, SF::R, r);  // x_N - r_{N-1}
                    pv[r] = Q[r] * eb;
                    lam[r] = Q[r] * (ST(N, SF::D, r) + eb);  // lam_N = Q e_{N-1}
                    if constexpr (XB) {  // barrier at x_N
                        PS(r, r) += (FT)ST(N - 1, SF::SG, r);
                        pv[r] += ST(N - 1, SF::BB, r);
                        lam[r] += ST(N - 1, SF::ZG, r);
                    }
                    lmax = fmax(lmax, fabs(lam[r]));
                }
                // software pipeline as in (1): x_{k-1}, u_{k-1} (model inputs of the next step) are loaded during
                // step k, everything else of step k before its model evaluation
                double xpf[NX], upf[NU];
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    unext[c] = 0.0;
                    upf[c] = ST(N - 1, FU, c);
                }
                double xk1[NX];   // x_{k+1} (MMPC_LANE_C_NOSTORE)
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    xpf[r] = ST(N - 1, FX, r);
                    xk1[r] = ST(N, FX, r);
                }
                #pragma unroll 1
                for (int k = N - 1; k >= 0; --k) {
                    gmem<double>* const sk = stage_ptr(wsb, k, SS, lane);
                    double x[NX], u[NU], um[NU], cc[NX], dk[NX], rkm[NX], xd[NX], hFq[SQ], hFqd[NA * NA],
                        hFu[NA * NU], tg[NU];
#pragma unroll
                    for (int r = 0; r < NX; ++r) {
                        x[r] = xpf[r];
                        if constexpr (!MMPC_LANE_C_NOSTORE) cc[r] = SK(0, SF::C, r);
                        dk[r] = SK(0, SF::D, r);
                    }
#pragma unroll
                    for (int c = 0; c < NU; ++c) u[c] = upf[c];
                    if (k >= 1) {
#pragma unroll
                        for (int r = 0; r < NX; ++r) {
                            rkm[r] = SK(-1, SF::R, r);
                            xpf[r] = SK(-1, FX, r);
                        }
#pragma unroll
                        for (int c = 0; c < NU; ++c) um[c] = SK(-1, FU, c);
                    } else {
#pragma unroll
                        for (int r = 0; r < NX; ++r) rkm[r] = 0.0;
#pragma unroll
                        for (int c = 0; c < NU; ++c) um[c] = up[c];
                    }
#pragma unroll
                    for (int c = 0; c < NU; ++c) upf[c] = um[c];
                    // XB: the barrier pieces this stage adds (u part of stage k, x part of stage k-1), loaded before the
                    // model evaluation so that their latency hides behind it (read at their uses they stalled the sweep)
                    constexpr int XE = (XB && MMPC_LANE_XB_EARLY) ? 1 : 0;
                    double zgu[XE ? NU : 1], sgu[XE ? NU : 1], bbu[XE ? NU : 1], zgx[XE ? NX : 1], sgx[XE ? NX : 1],
                        bbx[XE ? NX : 1];
                    if constexpr (XE) {
#pragma unroll
                        for (int c = 0; c < NU; ++c) {
                            zgu[c] = SK(0, SF::ZG, NX + c);
                            sgu[c] = SK(0, SF::SG, NX + c);
                            bbu[c] = SK(0, SF::BB, NX + c);
                        }
                        if (k >= 1) {
#pragma unroll
                            for (int r = 0; r < NX; ++r) {
                                zgx[r] = SK(-1, SF::ZG, r);
                                sgx[r] = SK(-1, SF::SG, r);
                                bbx[r] = SK(-1, SF::BB, r);
                            }
                        }
                    }
                    auto xb_zgu = [&](int c) { if constexpr (XE) return zgu[c]; else return (double)SK(0, SF::ZG, NX + c); };
                    auto xb_sgu = [&](int c) { if constexpr (XE) return sgu[c]; else return (double)SK(0, SF::SG, NX + c); };
                    auto xb_bbu = [&](int c) { if constexpr (XE) return bbu[c]; else return (double)SK(0, SF::BB, NX + c); };
                    auto xb_zgx = [&](int r) { if constexpr (XE) return zgx[r]; else return (double)SK(-1, SF::ZG, r); };
                    auto xb_sgx = [&](int r) { if constexpr (XE) return sgx[r]; else return (double)SK(-1, SF::SG, r); };
                    auto xb_bbx = [&](int r) { if constexpr (XE) return bbx[r]; else return (double)SK(-1, SF::BB, r); };
                    STAGE_EVAL(x, u, xd, hFq, hFqd, hFu, true);
                    if constexpr (MMPC_LANE_C_NOSTORE) {
                        // c_k = F(x_k, u_k) - x_{k+1} from this sweep's own evaluation (round 6: no C record in the
                        // workspace; the Jacobian evaluation's value is pass (1)'s bit for bit on cfg#3/#5, exact, |u|
                        // <= 0.5: profiles/r06/cns)
#pragma unroll
                        for (int r = 0; r < NX; ++r) {
                            cc[r] = fma(h, xd[r], x[r]) - xk1[r];
                            xk1[r] = x[r];
                        }
                    }
                    // exact Hessian: W_k at (x_k, u_k) with lam_{k+1} (lam holds it until the adjoint step below)
                    constexpr int KZ = NX + NU;
                    double Wk[EXACT ? KZ * KZ : 1];
                    if constexpr (EXACT) {
                        if (useW) {
                            double la[NA];
#pragma unroll
                            for (int s2 = 0; s2 < NA; ++s2) la[s2] = h * lam[NQ + s2];
                            Model::eval_hess(x, u, la, Wk);
                        } else {
#pragma unroll
                            for (int i = 0; i < KZ * KZ; ++i) Wk[i] = 0.0;
                        }
                    }
                    // reduced gradient g_k = B_k^T lam_{k+1} + R/Rm terms (same expression as sqp_wave.h)
#pragma unroll
                    for (int c = 0; c < NU; ++c) {
                        double g = 0.0;
#pragma unroll
                        for (int s = 0; s < NA; ++s) g = fma(hFu[s * NU + c], lam[NQ + s], g);
                        g = fma(R[c], u[c] - um[c], fma(Rm[c], u[c], g));
                        if (k + 1 < N) g -= R[c] * (unext[c] - u[c]);
                        if (XB) g += xb_zgu(c);  // reduced Lagrangian gradient
                        if (!BOUNDED) {
                            gmax = fmax(gmax, fabs(2.0 * g));
                        } else {  // projected gradient; hold rule (pass 0) or the holds of the previous solve
                            gmax = fmax(gmax, fabs(u[c] - proj(u[c] - 2.0 * g, lbv[c], ubv[c])));
                            if (pass == 0) {
                                tg[c] = (u[c] <= lbv[c] + beps && g > 0.0)   ? lbv[c]
                                        : (u[c] >= ubv[c] - beps && g < 0.0) ? ubv[c]
                                                                              : NAN;
                                SK(0, SF::HOLD, c) = tg[c];
                            } else {
                                tg[c] = SK(0, SF::HOLD, c);
                            }
                        }
                        nonfinite |= !isfinite(g);
                        unext[c] = u[c];
                    }
                    // adjoint lam_k = Q e_{k-1} + A_k^T lam_{k+1},  e_{k-1} = d_k + x_k - r_{k-1}
                    if (k >= 1) {
                        double ln[NX];
                        at_mul<NQ, NA>(h, hFq, hFqd, lam, ln);
#pragma unroll
                        for (int r = 0; r < NX; ++r) {
                            lam[r] = fma(Q[r], dk[r] + x[r] - rkm[r], ln[r]);
                            if (XB) lam[r] += xb_zgx(r);
                            lmax = fmax(lmax, fabs(lam[r]));
                        }
                    }
                    // ---- Riccati step ----
                    // Matrix recursion (P, G, H_ww, its Cholesky factor, the matrix part of Y and K) in FT; the
                    // right-hand side (p, m = P_xx c + p_x, h_w, y, kff) in fp64 with FT matrices: with FT = float
                    // this is an fp32 factorisation applied to fp64 residuals, so each SQP iteration is a
                    // refinement step (the linear terms cancel down to the gradient and need fp64).
                    FT fq[SQ], fqd[NA * NA], fu[NA * NU];
                    const FT hf = (FT)h;
#pragma unroll
                    for (int i = 0; i < NA * NQ; ++i) fq[i] = (FT)hFq[i];
#pragma unroll
                    for (int i = 0; i < NA * NA; ++i) fqd[i] = (FT)hFqd[i];
#pragma unroll
                    for (int i = 0; i < NA * NU; ++i) fu[i] = (FT)hFu[i];
                    FT G[NX][NU];  // P_xx B + P_xu   (B = [0; hFu])
#pragma unroll
                    for (int r = 0; r < NX; ++r)
#pragma unroll
                        for (int c = 0; c < NU; ++c) {
                            FT t = PS(r, NX + c);
#pragma unroll
                            for (int s = 0; s < NA; ++s) t = fma(PS(r, NQ + s), fu[s * NU + c], t);
                            G[r][c] = t;
                        }
                    double mv[NX];  // P_xx c + p_x (fp64)
#pragma unroll
                    for (int r = 0; r < NX; ++r) {
                        double t = pv[r];
#pragma unroll
                        for (int q = 0; q < NX; ++q) t = fma((double)PS(r, q), cc[q], t);
                        mv[r] = t;
                    }
                    FT Hww[NU][NU], Y[NU][NS];  // Y rows: L^-1 [H_wx | -R]
                    double yh[NU];              // L^-1 h_w (fp64)
#pragma unroll
                    for (int a = 0; a < NU; ++a) {
#pragma unroll
                        for (int b = a; b < NU; ++b) {
                            FT t = PS(NX + a, NX + b);
#pragma unroll
                            for (int s = 0; s < NA; ++s)
                                t = fma(fu[s * NU + a], G[NQ + s][b], fma(PS(NQ + s, NX + a), fu[s * NU + b], t));
                            if (a == b) t += (FT)(R[a] + Rm[a]);
                            if (XB && a == b) t += (FT)xb_sgu(a);
                            if constexpr (EXACT) t += Wk[(NX + a) * KZ + NX + b];
                            Hww[a][b] = t;
                        }
                        double t = fma(R[a], u[a] - um[a], fma(Rm[a], u[a], pv[NX + a]));
                        if (XB) t += xb_bbu(a);
#pragma unroll
                        for (int s = 0; s < NA; ++s) t = fma(hFu[s * NU + a], mv[NQ + s], t);
#pragma unroll
                        for (int r = 0; r < NX; ++r) t = fma((double)PS(r, NX + a), cc[r], t);
                        yh[a] = t;
                        FT ga[NX];
#pragma unroll
                        for (int r = 0; r < NX; ++r) ga[r] = G[r][a];
                        at_mul<NQ, NA, FT>(hf, fq, fqd, ga, &Y[a][0]);  // H_wx row a = (A^T G[:, a])^T
                        if constexpr (EXACT) {   // + W_ux row a
#pragma unroll
                            for (int j = 0; j < NX; ++j) Y[a][j] += Wk[(NX + a) * KZ + j];
                        }
#pragma unroll
                        for (int c = 0; c < NU; ++c) Y[a][NX + c] = (FT)((a == c) ? -R[a] : 0.0);
                    }
                    // Held controls (bounded solves): the stage QP with w_A = delta_A = target - u fixed --
                    // h_F += H_FA delta_A, rows/cols A of H_ww -> identity, rows A of [H_wx | -R] -> 0, so that
                    // K_A = 0 and kff_A = delta_A; p~_k gains [H_wx | -R]_A^T delta_A (pex).
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
                                for (int j = 0; j < NS; ++j) pex[j] = fma((double)Y[a][j], dl[a], pex[j]);
#pragma unroll
                            for (int b = 0; b < NU; ++b) {
                                double t = yh[b];
#pragma unroll
                                for (int a = 0; a < NU; ++a) t = fma((double)Hww[a < b ? a : b][a < b ? b : a], dl[a], t);
                                yh[b] = hd[b] ? -dl[b] : t;
                            }
#pragma unroll
                            for (int a = 0; a < NU; ++a) {
#pragma unroll
                                for (int b = a; b < NU; ++b)
                                    if (hd[a] || hd[b]) Hww[a][b] = (FT)((a == b) ? 1.0 : 0.0);
                                if (hd[a])
#pragma unroll
                                    for (int j = 0; j < NS; ++j) Y[a][j] = (FT)0;
                            }
                        }
                    }
                    // W = P_xx A (row r of W = (A^T P_xx[r][:])^T), streamed through the lane's scratch stage of the
                    // workspace (in registers next to G, Y and the stage blocks it spills).
                    // p~_k x part: A^T mv + Q (x_k - r_{k-1}) (fp64).
                    double pn[NS];
                    gmem<FT>* const sw = (gmem<FT>*)(stage_ptr(wsb, kScratch, SS, 0)) + lane;  // per-lane scratch stage
                    if (k >= 1) {
                        if constexpr (!WLDS)
#pragma unroll
                        for (int r = 0; r < NX; ++r) {
                            FT prow[NX], wrow[NX];
#pragma unroll
                            for (int q = 0; q < NX; ++q) prow[q] = PS(r, q);
                            at_mul<NQ, NA, FT>(hf, fq, fqd, prow, wrow);
#pragma unroll
                            for (int b = 0; b < NX; ++b) sw[(r * NX + b) * 64] = wrow[b];
                        }
                        double t[NX];
                        at_mul<NQ, NA, double>(h, hFq, hFqd, mv, t);
#pragma unroll
                        for (int q = 0; q < NX; ++q) {
                            pn[q] = fma(Q[q], x[q] - rkm[q], t[q]);
                            if (XB) pn[q] += xb_bbx(q);
                        }
#pragma unroll
                        for (int c = 0; c < NU; ++c) pn[NX + c] = -R[c] * (u[c] - um[c]);
                    }
                    // Cholesky H_ww = L L^T (FT), then Y <- L^-1 Y (FT) and yh <- L^-1 yh (fp64)
                    FT Ld[NU][NU], il[NU];
#pragma unroll
                    for (int a = 0; a < NU; ++a) {
                        FT s = Hww[a][a];
#pragma unroll
                        for (int q = 0; q < a; ++q) s = fma(-Ld[a][q], Ld[a][q], s);
                        fact_ok &= (s > (FT)0) && isfinite(s);
                        if constexpr (std::is_same<FT, double>::value) {   // no sqrt + division sequences (device.h)
                            sqrt_rsqrt(fmax(s, std::numeric_limits<FT>::min()), Ld[a][a], il[a]);
                        } else {
                            const FT lj = sqrt(fmax(s, std::numeric_limits<FT>::min()));
                            Ld[a][a] = lj;
                            il[a] = (FT)1 / lj;
                        }
#pragma unroll
                        for (int b = a + 1; b < NU; ++b) {
                            FT t = Hww[a][b];
#pragma unroll
                            for (int q = 0; q < a; ++q) t = fma(-Ld[b][q], Ld[a][q], t);
                            Ld[b][a] = t * il[a];
                        }
                    }
#pragma unroll
                    for (int a = 0; a < NU; ++a) {
#pragma unroll
                        for (int j = 0; j < NS; ++j) {
                            // the -R columns stay lower triangular (L^-1 (-R), R diagonal): Y[q][NX + c] = 0 for q < c.
                            // Multiplications by those zeros are not folded (0 * x is not 0 for x = inf / NaN), so
                            // every loop over q below starts at the first row that can be nonzero (ylo)
                            if (j >= NX && j - NX > a) {
                                Y[a][j] = (FT)0;
                                continue;
                            }
                            FT t = Y[a][j];
#pragma unroll
                            for (int q = ylo(j); q < a; ++q) t = fma(-Ld[a][q], Y[q][j], t);
                            Y[a][j] = t * il[a];
                        }
                        double t = yh[a];
#pragma unroll
                        for (int q = 0; q < a; ++q) t = fma(-(double)Ld[a][q], yh[q], t);
                        yh[a] = std::is_same<FT, double>::value ? t * (double)il[a] : t / (double)Ld[a][a];
                    }
                    // [K_k | kff_k] = -L^-T [Y | yh]: kff (fp64) in the first NU slots of the K field, K (FT) after it
                    // One column of K at a time, stored as soon as it is formed (the same expressions as a row-wise
                    // back substitution, so the same values): 4 live gains instead of 48 (round 5 register diet)
                    {
                        gmem<double>* const kb = stage_ptr(wsb, k, SS, 0) + SF::K * 64;
                        gmem<FT>* const kk = (gmem<FT>*)(kb + NU * 64) + lane;
                        double kh[NU];
#pragma unroll
                        for (int a = NU - 1; a >= 0; --a) {
                            double t = yh[a];
#pragma unroll
                            for (int q = a + 1; q < NU; ++q) t = fma(-(double)Ld[q][a], kh[q], t);
                            kh[a] = std::is_same<FT, double>::value ? t * (double)il[a] : t / (double)Ld[a][a];
                        }
#pragma unroll
                        for (int a = 0; a < NU; ++a) kb[a * 64 + lane] = -kh[a];
#pragma unroll
                        for (int j = 0; j < (KPACK ? NX : NS); ++j) {
                            FT kc[NU];
#pragma unroll
                            for (int a = NU - 1; a >= 0; --a) {
                                FT t = Y[a][j];
#pragma unroll
                                for (int q = a + 1; q < NU; ++q) t = fma(-Ld[q][a], kc[q], t);
                                kc[a] = t * il[a];
                            }
#pragma unroll
                            for (int a = 0; a < NU; ++a) kk[kgain_idx<NX, NU, KPACK>(a, j) * 64] = -kc[a];
                        }
                        if constexpr (KPACK) {   // H_ww^-1 column c, rows a >= c: L^-T (L^-1 e_c)
#pragma unroll
                            for (int c = 0; c < NU; ++c) {
                                FT z[NU], hc[NU];
#pragma unroll
                                for (int q = c; q < NU; ++q) {
                                    FT t = q == c ? (FT)1 : (FT)0;
#pragma unroll
                                    for (int m = c; m < q; ++m) t = fma(-Ld[q][m], z[m], t);
                                    z[q] = t * il[q];
                                }
#pragma unroll
                                for (int a = NU - 1; a >= c; --a) {
                                    FT t = z[a];
#pragma unroll
                                    for (int q = a + 1; q < NU; ++q) t = fma(-Ld[q][a], hc[q], t);
                                    hc[a] = t * il[a];
                                    kk[kgain_idx<NX, NU, KPACK>(a, NX + c) * 64] = hc[a];
                                }
                            }
                        }
                    }
                    if (k == 0) break;  // s_0 = 0: P~_0 is never used
                    // P~_k = blkdiag(A^T W + Q, R) - Y^T Y (old P is dead: overwrite it in place), p~_k = pn - Y^T yh
                    if constexpr (WLDS) {
                        // W in LDS: the a-rows of W (used by every output row) go to the dead P_xu / P_uu slots; the
                        // q-rows are formed one at a time in registers, in descending order, each right before the
                        // two output rows that use it (a and NQ + a): every P~_xx entry a later W row still reads
                        // lies in a row not yet rewritten.
                        auto WB = [&](int s2, int b) -> FT& { return Pl[lane_dead_slot(NX, NU, s2 * NX + b) * 64]; };
#pragma unroll
                        for (int s2 = 0; s2 < NA; ++s2) {
                            FT prow[NX], wrow[NX];
#pragma unroll
                            for (int q = 0; q < NX; ++q) prow[q] = PS(NQ + s2, q);
                            at_mul<NQ, NA, FT>(hf, fq, fqd, prow, wrow);
#pragma unroll
                            for (int b = 0; b < NX; ++b) WB(s2, b) = wrow[b];
                        }
                        auto out = [&](int a, int b, FT v) {
                            v += (FT)((a == b) ? Q[a] + (XB ? xb_sgx(a) : 0.0) : 0.0);
                            if constexpr (EXACT) v += Wk[a * KZ + b];   // + W_xx
#pragma unroll
                            for (int q = 0; q < NU; ++q) v = fma(-Y[q][a], Y[q][b], v);
                            PS(a, b) = v;
                        };
                        // rows NQ + a for a >= NQ (first-order part beyond the kinematic pairs): W a-rows only
#pragma unroll
                        for (int a = NQ; a < NA; ++a)
#pragma unroll
                            for (int b = NQ + a; b < NX; ++b) {
                                FT t = WB(a, b);
#pragma unroll
                                for (int s2 = 0; s2 < NA; ++s2) t = fma(fqd[s2 * NA + a], WB(s2, b), t);
                                out(NQ + a, b, t);
                            }
#pragma unroll
                        for (int a = NQ - 1; a >= 0; --a) {
                            FT prow[NX], wt[NX];
#pragma unroll
                            for (int q = 0; q < NX; ++q) prow[q] = PS(a, q);
                            at_mul<NQ, NA, FT>(hf, fq, fqd, prow, wt);   // row a of W
#pragma unroll
                            for (int b = a; b < NX; ++b) {   // output row a: W[a] + sum_s hFq[s][a] W[NQ+s]
                                FT t = wt[b];
#pragma unroll
                                for (int s2 = 0; s2 < NA; ++s2) t = fma(fq[s2 * NQ + a], WB(s2, b), t);
                                out(a, b, t);
                            }
#pragma unroll
                            for (int b = NQ + a; b < NX; ++b) {   // output row NQ+a: h W[a] + W[NQ+a] + sum hFqd W
                                FT t = fma(hf, wt[b], WB(a, b));
#pragma unroll
                                for (int s2 = 0; s2 < NA; ++s2) t = fma(fqd[s2 * NA + a], WB(s2, b), t);
                                out(NQ + a, b, t);
                            }
                        }
                    } else {
                    asm volatile("" ::: "memory");  // W comes back from memory, not from forwarded registers
#pragma unroll
                    for (int b = 0; b < NX; ++b) {
                        FT wcol[NX], col[NX];
#pragma unroll
                        for (int r = 0; r < NX; ++r) wcol[r] = sw[(r * NX + b) * 64];
                        at_mul<NQ, NA, FT>(hf, fq, fqd, wcol, col);
#pragma unroll
                        for (int a = 0; a <= b; ++a) {
                            FT v = col[a] + (FT)((a == b) ? Q[a] + (XB ? xb_sgx(a) : 0.0) : 0.0);
                            if constexpr (EXACT) v += Wk[a * KZ + b];   // + W_xx
#pragma unroll
                            for (int q = 0; q < NU; ++q) v = fma(-Y[q][a], Y[q][b], v);
                            PS(a, b) = v;
                        }
                    }
                    }
#pragma unroll
                    for (int a = 0; a < NS; ++a) {
                        double t = pn[a];
#pragma unroll
                        for (int q = ylo(a); q < NU; ++q) t = fma(-(double)Y[q][a], yh[q], t);
                        if (BOUNDED) t += pex[a];
                        pv[a] = t;
#pragma unroll
                        for (int b = (a < NX ? NX : a); b < NS; ++b) {
                            FT v = (FT)((a == b) ? R[a - NX] : 0.0);
#pragma unroll
                            for (int q = ylo(b); q < NU; ++q) v = fma(-Y[q][a], Y[q][b], v);   // b >= a: ylo(b) >= ylo(a)
                            PS(a, b) = v;
                        }
                    }
                }
            }
            // exact KKT matrix not positive definite on the null space: this iteration takes the Gauss-Newton step
            if (!(EXACT && useW && !fact_ok)) break;
            useW = false;
            }
            MMPC_PHASE(2);
            if (pass == 0) {
                kkt = fmax(gmax, cmax);
                if (XB) kkt = fmax(kkt, 2.0 * cmpl0);  // J-scale complementarity
                if (trc) {
                    trc[0] = gmax;
                    trc[1] = cmax;
                    trc[2] = J0;
                    trc[3] = c1;
                    trc[7] = lmax;
                }
                if (nonfinite || !isfinite(kkt)) {
                    status = ST_NONFINITE;
                    done = true;
                    break;
                }
                if (gmax <= p.tol_grad && cmax <= p.tol_defect && (!XB || 2.0 * cmpl0 <= kIpTolCompl)) {
                    status = ST_CONVERGED;
                    done = true;
                    break;
                }
                if (it == p.max_iter) {
                    status = ST_MAX_ITER;
                    done = true;
                    break;
                }
                // tail hand-over (unbounded solves): the instance continues in a 16-lane resume launch from this
                // iterate, iteration count and merit weight -- the wave no longer waits for it.  At iteration
                // tail_cap (and later, after an overflow), or earlier (from iteration 2) once at most tail_wave_max
                // lanes of the wave are still iterating: the active lanes here are exactly the unconverged ones
                bool hand = p.tail_cap > 0 && !lean_off && it >= p.tail_cap;   // lean_off: the list is full
                if (p.tail_cap > 0 && !lean_off && !hand && it >= 2 && p.tail_wave_max > 0)
                    hand = __popcll(__ballot(1)) <= p.tail_wave_max;
                if (hand) {
                    const int slot = atomicAdd(p.tail_count, 1);
                    if (slot < p.tail_slots) {
                        p.tail_idx[slot] = (int32_t)inst;
                        p.tail_it[slot] = it;
                        p.tail_mu[slot] = mu;
                        if constexpr (XB) p.tail_mub[slot] = mub;   // the duals stay in this launch's workspace
                        if constexpr (BOUNDED) p.tail_mub[slot] = pg_prev;   // the epsilon of the hold rule
                        status = ST_HANDED_OVER;
                        done = true;
                        break;
                    }
                    lean_off = true;
                }
                if (BOUNDED) pg_prev = gmax;
                // barrier update for the next iteration (IPOPT monotone rule, lagged; oracle solve_one_ip)
                if (XB && fmax(fmax(0.5 * gmax, cmax), cmplmu) <= kIpKappaEps * mub)
                    mub_next = fmax(kIpTolCompl / 20.0, fmin(kIpKappaMu * mub, pow(mub, kIpThetaMu)));
            }
            if (!fact_ok) {
                status = ST_FACT_FAILED;
                done = true;
                break;
            }

            // ---- (3) forward: step (dx, du) and the directional derivative of J ----
            // Unbounded solves also evaluate the line search's first trial (alpha = 1) here, stage by stage, with
            // the operands already in registers: same values and summation order as the trial loop of (4).
            dJ = 0.0;
            Jt1 = 0.0;
            ct1 = 0.0;
            cmt1 = 0.0;
            nft1 = false;
            amax = 1.0;
            az = 1.0;
            dbar = 0.0;
            {
                double dx[NX], dup[NU], um[NU];
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    dx[r] = 0.0;
                    ST(0, SF::DX, r) = 0.0;
                }
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    dup[c] = 0.0;
                    um[c] = up[c];
                }
                // software pipeline as in (1); the feedback gains K_k are consumed (and loaded) before the model
                // evaluation, whose compute then covers the remaining loads of the stage
                double xpf[NX], upf[NU], umt[NU], dt[NX];  // dt: d of the alpha = 1 trial point (FUSE_FWD)
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    xpf[r] = ST(0, FX, r);
                    dt[r] = 0.0;
                }
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    upf[c] = ST(0, FU, c);
                    umt[c] = up[c];
                }
                #pragma unroll 1
                for (int k = 0; k < N; ++k) {
                    gmem<double>* const sk = stage_ptr(wsb, k, SS, lane);
                    double x[NX], u[NU], xd[NX], rk[NX], ck[NX], hFq[SQ], hFqd[NA * NA], hFu[NA * NU], dxk[NX];
#pragma unroll
                    for (int r = 0; r < NX; ++r) dxk[r] = dx[r];
#pragma unroll
                    for (int r = 0; r < NX; ++r) {
                        x[r] = xpf[r];
                        xpf[r] = SK(1, FX, r);
                        rk[r] = SK(0, SF::R, r);
                        if constexpr (!MMPC_LANE_C_RECOMPUTE) ck[r] = SK(0, SF::C, r);
                    }
#pragma unroll
                    for (int c = 0; c < NU; ++c) {
                        u[c] = upf[c];
                        upf[c] = SK(1, FU, c);  // stage N's U slot exists (unused) when k = N-1
                    }
                    // XB: the duals and barrier gradient of this stage for the fraction to the boundary, loaded before
                    // the model evaluation (read at their use, at the end of the stage, they stalled the sweep)
                    constexpr int XS = (XB && MMPC_LANE_XB_EARLY_STEP) ? NY : 1;
                    double zls[XS], zus[XS], bbs[XS];
                    if constexpr (XB && MMPC_LANE_XB_EARLY_STEP) {
#pragma unroll
                        for (int j = 0; j < NY; ++j) {
                            zls[j] = SK(0, SF::ZL, j);
                            zus[j] = SK(0, SF::ZU, j);
                            bbs[j] = SK(0, SF::BB, j);
                        }
                    }
                    double du[NU];
                    const gmem<double>* const kb = stage_ptr(wsb, k, SS, 0) + SF::K * 64;
                    const gmem<FT>* const kk = (const gmem<FT>*)(kb + NU * 64) + lane;
                    if constexpr (!XB || MMPC_LANE_XB_BATCHED) {
                        // all loads of [K_k | kff_k] issued before the first use: under register pressure the
                        // scheduler otherwise interleaves load -> vmcnt(0) -> fma, one memory round trip per gain
                        FT kv[KN];
                        double kf[NU];
#pragma unroll
                        for (int a = 0; a < NU; ++a) kf[a] = kb[a * 64 + lane];
#pragma unroll
                        for (int e = 0; e < KN; ++e) kv[e] = kk[e * 64];
                        __builtin_amdgcn_sched_barrier(0);
#if MMPC_LANE_XTRA_K   // diagnostic A/B only: the gains stored back (same values): + the K record's write traffic
#pragma unroll
                        for (int e = 0; e < KN; ++e) ((gmem<FT>*)kk)[e * 64] = kv[e];
#endif
                        double dr[NU];   // the vector K_u multiplies: du_{k-1}, or R o du_{k-1} (KPACK)
#pragma unroll
                        for (int c = 0; c < NU; ++c) dr[c] = KPACK ? R[c] * dup[c] : dup[c];
#pragma unroll
                        for (int a = 0; a < NU; ++a) {
                            double t = kf[a];
#pragma unroll
                            for (int q = 0; q < NX; ++q) t = fma((double)kv[kgain_idx<NX, NU, KPACK>(a, q)], dx[q], t);
#pragma unroll
                            for (int c = 0; c < NU; ++c) t = fma((double)kv[kgain_idx<NX, NU, KPACK>(a, NX + c)], dr[c], t);
                            du[a] = t;
                            if (wdxu) SK(0, SF::DU, a) = t;
                        }
                    } else {
                        // loads at their uses (MMPC_LANE_XB_BATCHED=0 only).  The batched form above computed wrong
                        // steps in the exo interior-point instantiation under ROCm 7.2's greedy SGPR allocator (a
                        // register-allocation defect, not the source); with the basic allocator this
                        // unit is built with it is right, and it made the exo state-bounded cfg#3-size solve
                        // 92.4 -> 74.3 ms (round 4, profiles/r04/ab_xbb).
#pragma unroll
                        for (int a = 0; a < NU; ++a) {
                            double t = kb[a * 64 + lane];
#pragma unroll
                            for (int q = 0; q < NX; ++q) t = fma((double)kk[kgain_idx<NX, NU, KPACK>(a, q) * 64], dx[q], t);
#pragma unroll
                            for (int c = 0; c < NU; ++c)
                                t = fma((double)kk[kgain_idx<NX, NU, KPACK>(a, NX + c) * 64], KPACK ? R[c] * dup[c] : dup[c], t);
                            du[a] = t;
                            SK(0, SF::DU, a) = t;
                        }
                    }
                    if (BOUNDED && pass + 1 < kBoundPasses) {  // a free control whose step crosses a bound: hold it
#pragma unroll
                        for (int a = 0; a < NU; ++a) {
                            const double hv = SK(0, SF::HOLD, a), t = u[a] + du[a];
                            if (hv != hv && (t < lbv[a] || t > ubv[a])) {
                                SK(0, SF::HOLD, a) = t < lbv[a] ? lbv[a] : ubv[a];
                                resolve = true;
                            }
                        }
                    }
                    double ad[NX];   // A_k dx_k + B_k du_k
                    if (JVP && !lin) {
                        double jv[NA];
                        model_jvp<Model>(x, u, dx, du, xd, jv);
                        jvp_step<NQ, NA>(h, dx, jv, ad);
                    } else {
                        STAGE_EVAL(x, u, xd, hFq, hFqd, hFu, true);
                        a_mul<NQ, NA>(h, hFq, hFqd, dx, ad);
#pragma unroll
                        for (int s = 0; s < NA; ++s)
#pragma unroll
                            for (int c = 0; c < NU; ++c) ad[NQ + s] = fma(hFu[s * NU + c], du[c], ad[NQ + s]);
                    }
#pragma unroll
                    for (int r = 0; r < NX; ++r) {
                        const double F = fma(h, xd[r], x[r]);
                        // c_k = F(x_k, u_k) - x_{k+1} from this evaluation: the stored C_k is the same expression of the
                        // same model function at the same point (pass (1) or the previous iteration's fused trial), so
                        // the same bits, without its load (round 6)
                        if constexpr (MMPC_LANE_C_RECOMPUTE) ck[r] = F - xpf[r];
                        const double qe = 2.0 * Q[r] * (F - rk[r]);
                        dJ = fma(qe, ad[r], dJ);
                        dx[r] = ad[r] + ck[r];
                        if (wdxu) SK(1, SF::DX, r) = dx[r];
                    }
#pragma unroll
                    for (int c = 0; c < NU; ++c) {
                        const double dif = u[c] - um[c];
                        dJ = fma(2.0 * R[c] * dif, du[c] - dup[c], fma(2.0 * Rm[c] * u[c], du[c], dJ));
                        um[c] = u[c];
                        dup[c] = du[c];
                    }
                    if constexpr (FUSE_TRIAL) {   // trial point (x_k + dx_k, u_k + du_k), its defect to x_{k+1} + dx_{k+1}
                        // = pass (1) at the iterate the full step gives (the update's fma(1, dx, x) is x + dx): the
                        // same expressions in the same order, C_k and d_{k+1} stored for the next iteration (C_k of
                        // this iteration was read above; a rejected full step recomputes both in (1))
                        double xt[NX], ut[NU], xdt[NX];
#pragma unroll
                        for (int r = 0; r < NX; ++r) xt[r] = x[r] + dxk[r];
#pragma unroll
                        for (int c = 0; c < NU; ++c) ut[c] = u[c] + du[c];
                        if constexpr (FUSE_FWD) {
                            double dn[NX];   // A d at the trial point, as pass (1)
                            if (JVP && !lin) {
                                double zu[NU], jv[NA];
#pragma unroll
                                for (int c = 0; c < NU; ++c) zu[c] = 0.0;
                                model_jvp<Model>(xt, ut, dt, zu, xdt, jv);
                                jvp_step<NQ, NA>(h, dt, jv, dn);
                            } else {
                                double tFq[SQ], tFqd[NA * NA], tFu[NA * NU];
                                STAGE_EVAL(xt, ut, xdt, tFq, tFqd, tFu, true);
                                a_mul<NQ, NA>(h, tFq, tFqd, dt, dn);
                            }
#pragma unroll
                            for (int r = 0; r < NX; ++r) {
                                const double F = fma(h, xdt[r], xt[r]);
                                const double xn1 = xpf[r] + dx[r];   // x_{k+1} + dx_{k+1}: the update's fma(1, dx, x)
                                if constexpr (SWAP) SK(1, FXo, r) = xn1;
                                const double c = F - xn1;
                                if constexpr (!MMPC_LANE_C_NOSTORE) SK(0, SF::C, r) = c;
                                cmt1 = fmax(cmt1, fabs(c));
                                ct1 += fabs(c);
                                nft1 |= !isfinite(c);
                                const double er = F - rk[r];
                                Jt1 = fma(er * Q[r], er, Jt1);
                                dt[r] = dn[r] + c;
                                SK(1, SF::D, r) = dt[r];
                            }
                        } else {
                            double* nil_ = nullptr;
                            STAGE_EVAL(xt, ut, xdt, nil_, nil_, nil_, false);
#pragma unroll
                            for (int r = 0; r < NX; ++r) {
                                const double F = fma(h, xdt[r], xt[r]);
                                const double er = F - rk[r];
                                Jt1 = fma(er * Q[r], er, Jt1);
                                const double xn1 = xpf[r] + dx[r];
                                if constexpr (SWAP) SK(1, FXo, r) = xn1;
                                ct1 += fabs(F - xn1);
                            }
                        }
#pragma unroll
                        for (int c = 0; c < NU; ++c) {
                            const double dif = ut[c] - umt[c];
                            Jt1 = fma(dif * R[c], dif, fma(ut[c] * Rm[c], ut[c], Jt1));
                            umt[c] = ut[c];
                            if constexpr (SWAP) SK(0, FUo, c) = ut[c];
                        }
                    }
                    if constexpr (XB) {  // fraction to the boundary of (x_{k+1} | u_k), barrier directional derivative
#pragma unroll
                        for (int j = 0; j < NY; ++j) {
                            double zl, zu, bb;
                            if constexpr (MMPC_LANE_XB_EARLY_STEP) {
                                zl = zls[j];
                                zu = zus[j];
                                bb = bbs[j];
                            } else {
                                zl = SK(0, SF::ZL, j);
                                zu = SK(0, SF::ZU, j);
                                bb = SK(0, SF::BB, j);
                            }
                            ip_step_limits(j < NX ? xpf[j] : u[j - NX], j < NX ? dx[j] : du[j - NX], yl[j], yu[j], zl,
                                           zu, mub, kIpTau, bb, amax, az, dbar);
                        }
                    }
                }
            }

            MMPC_PHASE(4);
            if (!BOUNDED || !resolve || pass + 1 >= kBoundPasses) break;
        }
        if (done) break;
        // ---- (4) l1-merit Armijo line search (noise-aware, as sqp_wave.h) ----
        if constexpr (LAZY && MMPC_LANE_LS_HANDOVER) {
            // a full step rejected after the first iteration: the instance is handed over as at this iteration's stop
            // test (iterate, count, merit weight before this update) instead of running its line search, the step
            // records' regeneration and the extra forward pass with its whole wave waiting (round 6: one such
            // instance in a cfg#3 batch made the launch 7.4 ms instead of 5.8, profiles/r06/blocks/)
            if (p.tail_cap > 0 && !lean_off && it >= 1) {
                const double mu1 = fmax(mu, 4.0 * lmax + 1.0);
                const double phi0 = fma(mu1, c1, J0), dphi = dJ - mu1 * c1, phit = fma(mu1, ct1, Jt1);
                const double noise = 1.0 + fabs(phi0);
                // the line search's test at alpha = 1 (no filter clause after the first iteration)
                if (!(dphi >= -1e-11 * noise || phit <= phi0 + 1e-4 * dphi + 1e-13 * noise)) {
                    const int slot = atomicAdd(p.tail_count, 1);
                    if (slot < p.tail_slots) {
                        p.tail_idx[slot] = (int32_t)inst;
                        p.tail_it[slot] = it;
                        p.tail_mu[slot] = mu;
                        status = ST_HANDED_OVER;
                        break;
                    }
                    lean_off = true;
                }
            }
        }
        mu = fmax(mu, 4.0 * lmax + 1.0);
        const double phi0 = XB ? fma(mu, c1, fma(-2.0 * mub, lsum, J0)) : fma(mu, c1, J0);
        const double dphi = XB ? dJ + dbar - mu * c1 : dJ - mu * c1;
        double alpha = XB ? amax : 1.0;
        bool accepted = false;
        #pragma unroll 1
        for (int ls = 0; ls < 30; ++ls) {
            double Jt = 0.0, ct = 0.0, lt = 0.0, xk[NX], umt[NU], upf[NU], dupf[NU];
            if (FUSE_TRIAL && ls == 0) {   // alpha = 1: evaluated in the step sweep
                Jt = Jt1;
                ct = ct1;
            } else {
            if constexpr (LAZY) {
                if (!have_dxu) {   // the step sweep's du_k, dx_{k+1} again (its expressions, in its order), stored
                    double dx[NX], dup[NU];
#pragma unroll
                    for (int r = 0; r < NX; ++r) dx[r] = 0.0;
#pragma unroll
                    for (int c = 0; c < NU; ++c) dup[c] = 0.0;
                    #pragma unroll 1
                    for (int k = 0; k < N; ++k) {
                        gmem<double>* const sk = stage_ptr(wsb, k, SS, lane);
                        double x[NX], u[NU], xn[NX], xd[NX], du[NU], ad[NX];
#pragma unroll
                        for (int r = 0; r < NX; ++r) {
                            x[r] = SK(0, FX, r);
                            xn[r] = SK(1, FX, r);
                        }
#pragma unroll
                        for (int c = 0; c < NU; ++c) u[c] = SK(0, FU, c);
                        const gmem<double>* const kb = stage_ptr(wsb, k, SS, 0) + SF::K * 64;
                        const gmem<FT>* const kk = (const gmem<FT>*)(kb + NU * 64) + lane;
                        double dr[NU];
#pragma unroll
                        for (int c = 0; c < NU; ++c) dr[c] = KPACK ? R[c] * dup[c] : dup[c];
#pragma unroll
                        for (int a = 0; a < NU; ++a) {
                            double t = kb[a * 64 + lane];
#pragma unroll
                            for (int q = 0; q < NX; ++q) t = fma((double)kk[kgain_idx<NX, NU, KPACK>(a, q) * 64], dx[q], t);
#pragma unroll
                            for (int c = 0; c < NU; ++c) t = fma((double)kk[kgain_idx<NX, NU, KPACK>(a, NX + c) * 64], dr[c], t);
                            du[a] = t;
                            SK(0, SF::DU, a) = t;
                        }
                        if (JVP && !lin) {
                            double jv[NA];
                            model_jvp<Model>(x, u, dx, du, xd, jv);
                            jvp_step<NQ, NA>(h, dx, jv, ad);
                        } else {
                            double hFq[SQ], hFqd[NA * NA], hFu[NA * NU];
                            STAGE_EVAL(x, u, xd, hFq, hFqd, hFu, true);
                            a_mul<NQ, NA>(h, hFq, hFqd, dx, ad);
#pragma unroll
                            for (int s2 = 0; s2 < NA; ++s2)
#pragma unroll
                                for (int c = 0; c < NU; ++c) ad[NQ + s2] = fma(hFu[s2 * NU + c], du[c], ad[NQ + s2]);
                        }
#pragma unroll
                        for (int r = 0; r < NX; ++r) {
                            const double F = fma(h, xd[r], x[r]);
                            dx[r] = ad[r] + (F - xn[r]);
                            SK(1, SF::DX, r) = dx[r];
                        }
#pragma unroll
                        for (int c = 0; c < NU; ++c) dup[c] = du[c];
                    }
                    have_dxu = true;
                }
            }
#pragma unroll
            for (int r = 0; r < NX; ++r) xk[r] = ST(0, FX, r);  // dx_0 = 0
#pragma unroll
            for (int c = 0; c < NU; ++c) {
                umt[c] = up[c];
                upf[c] = ST(0, FU, c);
                dupf[c] = ST(0, SF::DU, c);
            }
            #pragma unroll 1
            for (int k = 0; k < N; ++k) {
                gmem<double>* const sk = stage_ptr(wsb, k, SS, lane);
                double u[NU], xn[NX], xd[NX], rk[NX];
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    u[c] = fma(alpha, dupf[c], upf[c]);
                    if (BOUNDED) u[c] = proj(u[c], lbv[c], ubv[c]);  // projected trial point
                    upf[c] = SK(1, FU, c);   // software pipeline as in (1)
                    dupf[c] = SK(1, SF::DU, c);
                }
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    xn[r] = fma(alpha, SK(1, SF::DX, r), SK(1, FX, r));
                    rk[r] = SK(0, SF::R, r);
                }
                {
                    double* nil_ = nullptr;
                    STAGE_EVAL(xk, u, xd, nil_, nil_, nil_, false);
                }
#pragma unroll
                for (int r = 0; r < NX; ++r) {
                    const double F = fma(h, xd[r], xk[r]);
                    const double er = F - rk[r];
                    Jt = fma(er * Q[r], er, Jt);
                    ct += fabs(F - xn[r]);
                    xk[r] = xn[r];
                }
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    const double dif = u[c] - umt[c];
                    Jt = fma(dif * R[c], dif, fma(u[c] * Rm[c], u[c], Jt));
                    umt[c] = u[c];
                }
                if constexpr (XB) {
#pragma unroll
                    for (int j = 0; j < NY; ++j) lt += ip_log_slacks(j < NX ? xn[j] : u[j - NX], yl[j], yu[j]);
                }
            }
            }
            const double phit = XB ? fma(mu, ct, fma(-2.0 * mub, lt, Jt)) : fma(mu, ct, Jt);
            const double noise = 1.0 + fabs(phi0);
            if (dphi >= -1e-11 * noise || phit <= phi0 + 1e-4 * alpha * dphi + 1e-13 * noise ||
                (!XB && it == 0 && first_iter_filter_accepts(J0, c1, Jt, ct, dJ, alpha))) {
                accepted = true;
                break;
            }
            alpha *= 0.5;
        }
        MMPC_PHASE(5);
        if (trc) {
            trc[4] = XB ? amax : dJ;
            trc[5] = alpha;
            trc[6] = XB ? mub : mu;
            if (XB) trc[3] = cmpl0;
        }
        if (!accepted) {
            status = ST_LS_FAILED;
            break;
        }
        if (FUSE_FWD && alpha == 1.0) {  // the step sweep already formed pass (1) at the new iterate
            fwd_ready = true;
            J0n = Jt1;
            c1n = ct1;
            cmaxn = cmt1;
            nfn = nft1;
        }
        if constexpr (XB) {  // y and the duals of stage k's (x_{k+1} | u_k), as oracle solve_one_ip
            #pragma unroll 1
            for (int k = 0; k < N; ++k) {
                gmem<double>* const sk = stage_ptr(wsb, k, SS, lane);
#pragma unroll
                for (int j = 0; j < NY; ++j) {
                    gmem<double>& y = j < NX ? SK(1, FX, j) : SK(0, FU, j - NX);
                    const double dy = j < NX ? SK(1, SF::DX, j) : SK(0, SF::DU, j - NX);
                    double zl = SK(0, SF::ZL, j), zu = SK(0, SF::ZU, j), yn;
                    ip_update(y, dy, yl[j], yu[j], zl, zu, mub, alpha, az, yn);
                    y = yn;
                    SK(0, SF::ZL, j) = zl;
                    SK(0, SF::ZU, j) = zu;
                }
            }
            mub = mub_next;
        } else if constexpr (SWAP) {
            // the other buffer holds the full-step point; after a shorter step it gets fma(alpha, d, v) instead
            if (alpha != 1.0) {
                #pragma unroll 1
                for (int k = 0; k <= N; ++k) {
                    gmem<double>* const sk = stage_ptr(wsb, k, SS, lane);
                    if (k > 0) {
#pragma unroll
                        for (int r = 0; r < NX; ++r) SK(0, FXo, r) = fma(alpha, SK(0, SF::DX, r), SK(0, FX, r));
                    }
                    if (k < N) {
#pragma unroll
                        for (int c = 0; c < NU; ++c) SK(0, FUo, c) = fma(alpha, SK(0, SF::DU, c), SK(0, FU, c));
                    }
                }
            }
            const int tx = FX, tu = FU;
            FX = FXo;
            FU = FUo;
            FXo = tx;
            FUo = tu;
        } else {
            #pragma unroll 1
            for (int k = 0; k <= N; ++k) {
                gmem<double>* const sk = stage_ptr(wsb, k, SS, lane);
                if (k > 0) {
#pragma unroll
                    for (int r = 0; r < NX; ++r) SK(0, FX, r) = fma(alpha, SK(0, SF::DX, r), SK(0, FX, r));
                }
                if (k < N) {
#pragma unroll
                    for (int c = 0; c < NU; ++c) {
                        const double un = fma(alpha, SK(0, SF::DU, c), SK(0, FU, c));
                        SK(0, FU, c) = BOUNDED ? proj(un, lbv[c], ubv[c]) : un;
                    }
                }
            }
        }
    }

    MMPC_PHASE(6);
    // ---- write back V (reference layout) ----
    double* Vout = p.V + inst * (int64_t)NV;
    for (int k0 = 0; k0 < N; k0 += LB) {   // LB stages loaded before they are stored (see the load phase)
        double v[LB][ND];
#pragma unroll
        for (int j = 0; j < LB; ++j) {
            const int k = k0 + j < N ? k0 + j : N - 1;
#pragma unroll
            for (int r = 0; r < NX; ++r) v[j][r] = ST(k, FX, r);
#pragma unroll
            for (int c = 0; c < NU; ++c) v[j][NX + c] = ST(k, FU, c);
        }
#pragma unroll
        for (int j = 0; j < LB; ++j)
            if (k0 + j < N)
#pragma unroll
                for (int e = 0; e < ND; ++e) Vout[(k0 + j) * ND + e] = v[j][e];
    }
#pragma unroll
    for (int r = 0; r < NX; ++r) Vout[N * ND + r] = ST(N, FX, r);
    if (p.u0_out) {
#pragma unroll
        for (int c = 0; c < NU; ++c) p.u0_out[inst * NU + c] = ST(0, FU, c);
    }
    if (p.status) p.status[inst] = status;
    if (p.iters) p.iters[inst] = it;
    if (p.kkt) p.kkt[inst] = kkt;
    MMPC_PHASE(7);
    MMPC_PHASE_FLUSH
#undef ST
#undef SK
#undef PS
#undef STAGE_EVAL
}

}  // namespace mmpc
