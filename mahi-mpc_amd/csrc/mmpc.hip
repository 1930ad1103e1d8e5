// mmpc.hip -- C-ABI (include/mmpc.h) of the MI355X batched NMPC solve path.
//
// Host side of the drop-in boundary: loads the reference's <name>.json model file
// (src/Mahi/Mpc/ModelParameters.cpp:52-72 semantics), validates every launch shape on
// the host, and launches the gfx950 kernels of sqp_wave.h / below.  No CPU fallback
// exists: every compute entry point runs on the GPU or returns an error.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <mutex>
#include <thread>
#include <sstream>
#include <string>
#include <type_traits>
#include <vector>

#include <dlfcn.h>
#include <rccl/rccl.h>   // types and enums only: RCCL itself is loaded with dlopen at the first RCCL call

#include "../../include/mmpc.h"
#include "json_lite.h"
#include "group_launch.h"
#include "lane_launch.h"
#include "models.h"
#include "sqp_group.h"
#include "sqp_lane.h"
#include "sqp_wave.h"

// A library built by ModelGenerator::compile_model for SX-defined dynamics (mahi-mpc's <name>.so,
// ModelGenerator.cpp:254-259) compiles this same file with -DMMPC_USER_MODEL_HEADER="<name>_model.h", which
// defines mmpc::UserModel; it then serves that one model (MMPC_MODEL_USER) and none of the built-in ones.
#ifdef MMPC_USER_MODEL_HEADER
#include MMPC_USER_MODEL_HEADER
#define MMPC_BUILTIN_MODELS 0
#else
#define MMPC_BUILTIN_MODELS 1
#endif

using namespace mmpc;

// ---------------------------------------------------------------- errors
namespace {
thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}
int hip_fail(hipError_t e, const char* where) {
    return fail(MMPC_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}
#define MMPC_HIP(call)                                    \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return hip_fail(e_, #call); \
    } while (0)
}  // namespace

// ---------------------------------------------------------------- handle
struct mmpc_handle {
    mmpc_model_info info;
    int nq = 0;  // kinematic rows of the model's dynamics (sqp_lane.h a_mul)
    mmpc_opts opts;
    std::mutex host_mu;  // serialises the *_host entry points
    hipStream_t host_stream = nullptr;
    int host_dev = -1;
    // device staging for the *_host entry points (grown on demand)
    double* d_buf = nullptr;
    size_t d_buf_bytes = 0;
    // Riccati solver workspace (SoA, sqp_lane.h LaneLayout), grown on demand
    std::mutex ws_mu;
    double* ws = nullptr;
    size_t ws_bytes = 0;
    int ws_dev = -1;
    // iteration-tail hand-over: cap override from MMPC_TAIL_CAP at creation (-1: the default policy),
    // compute units of the device (slots of the resume launch)
    int tail_cap_env = -1;      // MMPC_TAIL_CAP (test / A/B override of opts.tail_cap; -1: not set)
    int tail_wave_env = -1;     // MMPC_TAIL_WAVE (override of opts.tail_wave_max)
    int tail_rounds_env = -1;   // MMPC_TAIL_ROUNDS (override of opts.tail_rounds)
    int cu_count = 0;
    // state bounds of x_1..x_N (JSON x_min/x_max, or mmpc_set_state_bounds); copied into each launch's arguments
    double x_lb[16], x_ub[16];
    bool x_bounded = false;
    std::mutex xb_mu;
};

namespace {

struct DeviceGuard {
    int prev = -1;
    bool changed = false;
    int err = 0;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) {
            err = 1;
            return;
        }
        if (dev >= 0 && dev != prev) {
            if (hipSetDevice(dev) != hipSuccess) {
                err = 1;
                return;
            }
            changed = true;
        }
    }
    ~DeviceGuard() {
        if (changed) (void)hipSetDevice(prev);
    }
};

int parse_model(const std::string& text, mmpc_model_info* info) {
    json::Value root;
    try {
        root = json::parse(text);
    } catch (const std::exception& ex) {
        return fail(MMPC_ERR_PARSE, ex.what());
    }
    const json::Value* m = root.get("model");  // ModelGenerator.cpp:264 writes j["model"]
    if (!m) m = &root;
    if (m->kind != json::Value::Object) return fail(MMPC_ERR_PARSE, "model entry is not an object");
    auto num = [&](const char* k, double* out) -> bool {
        const json::Value* v = m->get(k);
        if (!v || v->kind != json::Value::Number) return false;
        *out = v->num;
        return true;
    };
    std::memset(info, 0, sizeof(*info));
    const json::Value* nm = m->get("name");
    if (!nm || nm->kind != json::Value::String) return fail(MMPC_ERR_PARSE, "missing \"name\"");
    std::snprintf(info->name, sizeof(info->name), "%s", nm->str.c_str());
    double nx, nu, N, step_us, span_us = 0.0;
    if (!num("num_x", &nx) || !num("num_u", &nu) || !num("num_shooting_nodes", &N) || !num("step_size", &step_us))
        return fail(MMPC_ERR_PARSE, "missing num_x / num_u / num_shooting_nodes / step_size");
    num("timespan", &span_us);
    info->num_x = static_cast<int32_t>(nx);
    info->num_u = static_cast<int32_t>(nu);
    info->num_shooting_nodes = static_cast<int32_t>(N);
    if (info->num_x < 1 || info->num_x > 16 || info->num_u < 1 || info->num_u > 16 || info->num_shooting_nodes < 1)
        return fail(MMPC_ERR_PARSE, "num_x / num_u / num_shooting_nodes out of range");
    info->step_size_us = static_cast<int64_t>(std::llround(step_us));
    info->timespan_us = static_cast<int64_t>(std::llround(span_us));
    info->step_size = step_us * 1e-6;  // mahi::util::microseconds(j.at("step_size"))
    info->num_v = info->num_x * (info->num_shooting_nodes + 1) + info->num_u * info->num_shooting_nodes;
    info->num_g = info->num_x * info->num_shooting_nodes;
    const json::Value* lin = m->get("is_linear");
    info->is_linear = (lin && lin->kind == json::Value::Bool && lin->b) ? 1 : 0;
    // bounds: default +-10e30 (ModelParameters.cpp:21-24); x bounds of exactly +-10e30 become +-inf on
    // load (ModelParameters.cpp:66-69); nlohmann writes +-inf as null, read back here as unbounded.
    auto bounds = [&](const char* k, double* out, int n, double dflt, bool inf_map) -> int {
        for (int i = 0; i < n; ++i) out[i] = dflt;
        const json::Value* v = m->get(k);
        if (!v || v->kind == json::Value::Null) return 0;
        if (v->kind != json::Value::Array) return fail(MMPC_ERR_PARSE, std::string(k) + " is not an array");
        if (static_cast<int>(v->arr.size()) != n && !v->arr.empty())
            return fail(MMPC_ERR_PARSE, std::string(k) + " has the wrong length");
        for (size_t i = 0; i < v->arr.size(); ++i) {
            const json::Value& e = v->arr[i];
            if (e.kind == json::Value::Null) out[i] = dflt;
            else if (e.kind == json::Value::Number) out[i] = e.num;
            else return fail(MMPC_ERR_PARSE, std::string(k) + " has a non-number entry");
            if (inf_map && std::fabs(out[i]) == 10e30) out[i] = std::copysign(INFINITY, out[i]);
        }
        return 0;
    };
    int rc;
    if ((rc = bounds("x_min", info->x_min, info->num_x, -INFINITY, true))) return rc;
    if ((rc = bounds("x_max", info->x_max, info->num_x, INFINITY, true))) return rc;
    if ((rc = bounds("u_min", info->u_min, info->num_u, -10e30, false))) return rc;
    if ((rc = bounds("u_max", info->u_max, info->num_u, 10e30, false))) return rc;
    // dynamics: explicit "mmpc_model" key, else the only built-in model with these dimensions
    const json::Value* mdl = m->get("mmpc_model");
#if !MMPC_BUILTIN_MODELS
    // a generated library serves exactly its own model
    if (mdl && mdl->kind == json::Value::String && mdl->str != UserModel::kName)
        return fail(MMPC_ERR_UNSUPPORTED, "this library was generated for model \"" + std::string(UserModel::kName) +
                                              "\", not \"" + mdl->str + "\"");
    if (info->num_x != UserModel::NX || info->num_u != UserModel::NU)
        return fail(MMPC_ERR_PARSE, "num_x / num_u differ from the generated model's dimensions");
    info->model_id = MMPC_MODEL_USER;
    return MMPC_OK;
#endif
    if (mdl && mdl->kind == json::Value::String) {
        if (mdl->str == "two_link_arm" || mdl->str == "double_pendulum") info->model_id = MMPC_MODEL_TWO_LINK_ARM;
        else if (mdl->str == "exo_arm" || mdl->str == "exo") info->model_id = MMPC_MODEL_EXO_ARM;
        else return fail(MMPC_ERR_UNSUPPORTED, "unknown mmpc_model \"" + mdl->str + "\"");
    } else if (info->num_x == 4 && info->num_u == 2) {
        info->model_id = MMPC_MODEL_TWO_LINK_ARM;
    } else if (info->num_x == 8 && info->num_u == 4) {
        info->model_id = MMPC_MODEL_EXO_ARM;
    } else {
        return fail(MMPC_ERR_UNSUPPORTED, "no built-in dynamics for these dimensions (set \"mmpc_model\")");
    }
    if (info->model_id == MMPC_MODEL_TWO_LINK_ARM && (info->num_x != 4 || info->num_u != 2))
        return fail(MMPC_ERR_PARSE, "two_link_arm needs num_x = 4, num_u = 2");
    if (info->model_id == MMPC_MODEL_EXO_ARM && (info->num_x != 8 || info->num_u != 4))
        return fail(MMPC_ERR_PARSE, "exo_arm needs num_x = 8, num_u = 4");
    return MMPC_OK;
}

int validate_opts(const mmpc_opts* o) {
    if (o->max_iter < 0 || o->max_iter > 100000) return fail(MMPC_ERR_INVALID_ARG, "max_iter out of range");
    if (!(o->tol_grad > 0.0) || !(o->tol_defect > 0.0)) return fail(MMPC_ERR_INVALID_ARG, "tolerances must be > 0");
    if (o->kkt_solver < MMPC_KKT_AUTO || o->kkt_solver > MMPC_KKT_RICCATI_GROUP)
        return fail(MMPC_ERR_INVALID_ARG, "unknown kkt_solver");
    if (o->factor_fp32 != 0 && o->factor_fp32 != 1) return fail(MMPC_ERR_INVALID_ARG, "factor_fp32 must be 0 or 1");
    if (o->init_states != MMPC_INIT_AS_GIVEN && o->init_states != MMPC_INIT_HOLD_X0 && o->init_states != MMPC_INIT_ZERO)
        return fail(MMPC_ERR_INVALID_ARG, "unknown init_states");
    if (o->hessian < MMPC_HESSIAN_AUTO || o->hessian > MMPC_HESSIAN_EXACT)
        return fail(MMPC_ERR_INVALID_ARG, "unknown hessian");
    if (o->tail_cap < -1 || o->tail_cap >= 1000) return fail(MMPC_ERR_INVALID_ARG, "tail_cap must be -1 .. 999");
    if (o->tail_wave_max < -1 || o->tail_wave_max > 64)
        return fail(MMPC_ERR_INVALID_ARG, "tail_wave_max must be -1 .. 64");
    if (o->tail_rounds < -1 || o->tail_rounds == 0 || o->tail_rounds >= 1000)
        return fail(MMPC_ERR_INVALID_ARG, "tail_rounds must be -1 or 1 .. 999");
    return MMPC_OK;
}

int resolve_device(mmpc_handle* h, int* dev) {
    if (h->opts.device >= 0) {
        *dev = h->opts.device;
        return MMPC_OK;
    }
    int d = -1;
    hipError_t e = hipGetDevice(&d);
    if (e != hipSuccess) return fail(MMPC_ERR_NO_DEVICE, std::string("no HIP device: ") + hipGetErrorString(e));
    *dev = d;
    return MMPC_OK;
}

// ---------------------------------------------------------------- auxiliary kernels
template <class Model>
__global__ __launch_bounds__(256) void linearize_kernel(int64_t B, const double* __restrict__ x,
                                                        const double* __restrict__ u, double* A, double* Bm,
                                                        double* xdot) {
    constexpr int NX = Model::NX, NU = Model::NU;
    const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (b >= B) return;
    double xv[NX], uv[NU], xd[NX], fx[NX * NX], fu[NX * NU];
#pragma unroll
    for (int i = 0; i < NX; ++i) xv[i] = x[b * NX + i];
#pragma unroll
    for (int i = 0; i < NU; ++i) uv[i] = u[b * NU + i];
    model_eval_jac<Model>(xv, uv, xd, fx, fu);
    // column-major, as CasADi DM -> std::vector (ModelControl.cpp:127-129)
#pragma unroll
    for (int r = 0; r < NX; ++r) {
        if (xdot) xdot[b * NX + r] = xd[r];
#pragma unroll
        for (int c = 0; c < NX; ++c)
            if (A) A[b * NX * NX + c * NX + r] = fx[r * NX + c];
#pragma unroll
        for (int c = 0; c < NU; ++c)
            if (Bm) Bm[b * NX * NU + c * NX + r] = fu[r * NU + c];
    }
}

template <class Model>
__global__ __launch_bounds__(256) void nlp_eval_kernel(int64_t B, int N, double h, int is_linear,
                                                       const double* __restrict__ V, const double* __restrict__ u_prev,
                                                       const double* __restrict__ traj,
                                                       const double* __restrict__ weights, int64_t w_stride,
                                                       double* J, double* ginf) {
    constexpr int NX = Model::NX, NU = Model::NU, ND = NX + NU;
    const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int NV = NX * (N + 1) + NU * N;
    const double* v = V + b * NV;
    const double* w = weights + b * w_stride;
    const double* up = u_prev + b * NU;
    const double* tr = traj + b * (int64_t)N * NX;
    double lin[NX * NX + NX * NU + NX];
    if (is_linear) {  // F_lin at (x*, u*) = (x_0, u_prev), ModelGenerator.cpp:47-48
        double xd[NX], fx[NX * NX], fu[NX * NU];
        model_eval_jac<Model>(v, up, xd, fx, fu);
        for (int i = 0; i < NX * NX; ++i) lin[i] = fx[i];
        for (int i = 0; i < NX * NU; ++i) lin[NX * NX + i] = fu[i];
        for (int i = 0; i < NX; ++i) lin[NX * NX + NX * NU + i] = xd[i];
    }
    double Jv = 0.0, gm = 0.0;
    for (int k = 0; k < N; ++k) {
        const double* xk = v + k * ND;
        const double* uk = xk + NX;
        double xd[NX];
        if (!is_linear) {
            model_eval<Model>(xk, uk, xd);
        } else {
            for (int r = 0; r < NX; ++r) {
                double s = lin[NX * NX + NX * NU + r];
                for (int c = 0; c < NX; ++c) s += lin[r * NX + c] * (xk[c] - v[c]);
                for (int c = 0; c < NU; ++c) s += lin[NX * NX + r * NU + c] * (uk[c] - up[c]);
                xd[r] = s;
            }
        }
        for (int r = 0; r < NX; ++r) {
            const double F = xk[r] + h * xd[r];
            const double e = F - tr[k * NX + r];
            Jv += e * w[r] * e;
            const double gk = F - v[(k + 1) * ND + r];
            gm = (std::fabs(gk) > gm || gk != gk) ? std::fabs(gk) : gm;
        }
        for (int c = 0; c < NU; ++c) {
            const double um = (k == 0) ? up[c] : v[(k - 1) * ND + NX + c];
            const double du = uk[c] - um;
            Jv += du * w[NX + c] * du + uk[c] * w[NX + NU + c] * uk[c];
        }
    }
    if (J) J[b] = Jv;
    if (ginf) ginf[b] = gm;
}

// nlp_grad_f / nlp_jac_g of the generated NLP (ModelGenerator.cpp:238, CasADi generate_dependencies): per
// instance J, dJ/dV [NV] (V layout) and the nonzero blocks of dg/dV, [dg_k/dx_k | dg_k/du_k] = [I + h f_x | h f_u]
// (row-major nx x (nx+nu) per stage; dg_k/dx_{k+1} = -I).  Linear mode: F_lin with A*, B* at (x_0, u_prev).
template <class Model>
__global__ __launch_bounds__(256) void nlp_derivs_kernel(int64_t B, int N, double h, int is_linear,
                                                         const double* __restrict__ V, const double* __restrict__ u_prev,
                                                         const double* __restrict__ traj,
                                                         const double* __restrict__ weights, int64_t w_stride,
                                                         double* J, double* grad, double* jac_blocks) {
    constexpr int NX = Model::NX, NU = Model::NU, ND = NX + NU;
    const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int NV = NX * (N + 1) + NU * N;
    const double* v = V + b * NV;
    const double* w = weights + b * w_stride;
    const double* up = u_prev + b * NU;
    const double* tr = traj + b * (int64_t)N * NX;
    double* gr = grad ? grad + b * NV : nullptr;
    double lin[NX * NX + NX * NU + NX];
    if (is_linear) {
        double xd[NX], fx[NX * NX], fu[NX * NU];
        model_eval_jac<Model>(v, up, xd, fx, fu);
        for (int i = 0; i < NX * NX; ++i) lin[i] = fx[i];
        for (int i = 0; i < NX * NU; ++i) lin[NX * NX + i] = fu[i];
        for (int i = 0; i < NX; ++i) lin[NX * NX + NX * NU + i] = xd[i];
    }
    double Jv = 0.0;
    if (gr)
        for (int r = 0; r < NX; ++r) gr[N * ND + r] = 0.0;  // x_N does not enter J
    for (int k = 0; k < N; ++k) {
        const double* xk = v + k * ND;
        const double* uk = xk + NX;
        double xd[NX], fx[NX * NX], fu[NX * NU];
        if (!is_linear) {
            model_eval_jac<Model>(xk, uk, xd, fx, fu);
        } else {
            for (int r = 0; r < NX; ++r) {
                double s = lin[NX * NX + NX * NU + r];
                for (int c = 0; c < NX; ++c) s += lin[r * NX + c] * (xk[c] - v[c]);
                for (int c = 0; c < NU; ++c) s += lin[NX * NX + r * NU + c] * (uk[c] - up[c]);
                xd[r] = s;
            }
            for (int i = 0; i < NX * NX; ++i) fx[i] = lin[i];
            for (int i = 0; i < NX * NU; ++i) fu[i] = lin[NX * NX + i];
        }
        double qe[NX];
        for (int r = 0; r < NX; ++r) {
            const double e = xk[r] + h * xd[r] - tr[k * NX + r];
            Jv += e * w[r] * e;
            qe[r] = 2.0 * w[r] * e;
        }
        if (jac_blocks) {
            double* jb = jac_blocks + (b * N + k) * (int64_t)(NX * ND);
            for (int r = 0; r < NX; ++r) {
                for (int c = 0; c < NX; ++c) jb[r * ND + c] = (r == c ? 1.0 : 0.0) + h * fx[r * NX + c];
                for (int c = 0; c < NU; ++c) jb[r * ND + NX + c] = h * fu[r * NU + c];
            }
        }
        for (int c = 0; c < NU; ++c) {
            const double um = (k == 0) ? up[c] : v[(k - 1) * ND + NX + c];
            const double du = uk[c] - um;
            Jv += du * w[NX + c] * du + uk[c] * w[NX + NU + c] * uk[c];
        }
        if (gr) {
            for (int c = 0; c < NX; ++c) {  // dJ/dx_k = 2 (I + h f_x)^T Q e_k
                double t = qe[c];
                for (int r = 0; r < NX; ++r) t += h * fx[r * NX + c] * qe[r];
                gr[k * ND + c] = t;
            }
            for (int c = 0; c < NU; ++c) {  // dJ/du_k = 2 h f_u^T Q e_k + Delta-u and Rm terms
                double t = 0.0;
                for (int r = 0; r < NX; ++r) t += h * fu[r * NU + c] * qe[r];
                const double um = (k == 0) ? up[c] : v[(k - 1) * ND + NX + c];
                t += 2.0 * w[NX + c] * (uk[c] - um) + 2.0 * w[NX + NU + c] * uk[c];
                if (k + 1 < N) t -= 2.0 * w[NX + c] * (v[(k + 1) * ND + NX + c] - uk[c]);
                gr[k * ND + NX + c] = t;
            }
        }
    }
    if (J) J[b] = Jv;
}

// nlp_hess_l of the generated NLP (ModelGenerator.cpp:238; CasADi's Hessian of the Lagrangian
// lam_f J + lam_g^T g): the nonzero stage blocks, one thread per (instance, stage).  Block k on (x_k, u_k) [K x K]:
//   lam_f [2 J_Fk^T Q J_Fk + blkdiag(0, 2R + 2Rm (+ 2R for k + 1 < N))] + h sum_r nu_r d^2 f_r/d(x_k,u_k)^2,
//   nu = 2 lam_f Q e_k + lam_g,k,  J_Fk = [I + h f_x | h f_u],  e_k = F(x_k,u_k) - r_k;
// the other nonzeros are constant (d^2/du_k du_{k-1} = -2 lam_f R) and x_N enters L linearly.
template <class Model>
__global__ __launch_bounds__(256) void nlp_hess_kernel(int64_t B, int N, double h, int is_linear,
                                                       const double* __restrict__ V, const double* __restrict__ u_prev,
                                                       const double* __restrict__ traj,
                                                       const double* __restrict__ weights, int64_t w_stride,
                                                       double lam_f, const double* __restrict__ lam_g, double* blocks) {
    constexpr int NX = Model::NX, NU = Model::NU, ND = NX + NU, NQ = Model::NQ, NA = NX - NQ;
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= B * N) return;
    const int64_t b = t / N;
    const int k = static_cast<int>(t - b * N);
    const int NV = NX * (N + 1) + NU * N;
    const double* v = V + b * NV;
    const double* w = weights + b * w_stride;
    const double* up = u_prev + b * NU;
    const double* xk = v + k * ND;
    const double* uk = xk + NX;
    double xd[NX], fx[NX * NX], fu[NX * NU];
    if (!is_linear) {
        model_eval_jac<Model>(xk, uk, xd, fx, fu);
    } else {   // F_lin: A*, B*, xdot* at (x_0, u_prev)
        double xs[NX], fxs[NX * NX], fus[NX * NU];
        model_eval_jac<Model>(v, up, xs, fxs, fus);
        for (int r = 0; r < NX; ++r) {
            double s = xs[r];
            for (int c = 0; c < NX; ++c) s += fxs[r * NX + c] * (xk[c] - v[c]);
            for (int c = 0; c < NU; ++c) s += fus[r * NU + c] * (uk[c] - up[c]);
            xd[r] = s;
        }
        for (int i = 0; i < NX * NX; ++i) fx[i] = fxs[i];
        for (int i = 0; i < NX * NU; ++i) fu[i] = fus[i];
    }
    double JF[NX][ND], nu[NX];
    for (int r = 0; r < NX; ++r) {
        for (int c = 0; c < NX; ++c) JF[r][c] = (r == c ? 1.0 : 0.0) + h * fx[r * NX + c];
        for (int c = 0; c < NU; ++c) JF[r][NX + c] = h * fu[r * NU + c];
        const double e = xk[r] + h * xd[r] - traj[(b * N + k) * NX + r];
        nu[r] = 2.0 * lam_f * w[r] * e + (lam_g ? lam_g[b * (int64_t)N * NX + k * NX + r] : 0.0);
    }
    double W[ND * ND];
    for (int i = 0; i < ND * ND; ++i) W[i] = 0.0;
    if constexpr (HasHess<Model>::value) {
        if (!is_linear) {
            double la[NA];
            for (int s2 = 0; s2 < NA; ++s2) la[s2] = h * nu[NQ + s2];
            Model::eval_hess(xk, uk, la, W);
        }
    }
    double* out = blocks + t * (int64_t)(ND * ND);
    for (int i = 0; i < ND; ++i)
        for (int j = i; j < ND; ++j) {   // upper triangle, mirrored: the block is symmetric bit for bit
            double s = W[i * ND + j];
            for (int r = 0; r < NX; ++r) s += 2.0 * lam_f * w[r] * JF[r][i] * JF[r][j];
            if (i == j && i >= NX) {
                const int c = i - NX;
                s += lam_f * (2.0 * w[NX + c] + 2.0 * w[NX + NU + c] + (k + 1 < N ? 2.0 * w[NX + c] : 0.0));
            }
            out[i * ND + j] = s;
            out[j * ND + i] = s;
        }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ double unit_draw(uint64_t seed, int64_t index, int j) {
    const uint64_t v = splitmix64(seed ^ splitmix64((uint64_t)index * 16ull + (uint64_t)j));
    return (double)(v >> 11) * 0x1.0p-53;
}

// lo + span*u with an unfused product (bit-identical to the oracle's and make_golden.py's generator)
__device__ __forceinline__ double affine_draw(double lo, double span, double u) {
#pragma clang fp contract(off)
    const double p = span * u;
    return lo + p;
}

// SURVEY.md 8d instance generators (identical recipes in oracle/mmpc_oracle.c and tests/golden/).  bench.py generates
// every step's instances inside its clock, so they are built for throughput: a 256-thread block takes
// I = max(1, 256 / N) instances; its threads first form the instances' unit draws (each exactly once, into LDS; the
// x0 / u_prev draws go straight to memory), then one thread per (instance, stage) forms that stage's targets (sin /
// cos of the phase, stores contiguous across the block).  Round 4 ran one thread per instance (30-50 sin / cos in
// series, strided stores, 16 CUs busy at cfg#2: 12.3 us per batch); a first round-5 version redrew every instance's
// parameters in each stage's thread (5.2 us at cfg#2 but 165 us at cfg#3: the 64-bit multiplies of splitmix64).
// The phase argument is formed without FMA contraction, as the C oracle.
// Round 6: the block's target rows (I N nx doubles, contiguous in traj) are staged in LDS and written out with
// consecutive lanes on consecutive doubles: one thread per stage wrote its row with nx stores of 8 bytes at a 64-byte
// lane stride (8 cache-line segments per store instruction; 131 us per cfg#3 batch).  N <= 256 always fits (I N <= 256).
constexpr int kSynthThreads = 256;
constexpr int kSynthStaged = 2048;   // doubles of LDS for the staged rows

// cfg#2: q ~ U[-pi/4, pi/4], qdot ~ U[-1, 1], u_prev ~ U[-5, 5]; a ~ U[0.5, 1], f ~ U[0.25, 1] Hz, phase ~ U[0, 2 pi];
// r_k = [a sin(2 pi f t_k + phase), -a sin(.), 2 pi f a cos(.), -2 pi f a cos(.)], t_k = k h
__global__ __launch_bounds__(kSynthThreads) void synth_two_link_kernel(uint64_t seed, int64_t first, int64_t B, int N,
                                                                       double h, double* x0, double* u_prev,
                                                                       double* traj) {
    constexpr int ND = 9;   // draws per instance: x0 (4), u_prev (2), a, f, phase
    __shared__ double dr[kSynthThreads][3];
    const int I = N < kSynthThreads ? kSynthThreads / N : 1;
    const int64_t b0 = (int64_t)blockIdx.x * I;
    const double PI = 3.14159265358979323846;
    for (int t = threadIdx.x; t < I * ND; t += kSynthThreads) {
        const int i = t / ND, j = t - i * ND;
        const int64_t b = b0 + i;
        if (b >= B) continue;
        const double u = unit_draw(seed, first + b, j);
        if (j < 2) x0[b * 4 + j] = affine_draw(-PI / 4, PI / 2, u);
        else if (j < 4) x0[b * 4 + j] = affine_draw(-1.0, 2.0, u);
        else if (j < 6) u_prev[b * 2 + j - 4] = affine_draw(-5.0, 10.0, u);
        else if (j == 6) dr[i][0] = affine_draw(0.5, 0.5, u);
        else if (j == 7) dr[i][1] = affine_draw(0.25, 0.75, u);
        else dr[i][2] = affine_draw(0.0, 2.0 * PI, u);
    }
    __syncthreads();
    __shared__ double so[kSynthStaged];
    const bool staged = I * N * 4 <= kSynthStaged;
    for (int t = threadIdx.x; t < I * N; t += kSynthThreads) {
        const int i = t / N, k = t - i * N;
        const int64_t b = b0 + i;
        if (b >= B) continue;
        const double a = dr[i][0], f = dr[i][1], ph = dr[i][2];
        double arg, cs;
        {
#pragma clang fp contract(off)
            arg = 2.0 * PI * f * (k * h) + ph;
            cs = 2.0 * PI * f * a;
        }
        double sn, cn;
        sincos(arg, &sn, &cn);   // one argument reduction for both (the device library's sin and cos values)
        const double sv = a * sn, cv = cs * cn;
        double* r = staged ? so + t * 4 : traj + (b * N + k) * 4;
        r[0] = sv;
        r[1] = -sv;
        r[2] = cv;
        r[3] = -cv;
    }
    if (staged) {   // the block's rows are contiguous in traj: coalesced copy-out
        __syncthreads();
        const int64_t nb = B - b0 < I ? B - b0 : I;
        double* const dst = traj + b0 * N * 4;
        for (int t = threadIdx.x; t < nb * N * 4; t += kSynthThreads) dst[t] = so[t];
    }
}

// cfg#3: q, qd ~ U[-0.5, 0.5], tau_prev ~ U[-1, 1], per joint a ~ U[0.1, 0.4], f ~ U[0.25, 1] Hz, phase ~ U[0, 2 pi];
// r_k = [a sin(2 pi f t_k + phase); 2 pi f a cos(2 pi f t_k + phase)], t_k = k h
__device__ __forceinline__ double unit_draw_exo(uint64_t seed, int64_t index, int j) {
    const uint64_t v = splitmix64((seed + 0x3C6EF372FE94F82Aull) ^ splitmix64((uint64_t)index * 32ull + (uint64_t)j));
    return (double)(v >> 11) * 0x1.0p-53;
}
__global__ __launch_bounds__(kSynthThreads) void synth_exo_kernel(uint64_t seed, int64_t first, int64_t B, int N,
                                                                  double h, double* x0, double* u_prev, double* traj) {
    constexpr int ND = 24;   // draws per instance: x0 (8), u_prev (4), per joint a, f, phase (12)
    __shared__ double dr[kSynthThreads][12];
    const int I = N < kSynthThreads ? kSynthThreads / N : 1;
    const int64_t b0 = (int64_t)blockIdx.x * I;
    const double PI = 3.14159265358979323846;
    for (int t = threadIdx.x; t < I * ND; t += kSynthThreads) {
        const int i = t / ND, j = t - i * ND;
        const int64_t b = b0 + i;
        if (b >= B) continue;
        const double u = unit_draw_exo(seed, first + b, j);
        if (j < 8) x0[b * 8 + j] = affine_draw(-0.5, 1.0, u);
        else if (j < 12) u_prev[b * 4 + j - 8] = affine_draw(-1.0, 2.0, u);
        else if (j < 16) dr[i][j - 12] = affine_draw(0.1, 0.3, u);
        else if (j < 20) dr[i][j - 12] = affine_draw(0.25, 0.75, u);
        else dr[i][j - 12] = affine_draw(0.0, 2.0 * PI, u);
    }
    __syncthreads();
    __shared__ double so[kSynthStaged];
    const bool staged = I * N * 8 <= kSynthStaged;
    for (int t = threadIdx.x; t < I * N; t += kSynthThreads) {
        const int i = t / N, k = t - i * N;
        const int64_t b = b0 + i;
        if (b >= B) continue;
        double* r = staged ? so + t * 8 : traj + (b * N + k) * 8;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double a = dr[i][j], f = dr[i][4 + j], ph = dr[i][8 + j];
            double arg, cs;
            {
#pragma clang fp contract(off)
                arg = 2.0 * PI * f * (k * h) + ph;
                cs = 2.0 * PI * f * a;
            }
            double sn, cn;
            sincos(arg, &sn, &cn);
            r[j] = a * sn;
            r[4 + j] = cs * cn;
        }
    }
    if (staged) {   // the block's rows are contiguous in traj: coalesced copy-out
        __syncthreads();
        const int64_t nb = B - b0 < I ? B - b0 : I;
        double* const dst = traj + b0 * N * 8;
        for (int t = threadIdx.x; t < nb * N * 8; t += kSynthThreads) dst[t] = so[t];
    }
}

inline unsigned grid1d(int64_t B, int threads) { return static_cast<unsigned>((B + threads - 1) / threads); }
// blocks of the instance generators: I = max(1, kSynthThreads / N) instances per block
inline unsigned synth_blocks(int64_t B, int N) {
    const int64_t I = N < kSynthThreads ? kSynthThreads / N : 1;
    return static_cast<unsigned>((B + I - 1) / I);
}

// Calls f((Model*)nullptr) for the model compiled into this library under model_id.
template <class F>
int with_model(int model_id, F&& f) {
#if MMPC_BUILTIN_MODELS
    if (model_id == MMPC_MODEL_TWO_LINK_ARM) return f(static_cast<TwoLinkArm*>(nullptr));
    if (model_id == MMPC_MODEL_EXO_ARM) return f(static_cast<ExoArm*>(nullptr));
#else
    if (model_id == MMPC_MODEL_USER) return f(static_cast<UserModel*>(nullptr));
#endif
    return fail(MMPC_ERR_UNSUPPORTED, "model not compiled into this library");
}
int model_nq(int model_id) {
    int nq = 0;
    with_model(model_id, [&](auto* m) {
        nq = std::remove_pointer_t<decltype(m)>::NQ;
        return MMPC_OK;
    });
    return nq;
}

size_t workspace_bytes(const mmpc_model_info& mi, int nq, int64_t B, bool xb = true) {
    const int64_t blocks = (B + 63) / 64;
    return static_cast<size_t>(lane_ws_doubles(mi.num_x, mi.num_u, nq, mi.num_shooting_nodes, xb)) * 64u *
           static_cast<size_t>(blocks) * sizeof(double);
}

size_t group_workspace_bytes(const mmpc_model_info& mi, int64_t B) {   // the largest variant's (bounded or xb)
    const int nx = mi.num_x, nu = mi.num_u, N = mi.num_shooting_nodes;
    const int per = std::max(group_ws_doubles(nx, nu, N, true, false), group_ws_doubles(nx, nu, N, false, true));
    return static_cast<size_t>(per) * static_cast<size_t>(B) * sizeof(double);
}
size_t group_lds_bytes(const mmpc_model_info& mi, int nq, bool bounded = true, bool xb = false) {
    return static_cast<size_t>(group_lds_doubles(mi.num_x, mi.num_u, nq, mi.num_shooting_nodes, bounded && !xb,
                                                 mi.is_linear != 0, xb)) * kGroupsPerWave *
           sizeof(double);
}
constexpr size_t kMaxGroupLds = 160 * 1024;  // gfx950: 160 KB of LDS per workgroup (attribute raised above 64 KB)

template <class K>
int set_dynamic_lds(K kernel, size_t bytes) {
    if (bytes <= 64 * 1024) return MMPC_OK;
    MMPC_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                 static_cast<int>(bytes)));
    return MMPC_OK;
}

// the KKT solver a solve of B instances runs (opts.kkt_solver, or the AUTO choice)
int resolve_kkt_solver_base(const mmpc_handle* h, int64_t B);
int resolve_kkt_solver(const mmpc_handle* h, int64_t B) {
    const int s = resolve_kkt_solver_base(h, B);
    // state bounds (interior-point variant): the Riccati solvers only; the group kernel when its LDS layout fits
    if (h->x_bounded && h->opts.kkt_solver == MMPC_KKT_AUTO && s == MMPC_KKT_CONDENSED)
        return group_lds_bytes(h->info, h->nq, true, true) <= kMaxGroupLds ? MMPC_KKT_RICCATI_GROUP : MMPC_KKT_RICCATI;
    return s;
}
int resolve_kkt_solver_base(const mmpc_handle* h, int64_t B) {
    const mmpc_model_info& mi = h->info;
    if (h->opts.kkt_solver != MMPC_KKT_AUTO) return h->opts.kkt_solver;
    if (h->opts.factor_fp32) return MMPC_KKT_RICCATI;
    // measured on one MI355X (tools/solver_sweep.py): 2-link arm -- condensed for small batches
    // (B <= 2560 at N*nu <= 64), the 16-lane Riccati kernel up to B*N = 1e6, one lane per instance beyond;
    // exo -- the 16-lane kernel while at least two of its workgroups fit a CU's LDS and B <= 4096
    const int N = mi.num_shooting_nodes;
    // LDS of the layout launch_kernel will use: the interior-point fields with state bounds, else the bounded
    // solves' hold targets (the larger of the two control-bound variants)
    const size_t glds = group_lds_bytes(mi, h->nq, true, h->x_bounded);
    if (mi.model_id == MMPC_MODEL_USER) {  // SX-generated dynamics: no condensed kernel (it is 2-link specific)
        if (glds <= kMaxGroupLds / 2 && B * static_cast<int64_t>(N) <= 1000000) return MMPC_KKT_RICCATI_GROUP;
        return MMPC_KKT_RICCATI;
    }
    if (mi.model_id == MMPC_MODEL_TWO_LINK_ARM) {
        // the condensed kernel is Gauss-Newton only: with the exact Hessian (AUTO) the 16-lane kernel takes the
        // small batches too (fewer SQP iterations outweigh its higher per-iteration cost)
        if (N * TwoLinkArm::NU <= 64 && B <= 2560 && (h->opts.hessian == MMPC_HESSIAN_GAUSS_NEWTON || mi.is_linear))
            return MMPC_KKT_CONDENSED;
        if (glds <= kMaxGroupLds && B * static_cast<int64_t>(N) <= 1000000) return MMPC_KKT_RICCATI_GROUP;
        return MMPC_KKT_RICCATI;
    }
    if (glds <= kMaxGroupLds / 2 && B <= 4096) return MMPC_KKT_RICCATI_GROUP;
    return MMPC_KKT_RICCATI;
}

// Exact-Hessian support of a model / solve (mmpc_opts.hessian): second derivatives, the lane-distributed path
// of the group kernel (nx + nu < 16, no bounds), nonlinear dynamics.  AUTO also needs the model's default
// (kExactDefault: the exo keeps Gauss-Newton -- its small-residual fits converge in 3-5 Gauss-Newton
// iterations and the exact Hessian did not cut them in the prototype sweep).
template <class M>
constexpr bool exact_capable() {
    return HasHess<M>::value && (M::NX + M::NU < kGroupLanes);
}
template <class M, class = void>
struct ExactDefault {
    static constexpr bool value = true;
};
template <class M>
struct ExactDefault<M, std::enable_if_t<!M::kExactDefault || M::kExactDefault>> {
    static constexpr bool value = M::kExactDefault;
};
// MMPC_HESSIAN_GAUSS_NEWTON / _EXACT for a solve under solver with/without control bounds; <0 = error
int resolve_hessian(const mmpc_handle* h, int solver, bool u_bounded) {
    const int want = h->opts.hessian;
    if (want == MMPC_HESSIAN_GAUSS_NEWTON) return MMPC_HESSIAN_GAUSS_NEWTON;
    bool group_capable = false, lane_capable = false, dflt = false;
    with_model(h->info.model_id, [&](auto* m) {
        using M = std::remove_pointer_t<decltype(m)>;
        group_capable = exact_capable<M>();
        lane_capable = HasHess<M>::value;
        dflt = ExactDefault<M>::value;
        return MMPC_OK;
    });
    // control bounds (the projected SQP): EXACT fixes the held controls in the exact QP as in the Gauss-Newton one
    // (group kernel; lane kernel since round 5); AUTO keeps Gauss-Newton there -- measured faster at cfg#2 with +-2 Nm
    // (0.77 vs 0.91 ms: the exact solves take fewer iterations, but every re-solve after a hold repeats the costlier
    // exact Riccati sweep).  The lane kernel (round 4) takes EXACT on request; AUTO there stays
    // Gauss-Newton (its backward sweep evaluates the model's Hessian per stage).
    // state bounds (round 6): EXACT on request (IPOPT's exact Hessian under the barrier, ModelGenerator.cpp:232,238);
    // AUTO keeps Gauss-Newton for state-bounded solves like for control-bounded ones
    const bool common = !h->info.is_linear && !h->opts.factor_fp32;
    const bool group_ok = common && group_capable && solver == MMPC_KKT_RICCATI_GROUP;
    const bool lane_ok = common && lane_capable && solver == MMPC_KKT_RICCATI;
    if (want == MMPC_HESSIAN_EXACT) {
        if (!group_ok && !lane_ok)
            return fail(MMPC_ERR_UNSUPPORTED, "exact Hessian: needs a model with second derivatives, a Riccati "
                                              "solver (RICCATI_GROUP or RICCATI, fp64 factor) and a nonlinear solve");
        return MMPC_HESSIAN_EXACT;
    }
    return group_ok && dflt && !u_bounded && !h->x_bounded ? MMPC_HESSIAN_EXACT : MMPC_HESSIAN_GAUSS_NEWTON;
}

template <class Model, bool BOUNDED, bool XB = false, bool EXACT = false>
int launch_group(dim3 grid, dim3 block, size_t lds, hipStream_t stream, const SolveParams& p, GroupWork gwk) {
    int rc = set_dynamic_lds(sqp_group_kernel<Model, BOUNDED, XB, EXACT>, lds);
    if (rc) return rc;
    sqp_group_kernel<Model, BOUNDED, XB, EXACT><<<grid, block, lds, stream>>>(p, gwk);
    return MMPC_OK;
}

// Riccati workspace (sqp_lane.h / sqp_group.h layouts), grown on demand.  Growth is synchronous:
// hipFree waits for the kernels still using the old buffer.
constexpr size_t kExitCountBytes = 256;
int ensure_workspace_bytes(mmpc_handle* h, size_t bytes, double** out) {
    int dev = -1;
    MMPC_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(h->ws_mu);
    if (h->ws && h->ws_dev != dev) return fail(MMPC_ERR_INVALID_ARG, "handle used on two devices");
    if (bytes > h->ws_bytes) {
        if (h->ws) MMPC_HIP(hipFree(h->ws));
        h->ws = nullptr;
        h->ws_bytes = 0;
        // + the 16-lane kernel's finish counter (SolveParams::exit_count), zeroed once here and reset by every launch
        MMPC_HIP(hipMalloc(reinterpret_cast<void**>(&h->ws), bytes + kExitCountBytes));
        MMPC_HIP(hipMemset(reinterpret_cast<char*>(h->ws) + bytes, 0, kExitCountBytes));
        h->ws_bytes = bytes;
        h->ws_dev = dev;
    }
    *out = h->ws;
    return MMPC_OK;
}
// iteration-tail hand-over list after the solver workspace: [count | pad][idx: slots x i32][it: slots x i32][mu][mub]
// (a state-bounded solve's resume workspace follows it: its duals stay in the lane launch's workspace)
constexpr int kTailMaxSlots = 65536;
constexpr size_t kTailBytes = 256 + static_cast<size_t>(kTailMaxSlots) * 24;
size_t solver_workspace_bytes(const mmpc_handle* h, int64_t B) {
    return (std::max(workspace_bytes(h->info, h->nq, B), group_workspace_bytes(h->info, B)) + 255) / 256 * 256;
}
int ensure_workspace(mmpc_handle* h, int64_t B, LaneWork* lw) {
    return ensure_workspace_bytes(h, solver_workspace_bytes(h, B) + kTailBytes, &lw->ws);
}

int launch_kernel(mmpc_handle* h, int solver, const SolveParams& p, bool bounded, hipStream_t stream);

// Iteration-tail hand-over of a lane-kernel solve: the lane kernel's wave runs until its slowest lane
// converges (cfg#3: 1 % of the instances need a 5th iteration, and the waves holding them set the kernel time), so
// instances still unconverged at the stop test of iteration `cap` continue in a 16-lane resume launch, whose
// per-iteration latency is ~5x lower (exo N = 24, B = 256: 0.30 vs 1.68 ms). Unbounded nonlinear solves of models
// the 16-lane kernel runs (nx + nu < 16), without the diagnostic trace; a solve with the fp32 Riccati factor continues
// its tail with the fp64 factor (precision escalation: same stop test, same iterate). cap: 4 (Gauss-Newton and exact
// Hessian; 3 hands over too many: cfg#3 12.8 ms), MMPC_TAIL_CAP overrides (0 = off). slots: four rounds of resume
// workgroups (groups per workgroup gpw with <= 64 KB of LDS, up to 4 one-wave workgroups per CU per round),
// MMPC_TAIL_ROUNDS overrides.
// Bounded solves hand over by the wave rule alone (their counts spread: no common cap). State bounds: the duals are
// read from the lane launch's workspace by the resume launch, whose own workspace then lies after the hand-over list
// (xb_ws_bytes). Control bounds: the resume launch runs the lane kernel's active-set rule (no_release) from the
// handed-over hold epsilon (tail_mub).
struct TailPlan {
    int cap = 0, wave_max = 0, slots = 0, gpw = 1;
    size_t lds = 0, xb_ws_bytes = 0;
};
TailPlan tail_plan(const mmpc_handle* h, const SolveParams& p, bool bounded, int cu) {
    TailPlan t;
    const mmpc_model_info& mi = h->info;
    const bool xb = p.x_bounded != 0;
    if (mi.is_linear || p.trace || cu <= 0) return t;
    if (mi.num_x + mi.num_u >= kGroupLanes) return t;
    constexpr int kNoCap = 1 << 20;
    // bounded solves (state: interior point; control: projected SQP with its QP re-solves) hand over by the wave rule
    // alone: their counts spread (exo |u| <= 0.5: 4.3 mean, 12 max), and a cap either hands over too many or none
    const bool spread = xb || bounded;
    // opts.tail_* (ABI 6), the MMPC_TAIL_* environment overriding them (A/B and tests); -1: the default policy
    const int cap_o = h->tail_cap_env >= 0 ? h->tail_cap_env : h->opts.tail_cap;
    const int wave_o = h->tail_wave_env >= 0 ? h->tail_wave_env : h->opts.tail_wave_max;
    const int rounds_o = h->tail_rounds_env > 0 ? h->tail_rounds_env : h->opts.tail_rounds;
    const int cap = cap_o >= 0 ? cap_o : (spread ? kNoCap : 4);
    if (cap <= 0 || (cap >= p.max_iter && !spread)) return t;
    // wave rule threshold: 8 lanes (unbounded: only the thin tails of loose tolerances use it), 4 for bounded solves,
    // whose handed-over instances need several more iterations (exo at cfg#3 size, ms without / with 4: |qdot| <= 1.5
    // 65.3 / 60.5 (1 / 2 / 3 / 6 lanes: 62.2 / 61.0 / 61.0 / 67.6, profiles/r05/xbwave); |u| <= 0.5 36.9 / 30.1, |u| <= 2
    // 22.7 / 22.2 (8 lanes: 38.4 / 21.0; caps 4-8 beside it, profiles/r05/ubsweep))
    const int wave_max = wave_o >= 0 ? wave_o : (spread ? 4 : 8);
    if (spread && cap >= p.max_iter && wave_max <= 0) return t;
    const size_t inst = static_cast<size_t>(group_lds_doubles(mi.num_x, mi.num_u, h->nq, mi.num_shooting_nodes,
                                                              bounded && !xb, false, xb)) * sizeof(double);
    if (inst > 64 * 1024) return t;
    const int gpw = static_cast<int>(std::max<size_t>(1, std::min<size_t>(kGroupsPerWave, (64 * 1024) / inst)));
    const int per_cu = static_cast<int>(std::min<size_t>(4, (160 * 1024) / (gpw * inst)));
    t.cap = cap;
    t.wave_max = wave_max;
    t.gpw = gpw;
    t.lds = gpw * inst;
    // up to four rounds of resume workgroups (slots nobody claimed exit at once, so spare slots cost nothing)
    const int rounds = rounds_o > 0 ? rounds_o : 4;
    t.slots = static_cast<int>(std::min<int64_t>({p.B, kTailMaxSlots, (int64_t)rounds * per_cu * cu * gpw}));
    if (xb)
        t.xb_ws_bytes = static_cast<size_t>(group_ws_doubles(mi.num_x, mi.num_u, mi.num_shooting_nodes, false, true)) *
                        static_cast<size_t>(t.slots) * sizeof(double);
    return t;
}
// the device's compute units (the resume launch's slots scale with them), queried once per handle
int query_cu_count(mmpc_handle* h) {
    if (h->cu_count == 0) {
        int dev = 0, n = 0;
        MMPC_HIP(hipGetDevice(&dev));
        MMPC_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
        h->cu_count = n;
    }
    return MMPC_OK;
}

int launch_solve(mmpc_handle* h, int64_t B, const double* x0, const double* u_prev, const double* traj,
                 const double* weights, int64_t w_stride, const double* u_lb, const double* u_ub, double* V,
                 int32_t* status, int32_t* iters, double* kkt, hipStream_t stream, double* trace = nullptr,
                 double* u0_out = nullptr) {
    const mmpc_model_info& mi = h->info;
    if (B < 0) return fail(MMPC_ERR_INVALID_ARG, "B < 0");
    if (B == 0) return MMPC_OK;
    if (!x0 || !u_prev || !traj || !weights || !V) return fail(MMPC_ERR_INVALID_ARG, "null input pointer");
    const int nw = mi.num_x + 2 * mi.num_u;
    if (w_stride != 0 && w_stride < nw) return fail(MMPC_ERR_INVALID_ARG, "weights_stride must be 0 or >= nx+2nu");
    if (B > 0x7fffffffLL) return fail(MMPC_ERR_INVALID_ARG, "B exceeds the grid limit (2^31-1)");
    SolveParams p;
    p.B = B;
    p.N = mi.num_shooting_nodes;
    p.max_iter = h->opts.max_iter;
    p.h = mi.step_size;
    p.tol_grad = h->opts.tol_grad;
    p.tol_defect = h->opts.tol_defect;
    p.is_linear = mi.is_linear;
    p.x0 = x0;
    p.u_prev = u_prev;
    p.traj = traj;
    p.weights = weights;
    p.w_stride = w_stride;
    p.u_lb = u_lb;
    p.u_ub = u_ub;
    p.V = V;
    p.status = status;
    p.iters = iters;
    p.kkt = kkt;
    p.trace = trace;
    p.u0_out = u0_out;
    p.init_hold = h->opts.init_states == MMPC_INIT_HOLD_X0;
    p.init_zero = h->opts.init_states == MMPC_INIT_ZERO;
    p.tail_cap = 0;
    p.tail_wave_max = 0;
    p.tail_slots = 0;
    p.tail_count = p.tail_idx = p.tail_it = nullptr;
    p.tail_mu = p.tail_mub = nullptr;
    p.tail_lws = nullptr;
    p.no_release = 0;
    p.tail_lws_block = 0;
    p.tail_lws_ss = p.tail_lws_zl = 0;
    p.gpw = kGroupsPerWave;
    p.exit_count = nullptr;
    // any bound pointer selects the kernels' BOUNDED variant (projected GN-SQP, sqp_wave.h); host entry
    // points pass NULL for bounds that are all infinite
    const bool bounded = u_lb || u_ub;
    {  // state bounds: the interior-point variant (sqp_wave.h "state bounds"), by value in the launch arguments
        std::lock_guard<std::mutex> lk(h->xb_mu);
        p.x_bounded = h->x_bounded;
        for (int i = 0; i < 16; ++i) {
            p.x_lb[i] = i < mi.num_x ? h->x_lb[i] : -INFINITY;
            p.x_ub[i] = i < mi.num_x ? h->x_ub[i] : INFINITY;
        }
    }
    const int solver = resolve_kkt_solver(h, B);
    return launch_kernel(h, solver, p, bounded, stream);
}

// one kernel launch for solver (not AUTO) on p.B instances
int launch_kernel(mmpc_handle* h, int solver, const SolveParams& p, bool bounded, hipStream_t stream) {
    const mmpc_model_info& mi = h->info;
    const int64_t B = p.B;
    const int N = mi.num_shooting_nodes;
    if (solver == MMPC_KKT_RICCATI_GROUP) {
        if (h->opts.factor_fp32) return fail(MMPC_ERR_UNSUPPORTED, "factor_fp32 needs the lane Riccati solver");
        const bool xb = p.x_bounded != 0;
        const size_t lds = group_lds_bytes(mi, h->nq, bounded, xb);
        if (lds > kMaxGroupLds) return fail(MMPC_ERR_UNSUPPORTED, "group Riccati solver: stage data exceeds 160 KB LDS");
        LaneWork lw;
        int rc = ensure_workspace(h, B, &lw);
        if (rc) return rc;
        GroupWork gwk{lw.ws};
        dim3 grid(grid1d(B, kGroupsPerWave)), block(64);
        const int hess = resolve_hessian(h, solver, bounded);
        if (hess < 0) return hess;
        SolveParams pg = p;
#if MMPC_GROUP_EXIT_HOLD
        // resident finish: when the whole grid is resident at once (one wave per SIMD by registers, the
        // workgroups per CU the LDS allows), finished waves stay resident until the launch's last waves have finished
        if ((rc = query_cu_count(h))) return rc;
        const int64_t resident = static_cast<int64_t>(h->cu_count) * std::min<int64_t>(4, (160 * 1024) / std::max<size_t>(lds, 1));
        if (grid.x >= 2 && static_cast<int64_t>(grid.x) <= resident)
            pg.exit_count = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(lw.ws) + h->ws_bytes);
#endif
        rc = with_model(mi.model_id, [&](auto* m) {
            using M = std::remove_pointer_t<decltype(m)>;
            if constexpr (std::is_same<M, TwoLinkArm>::value) {   // the units of group_launch.h
                const bool exact = hess == MMPC_HESSIAN_EXACT;
                const hipError_t e =
                    (bounded || xb) ? launch_group_two_link_bounded(xb, exact, grid, block, lds, stream, pg, gwk)
                                    : launch_group_two_link(exact, grid, block, lds, stream, pg, gwk);
                return e == hipSuccess ? MMPC_OK : fail(MMPC_ERR_HIP, std::string("group kernel launch: ") +
                                                                          hipGetErrorString(e));
            } else {
                if constexpr (exact_capable<M>()) {
                    if (hess == MMPC_HESSIAN_EXACT)
                        return xb        ? launch_group<M, false, true, true>(grid, block, lds, stream, pg, gwk)
                               : bounded ? launch_group<M, true, false, true>(grid, block, lds, stream, pg, gwk)
                                         : launch_group<M, false, false, true>(grid, block, lds, stream, pg, gwk);
                }
                if (xb) return launch_group<M, false, true>(grid, block, lds, stream, pg, gwk);
                return bounded ? launch_group<M, true>(grid, block, lds, stream, pg, gwk)
                               : launch_group<M, false>(grid, block, lds, stream, pg, gwk);
            }
        });
        if (rc) return rc;
        MMPC_HIP(hipGetLastError());
        return MMPC_OK;
    }
    if (p.x_bounded && solver == MMPC_KKT_CONDENSED)
        return fail(MMPC_ERR_UNSUPPORTED, "state bounds need a Riccati solver (MMPC_KKT_RICCATI[_GROUP])");
    const int hess = resolve_hessian(h, solver, bounded);   // EXACT requested on an unsupported solver: error
    if (hess < 0) return hess;
    if (solver == MMPC_KKT_CONDENSED) {
        if (h->opts.factor_fp32) return fail(MMPC_ERR_UNSUPPORTED, "factor_fp32 is a Riccati-solver option");
#if MMPC_BUILTIN_MODELS
        // host-side shape checks: the kernel holds one condensed-Hessian row per lane
        if (mi.model_id != MMPC_MODEL_TWO_LINK_ARM || N * TwoLinkArm::NU > 64)
            return fail(MMPC_ERR_UNSUPPORTED, "condensed solver needs the 2-link arm and N*nu <= 64");
        dim3 grid(static_cast<unsigned>(B)), block(64);
        if (bounded) {
            if (N <= 16) sqp_wave_kernel<TwoLinkArm, 16, true><<<grid, block, 0, stream>>>(p);
            else if (N <= 30) sqp_wave_kernel<TwoLinkArm, 30, true><<<grid, block, 0, stream>>>(p);
            else sqp_wave_kernel<TwoLinkArm, 32, true><<<grid, block, 0, stream>>>(p);
        } else {
            if (N <= 16) sqp_wave_kernel<TwoLinkArm, 16><<<grid, block, 0, stream>>>(p);
            else if (N <= 30) sqp_wave_kernel<TwoLinkArm, 30><<<grid, block, 0, stream>>>(p);
            else sqp_wave_kernel<TwoLinkArm, 32><<<grid, block, 0, stream>>>(p);
        }
#else
        return fail(MMPC_ERR_UNSUPPORTED, "condensed solver needs the built-in 2-link arm");
#endif
    } else {
        int rc = query_cu_count(h);
        if (rc) return rc;
        const TailPlan tp = tail_plan(h, p, bounded, h->cu_count);
        LaneWork lw;
        rc = ensure_workspace_bytes(h, solver_workspace_bytes(h, B) + kTailBytes + tp.xb_ws_bytes, &lw.ws);
        if (rc) return rc;
        dim3 grid(grid1d(B, 64)), block(64);
        SolveParams pl = p;
        if (tp.cap > 0) {   // the lane kernel hands instances still unconverged at iteration cap to a 16-lane launch
            char* const tb = reinterpret_cast<char*>(lw.ws) + solver_workspace_bytes(h, B);
            pl.tail_cap = tp.cap;
            pl.tail_wave_max = tp.wave_max;
            pl.tail_slots = tp.slots;
            pl.tail_count = reinterpret_cast<int32_t*>(tb);
            pl.tail_idx = reinterpret_cast<int32_t*>(tb + 256);
            pl.tail_it = pl.tail_idx + kTailMaxSlots;
            pl.tail_mu = reinterpret_cast<double*>(pl.tail_it + kTailMaxSlots);
            pl.tail_mub = pl.tail_mu + kTailMaxSlots;
            MMPC_HIP(hipMemsetAsync(pl.tail_count, 0, sizeof(int32_t), stream));
        }
        // lane kernels: their own translation unit (lane_kernels.hip, lane_launch.h)
        if (launch_lane_kernels(mi.model_id, h->opts.factor_fp32 != 0, bounded, p.x_bounded != 0,
                                hess == MMPC_HESSIAN_EXACT, grid, block, stream, pl, lw) != 0)
            return fail(MMPC_ERR_UNSUPPORTED, "model not compiled into this library");
        if (tp.cap > 0) {   // resume launch over the hand-over list (slots the lane kernel did not claim exit at once)
            MMPC_HIP(hipGetLastError());
            SolveParams pr = pl;
            pr.tail_cap = 0;
            pr.gpw = tp.gpw;
            pr.init_hold = pr.init_zero = 0;   // the handed-over iterate is in V
            pr.no_release = 1;                 // control bounds: the lane kernel's active-set rule
            const bool xb = p.x_bounded != 0;
            const bool ub = bounded && !xb;
            GroupWork gwk{lw.ws};
            if (xb) {   // duals from the lane workspace; the resume workspace after the hand-over list
                const int nx = mi.num_x, nu = mi.num_u, N = mi.num_shooting_nodes;
                pr.tail_lws = lw.ws;
                pr.tail_lws_block = static_cast<int64_t>(lane_ws_doubles(nx, nu, h->nq, N, true)) * 64;
                pr.tail_lws_ss = lane_stage_stride(nx, nu, true);
                pr.tail_lws_zl = lane_zl_offset(nx, nu);
                gwk.ws = lw.ws + (solver_workspace_bytes(h, B) + kTailBytes) / sizeof(double);
            }
            dim3 rgrid(static_cast<unsigned>((tp.slots + tp.gpw - 1) / tp.gpw)), rblock(64);
            rc = with_model(mi.model_id, [&](auto* m) {
                using M = std::remove_pointer_t<decltype(m)>;
                if constexpr (M::NX + M::NU < kGroupLanes) {
                    if constexpr (std::is_same<M, TwoLinkArm>::value) {
                        const bool ex = hess == MMPC_HESSIAN_EXACT;
                        const hipError_t e =
                            (xb || ub) ? launch_group_two_link_bounded(xb, ex, rgrid, rblock, tp.lds, stream, pr, gwk)
                                       : launch_group_two_link(ex, rgrid, rblock, tp.lds, stream, pr, gwk);
                        return e == hipSuccess ? MMPC_OK : fail(MMPC_ERR_HIP, std::string("resume launch: ") +
                                                                                  hipGetErrorString(e));
                    } else {
                        if constexpr (exact_capable<M>()) {
                            if (xb && hess == MMPC_HESSIAN_EXACT)
                                return launch_group<M, false, true, true>(rgrid, rblock, tp.lds, stream, pr, gwk);
                        }
                        if (xb) return launch_group<M, false, true>(rgrid, rblock, tp.lds, stream, pr, gwk);
                        if constexpr (exact_capable<M>()) {
                            if (hess == MMPC_HESSIAN_EXACT)
                                return ub ? launch_group<M, true, false, true>(rgrid, rblock, tp.lds, stream, pr, gwk)
                                          : launch_group<M, false, false, true>(rgrid, rblock, tp.lds, stream, pr, gwk);
                        }
                        return ub ? launch_group<M, true>(rgrid, rblock, tp.lds, stream, pr, gwk)
                                  : launch_group<M, false>(rgrid, rblock, tp.lds, stream, pr, gwk);
                    }
                } else {
                    return fail(MMPC_ERR_UNSUPPORTED, "tail hand-over: nx + nu >= 16");   // tail_plan excludes it
                }
            });
            if (rc) return rc;
        }
    }
    MMPC_HIP(hipGetLastError());
    return MMPC_OK;
}

int ensure_host_ctx(mmpc_handle* h, size_t bytes) {
    int dev;
    int rc = resolve_device(h, &dev);
    if (rc) return rc;
    if (h->host_stream && h->host_dev != dev) return fail(MMPC_ERR_INVALID_ARG, "handle used on two devices");
    if (!h->host_stream) {
        MMPC_HIP(hipStreamCreateWithFlags(&h->host_stream, hipStreamNonBlocking));
        h->host_dev = dev;
    }
    if (bytes > h->d_buf_bytes) {
        if (h->d_buf) MMPC_HIP(hipFree(h->d_buf));
        h->d_buf = nullptr;
        h->d_buf_bytes = 0;
        MMPC_HIP(hipMalloc(reinterpret_cast<void**>(&h->d_buf), bytes));
        h->d_buf_bytes = bytes;
    }
    return MMPC_OK;
}

}  // namespace

// ---------------------------------------------------------------- C-ABI
extern "C" {

int mmpc_abi_version(void) { return MMPC_ABI_VERSION; }

void mmpc_default_opts(mmpc_opts* o) {
    if (!o) return;
    o->max_iter = 200;  // reference IPOPT option, ModelControl.cpp:55
    o->device = -1;
    o->tol_grad = 1e-8;
    o->tol_defect = 1e-10;
    o->kkt_solver = MMPC_KKT_AUTO;
    o->factor_fp32 = 0;
    o->init_states = MMPC_INIT_AS_GIVEN;
    o->hessian = MMPC_HESSIAN_AUTO;
    o->tail_cap = -1;   // the iteration-tail hand-over's default policy
    o->tail_wave_max = -1;
    o->tail_rounds = -1;
}

int mmpc_create_from_json(const char* json_text, const mmpc_opts* opts, mmpc_handle** out) {
    if (!json_text || !out) return fail(MMPC_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    mmpc_opts o;
    mmpc_default_opts(&o);
    if (opts) o = *opts;
    int rc = validate_opts(&o);
    if (rc) return rc;
    mmpc_model_info info;
    rc = parse_model(json_text, &info);
    if (rc) return rc;
    mmpc_handle* h = new (std::nothrow) mmpc_handle();
    if (!h) return fail(MMPC_ERR_INVALID_ARG, "out of memory");
    h->info = info;
    h->nq = model_nq(info.model_id);
    for (int i = 0; i < info.num_x; ++i) {  // x_min/x_max of the JSON (ModelControl.cpp:37-50)
        h->x_lb[i] = info.x_min[i];
        h->x_ub[i] = info.x_max[i];
        h->x_bounded |= info.x_min[i] > -1e19 || info.x_max[i] < 1e19;
    }
    h->opts = o;
    if (const char* e = std::getenv("MMPC_TAIL_CAP")) {   // A/B and tests: the tail hand-over's cap (0 = off)
        char* end = nullptr;
        const long v = std::strtol(e, &end, 10);
        if (end != e && v >= 0 && v < 1000) h->tail_cap_env = static_cast<int>(v);
    }
    if (const char* e = std::getenv("MMPC_TAIL_WAVE")) {
        char* end = nullptr;
        const long v = std::strtol(e, &end, 10);
        if (end != e && v >= 0 && v <= 64) h->tail_wave_env = static_cast<int>(v);
    }
    if (const char* e = std::getenv("MMPC_TAIL_ROUNDS")) {
        char* end = nullptr;
        const long v = std::strtol(e, &end, 10);
        if (end != e && v > 0 && v < 1000) h->tail_rounds_env = static_cast<int>(v);
    }
    *out = h;
    g_last_error.clear();
    return MMPC_OK;
}

int mmpc_create(const char* path, const mmpc_opts* opts, mmpc_handle** out) {
    if (!path || !out) return fail(MMPC_ERR_INVALID_ARG, "null argument");
    std::ifstream f(path);  // ModelControl.cpp:24 reads <model_name>.json
    if (!f) return fail(MMPC_ERR_IO, std::string("cannot open ") + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return mmpc_create_from_json(ss.str().c_str(), opts, out);
}

int mmpc_destroy(mmpc_handle* h) {
    if (!h) return MMPC_OK;
    if (h->host_stream || h->d_buf) {
        DeviceGuard g(h->host_dev);
        if (h->d_buf) (void)hipFree(h->d_buf);
        if (h->host_stream) (void)hipStreamDestroy(h->host_stream);
    }
    if (h->ws) {
        DeviceGuard g(h->ws_dev);
        (void)hipFree(h->ws);
    }
    delete h;
    return MMPC_OK;
}

int mmpc_get_model_info(const mmpc_handle* h, mmpc_model_info* info) {
    if (!h || !info) return fail(MMPC_ERR_INVALID_ARG, "null argument");
    *info = h->info;
    return MMPC_OK;
}

int mmpc_set_opts(mmpc_handle* h, const mmpc_opts* opts) {
    if (!h || !opts) return fail(MMPC_ERR_INVALID_ARG, "null argument");
    int rc = validate_opts(opts);
    if (rc) return rc;
    h->opts = *opts;
    return MMPC_OK;
}

int mmpc_set_state_bounds(mmpc_handle* h, const double* x_lb, const double* x_ub) {
    if (!h) return fail(MMPC_ERR_INVALID_ARG, "null handle");
    std::lock_guard<std::mutex> lk(h->xb_mu);
    bool any = false;
    for (int i = 0; i < h->info.num_x; ++i) {
        const double l = x_lb ? x_lb[i] : -INFINITY, u = x_ub ? x_ub[i] : INFINITY;
        if (l != l || u != u || l > u) return fail(MMPC_ERR_INVALID_ARG, "state bounds: NaN or lower > upper");
        h->x_lb[i] = l;
        h->x_ub[i] = u;
        any |= l > -1e19 || u < 1e19;
    }
    h->x_bounded = any;
    return MMPC_OK;
}

int mmpc_get_state_bounds(const mmpc_handle* h, double* x_lb, double* x_ub) {
    if (!h || !x_lb || !x_ub) return fail(MMPC_ERR_INVALID_ARG, "null argument");
    for (int i = 0; i < h->info.num_x; ++i) {
        x_lb[i] = h->x_lb[i];
        x_ub[i] = h->x_ub[i];
    }
    return MMPC_OK;
}

int mmpc_reserve_workspace(mmpc_handle* h, int64_t B, uint64_t* bytes) {
    if (!h) return fail(MMPC_ERR_INVALID_ARG, "null handle");
    if (B < 0) return fail(MMPC_ERR_INVALID_ARG, "B < 0");
    // + the tail hand-over list + a state-bounded solve's resume workspace (sized by the device's CUs: 256 until a
    // device was queried), reserved whether or not the handle has state bounds now: a later mmpc_set_state_bounds must
    // not make a solve grow the workspace (a hipFree / hipMalloc inside a stream-ordered solve, or under a captured
    // hipGraph that still points at the old buffer)
    auto total = [&]() {
        SolveParams p{};
        p.B = B;
        p.max_iter = h->opts.max_iter;
        p.x_bounded = 1;
        p.is_linear = h->info.is_linear;
        const int cu = h->cu_count > 0 ? h->cu_count : 256;
        return solver_workspace_bytes(h, B) + kTailBytes + tail_plan(h, p, false, cu).xb_ws_bytes;
    };
    if (bytes) *bytes = B == 0 ? 0 : total();
    if (B == 0) return MMPC_OK;
    int dev;
    int rc = resolve_device(h, &dev);
    if (rc) return rc;
    DeviceGuard g(dev);
    if (g.err) return fail(MMPC_ERR_NO_DEVICE, "cannot select device");
    if ((rc = query_cu_count(h))) return rc;
    if (bytes) *bytes = total();
    double* ws = nullptr;
    return ensure_workspace_bytes(h, total(), &ws);
}

int mmpc_solve_batch(mmpc_handle* h, int64_t B, const double* x0, const double* u_prev, const double* traj,
                     const double* weights, int64_t weights_stride, const double* u_lb, const double* u_ub,
                     double* V_inout, int32_t* status, int32_t* iters, double* kkt_res, void* stream) {
    return mmpc_solve_batch_u0(h, B, x0, u_prev, traj, weights, weights_stride, u_lb, u_ub, V_inout, status, iters,
                               kkt_res, nullptr, stream);
}

int mmpc_solve_batch_u0(mmpc_handle* h, int64_t B, const double* x0, const double* u_prev, const double* traj,
                        const double* weights, int64_t weights_stride, const double* u_lb, const double* u_ub,
                        double* V_inout, int32_t* status, int32_t* iters, double* kkt_res, double* u0_out,
                        void* stream) {
    if (!h) return fail(MMPC_ERR_INVALID_ARG, "null handle");
    if (B < 0) return fail(MMPC_ERR_INVALID_ARG, "B < 0");
    if (B == 0) return MMPC_OK;
    if (!x0 || !u_prev || !traj || !weights || !V_inout) return fail(MMPC_ERR_INVALID_ARG, "null input pointer");
    int dev;
    int rc = resolve_device(h, &dev);
    if (rc) return rc;
    DeviceGuard g(dev);
    if (g.err) return fail(MMPC_ERR_NO_DEVICE, "cannot select device");
    return launch_solve(h, B, x0, u_prev, traj, weights, weights_stride, u_lb, u_ub, V_inout, status, iters,
                        kkt_res, reinterpret_cast<hipStream_t>(stream), nullptr, u0_out);
}

int mmpc_host_alloc(uint64_t bytes, void** out) {
    if (!out) return fail(MMPC_ERR_INVALID_ARG, "null output pointer");
    *out = nullptr;
    if (bytes == 0) return MMPC_OK;
    // pinned, mapped into every device's address space at the same address, coherent (uncached on the device
    // side): a kernel's stores land in host memory, visible to the host once the stream's work has completed
    if (hipHostMalloc(out, bytes, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess) {
        *out = nullptr;
        return fail(MMPC_ERR_HIP, "hipHostMalloc failed");
    }
    return MMPC_OK;
}

int mmpc_host_free(void* p) {
    if (p && hipHostFree(p) != hipSuccess) return fail(MMPC_ERR_HIP, "hipHostFree failed");
    return MMPC_OK;
}

int mmpc_solve_batch_host(mmpc_handle* h, int64_t B, const double* x0, const double* u_prev, const double* traj,
                          const double* weights, int64_t weights_stride, const double* u_lb, const double* u_ub,
                          double* V_inout, int32_t* status, int32_t* iters, double* kkt_res) {
    if (!h) return fail(MMPC_ERR_INVALID_ARG, "null handle");
    if (B < 0) return fail(MMPC_ERR_INVALID_ARG, "B < 0");
    if (B == 0) return MMPC_OK;
    if (!x0 || !u_prev || !traj || !weights || !V_inout) return fail(MMPC_ERR_INVALID_ARG, "null input pointer");
    std::lock_guard<std::mutex> lk(h->host_mu);
    const mmpc_model_info& mi = h->info;
    const size_t nx = mi.num_x, nu = mi.num_u, N = mi.num_shooting_nodes, NV = mi.num_v;
    // bounds that are all infinite (|b| >= 1e19, the reference's +-1e31 defaults) select the unbounded kernels
    bool lb_finite = false, ub_finite = false;
    for (size_t c = 0; c < nu; ++c) {
        lb_finite |= u_lb && u_lb[c] > -1e19;
        ub_finite |= u_ub && u_ub[c] < 1e19;
    }
    if (!lb_finite && !ub_finite) u_lb = u_ub = nullptr;
    const size_t nw = nx + 2 * nu;
    const size_t nW = weights_stride ? (size_t)B * (size_t)weights_stride : nw;
    // doubles: x0, u_prev, traj, weights, lb, ub, V, kkt ; ints: status, iters (as doubles' room)
    const size_t off_x0 = 0, off_up = off_x0 + B * nx, off_tr = off_up + B * nu, off_w = off_tr + B * N * nx;
    const size_t off_lb = off_w + nW, off_ub = off_lb + nu, off_V = off_ub + nu, off_kkt = off_V + B * NV;
    const size_t off_st = off_kkt + B, off_it = off_st + (B + 1) / 2, total = off_it + (B + 1) / 2;
    int dev;
    int rc = resolve_device(h, &dev);
    if (rc) return rc;
    DeviceGuard g(dev);
    if (g.err) return fail(MMPC_ERR_NO_DEVICE, "cannot select device");
    rc = ensure_host_ctx(h, total * sizeof(double));
    if (rc) return rc;
    double* d = h->d_buf;
    hipStream_t s = h->host_stream;
    MMPC_HIP(hipMemcpyAsync(d + off_x0, x0, B * nx * sizeof(double), hipMemcpyHostToDevice, s));
    MMPC_HIP(hipMemcpyAsync(d + off_up, u_prev, B * nu * sizeof(double), hipMemcpyHostToDevice, s));
    MMPC_HIP(hipMemcpyAsync(d + off_tr, traj, B * N * nx * sizeof(double), hipMemcpyHostToDevice, s));
    MMPC_HIP(hipMemcpyAsync(d + off_w, weights, nW * sizeof(double), hipMemcpyHostToDevice, s));
    if (u_lb) MMPC_HIP(hipMemcpyAsync(d + off_lb, u_lb, nu * sizeof(double), hipMemcpyHostToDevice, s));
    if (u_ub) MMPC_HIP(hipMemcpyAsync(d + off_ub, u_ub, nu * sizeof(double), hipMemcpyHostToDevice, s));
    MMPC_HIP(hipMemcpyAsync(d + off_V, V_inout, B * NV * sizeof(double), hipMemcpyHostToDevice, s));
    int32_t* dst = reinterpret_cast<int32_t*>(d + off_st);
    int32_t* dit = reinterpret_cast<int32_t*>(d + off_it);
    rc = launch_solve(h, B, d + off_x0, d + off_up, d + off_tr, d + off_w, weights_stride, u_lb ? d + off_lb : nullptr,
                      u_ub ? d + off_ub : nullptr, d + off_V, dst, dit, d + off_kkt, s);
    if (rc) return rc;
    MMPC_HIP(hipMemcpyAsync(V_inout, d + off_V, B * NV * sizeof(double), hipMemcpyDeviceToHost, s));
    if (status) MMPC_HIP(hipMemcpyAsync(status, dst, B * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (iters) MMPC_HIP(hipMemcpyAsync(iters, dit, B * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (kkt_res) MMPC_HIP(hipMemcpyAsync(kkt_res, d + off_kkt, B * sizeof(double), hipMemcpyDeviceToHost, s));
    MMPC_HIP(hipStreamSynchronize(s));
    return MMPC_OK;
}

int mmpc_resolve_kkt_solver(const mmpc_handle* h, int64_t B, int32_t* solver) {
    if (!h || !solver || B < 0) return fail(MMPC_ERR_INVALID_ARG, "bad argument");
    *solver = resolve_kkt_solver(h, B);
    return MMPC_OK;
}

int mmpc_resolve_hessian(const mmpc_handle* h, int64_t B, int32_t u_bounded, int32_t* hessian) {
    if (!h || !hessian || B < 0) return fail(MMPC_ERR_INVALID_ARG, "null argument or B < 0");
    const int r = resolve_hessian(h, resolve_kkt_solver(h, B), u_bounded != 0);
    if (r < 0) return r;
    *hessian = r;
    return MMPC_OK;
}

int mmpc_linearize_batch(mmpc_handle* h, int64_t B, const double* x, const double* u, double* A_colmajor,
                         double* B_colmajor, double* xdot, void* stream) {
    if (!h) return fail(MMPC_ERR_INVALID_ARG, "null handle");
    if (B < 0) return fail(MMPC_ERR_INVALID_ARG, "B < 0");
    if (B == 0) return MMPC_OK;
    if (!x || !u) return fail(MMPC_ERR_INVALID_ARG, "null input pointer");
    int dev;
    int rc = resolve_device(h, &dev);
    if (rc) return rc;
    DeviceGuard g(dev);
    if (g.err) return fail(MMPC_ERR_NO_DEVICE, "cannot select device");
    rc = with_model(h->info.model_id, [&](auto* m) {
        using M = std::remove_pointer_t<decltype(m)>;
        linearize_kernel<M><<<grid1d(B, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
            B, x, u, A_colmajor, B_colmajor, xdot);
        return MMPC_OK;
    });
    if (rc) return rc;
    MMPC_HIP(hipGetLastError());
    return MMPC_OK;
}

int mmpc_linearize_batch_host(mmpc_handle* h, int64_t B, const double* x, const double* u, double* A_colmajor,
                              double* B_colmajor, double* xdot) {
    if (!h) return fail(MMPC_ERR_INVALID_ARG, "null handle");
    if (B < 0) return fail(MMPC_ERR_INVALID_ARG, "B < 0");
    if (B == 0) return MMPC_OK;
    if (!x || !u) return fail(MMPC_ERR_INVALID_ARG, "null input pointer");
    std::lock_guard<std::mutex> lk(h->host_mu);
    const size_t nx = h->info.num_x, nu = h->info.num_u;
    const size_t off_x = 0, off_u = B * nx, off_A = off_u + B * nu, off_B = off_A + B * nx * nx,
                 off_f = off_B + B * nx * nu, total = off_f + B * nx;
    int dev;
    int rc = resolve_device(h, &dev);
    if (rc) return rc;
    DeviceGuard g(dev);
    if (g.err) return fail(MMPC_ERR_NO_DEVICE, "cannot select device");
    rc = ensure_host_ctx(h, total * sizeof(double));
    if (rc) return rc;
    double* d = h->d_buf;
    hipStream_t s = h->host_stream;
    MMPC_HIP(hipMemcpyAsync(d + off_x, x, B * nx * sizeof(double), hipMemcpyHostToDevice, s));
    MMPC_HIP(hipMemcpyAsync(d + off_u, u, B * nu * sizeof(double), hipMemcpyHostToDevice, s));
    rc = mmpc_linearize_batch(h, B, d + off_x, d + off_u, d + off_A, d + off_B, d + off_f, s);
    if (rc) return rc;
    if (A_colmajor) MMPC_HIP(hipMemcpyAsync(A_colmajor, d + off_A, B * nx * nx * sizeof(double), hipMemcpyDeviceToHost, s));
    if (B_colmajor) MMPC_HIP(hipMemcpyAsync(B_colmajor, d + off_B, B * nx * nu * sizeof(double), hipMemcpyDeviceToHost, s));
    if (xdot) MMPC_HIP(hipMemcpyAsync(xdot, d + off_f, B * nx * sizeof(double), hipMemcpyDeviceToHost, s));
    MMPC_HIP(hipStreamSynchronize(s));
    return MMPC_OK;
}

int mmpc_nlp_eval_batch(mmpc_handle* h, int64_t B, const double* V, const double* u_prev, const double* traj,
                        const double* weights, int64_t weights_stride, double* J, double* defect_inf, void* stream) {
    if (!h) return fail(MMPC_ERR_INVALID_ARG, "null handle");
    if (B < 0) return fail(MMPC_ERR_INVALID_ARG, "B < 0");
    if (B == 0) return MMPC_OK;
    if (!V || !u_prev || !traj || !weights) return fail(MMPC_ERR_INVALID_ARG, "null input pointer");
    int dev;
    int rc = resolve_device(h, &dev);
    if (rc) return rc;
    DeviceGuard g(dev);
    if (g.err) return fail(MMPC_ERR_NO_DEVICE, "cannot select device");
    rc = with_model(h->info.model_id, [&](auto* m) {
        using M = std::remove_pointer_t<decltype(m)>;
        nlp_eval_kernel<M><<<grid1d(B, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
            B, h->info.num_shooting_nodes, h->info.step_size, h->info.is_linear, V, u_prev, traj, weights,
            weights_stride, J, defect_inf);
        return MMPC_OK;
    });
    if (rc) return rc;
    MMPC_HIP(hipGetLastError());
    return MMPC_OK;
}

int mmpc_nlp_derivs_batch(mmpc_handle* h, int64_t B, const double* V, const double* u_prev, const double* traj,
                          const double* weights, int64_t weights_stride, double* J, double* grad, double* jac_blocks,
                          void* stream) {
    if (!h) return fail(MMPC_ERR_INVALID_ARG, "null handle");
    if (B < 0) return fail(MMPC_ERR_INVALID_ARG, "B < 0");
    if (B == 0) return MMPC_OK;
    if (!V || !u_prev || !traj || !weights) return fail(MMPC_ERR_INVALID_ARG, "null input pointer");
    const int nw = h->info.num_x + 2 * h->info.num_u;
    if (weights_stride != 0 && weights_stride < nw) return fail(MMPC_ERR_INVALID_ARG, "weights_stride must be 0 or >= nx+2nu");
    int dev;
    int rc = resolve_device(h, &dev);
    if (rc) return rc;
    DeviceGuard g(dev);
    if (g.err) return fail(MMPC_ERR_NO_DEVICE, "cannot select device");
    rc = with_model(h->info.model_id, [&](auto* m) {
        using M = std::remove_pointer_t<decltype(m)>;
        nlp_derivs_kernel<M><<<grid1d(B, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
            B, h->info.num_shooting_nodes, h->info.step_size, h->info.is_linear, V, u_prev, traj, weights,
            weights_stride, J, grad, jac_blocks);
        return MMPC_OK;
    });
    if (rc) return rc;
    MMPC_HIP(hipGetLastError());
    return MMPC_OK;
}

int mmpc_nlp_hess_batch(mmpc_handle* h, int64_t B, const double* V, const double* u_prev, const double* traj,
                        const double* weights, int64_t weights_stride, double lam_f, const double* lam_g,
                        double* hess_blocks, void* stream) {
    if (!h || B < 0) return fail(MMPC_ERR_INVALID_ARG, "null handle or B < 0");
    if (B == 0) return MMPC_OK;
    if (!V || !u_prev || !traj || !weights || !hess_blocks) return fail(MMPC_ERR_INVALID_ARG, "null pointer");
    const mmpc_model_info& mi = h->info;
    if (weights_stride != 0 && weights_stride < mi.num_x + 2 * mi.num_u)
        return fail(MMPC_ERR_INVALID_ARG, "weights_stride must be 0 or >= nx+2nu");
    const int64_t n = B * mi.num_shooting_nodes;
    if (n > 0x7fffffffLL * 256) return fail(MMPC_ERR_INVALID_ARG, "B*N too large");
    int dev;
    int rc = resolve_device(h, &dev);
    if (rc) return rc;
    DeviceGuard g(dev);
    if (g.err) return fail(MMPC_ERR_NO_DEVICE, "cannot select device");
    rc = with_model(mi.model_id, [&](auto* m) {
        using M = std::remove_pointer_t<decltype(m)>;
        if (!HasHess<M>::value && !mi.is_linear)
            return fail(MMPC_ERR_UNSUPPORTED, "nlp_hess: the model has no second derivatives");
        nlp_hess_kernel<M><<<grid1d(n, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
            B, mi.num_shooting_nodes, mi.step_size, mi.is_linear, V, u_prev, traj, weights, weights_stride, lam_f,
            lam_g, hess_blocks);
        return static_cast<int>(MMPC_OK);
    });
    if (rc) return rc;
    MMPC_HIP(hipGetLastError());
    return MMPC_OK;
}

int mmpc_synth_batch(mmpc_handle* h, uint64_t seed, int64_t first_index, int64_t B, double* x0, double* u_prev,
                     double* traj, void* stream) {
    if (!h) return fail(MMPC_ERR_INVALID_ARG, "null handle");
    if (B < 0 || first_index < 0) return fail(MMPC_ERR_INVALID_ARG, "negative B / first_index");
    if (B == 0) return MMPC_OK;
    if (!x0 || !u_prev || !traj) return fail(MMPC_ERR_INVALID_ARG, "null output pointer");
    if (h->info.model_id == MMPC_MODEL_USER)
        return fail(MMPC_ERR_UNSUPPORTED, "no synthetic-instance recipe for generated models");
    int dev;
    int rc = resolve_device(h, &dev);
    if (rc) return rc;
    DeviceGuard g(dev);
    if (g.err) return fail(MMPC_ERR_NO_DEVICE, "cannot select device");
    if (h->info.model_id == MMPC_MODEL_EXO_ARM)
        synth_exo_kernel<<<synth_blocks(B, h->info.num_shooting_nodes), kSynthThreads, 0,
                           reinterpret_cast<hipStream_t>(stream)>>>(
            seed, first_index, B, h->info.num_shooting_nodes, h->info.step_size, x0, u_prev, traj);
    else
        synth_two_link_kernel<<<synth_blocks(B, h->info.num_shooting_nodes), kSynthThreads, 0,
                                reinterpret_cast<hipStream_t>(stream)>>>(
            seed, first_index, B, h->info.num_shooting_nodes, h->info.step_size, x0, u_prev, traj);
    MMPC_HIP(hipGetLastError());
    return MMPC_OK;
}

// ---------------------------------------------------------------- multi-device (one process, G devices)
int mmpc_shard(int64_t B, int32_t n, int32_t i, int64_t* first, int64_t* count) {
    if (B < 0 || n < 1 || i < 0 || i >= n || !first || !count) return fail(MMPC_ERR_INVALID_ARG, "bad shard arguments");
    if (B > (int64_t(1) << 40)) return fail(MMPC_ERR_INVALID_ARG, "B too large");
    const int64_t lo = (static_cast<int64_t>(i) * B) / n, hi = (static_cast<int64_t>(i + 1) * B) / n;
    *first = lo;
    *count = hi - lo;
    return MMPC_OK;
}

}  // extern "C"

namespace {
// RCCL entry points, resolved from librccl at the first RCCL call (no link-time dependency of libmmpc.so on it)
struct RcclApi {
    void* lib = nullptr;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclGetVersion) get_version = nullptr;
};
const RcclApi* rccl_api() {
    static const RcclApi api = [] {
        RcclApi a;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            a.lib = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (a.lib) break;
        }
        if (!a.lib) return a;
        bool ok = true;
        auto sym = [&](auto& fn, const char* n) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(a.lib, n));
            ok &= fn != nullptr;
        };
        sym(a.comm_init_all, "ncclCommInitAll");
        sym(a.comm_destroy, "ncclCommDestroy");
        sym(a.group_start, "ncclGroupStart");
        sym(a.group_end, "ncclGroupEnd");
        sym(a.send, "ncclSend");
        sym(a.recv, "ncclRecv");
        sym(a.broadcast, "ncclBroadcast");
        sym(a.error_string, "ncclGetErrorString");
        sym(a.get_version, "ncclGetVersion");
        if (!ok) a.lib = nullptr;
        return a;
    }();
    return api.lib ? &api : nullptr;
}
}  // namespace

struct mmpc_multi {
    std::vector<mmpc_handle*> h;  // one handle (own stream, workspace, staging) per listed device
    std::vector<int32_t> dev;
    std::mutex mu;                // one multi-device solve at a time
    // RCCL path (mmpc_multi_solve_batch_rccl): one communicator and stream per device, grown-only shard buffers
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> st;
    std::vector<char*> buf;
    std::vector<size_t> buf_bytes;
};

extern "C" {

int mmpc_multi_create(const char* model_json_path, const mmpc_opts* opts, const int32_t* devices, int32_t n_devices,
                      mmpc_multi** out) {
    if (!model_json_path || !devices || n_devices < 1 || n_devices > 1024 || !out)
        return fail(MMPC_ERR_INVALID_ARG, "bad multi-device arguments");
    *out = nullptr;
    std::unique_ptr<mmpc_multi> m(new mmpc_multi());
    mmpc_opts o;
    mmpc_default_opts(&o);
    if (opts) o = *opts;
    for (int32_t g = 0; g < n_devices; ++g) {
        if (devices[g] < 0) {
            for (mmpc_handle* x : m->h) mmpc_destroy(x);
            return fail(MMPC_ERR_INVALID_ARG, "device ordinals must be >= 0");
        }
        o.device = devices[g];
        mmpc_handle* h = nullptr;
        const int rc = mmpc_create(model_json_path, &o, &h);
        if (rc) {
            for (mmpc_handle* x : m->h) mmpc_destroy(x);
            return rc;
        }
        m->h.push_back(h);
        m->dev.push_back(devices[g]);
    }
    *out = m.release();
    return MMPC_OK;
}

int mmpc_multi_destroy(mmpc_multi* m) {
    if (!m) return MMPC_OK;
    if (const RcclApi* R = rccl_api())
        for (ncclComm_t c : m->comm)
            if (c) R->comm_destroy(c);
    for (size_t g = 0; g < m->st.size(); ++g) {
        DeviceGuard dg(m->dev[g]);
        if (m->st[g]) (void)hipStreamDestroy(m->st[g]);
        if (m->buf[g]) (void)hipFree(m->buf[g]);
    }
    for (mmpc_handle* h : m->h) mmpc_destroy(h);
    delete m;
    return MMPC_OK;
}

int mmpc_multi_num_devices(const mmpc_multi* m, int32_t* n) {
    if (!m || !n) return fail(MMPC_ERR_INVALID_ARG, "null argument");
    *n = static_cast<int32_t>(m->h.size());
    return MMPC_OK;
}

int mmpc_multi_handle(mmpc_multi* m, int32_t g, mmpc_handle** h) {
    if (!m || !h || g < 0 || g >= static_cast<int32_t>(m->h.size())) return fail(MMPC_ERR_INVALID_ARG, "bad device index");
    *h = m->h[static_cast<size_t>(g)];
    return MMPC_OK;
}

int mmpc_multi_solve_batch_host(mmpc_multi* m, int64_t B, const double* x0, const double* u_prev, const double* traj,
                                const double* weights, int64_t weights_stride, const double* u_lb, const double* u_ub,
                                double* V_inout, int32_t* status, int32_t* iters, double* kkt_res) {
    if (!m) return fail(MMPC_ERR_INVALID_ARG, "null multi-device handle");
    if (B < 0) return fail(MMPC_ERR_INVALID_ARG, "B < 0");
    if (B == 0) return MMPC_OK;
    if (!x0 || !u_prev || !traj || !weights || !V_inout) return fail(MMPC_ERR_INVALID_ARG, "null input pointer");
    std::lock_guard<std::mutex> lk(m->mu);
    const mmpc_model_info& mi = m->h[0]->info;
    const int64_t nx = mi.num_x, nu = mi.num_u, N = mi.num_shooting_nodes, NV = mi.num_v;
    const int32_t G = static_cast<int32_t>(m->h.size());
    std::vector<int> rcs(static_cast<size_t>(G), MMPC_OK);
    std::vector<std::string> errs(static_cast<size_t>(G));
    // each device solves its contiguous shard of the host arrays on its own thread (H2D, solve, D2H on the
    // handle's stream); shards are disjoint, so the results land in place without any assembly copy
    auto work = [&](int32_t g) {
        int64_t first = 0, count = 0;
        mmpc_shard(B, G, g, &first, &count);
        if (count == 0) return;
        const int rc = mmpc_solve_batch_host(
            m->h[static_cast<size_t>(g)], count, x0 + first * nx, u_prev + first * nu, traj + first * N * nx,
            weights_stride ? weights + first * weights_stride : weights, weights_stride, u_lb, u_ub,
            V_inout + first * NV, status ? status + first : nullptr, iters ? iters + first : nullptr,
            kkt_res ? kkt_res + first : nullptr);
        rcs[static_cast<size_t>(g)] = rc;
        if (rc) errs[static_cast<size_t>(g)] = g_last_error;   // thread-local: carried back to the caller
    };
    if (G == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        th.reserve(static_cast<size_t>(G));
        for (int32_t g = 0; g < G; ++g) th.emplace_back(work, g);
        for (std::thread& t : th) t.join();
    }
    for (int32_t g = 0; g < G; ++g)
        if (rcs[static_cast<size_t>(g)])
            return fail(rcs[static_cast<size_t>(g)], "device " + std::to_string(m->dev[static_cast<size_t>(g)]) + ": " +
                                                         errs[static_cast<size_t>(g)]);
    return MMPC_OK;
}

int mmpc_rccl_version(int32_t* version) {
    if (!version) return fail(MMPC_ERR_INVALID_ARG, "null argument");
    *version = 0;
    const RcclApi* R = rccl_api();
    if (!R) return fail(MMPC_ERR_UNSUPPORTED, "librccl not loadable");
    int v = 0;
    if (R->get_version(&v) != ncclSuccess) return fail(MMPC_ERR_UNSUPPORTED, "ncclGetVersion failed");
    *version = v;
    return MMPC_OK;
}

int mmpc_multi_solve_batch_rccl(mmpc_multi* m, int64_t B, const double* x0, const double* u_prev, const double* traj,
                                const double* weights, int64_t weights_stride, const double* u_lb, const double* u_ub,
                                double* V_inout, int32_t* status, int32_t* iters, double* kkt_res, void* stream) {
    if (!m) return fail(MMPC_ERR_INVALID_ARG, "null multi-device handle");
    if (B < 0 || weights_stride < 0) return fail(MMPC_ERR_INVALID_ARG, "B < 0 or weights_stride < 0");
    if (B == 0) return MMPC_OK;
    if (!x0 || !u_prev || !traj || !weights || !V_inout) return fail(MMPC_ERR_INVALID_ARG, "null input pointer");
    if ((u_lb == nullptr) != (u_ub == nullptr)) return fail(MMPC_ERR_INVALID_ARG, "u_lb and u_ub go together");
    std::lock_guard<std::mutex> lk(m->mu);
    const mmpc_model_info& mi = m->h[0]->info;
    const int64_t nx = mi.num_x, nu = mi.num_u, N = mi.num_shooting_nodes, NV = mi.num_v, nw = nx + 2 * nu;
    // checked before anything is sent: the scatter reads rows of weights_stride (mmpc_solve_batch checks it too, but
    // only after the shards have been sent)
    if (weights_stride != 0 && weights_stride < nw)
        return fail(MMPC_ERR_INVALID_ARG, "weights_stride must be 0 (shared) or >= nx + 2 nu");
    const int32_t G = static_cast<int32_t>(m->h.size());
    for (int32_t a = 0; a < G; ++a)
        for (int32_t b = 0; b < a; ++b)
            if (m->dev[a] == m->dev[b])
                return fail(MMPC_ERR_UNSUPPORTED, "RCCL needs distinct devices (device " + std::to_string(m->dev[a]) +
                                                      " listed twice); mmpc_multi_solve_batch_host shares a device");
    const RcclApi* R = rccl_api();
    if (!R) return fail(MMPC_ERR_UNSUPPORTED, "librccl not loadable");
    auto nccl = [&](ncclResult_t r, const char* what) {
        return r == ncclSuccess ? MMPC_OK : fail(MMPC_ERR_HIP, std::string(what) + ": " + R->error_string(r));
    };
    if (m->comm.empty()) {   // one communicator per device, in the listed order (rank g = device g of the handle)
        std::vector<ncclComm_t> comm(static_cast<size_t>(G), nullptr);
        std::vector<int> devs(m->dev.begin(), m->dev.end());
        if (int rc = nccl(R->comm_init_all(comm.data(), G, devs.data()), "ncclCommInitAll")) return rc;
        m->comm = comm;
        m->st.assign(static_cast<size_t>(G), nullptr);
        m->buf.assign(static_cast<size_t>(G), nullptr);
        m->buf_bytes.assign(static_cast<size_t>(G), 0);
        for (int32_t g = 0; g < G; ++g) {
            DeviceGuard dg(m->dev[g]);
            MMPC_HIP(hipStreamCreateWithFlags(&m->st[g], hipStreamNonBlocking));
        }
    }
    const bool shared_w = weights_stride == 0;
    const int64_t wst = shared_w ? 0 : weights_stride;
    struct Shard {
        int64_t first = 0, count = 0;
        double *x0, *up, *tr, *w, *lb, *ub, *V, *kkt;
        int32_t *st, *it;
    };
    std::vector<Shard> sh(static_cast<size_t>(G));
    for (int32_t g = 0; g < G; ++g) {   // shard buffers on device g (grown only)
        Shard& s = sh[static_cast<size_t>(g)];
        mmpc_shard(B, G, g, &s.first, &s.count);
        const int64_t c = s.count;
        const int64_t nd = c * (nx + nu + N * nx + NV + 1) + (shared_w ? nw : c * wst) + 2 * nu;
        const size_t bytes = static_cast<size_t>(nd) * sizeof(double) + static_cast<size_t>(2 * c) * sizeof(int32_t) + 64;
        DeviceGuard dg(m->dev[g]);
        if (bytes > m->buf_bytes[g]) {
            if (m->buf[g]) MMPC_HIP(hipFree(m->buf[g]));
            m->buf[g] = nullptr;
            m->buf_bytes[g] = 0;
            MMPC_HIP(hipMalloc(&m->buf[g], bytes));
            m->buf_bytes[g] = bytes;
        }
        double* p = reinterpret_cast<double*>(m->buf[g]);
        s.x0 = p; p += c * nx;
        s.up = p; p += c * nu;
        s.tr = p; p += c * N * nx;
        s.V = p; p += c * NV;
        s.kkt = p; p += c;
        s.w = p; p += shared_w ? nw : c * wst;
        s.lb = p; p += nu;
        s.ub = p; p += nu;
        s.st = reinterpret_cast<int32_t*>(p);
        s.it = s.st + c;
    }
    // the caller's inputs on the first device are complete before RCCL reads them: the first device's stream waits
    // for the caller's stream (no device-wide synchronisation); at the end the caller's stream waits for the results
    hipStream_t caller = reinterpret_cast<hipStream_t>(stream);
    if (caller) {   // the bridges below record on and wait with the caller's stream from the first device
        hipDevice_t sd = -1;
        MMPC_HIP(hipStreamGetDevice(caller, &sd));
        if (sd != m->dev[0])
            return fail(MMPC_ERR_INVALID_ARG, "stream belongs to device " + std::to_string(sd) +
                                                  ", not to the multi handle's first device " + std::to_string(m->dev[0]));
    }
    {
        DeviceGuard dg(m->dev[0]);
        hipEvent_t ev;
        MMPC_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        hipError_t e = hipEventRecord(ev, caller);
        if (e == hipSuccess) e = hipStreamWaitEvent(m->st[0], ev, 0);
        (void)hipEventDestroy(ev);
        MMPC_HIP(e);
    }
    // every stream of the call drained before an error after the first enqueue is returned (no RCCL operation or
    // solve of this call is still running when the caller sees the error)
    auto drain = [&](int rc) {
        for (int32_t g = 0; g < G; ++g) {
            DeviceGuard dg(m->dev[g]);
            (void)hipStreamSynchronize(m->st[static_cast<size_t>(g)]);
        }
        return rc;
    };
    // a group is always closed (ncclGroupEnd) even when an operation inside it failed; the first failure is reported
    int grp_rc = MMPC_OK;
    auto op = [&](ncclResult_t r, const char* what, int32_t g) {
        if (r != ncclSuccess && grp_rc == MMPC_OK)
            grp_rc = fail(MMPC_ERR_HIP, std::string(what) + " (shard " + std::to_string(g) + "): " + R->error_string(r));
    };
    // scatter: shard g of every input from rank 0 to rank g (rank 0 included: its shard goes through RCCL as well),
    // shared weights and the bounds by broadcast.  Per-instance weights: the last row of a shard is sent up to its
    // nx + 2 nu entries, so a caller's buffer of (B - 1) weights_stride + nx + 2 nu doubles is never over-read.
    const ncclDataType_t f64 = ncclFloat64, i32 = ncclInt32;
    if (int rc = nccl(R->group_start(), "ncclGroupStart")) return drain(rc);
    for (int32_t g = 0; g < G; ++g) {
        const Shard& s = sh[static_cast<size_t>(g)];
        ncclComm_t c0 = m->comm[0], cg = m->comm[static_cast<size_t>(g)];
        hipStream_t s0 = m->st[0], sg = m->st[static_cast<size_t>(g)];
        if (s.count > 0) {
            const size_t c = static_cast<size_t>(s.count);
            op(R->send(x0 + s.first * nx, c * nx, f64, g, c0, s0), "ncclSend x0", g);
            op(R->recv(s.x0, c * nx, f64, 0, cg, sg), "ncclRecv x0", g);
            op(R->send(u_prev + s.first * nu, c * nu, f64, g, c0, s0), "ncclSend u_prev", g);
            op(R->recv(s.up, c * nu, f64, 0, cg, sg), "ncclRecv u_prev", g);
            op(R->send(traj + s.first * N * nx, c * N * nx, f64, g, c0, s0), "ncclSend traj", g);
            op(R->recv(s.tr, c * N * nx, f64, 0, cg, sg), "ncclRecv traj", g);
            op(R->send(V_inout + s.first * NV, c * NV, f64, g, c0, s0), "ncclSend V", g);
            op(R->recv(s.V, c * NV, f64, 0, cg, sg), "ncclRecv V", g);
            if (!shared_w) {
                const size_t nwc = (c - 1) * static_cast<size_t>(wst) + static_cast<size_t>(nw);
                op(R->send(weights + s.first * wst, nwc, f64, g, c0, s0), "ncclSend weights", g);
                op(R->recv(s.w, nwc, f64, 0, cg, sg), "ncclRecv weights", g);
            }
        }
        // collectives run on every rank, shards of count 0 included (the broadcast lands in its unused buffer)
        if (shared_w) op(R->broadcast(weights, s.w, static_cast<size_t>(nw), f64, 0, cg, sg), "ncclBroadcast weights", g);
        if (u_lb) {
            op(R->broadcast(u_lb, s.lb, static_cast<size_t>(nu), f64, 0, cg, sg), "ncclBroadcast u_lb", g);
            op(R->broadcast(u_ub, s.ub, static_cast<size_t>(nu), f64, 0, cg, sg), "ncclBroadcast u_ub", g);
        }
    }
    if (int rc = nccl(R->group_end(), "ncclGroupEnd (scatter)")) return drain(rc);
    if (grp_rc) return drain(grp_rc);
    // solve: every device its shard, on its stream after its receives
    for (int32_t g = 0; g < G; ++g) {
        const Shard& s = sh[static_cast<size_t>(g)];
        if (s.count == 0) continue;
        const int rc = mmpc_solve_batch(m->h[static_cast<size_t>(g)], s.count, s.x0, s.up, s.tr, s.w, wst,
                                        u_lb ? s.lb : nullptr, u_lb ? s.ub : nullptr, s.V, s.st, s.it, s.kkt,
                                        m->st[static_cast<size_t>(g)]);
        if (rc) {
            const std::string err = "device " + std::to_string(m->dev[static_cast<size_t>(g)]) + ": " + g_last_error;
            return drain(fail(rc, err));
        }
    }
    // gather: V, status, iters, kkt_res of shard g back to rank 0 at the shard's offset
    if (int rc = nccl(R->group_start(), "ncclGroupStart")) return drain(rc);
    for (int32_t g = 0; g < G; ++g) {
        const Shard& s = sh[static_cast<size_t>(g)];
        if (s.count == 0) continue;
        const size_t c = static_cast<size_t>(s.count);
        ncclComm_t c0 = m->comm[0], cg = m->comm[static_cast<size_t>(g)];
        hipStream_t s0 = m->st[0], sg = m->st[static_cast<size_t>(g)];
        op(R->send(s.V, c * NV, f64, 0, cg, sg), "ncclSend V (gather)", g);
        op(R->recv(V_inout + s.first * NV, c * NV, f64, g, c0, s0), "ncclRecv V (gather)", g);
        if (status) {
            op(R->send(s.st, c, i32, 0, cg, sg), "ncclSend status", g);
            op(R->recv(status + s.first, c, i32, g, c0, s0), "ncclRecv status", g);
        }
        if (iters) {
            op(R->send(s.it, c, i32, 0, cg, sg), "ncclSend iters", g);
            op(R->recv(iters + s.first, c, i32, g, c0, s0), "ncclRecv iters", g);
        }
        if (kkt_res) {
            op(R->send(s.kkt, c, f64, 0, cg, sg), "ncclSend kkt", g);
            op(R->recv(kkt_res + s.first, c, f64, g, c0, s0), "ncclRecv kkt", g);
        }
    }
    if (int rc = nccl(R->group_end(), "ncclGroupEnd (gather)")) return drain(rc);
    if (grp_rc) return drain(grp_rc);
    {   // later work on the caller's stream sees the gathered results
        DeviceGuard dg(m->dev[0]);
        hipEvent_t ev;
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) return drain(fail(MMPC_ERR_HIP, std::string("event: ") + hipGetErrorString(e)));
        e = hipEventRecord(ev, m->st[0]);
        if (e == hipSuccess) e = hipStreamWaitEvent(caller, ev, 0);
        (void)hipEventDestroy(ev);
        if (e != hipSuccess) return drain(fail(MMPC_ERR_HIP, std::string("event: ") + hipGetErrorString(e)));
    }
    for (int32_t g = 0; g < G; ++g) {
        DeviceGuard dg(m->dev[g]);
        MMPC_HIP(hipStreamSynchronize(m->st[static_cast<size_t>(g)]));
    }
    return MMPC_OK;
}

const char* mmpc_status_string(int32_t s) {
    switch (s) {
        case MMPC_STATUS_CONVERGED: return "converged";
        case MMPC_STATUS_MAX_ITER: return "max_iter";
        case MMPC_STATUS_LINESEARCH_FAILED: return "linesearch_failed";
        case MMPC_STATUS_NONFINITE: return "nonfinite";
        case MMPC_STATUS_FACTORIZATION_FAILED: return "factorization_failed";
        case MMPC_STATUS_BOUNDS_VIOLATED: return "bounds_violated";
        default: return "unknown";
    }
}

const char* mmpc_last_error(void) { return g_last_error.c_str(); }

// Internal diagnostic: per-phase s_memtime cycle totals of the SQP kernel (all zero unless the library
// was built with -DMMPC_PHASE_TIMING, i.e. lib/libmmpc_timing.so).  out[15] = number of waves.
// sums, except slots 10-12 (latest end, ~earliest start, longest wave: sqp_wave.h MMPC_PHASE_FLUSH), which are maxima;
// the per-wave slots 16.. are written by one unit only per launch (the others hold zeros after a reset)
static void merge_phase_tables(unsigned long long* out, const unsigned long long* t, int n) {
    for (int i = 0; i < n; ++i) out[i] = (i >= 10 && i <= 12) ? std::max(out[i], t[i]) : out[i] + t[i];
}
// the first n (<= kPhaseSlots) slots of the merged tables of every translation unit
int mmpc_debug_phase_table(unsigned long long* out, int n, int reset) {
    if (!out || n < 16 || n > kPhaseSlots) return fail(MMPC_ERR_INVALID_ARG, "null or n out of 16 .. kPhaseSlots");
    MMPC_HIP(phase_table_read(out, n, reset != 0));   // this unit's table
    std::vector<unsigned long long> t(static_cast<size_t>(n));
    MMPC_HIP(lane_phase_cycles(t.data(), n, reset != 0));   // the lane kernels' unit (lane_launch.h)
    merge_phase_tables(out, t.data(), n);
#if MMPC_BUILTIN_MODELS
    MMPC_HIP(group_two_link_phase_cycles(t.data(), n, reset != 0));   // the 2-link group kernels' units (group_launch.h)
    merge_phase_tables(out, t.data(), n);
    MMPC_HIP(group_two_link_bounded_phase_cycles(t.data(), n, reset != 0));
    merge_phase_tables(out, t.data(), n);
#endif
    return MMPC_OK;
}
int mmpc_debug_phase_cycles(unsigned long long* out16, int reset) { return mmpc_debug_phase_table(out16, 16, reset); }

// Internal diagnostic (not part of include/mmpc.h): the handle's Riccati workspace (device pointer and size), e.g. to
// read the gains [K_k | kff_k] a solve left there (tools/xb_diag.py)
int mmpc_debug_workspace(mmpc_handle* h, void** ptr, uint64_t* bytes) {
    if (!h || !ptr || !bytes) return fail(MMPC_ERR_INVALID_ARG, "null argument");
    *ptr = h->ws;
    *bytes = h->ws_bytes;
    return MMPC_OK;
}

// Internal diagnostic (not part of include/mmpc.h): as mmpc_solve_batch, plus a per-iteration trace
// [B][max_iter+1][8] = (||2g||, ||c||, alpha, dphi, phi0, mu, ||du||, accepted).  Device pointers.
int mmpc_debug_solve_trace(mmpc_handle* h, int64_t B, const double* x0, const double* u_prev, const double* traj,
                           const double* weights, int64_t weights_stride, double* V_inout, int32_t* status,
                           int32_t* iters, double* kkt_res, double* trace, void* stream) {
    if (!h || B < 0 || !trace) return fail(MMPC_ERR_INVALID_ARG, "bad argument");
    int dev;
    int rc = resolve_device(h, &dev);
    if (rc) return rc;
    DeviceGuard g(dev);
    return launch_solve(h, B, x0, u_prev, traj, weights, weights_stride, nullptr, nullptr, V_inout, status, iters,
                        kkt_res, reinterpret_cast<hipStream_t>(stream), trace);
}

}  // extern "C"
