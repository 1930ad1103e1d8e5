// model_flops.hip -- one-thread kernels that call each built-in model function once, compiled to gfx950 assembly
// by tools/model_flops.py, which counts the FP64 VALU operations of each kernel body (FMA = 2 flops): the
// per-evaluation flop cost of the model evaluations the solve kernels run, reported separately from the KKT
// algebra in bench.py's roofline ("Dynamics/Jacobian evaluation flops ... reported separately").
// Diagnostic only; never linked into the library.
#include <hip/hip_runtime.h>

// sin and cos count as one op each: sincos is replaced by an opaque stub with no FP64 ops, whose
// asm marker tools/model_flops.py counts (2 flops per call).  Division and sqrt keep their expansions.
__device__ inline void mmpc_flops_sincos(double x, double* s, double* c) {
    double a = x, b = x;
    asm volatile("; sincos_stub" : "+v"(a));
    asm volatile("; sincos_stub" : "+v"(b));
    *s = a;
    *c = b;
}
#define sincos(x, s, c) mmpc_flops_sincos(x, s, c)
// the models call sincos_fast (fast_trig.h): define it first, then route the models' calls to the stub
#include "../mahi-mpc_amd/csrc/fast_trig.h"
#define sincos_fast(K, x, s, c) mmpc_flops_sincos(x, s, c)
#include "../mahi-mpc_amd/csrc/models.h"

using namespace mmpc;

template <class M>
__device__ void load(const double* in, double* x, double* u) {
#pragma unroll
    for (int i = 0; i < M::NX; ++i) x[i] = in[i];
#pragma unroll
    for (int i = 0; i < M::NU; ++i) u[i] = in[M::NX + i];
}

#define MODEL_KERNELS(M)                                                                              \
    extern "C" __global__ void flops_eval_##M(const double* in, double* out) {                      \
        double x[M::NX], u[M::NU], xd[M::NX];                                                          \
        load<M>(in, x, u);                                                                             \
        M::eval(x, u, xd);                                                                             \
        for (int i = 0; i < M::NX; ++i) out[i] = xd[i];                                                \
    }                                                                                                  \
    extern "C" __global__ void flops_acc_jac_##M(const double* in, double* out) {                   \
        constexpr int NQ = M::NQ, NA = M::NX - M::NQ;                                                 \
        double x[M::NX], u[M::NU], acc[NA], Fq[NA * NQ], Fqd[NA * NA], Fu[NA * M::NU];                \
        load<M>(in, x, u);                                                                             \
        M::eval_acc_jac(x, u, acc, Fq, Fqd, Fu);                                                       \
        int o = 0;                                                                                     \
        for (int i = 0; i < NA; ++i) out[o++] = acc[i];                                                \
        for (int i = 0; i < NA * NQ; ++i) out[o++] = Fq[i];                                            \
        for (int i = 0; i < NA * NA; ++i) out[o++] = Fqd[i];                                           \
        for (int i = 0; i < NA * M::NU; ++i) out[o++] = Fu[i];                                         \
    }

MODEL_KERNELS(TwoLinkArm)
MODEL_KERNELS(ExoArm)

// the lane kernel's exo evaluations: h-scaled Jacobian (backward sweep) and directional derivative (forward / step)
extern "C" __global__ void flops_acc_jac_h_ExoArm(const double* in, double* out) {
    double x[8], u[4], acc[4], Fq[16], Fqd[16], Fu[16];
    load<ExoArm>(in, x, u);
    ExoArm::eval_acc_jac_h(x, u, in[12], acc, Fq, Fqd, Fu);
    int o = 0;
    for (int i = 0; i < 4; ++i) out[o++] = acc[i];
    for (int i = 0; i < 16; ++i) out[o++] = Fq[i];
    for (int i = 0; i < 16; ++i) out[o++] = Fqd[i];
    for (int i = 0; i < 16; ++i) out[o++] = Fu[i];
}
extern "C" __global__ void flops_jvp_ExoArm(const double* in, double* out) {
    double x[8], u[4], xd[8], jv[4];
    load<ExoArm>(in, x, u);
    ExoArm::eval_jvp(x, u, in + 12, in + 20, xd, jv);
    for (int i = 0; i < 8; ++i) out[i] = xd[i];
    for (int i = 0; i < 4; ++i) out[8 + i] = jv[i];
}

extern "C" __global__ void flops_hess_TwoLinkArm(const double* in, double* out) {
    constexpr int NZ = TwoLinkArm::NX + TwoLinkArm::NU;
    double x[TwoLinkArm::NX], u[TwoLinkArm::NU], lam[2], W[NZ * NZ];
    load<TwoLinkArm>(in, x, u);
    lam[0] = in[6];
    lam[1] = in[7];
    TwoLinkArm::eval_hess(x, u, lam, W);
    for (int i = 0; i < NZ * NZ; ++i) out[i] = W[i];
}
