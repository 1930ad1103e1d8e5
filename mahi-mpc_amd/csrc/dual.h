// dual.h -- forward-mode dual numbers for the device dynamics.
//
// Replaces CasADi's symbolic jacobian(m_x_dot, m_x) / jacobian(m_x_dot, m_u)
// (src/Mahi/Mpc/ModelGenerator.cpp:45-46): the model's x_dot(x,u) is written
// once as a template over the scalar type and evaluated either with double
// (values) or with Dual<NX+NU> (values + the full [df/dx | df/du] row).
#pragma once
#include <hip/hip_runtime.h>

namespace mmpc {

template <int K>
struct Dual {
    double v;
    double d[K];
};

#define MMPC_HD __device__ __forceinline__

template <int K>
MMPC_HD Dual<K> dual_const(double c) {
    Dual<K> r;
    r.v = c;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = 0.0;
    return r;
}
template <int K>
MMPC_HD Dual<K> dual_var(double v, int idx) {
    Dual<K> r;
    r.v = v;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = (i == idx) ? 1.0 : 0.0;
    return r;
}

template <int K>
MMPC_HD Dual<K> operator+(const Dual<K>& a, const Dual<K>& b) {
    Dual<K> r;
    r.v = a.v + b.v;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = a.d[i] + b.d[i];
    return r;
}
template <int K>
MMPC_HD Dual<K> operator-(const Dual<K>& a, const Dual<K>& b) {
    Dual<K> r;
    r.v = a.v - b.v;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = a.d[i] - b.d[i];
    return r;
}
template <int K>
MMPC_HD Dual<K> operator-(const Dual<K>& a) {
    Dual<K> r;
    r.v = -a.v;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = -a.d[i];
    return r;
}
template <int K>
MMPC_HD Dual<K> operator*(const Dual<K>& a, const Dual<K>& b) {
    Dual<K> r;
    r.v = a.v * b.v;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = fma(a.d[i], b.v, a.v * b.d[i]);
    return r;
}
template <int K>
MMPC_HD Dual<K> operator*(double s, const Dual<K>& a) {
    Dual<K> r;
    r.v = s * a.v;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = s * a.d[i];
    return r;
}
template <int K>
MMPC_HD Dual<K> operator*(const Dual<K>& a, double s) {
    return s * a;
}
template <int K>
MMPC_HD Dual<K> operator+(const Dual<K>& a, double s) {
    Dual<K> r = a;
    r.v += s;
    return r;
}
template <int K>
MMPC_HD Dual<K> operator-(const Dual<K>& a, double s) {
    Dual<K> r = a;
    r.v -= s;
    return r;
}
template <int K>
MMPC_HD Dual<K> operator+(double s, const Dual<K>& a) {
    return a + s;
}
template <int K>
MMPC_HD Dual<K> operator-(double s, const Dual<K>& a) {
    Dual<K> r;
    r.v = s - a.v;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = -a.d[i];
    return r;
}
// a constant of the scalar type (generated model code)
template <class T>
struct Lift {
    static MMPC_HD T from(double c) { return c; }
};
template <int K>
struct Lift<Dual<K>> {
    static MMPC_HD Dual<K> from(double c) { return dual_const<K>(c); }
};
template <class T>
MMPC_HD T lift(double c) {
    return Lift<T>::from(c);
}
template <int K>
MMPC_HD Dual<K> operator/(const Dual<K>& a, const Dual<K>& b) {
    Dual<K> r;
    const double ib = 1.0 / b.v;
    r.v = a.v * ib;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = (a.d[i] - r.v * b.d[i]) * ib;
    return r;
}
template <int K>
MMPC_HD Dual<K> operator/(double s, const Dual<K>& b) {
    Dual<K> r;
    const double ib = 1.0 / b.v;
    r.v = s * ib;
    const double k = -r.v * ib;
#pragma unroll
    for (int i = 0; i < K; ++i) r.d[i] = k * b.d[i];
    return r;
}

// scalar-generic elementary functions used by the model templates
MMPC_HD void mm_sincos(double x, double& s, double& c) { sincos(x, &s, &c); }
MMPC_HD double mm_cos(double x) { return cos(x); }
MMPC_HD double mm_sin(double x) { return sin(x); }

template <int K>
MMPC_HD void mm_sincos(const Dual<K>& x, Dual<K>& s, Dual<K>& c) {
    double sv, cv;
    sincos(x.v, &sv, &cv);
    s.v = sv;
    c.v = cv;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        s.d[i] = cv * x.d[i];
        c.d[i] = -sv * x.d[i];
    }
}
template <int K>
MMPC_HD Dual<K> mm_cos(const Dual<K>& x) {
    Dual<K> s, c;
    mm_sincos(x, s, c);
    return c;
}
template <int K>
MMPC_HD Dual<K> mm_sin(const Dual<K>& x) {
    Dual<K> s, c;
    mm_sincos(x, s, c);
    return s;
}

}  // namespace mmpc
