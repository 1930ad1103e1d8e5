// CasADi-external-ABI loader (see Mahi/Mpc/External.hpp).  Sparse inputs/outputs are scattered from/to
// dense column-major storage through their CCS patterns [nrow, ncol, colind[ncol+1], row[nnz]]
// (src/codegen_usage.cpp:128-132).
#include <Mahi/Mpc/External.hpp>

#include <dlfcn.h>
#include <sys/stat.h>

#include <mutex>
#include <stdexcept>

namespace mahi {
namespace mpc {

namespace {
typedef long long casadi_int;
typedef int (*eval_t)(const double**, double**, casadi_int*, double*, int);
typedef casadi_int (*getint_t)(void);
typedef const casadi_int* (*sparsity_t)(casadi_int);
typedef int (*work_t)(casadi_int*, casadi_int*, casadi_int*, casadi_int*);
typedef int (*checkout_t)(void);
typedef void (*release_t)(int);
typedef void (*signal_t)(void);

struct Pattern {
    casadi_int nrow = 0, ncol = 0;
    std::vector<casadi_int> colind, row;
    casadi_int nnz() const { return colind.empty() ? 0 : colind.back(); }
};

Pattern read_pattern(const casadi_int* sp) {
    if (!sp) throw std::runtime_error("external: missing sparsity pattern");
    Pattern p;
    p.nrow = sp[0];
    p.ncol = sp[1];
    p.colind.assign(sp + 2, sp + 3 + p.ncol);
    p.row.assign(sp + 3 + p.ncol, sp + 3 + p.ncol + p.colind.back());
    return p;
}

template <class F>
F sym(void* dl, const std::string& name, bool required) {
    dlerror();
    void* s = dlsym(dl, name.c_str());
    if (!s && required) throw std::runtime_error("external: symbol " + name + " not found");
    return reinterpret_cast<F>(s);
}
}  // namespace

struct External::Impl {
    std::string name;
    void* dl = nullptr;
    eval_t eval = nullptr;
    checkout_t checkout = nullptr;
    release_t release = nullptr;
    signal_t decref = nullptr;
    std::vector<Pattern> in, out;
    casadi_int sz_arg = 0, sz_res = 0, sz_iw = 0, sz_w = 0;
    mutable std::mutex mu;
    ~Impl() {
        if (decref) decref();
        // the library stays mapped: its device handle lives until process exit
    }
};

External::External(const std::string& name, const std::string& library_path) : m_impl(std::make_shared<Impl>()) {
    Impl& m = *m_impl;
    m.name = name;
    std::string path = library_path;
    struct stat st;
    if (path.find('/') == std::string::npos && stat(path.c_str(), &st) == 0) path = "./" + path;  // cwd first
    m.dl = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!m.dl) throw std::runtime_error("external: cannot load " + library_path + ": " + dlerror());
    m.eval = sym<eval_t>(m.dl, name, true);
    getint_t n_in = sym<getint_t>(m.dl, name + "_n_in", true);
    getint_t n_out = sym<getint_t>(m.dl, name + "_n_out", true);
    sparsity_t sp_in = sym<sparsity_t>(m.dl, name + "_sparsity_in", true);
    sparsity_t sp_out = sym<sparsity_t>(m.dl, name + "_sparsity_out", true);
    work_t work = sym<work_t>(m.dl, name + "_work", false);
    m.checkout = sym<checkout_t>(m.dl, name + "_checkout", false);
    m.release = sym<release_t>(m.dl, name + "_release", false);
    signal_t incref = sym<signal_t>(m.dl, name + "_incref", false);
    m.decref = sym<signal_t>(m.dl, name + "_decref", false);
    for (casadi_int i = 0; i < n_in(); i++) m.in.push_back(read_pattern(sp_in(i)));
    for (casadi_int i = 0; i < n_out(); i++) m.out.push_back(read_pattern(sp_out(i)));
    m.sz_arg = n_in();
    m.sz_res = n_out();
    if (work && work(&m.sz_arg, &m.sz_res, &m.sz_iw, &m.sz_w)) throw std::runtime_error("external: work() failed");
    if (incref) incref();
}

std::vector<std::vector<double>> External::operator()(const std::vector<std::vector<double>>& args) const {
    const Impl& m = *m_impl;
    if (args.size() != m.in.size())
        throw std::invalid_argument("external " + m.name + ": expected " + std::to_string(m.in.size()) + " inputs");
    std::vector<std::vector<double>> nz_in(m.in.size());
    std::vector<const double*> arg(static_cast<size_t>(m.sz_arg), nullptr);
    for (size_t i = 0; i < m.in.size(); i++) {
        const Pattern& p = m.in[i];
        if (static_cast<casadi_int>(args[i].size()) != p.nrow * p.ncol)
            throw std::invalid_argument("external " + m.name + ": input " + std::to_string(i) + " has " +
                                        std::to_string(args[i].size()) + " entries, expected " +
                                        std::to_string(p.nrow * p.ncol));
        nz_in[i].resize(static_cast<size_t>(p.nnz()));
        for (casadi_int c = 0; c < p.ncol; c++)
            for (casadi_int e = p.colind[c]; e < p.colind[c + 1]; e++) nz_in[i][e] = args[i][c * p.nrow + p.row[e]];
        arg[i] = nz_in[i].data();
    }
    std::vector<std::vector<double>> nz_out(m.out.size());
    std::vector<double*> res(static_cast<size_t>(m.sz_res), nullptr);
    for (size_t i = 0; i < m.out.size(); i++) {
        nz_out[i].assign(static_cast<size_t>(m.out[i].nnz()), 0.0);
        res[i] = nz_out[i].data();
    }
    std::vector<casadi_int> iw(static_cast<size_t>(m.sz_iw));
    std::vector<double> w(static_cast<size_t>(m.sz_w));
    int rc;
    {
        std::lock_guard<std::mutex> lk(m.mu);  // checkout/release are not thread-safe (codegen_usage.cpp:176-181)
        const int mem = m.checkout ? m.checkout() : 0;
        rc = m.eval(arg.data(), res.data(), iw.data(), w.data(), mem);
        if (m.release) m.release(mem);
    }
    if (rc) throw std::runtime_error("external " + m.name + ": evaluation failed");
    std::vector<std::vector<double>> out(m.out.size());
    for (size_t i = 0; i < m.out.size(); i++) {
        const Pattern& p = m.out[i];
        out[i].assign(static_cast<size_t>(p.nrow * p.ncol), 0.0);
        for (casadi_int c = 0; c < p.ncol; c++)
            for (casadi_int e = p.colind[c]; e < p.colind[c + 1]; e++) out[i][c * p.nrow + p.row[e]] = nz_out[i][e];
    }
    return out;
}

const std::string& External::name() const { return m_impl->name; }
long long External::n_in() const { return static_cast<long long>(m_impl->in.size()); }
long long External::n_out() const { return static_cast<long long>(m_impl->out.size()); }
std::pair<long long, long long> External::size_in(long long i) const {
    return {m_impl->in.at(static_cast<size_t>(i)).nrow, m_impl->in.at(static_cast<size_t>(i)).ncol};
}
std::pair<long long, long long> External::size_out(long long i) const {
    return {m_impl->out.at(static_cast<size_t>(i)).nrow, m_impl->out.at(static_cast<size_t>(i)).ncol};
}

External external(const std::string& name, const std::string& library_path) { return External(name, library_path); }

}  // namespace mpc
}  // namespace mahi
