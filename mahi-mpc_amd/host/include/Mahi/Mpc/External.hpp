// Mahi/Mpc/External.hpp -- loader for functions with the CasADi external C ABI, standing in for
// casadi::external as the reference uses it: examples/model_control_example.cpp:46,81-82 and
// src/Mahi/Mpc/ModelControl.cpp:70-72 load <name>_get_A / _get_B / _get_x_dot_init from
// <name>_linear_functions.so (written by ModelGenerator::generate_linear_functions, ModelGenerator.cpp:241-251).
//
// The ABI (src/codegen_usage.cpp:73-181): int f(const double** arg, double** res, long long* iw, double* w,
// int mem) plus f_n_in / f_n_out / f_sparsity_in / f_sparsity_out / f_work / f_checkout / f_release /
// f_incref / f_decref.  Inputs and outputs are exchanged as dense column-major vectors (what
// std::vector<double>(casadi::DM) gives the reference's callers).
#pragma once
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include <Mahi/Mpc/SX.hpp>

namespace mahi {
namespace mpc {

class External {
public:
    External(const std::string& name, const std::string& library_path);
    // evaluate with dense inputs (sizes nrow*ncol of each input sparsity); returns dense outputs.
    // Throws std::invalid_argument on a size mismatch and std::runtime_error if the function reports failure.
    std::vector<std::vector<double>> operator()(const std::vector<std::vector<double>>& args) const;
    // the reference's call shape: std::vector<casadi::DM> in, std::vector<casadi::DM> out
    // (examples/model_control_example.cpp:81-82)
    // (a template, so that a braced list {state, control} still selects the overload above)
    template <class D, class = typename std::enable_if<std::is_same<D, DM>::value>::type>
    std::vector<DM> operator()(const std::vector<D>& args) const {
        std::vector<std::vector<double>> in(args.begin(), args.end());
        auto out = (*this)(in);
        return std::vector<DM>(out.begin(), out.end());
    }
    const std::string& name() const;
    long long n_in() const;
    long long n_out() const;
    // (nrow, ncol) of input / output i
    std::pair<long long, long long> size_in(long long i) const;
    std::pair<long long, long long> size_out(long long i) const;

private:
    struct Impl;
    std::shared_ptr<Impl> m_impl;
};

// same call shape as casadi::external(name, library)
External external(const std::string& name, const std::string& library_path);

}  // namespace mpc
}  // namespace mahi

namespace casadi {
using mahi::mpc::external;
}  // namespace casadi
