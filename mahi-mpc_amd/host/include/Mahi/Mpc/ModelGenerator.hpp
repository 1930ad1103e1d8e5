// Mahi/Mpc/ModelGenerator.hpp -- counterpart of include/Mahi/Mpc/ModelGenerator.hpp:10-30.
//
// Reference flow (ModelGenerator.cpp:23-270): the caller gives x, x_dot = f(x, u) and u as casadi::SX; create_model()
// builds the multiple-shooting NLP and the linearisation functions get_A/get_B/get_x_dot_init (compiled at once
// into <name>_linear_functions.so), generate_c_code() writes the NLP's C code, compile_model() compiles it into
// <name>.so and writes <name>.json.
//
// Here: the same calls on the build's SX type (Mahi/Mpc/SX.hpp).  create_model() differentiates f symbolically
// and writes <name>_linear_functions.{c,so} with the CasADi external ABI (host C, gcc, as the reference);
// generate_c_code() emits the dynamics and their Jacobian blocks as a gfx950 device model (<name>_model.h);
// compile_model() compiles the solver kernels (mahi-mpc_amd/csrc/mmpc.hip) for that model with hipcc into
// <name>.so -- a library exporting the C-ABI of include/mmpc.h for this one model -- and writes <name>.json with
// dll_filepath = <name>.so, which ModelControl / mmpc.Solver load.  The NLP itself needs no generated code: it is
// fixed by construction in the kernels (ModelGenerator.cpp:191-222).
//
// Build extension: ModelGenerator(params, "two_link_arm" | "exo_arm") selects a built-in device model of
// libmmpc.so instead of SX dynamics.
#pragma once
#include <string>

#include <Mahi/Mpc/ModelParameters.hpp>
#include <Mahi/Mpc/SX.hpp>

namespace mahi {
namespace mpc {

// Device code of the weighted second derivatives of the accelerations (the part of CasADi's nlp_hess_l,
// ModelGenerator.cpp:238, that depends on the dynamics): a member function
//   MMPC_HD static void eval_hess(const double* x, const double* u, const double* lam, double* W)
// with W = sum_{s < nx - nq} lam[s] d^2 x_dot[nq + s] / d(x, u)^2, (nx+nu) x (nx+nu) row-major (symmetric; the
// kinematic rows q_dot = z[0:nq] are linear).  Symbolic: jacobian of jacobian of lam^T acc, CSE'd straight-line code.
std::string emit_device_hessian(const SX& x, const SX& x_dot, const SX& u, int nq, const std::string& indent = "    ");

class ModelGenerator {
public:
    ModelGenerator(ModelParameters model_parameters, SX x, SX x_dot, SX u);  // ModelGenerator.hpp:23
    ModelGenerator(ModelParameters model_parameters, std::string builtin_dynamics = "two_link_arm");
    ~ModelGenerator();
    void create_model();
    void generate_c_code();
    // <name>_linear_functions.{c,so}: the three functions with the CasADi external C ABI (ModelGenerator.cpp:241-251)
    void generate_linear_functions(Function get_A, Function get_B, Function get_x_dot_init);
    void generate_linear_functions();  // built-in model: externals over libmmpc's device linearisation
    void compile_model();
    void save_param_file();

    const ModelParameters& parameters() const { return m_model_parameters; }
    // kinematic rows detected in x_dot (x = [q; z], q_dot = z[0:nq]); 0 = a general first-order model
    int kinematic_rows() const { return m_nq; }
    const std::string& c_file_filepath() const { return m_c_file_filepath; }

private:
    ModelParameters m_model_parameters;
    SX m_x, m_x_dot, m_u;
    bool m_symbolic = false;
    bool m_created = false;
    int m_nq = 0;
    SX m_A, m_B;  // jacobian(x_dot, x), jacobian(x_dot, u)
    std::string m_c_file_filepath;
};

}  // namespace mpc
}  // namespace mahi
