// Mahi/Mpc/ModelGenerator.hpp -- counterpart of include/Mahi/Mpc/ModelGenerator.hpp:10-30.
// The reference builds the NLP symbolically with CasADi and compiles generated C (ModelGenerator.cpp:23-259).
// Here the dynamics are built-in device models (mahi-mpc_amd/csrc/models.h) selected by name, the NLP is
// fixed by construction (the HIP kernel implements ModelGenerator.cpp:191-222 directly), and
// compile_model() writes the same <name>.json artefact the reference writes.
#pragma once
#include <string>

#include <Mahi/Mpc/ModelParameters.hpp>

namespace mahi {
namespace mpc {

class ModelGenerator {
public:
    // dynamics: name of a built-in model ("two_link_arm" == examples/ex_model_generate.cpp:24-43, "exo_arm")
    ModelGenerator(ModelParameters model_parameters, std::string dynamics = "two_link_arm");
    ~ModelGenerator();
    void create_model();      // validates dimensions, then generate_linear_functions()
    // <name>_linear_functions.{c,so}: <name>_get_A/_get_B/_get_x_dot_init with the CasADi external ABI
    void generate_linear_functions();
    void generate_c_code();   // nothing to generate: the device code is compiled into libmmpc.so
    void compile_model();     // sets dll_filepath to libmmpc.so and writes <name>.json
    void save_param_file();   // <name>.json (ModelGenerator.cpp:261-270)
    const ModelParameters& parameters() const { return m_model_parameters; }

private:
    ModelParameters m_model_parameters;
    bool m_created = false;
};

}  // namespace mpc
}  // namespace mahi
