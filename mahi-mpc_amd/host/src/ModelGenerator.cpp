// ModelGenerator: offline step of the reference (src/Mahi/Mpc/ModelGenerator.cpp:23-270) reduced to what a
// built-in device model needs: validation and the <name>.json artefact.
#include <Mahi/Mpc/ModelGenerator.hpp>

#include <fstream>
#include <iostream>
#include <stdexcept>

namespace mahi {
namespace mpc {

ModelGenerator::ModelGenerator(ModelParameters model_parameters, std::string dynamics)
    : m_model_parameters(std::move(model_parameters)) {
    m_model_parameters.mmpc_model = dynamics;
}

ModelGenerator::~ModelGenerator() {}

void ModelGenerator::create_model() {
    const ModelParameters& p = m_model_parameters;
    if (p.mmpc_model == "two_link_arm" || p.mmpc_model == "double_pendulum") {
        if (p.num_x != 4 || p.num_u != 2) throw std::invalid_argument("two_link_arm needs num_x = 4, num_u = 2");
    } else {
        throw std::invalid_argument("unknown built-in model \"" + p.mmpc_model + "\"");
    }
    if (p.num_shooting_nodes < 1 || p.num_shooting_nodes * p.num_u > 64)
        throw std::invalid_argument("num_shooting_nodes * num_u must be in [1, 64] for the single-wave kernel");
    std::cout << "generating a " << (p.is_linear ? "" : "non") << "linear model with " << p.num_shooting_nodes
              << " shooting nodes over " << p.timespan.as_seconds() << " seconds with " << p.num_x << " states, and "
              << p.num_u << " control variables" << std::endl;  // ModelGenerator.cpp:25
    m_created = true;
}

void ModelGenerator::generate_c_code() {
    if (!m_created) throw std::logic_error("create_model() first");
}

void ModelGenerator::compile_model() {
    if (!m_created) throw std::logic_error("create_model() first");
    m_model_parameters.dll_filepath = "libmmpc.so";
    save_param_file();
}

void ModelGenerator::save_param_file() {
    std::ofstream f(m_model_parameters.name + ".json");
    if (!f) throw std::runtime_error("cannot write " + m_model_parameters.name + ".json");
    f << to_json_string(m_model_parameters);
}

}  // namespace mpc
}  // namespace mahi
