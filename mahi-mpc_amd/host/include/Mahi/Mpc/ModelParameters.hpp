// Mahi/Mpc/ModelParameters.hpp -- same struct and JSON schema as the reference
// (include/Mahi/Mpc/ModelParameters.hpp:11-28, src/Mahi/Mpc/ModelParameters.cpp:7-72).
#pragma once
#include <string>
#include <vector>

#include <Mahi/Util/Time.hpp>

namespace mahi {
namespace mpc {

struct ModelParameters {
    ModelParameters(std::string name_, int num_x_, int num_u_, mahi::util::Time step_size_, size_t num_shooting_nodes_,
                    bool is_linear_, std::vector<double> u_min_ = {}, std::vector<double> u_max_ = {},
                    std::vector<double> x_min_ = {}, std::vector<double> x_max_ = {});
    ModelParameters() {}

    std::string name;
    mahi::util::Time timespan;
    mahi::util::Time step_size;
    int num_x = 0;
    int num_u = 0;
    int num_shooting_nodes = 0;
    std::vector<double> x_min;
    std::vector<double> u_min;
    std::vector<double> x_max;
    std::vector<double> u_max;
    std::string dll_filepath;
    bool is_linear = false;
    // build extension: which built-in device model the solver runs ("" = resolve by dimensions)
    std::string mmpc_model;
};

// JSON text of {"model": {...}} with the reference keys (ModelParameters.cpp:38-49)
std::string to_json_string(const ModelParameters& p);
// parse {"model": {...}} (or the bare object); x bounds of exactly +-10e30 become +-inf (ModelParameters.cpp:59-62)
ModelParameters model_parameters_from_json_string(const std::string& text);

}  // namespace mpc
}  // namespace mahi
