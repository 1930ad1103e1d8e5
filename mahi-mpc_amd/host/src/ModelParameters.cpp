// ModelParameters: constructor defaults (src/Mahi/Mpc/ModelParameters.cpp:7-25) and the JSON schema
// of to_json / from_json (:37-72), written without nlohmann/mahi-util.
#include <Mahi/Mpc/ModelParameters.hpp>

#include <cmath>
#include <cstdio>
#include <limits>
#include <sstream>
#include <stdexcept>

#include "../../csrc/json_lite.h"

namespace mahi {
namespace mpc {

ModelParameters::ModelParameters(std::string name_, int num_x_, int num_u_, mahi::util::Time step_size_,
                                 size_t num_shooting_nodes_, bool is_linear_, std::vector<double> u_min_,
                                 std::vector<double> u_max_, std::vector<double> x_min_, std::vector<double> x_max_)
    : name(name_),
      step_size(step_size_),
      num_x(num_x_),
      num_u(num_u_),
      num_shooting_nodes(static_cast<int>(num_shooting_nodes_)),
      x_min(x_min_),
      u_min(u_min_),
      x_max(x_max_),
      u_max(u_max_),
      is_linear(is_linear_) {
    timespan = mahi::util::microseconds(step_size.as_microseconds() * static_cast<int64_t>(num_shooting_nodes_));
    if (x_min.empty()) x_min = std::vector<double>(num_x, -10e30);
    if (x_max.empty()) x_max = std::vector<double>(num_x, 10e30);
    if (u_min.empty()) u_min = std::vector<double>(num_u, -10e30);
    if (u_max.empty()) u_max = std::vector<double>(num_u, 10e30);
}

namespace {
std::string num(double v) {
    if (std::isinf(v) || std::isnan(v)) return "null";  // what nlohmann::json writes for +-inf / nan
    char b[40];
    std::snprintf(b, sizeof b, "%.17g", v);
    return b;
}
std::string arr(const std::vector<double>& v) {
    std::string s = "[";
    for (size_t i = 0; i < v.size(); ++i) s += (i ? "," : "") + num(v[i]);
    return s + "]";
}
std::string quote(const std::string& s) {
    std::string o = "\"";
    for (char c : s) {
        if (c == '"' || c == '\\') o += '\\';
        o += c;
    }
    return o + "\"";
}
std::vector<double> get_vec(const mmpc::json::Value& m, const char* k, int n, double dflt) {
    std::vector<double> out(n, dflt);
    const mmpc::json::Value* v = m.get(k);
    if (!v || v->kind != mmpc::json::Value::Array) return out;
    out.assign(v->arr.size(), dflt);
    for (size_t i = 0; i < v->arr.size(); ++i)
        if (v->arr[i].kind == mmpc::json::Value::Number) out[i] = v->arr[i].num;
    return out;
}
double get_num(const mmpc::json::Value& m, const char* k) {
    const mmpc::json::Value* v = m.get(k);
    if (!v || v->kind != mmpc::json::Value::Number) throw std::runtime_error(std::string("model json: missing ") + k);
    return v->num;
}
}  // namespace

std::string to_json_string(const ModelParameters& p) {
    std::ostringstream o;
    o << "{\"model\":{\"name\":" << quote(p.name) << ",\"timespan\":" << p.timespan.as_microseconds()
      << ",\"step_size\":" << p.step_size.as_microseconds() << ",\"num_x\":" << p.num_x << ",\"num_u\":" << p.num_u
      << ",\"num_shooting_nodes\":" << p.num_shooting_nodes << ",\"x_min\":" << arr(p.x_min)
      << ",\"u_min\":" << arr(p.u_min) << ",\"x_max\":" << arr(p.x_max) << ",\"u_max\":" << arr(p.u_max)
      << ",\"dll_filepath\":" << quote(p.dll_filepath) << ",\"is_linear\":" << (p.is_linear ? "true" : "false");
    if (!p.mmpc_model.empty()) o << ",\"mmpc_model\":" << quote(p.mmpc_model);
    o << "}}";
    return o.str();
}

ModelParameters model_parameters_from_json_string(const std::string& text) {
    mmpc::json::Value root = mmpc::json::parse(text);
    const mmpc::json::Value* m = root.get("model");
    if (!m) m = &root;
    ModelParameters p;
    const mmpc::json::Value* nm = m->get("name");
    if (!nm || nm->kind != mmpc::json::Value::String) throw std::runtime_error("model json: missing name");
    p.name = nm->str;
    p.timespan = mahi::util::microseconds(static_cast<int64_t>(get_num(*m, "timespan")));
    p.step_size = mahi::util::microseconds(static_cast<int64_t>(get_num(*m, "step_size")));
    p.num_x = static_cast<int>(get_num(*m, "num_x"));
    p.num_u = static_cast<int>(get_num(*m, "num_u"));
    p.num_shooting_nodes = static_cast<int>(get_num(*m, "num_shooting_nodes"));
    const double inf = std::numeric_limits<double>::infinity();
    p.x_min = get_vec(*m, "x_min", p.num_x, -inf);
    p.u_min = get_vec(*m, "u_min", p.num_u, -10e30);
    p.x_max = get_vec(*m, "x_max", p.num_x, inf);
    p.u_max = get_vec(*m, "u_max", p.num_u, 10e30);
    const mmpc::json::Value* dl = m->get("dll_filepath");
    if (dl && dl->kind == mmpc::json::Value::String) p.dll_filepath = dl->str;
    const mmpc::json::Value* li = m->get("is_linear");
    p.is_linear = li && li->kind == mmpc::json::Value::Bool && li->b;
    const mmpc::json::Value* mm = m->get("mmpc_model");
    if (mm && mm->kind == mmpc::json::Value::String) p.mmpc_model = mm->str;
    for (size_t i = 0; i < p.x_min.size(); ++i) {  // ModelParameters.cpp:59-62
        if (p.x_min[i] == -10e30) p.x_min[i] = -inf;
        if (i < p.x_max.size() && p.x_max[i] == 10e30) p.x_max[i] = inf;
    }
    return p;
}

}  // namespace mpc
}  // namespace mahi
