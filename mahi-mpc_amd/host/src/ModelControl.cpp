// ModelControl: the reference's online controller (src/Mahi/Mpc/ModelControl.cpp) with the IPOPT call
// replaced by the C-ABI of include/mmpc.h.  Packing follows ModelControl.cpp:116-172; output formatting
// :174-190; control_at_time :192-197; the async thread :75-114.
#include <Mahi/Mpc/ModelControl.hpp>

#include <dlfcn.h>

#include <chrono>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>

#include "../../../include/mmpc.h"
#include "model_library.hpp"

namespace mahi {
namespace mpc {

using detail::ModelLibrary;

ModelControl::ModelControl(std::string model_name, std::vector<double> Q, std::vector<double> R,
                           std::vector<double> Rm, Dict solver_opts)
    : m_solver_opts(solver_opts), m_Q(Q), m_R(R), m_Rm(Rm) {
    // like the reference, solver_opts are stored but not applied (ModelControl.cpp:7-11 vs :52-62)
    load_model(model_name);
}

ModelControl::~ModelControl() {
    m_stop = true;
    if (m_thread.joinable()) m_thread.join();  // the reference busy-waits on m_done_calcing (:16-19)
    if (m_handle) m_backend->destroy(m_handle);
}

void ModelControl::load_model(const std::string& model_name) {
    const std::string path = model_name + ".json";  // ModelControl.cpp:24
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    model_parameters = model_parameters_from_json_string(ss.str());
    if (m_handle) m_backend->destroy(m_handle);
    m_handle = nullptr;
    m_backend = ModelLibrary::load(model_parameters, path);
    m_backend->check(m_backend->create_from_json(ss.str().c_str(), nullptr, &m_handle), "mmpc_create");
    mmpc_model_info info;
    m_backend->check(m_backend->get_model_info(m_handle, &info), "mmpc_get_model_info");
    m_V.assign(static_cast<size_t>(info.num_v), 0.0);  // v_init = 0 (ModelControl.cpp:29-50)
}

std::vector<double> ModelControl::packed_weights() {
    std::lock_guard<std::mutex> lg(m_weights_mutex);
    const size_t nx = model_parameters.num_x, nu = model_parameters.num_u;
    // the reference would hand CasADi a p of the wrong length here
    if (m_Q.size() != nx || m_R.size() != nu || m_Rm.size() != nu)
        throw std::invalid_argument("ModelControl: Q, R, Rm must have num_x, num_u, num_u entries");
    std::vector<double> w;
    w.insert(w.end(), m_Q.begin(), m_Q.end());     // ModelControl.cpp:120
    w.insert(w.end(), m_R.begin(), m_R.end());     // :121
    w.insert(w.end(), m_Rm.begin(), m_Rm.end());   // :122
    return w;
}

void ModelControl::calc_u(mahi::util::Time control_time, const std::vector<double>& state,
                          const std::vector<double>& control, std::vector<double> traj) {
    curr_time = control_time;
    const size_t nx = model_parameters.num_x, nu = model_parameters.num_u, N = model_parameters.num_shooting_nodes;
    if (state.size() != nx || control.size() != nu || traj.size() != N * nx)
        throw std::invalid_argument("ModelControl::calc_u: state/control/traj size mismatch");
    const std::vector<double> w = packed_weights();
    std::vector<double> lb, ub;
    {
        std::lock_guard<std::mutex> lg(m_control_limits_mutex);  // ModelControl.cpp:148-154
        lb = model_parameters.u_min;
        ub = model_parameters.u_max;
    }
    int32_t st = -1, it = 0;
    double kkt = 0.0;
    // linear mode: the per-step linearisation at (state, control) of ModelControl.cpp:125-135 happens on the
    // device inside the solve; x_0 is pinned to `state` (ModelControl.cpp:144-145)
    m_backend->check(m_backend->solve_batch_host(m_handle, 1, state.data(), control.data(), traj.data(), w.data(), 0,
                                lb.size() == nu ? lb.data() : nullptr, ub.size() == nu ? ub.data() : nullptr,
                                m_V.data(), &st, &it, &kkt),
          "mmpc_solve_batch_host");
    m_last_status = st;
    m_last_iters = it;
    m_last_kkt = kkt;
    format_outputs(m_V);  // m_V stays as the next warm start (ModelControl.cpp:160-161)
}

std::vector<std::vector<double>> ModelControl::calc_u_batch(const std::vector<std::vector<double>>& states,
                                                            const std::vector<std::vector<double>>& controls,
                                                            const std::vector<std::vector<double>>& trajs,
                                                            std::vector<int>* status) {
    const size_t nx = model_parameters.num_x, nu = model_parameters.num_u, N = model_parameters.num_shooting_nodes;
    const size_t B = states.size();
    if (controls.size() != B || trajs.size() != B) throw std::invalid_argument("calc_u_batch: batch size mismatch");
    std::vector<double> x0, up, tr, V(B * m_V.size(), 0.0);
    for (size_t b = 0; b < B; ++b) {
        if (states[b].size() != nx || controls[b].size() != nu || trajs[b].size() != N * nx)
            throw std::invalid_argument("calc_u_batch: instance size mismatch");
        x0.insert(x0.end(), states[b].begin(), states[b].end());
        up.insert(up.end(), controls[b].begin(), controls[b].end());
        tr.insert(tr.end(), trajs[b].begin(), trajs[b].end());
    }
    const std::vector<double> w = packed_weights();
    std::vector<double> lb, ub;
    {
        std::lock_guard<std::mutex> lg(m_control_limits_mutex);  // the limits calc_u enforces (ModelControl.cpp:148-154)
        lb = model_parameters.u_min;
        ub = model_parameters.u_max;
    }
    std::vector<int32_t> st(B, -1), it(B, 0);
    std::vector<double> kkt(B, 0.0);
    m_backend->check(m_backend->solve_batch_host(m_handle, static_cast<int64_t>(B), x0.data(), up.data(), tr.data(), w.data(), 0,
                                lb.size() == nu ? lb.data() : nullptr, ub.size() == nu ? ub.data() : nullptr,
                                V.data(), st.data(), it.data(), kkt.data()),
          "mmpc_solve_batch_host");
    std::vector<std::vector<double>> out(B);
    for (size_t b = 0; b < B; ++b) out[b].assign(V.begin() + b * m_V.size(), V.begin() + (b + 1) * m_V.size());
    if (status) status->assign(st.begin(), st.end());
    return out;
}

void ModelControl::format_outputs(const std::vector<double>& opt_output) {
    std::vector<ControlResult> local;
    const size_t nx = model_parameters.num_x, nu = model_parameters.num_u;
    for (size_t i = 0; i < static_cast<size_t>(model_parameters.num_shooting_nodes); i++) {
        std::vector<double> x(opt_output.begin() + i * (nx + nu), opt_output.begin() + i * (nx + nu) + nx);
        std::vector<double> u(opt_output.begin() + i * (nx + nu) + nx, opt_output.begin() + i * (nx + nu) + nx + nu);
        local.emplace_back(mahi::util::seconds(curr_time.as_seconds() + model_parameters.step_size.as_seconds() * i),
                           x, u);
    }
    std::lock_guard<std::mutex> lg(m_output_mutex);
    control_results = local;
}

ModelControl::ControlResult ModelControl::control_at_time(mahi::util::Time time) {
    std::lock_guard<std::mutex> lg(m_output_mutex);
    // the reference indexes an empty vector before the first solve (ModelControl.cpp:195); this throws instead
    if (control_results.empty()) throw std::logic_error("control_at_time before the first calc_u");
    size_t i = 0;
    while (i < control_results.size() && control_results[i].time < time) i++;
    return (i == 0) ? control_results[0] : control_results[i - 1];
}

void ModelControl::set_state(mahi::util::Time time, const std::vector<double>& state,
                             const std::vector<double>& control, std::vector<double> traj) {
    std::lock_guard<std::mutex> lg(m_state_mutex);
    m_time = time;
    m_state = state;
    m_control = control;
    m_traj = traj;
}

void ModelControl::start_calc() {
    if (m_thread.joinable()) {
        m_stop = true;
        m_thread.join();
    }
    m_stop = false;
    m_done_calcing = false;
    m_thread = std::thread([this] {
        double total_ms = 0.0;
        size_t n = 0;
        while (!m_stop) {
            mahi::util::Time t;
            std::vector<double> s, c, tr;
            {
                std::lock_guard<std::mutex> lg(m_state_mutex);
                t = m_time;
                s = m_state;
                c = m_control;
                tr = m_traj;
            }
            if (s.empty()) {
                std::this_thread::yield();
                continue;
            }
            const auto t0 = std::chrono::steady_clock::now();
            calc_u(t, s, c, tr);
            total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            ++n;
        }
        if (n) std::cout << "Average calc time: " << total_ms / n << " ms" << std::endl;  // ModelControl.cpp:108
        m_done_calcing = true;
    });
}

void ModelControl::stop_calc() {
    m_stop = true;
    if (m_thread.joinable()) m_thread.join();
}

void ModelControl::update_weights(std::vector<double> Q, std::vector<double> R, std::vector<double> Rm) {
    std::lock_guard<std::mutex> lg(m_weights_mutex);
    if (!Q.empty()) m_Q = Q;
    if (!R.empty()) m_R = R;
    if (!Rm.empty()) m_Rm = Rm;
}

void ModelControl::update_control_limits(std::vector<double> u_min, std::vector<double> u_max) {
    std::lock_guard<std::mutex> lg(m_control_limits_mutex);
    model_parameters.u_min = u_min;
    model_parameters.u_max = u_max;
}

}  // namespace mpc
}  // namespace mahi
