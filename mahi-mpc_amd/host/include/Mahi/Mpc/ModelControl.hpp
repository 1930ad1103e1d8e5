// Mahi/Mpc/ModelControl.hpp -- drop-in for the reference class (include/Mahi/Mpc/ModelControl.hpp:13-80).
// Same public members and method signatures; the IPOPT call of calc_u (ModelControl.cpp:159) is replaced by
// the MI355X batched SQP behind include/mmpc.h.  casadi::Dict is replaced by mahi::mpc::Dict.
#pragma once
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <Mahi/Mpc/External.hpp>
#include <Mahi/Mpc/ModelParameters.hpp>
#include <Mahi/Mpc/SX.hpp>
#include <Mahi/Util/Time.hpp>

struct mmpc_handle;

namespace mahi {
namespace mpc {
namespace detail {
struct ModelLibrary;
}

using Dict = std::map<std::string, double>;

class ModelControl {
public:
    struct ControlResult {
        ControlResult(mahi::util::Time time_, std::vector<double> x_est_, std::vector<double> u_)
            : time(time_), x_est(x_est_), u(u_) {}
        mahi::util::Time time;
        std::vector<double> x_est;
        std::vector<double> u;
    };

    ModelControl(std::string model_name, std::vector<double> Q = {}, std::vector<double> R = {},
                 std::vector<double> Rm = {}, Dict solver_opts = Dict());
    ~ModelControl();
    ModelControl(const ModelControl&) = delete;
    ModelControl& operator=(const ModelControl&) = delete;

    ModelParameters model_parameters;
    std::vector<ControlResult> control_results;

    void calc_u(mahi::util::Time time, const std::vector<double>& state, const std::vector<double>& control,
                std::vector<double> traj);
    void load_model(const std::string& model_name);

    ControlResult control_at_time(mahi::util::Time time);

    void start_calc();
    void stop_calc();

    void set_state(mahi::util::Time time, const std::vector<double>& state, const std::vector<double>& control,
                   std::vector<double> traj);

    void update_weights(std::vector<double> Q = {}, std::vector<double> R = {}, std::vector<double> Rm = {});
    void update_control_limits(std::vector<double> u_min, std::vector<double> u_max);

    // ---- build extensions (not in the reference) ----
    // solver status of the last calc_u (the reference ignores IPOPT's status, ModelControl.cpp:159-161)
    int last_status() const { return m_last_status; }
    int last_iterations() const { return m_last_iters; }
    double last_kkt_residual() const { return m_last_kkt; }
    // B independent instances in one GPU call (states/controls/trajs instance-major); returns V* per instance
    std::vector<std::vector<double>> calc_u_batch(const std::vector<std::vector<double>>& states,
                                                  const std::vector<std::vector<double>>& controls,
                                                  const std::vector<std::vector<double>>& trajs,
                                                  std::vector<int>* status = nullptr);

private:
    std::shared_ptr<detail::ModelLibrary> m_backend;  // C-ABI of the model's library (dll_filepath)
    Dict m_solver_opts;
    mahi::util::Time curr_time;
    mmpc_handle* m_handle = nullptr;
    std::vector<double> m_V;  // warm start = previous solution (ModelControl.cpp:160-161)

    std::vector<double> m_Q, m_R, m_Rm;

    std::atomic<bool> m_stop{true};
    std::atomic<bool> m_done_calcing{true};
    std::thread m_thread;

    mahi::util::Time m_time;
    std::vector<double> m_state, m_control, m_traj;

    std::mutex m_state_mutex;
    std::mutex m_output_mutex;
    std::mutex m_control_limits_mutex;
    std::mutex m_weights_mutex;

    int m_last_status = -1;
    int m_last_iters = 0;
    double m_last_kkt = 0.0;

    void format_outputs(const std::vector<double>& opt_output);
    std::vector<double> packed_weights();
};

}  // namespace mpc
}  // namespace mahi

namespace casadi {
using mahi::mpc::Dict;   // the solver_opts type of the reference's constructor (ModelControl.hpp:26)
}  // namespace casadi
