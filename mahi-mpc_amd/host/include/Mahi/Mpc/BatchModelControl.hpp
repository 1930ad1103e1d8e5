// Mahi/Mpc/BatchModelControl.hpp -- the reference's online controller (ModelControl, ModelControl.cpp:75-197)
// for B independent instances of one model.
//
// Reference semantics kept per instance: set_state() stores the latest measurement snapshot (:93-100 under
// m_state_mutex), the worker thread started by start_calc() solves from the latest snapshot, warm-started with
// the previous solution (:160-161), and publishes control_results (:174-190) that control_at_time() reads
// (:192-197).  Batched and MI355X-side:
//   * one GPU solve per tick for all B instances (mmpc_solve_batch, device pointers, stream-ordered);
//   * the warm start V stays resident in HBM between ticks (never copied back in to the device);
//   * inputs go through two pinned staging slots and a copy stream: the upload of tick i+1 overlaps the solve of
//     tick i, the download of tick i's solution (from a per-slot device copy, so the next solve may overwrite V)
//     overlaps the solve of tick i+1; results are published when their download event completes;
//   * optional warm-start shift (off by default, as the reference): V moved k stages earlier, k = elapsed
//     time / step, by two strided device copies.
#pragma once
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <Mahi/Mpc/ModelControl.hpp>
#include <Mahi/Mpc/ModelParameters.hpp>
#include <Mahi/Util/Time.hpp>

namespace mahi {
namespace mpc {

class BatchModelControl {
public:
    using ControlResult = ModelControl::ControlResult;

    // model_name: <model_name>.json (ModelControl.cpp:24); B instances; device -1 = current HIP device
    BatchModelControl(std::string model_name, int64_t B, std::vector<double> Q, std::vector<double> R,
                      std::vector<double> Rm, Dict solver_opts = Dict(), int device = -1);
    ~BatchModelControl();
    BatchModelControl(const BatchModelControl&) = delete;
    BatchModelControl& operator=(const BatchModelControl&) = delete;

    ModelParameters model_parameters;
    int64_t batch() const { return m_B; }

    // synchronous tick: states [B*nx], controls [B*nu] (previous inputs, the Delta-u reference), trajs [B*N*nx]
    void calc_u(mahi::util::Time time, const std::vector<double>& states, const std::vector<double>& controls,
                const std::vector<double>& trajs);

    // asynchronous loop (ModelControl.cpp:75-114)
    void set_state(mahi::util::Time time, const std::vector<double>& states, const std::vector<double>& controls,
                   const std::vector<double>& trajs);
    void start_calc();
    void stop_calc();

    // published results (latest completed tick)
    ControlResult control_at_time(int64_t b, mahi::util::Time time);  // instance b, as ModelControl.cpp:192-197
    std::vector<double> controls_at_time(mahi::util::Time time);      // [B*nu], every instance
    std::vector<double> solution(int64_t b);                          // V* of instance b (reference layout)
    std::vector<int> last_status();                                   // per instance
    std::vector<int> last_iterations();
    mahi::util::Time last_solve_time();                               // time stamp of the published tick
    int64_t ticks_published() const { return m_ticks; }
    double mean_tick_ms() const;                                      // worker: enqueue -> published

    void update_weights(std::vector<double> Q = {}, std::vector<double> R = {}, std::vector<double> Rm = {});
    void update_control_limits(std::vector<double> u_min, std::vector<double> u_max);
    // move the warm start k = round((t - t_prev) / step) stages earlier before each solve (default false)
    void set_warm_start_shift(bool on) { m_shift = on; }

private:
    struct Impl;
    std::unique_ptr<Impl> m;
    int64_t m_B;
    std::atomic<bool> m_shift{false};
    std::atomic<int64_t> m_ticks{0};
    std::atomic<bool> m_stop{true};
    std::thread m_thread;

    std::mutex m_state_mutex;  // snapshot (ModelControl.hpp:71)
    std::condition_variable m_state_cv;
    uint64_t m_state_version = 0;
    mahi::util::Time m_time;
    std::vector<double> m_states, m_controls, m_trajs;

    std::mutex m_output_mutex;  // published results (ModelControl.hpp:72)
    mahi::util::Time m_out_time;
    std::vector<double> m_out_V;
    std::vector<int> m_out_status, m_out_iters;

    std::mutex m_weights_mutex;
    std::vector<double> m_Q, m_R, m_Rm;
    std::mutex m_control_limits_mutex;

    std::mutex m_solve_mutex;  // one tick pipeline at a time (calc_u vs the worker)
    double m_tick_ms_sum = 0.0;

    void enqueue_tick(int slot, mahi::util::Time time, const double* states, const double* controls,
                      const double* trajs);
    void publish(int slot);
    void worker();
};

}  // namespace mpc
}  // namespace mahi
