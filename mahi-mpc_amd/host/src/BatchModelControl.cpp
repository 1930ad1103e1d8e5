// BatchModelControl: ModelControl's online loop (ModelControl.cpp:75-197) for B instances per GPU solve, with the
// warm start resident in HBM and the host<->device staging double-buffered on a copy stream (see the header).
#include <Mahi/Mpc/BatchModelControl.hpp>

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "../../../include/mmpc.h"
#include "model_library.hpp"

namespace mahi {
namespace mpc {

namespace {
void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
#define HIPC(call) hip_check((call), #call)
}  // namespace

struct BatchModelControl::Impl {
    std::shared_ptr<detail::ModelLibrary> lib;
    mmpc_handle* h = nullptr;
    int dev = -1;
    hipStream_t compute = nullptr, copy = nullptr;
    int nx = 0, nu = 0, N = 0, NV = 0;
    double step = 0.0;
    int64_t B = 0;
    // per-slot input block (device and pinned host): x0 [B nx] | u_prev [B nu] | traj [B N nx] | Q R Rm | lb | ub
    size_t off_up = 0, off_tr = 0, off_w = 0, off_lb = 0, off_ub = 0, in_doubles = 0;
    double* d_in[2] = {nullptr, nullptr};
    double* h_in[2] = {nullptr, nullptr};
    bool bounded[2] = {false, false};
    // solution: resident warm start, per-slot copies for the download, per-slot status/iterations
    double* d_V = nullptr;
    double* d_tmp = nullptr;  // warm-start shift
    double* d_Vout[2] = {nullptr, nullptr};
    int32_t* d_st[2] = {nullptr, nullptr};
    int32_t* d_it[2] = {nullptr, nullptr};
    double* h_V[2] = {nullptr, nullptr};
    int32_t* h_st[2] = {nullptr, nullptr};
    int32_t* h_it[2] = {nullptr, nullptr};
    hipEvent_t h2d_done[2] = {nullptr, nullptr}, solved[2] = {nullptr, nullptr}, d2h_done[2] = {nullptr, nullptr};
    bool pending[2] = {false, false};
    mahi::util::Time pend_time[2];
    std::chrono::steady_clock::time_point pend_t0[2];
    int next_slot = 0;
    bool have_prev = false;
    mahi::util::Time prev_time;

    void check(int rc, const char* what) const { lib->check(rc, what); }
};

BatchModelControl::BatchModelControl(std::string model_name, int64_t B, std::vector<double> Q, std::vector<double> R,
                                     std::vector<double> Rm, Dict solver_opts, int device)
    : m(new Impl), m_B(B), m_Q(std::move(Q)), m_R(std::move(R)), m_Rm(std::move(Rm)) {
    (void)solver_opts;  // stored-but-ignored in the reference (ModelControl.cpp:7-11 vs :52-62)
    if (B < 1) throw std::invalid_argument("BatchModelControl: B must be >= 1");
    const std::string path = model_name + ".json";
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    model_parameters = model_parameters_from_json_string(ss.str());
    m->lib = detail::ModelLibrary::load(model_parameters, path);
    mmpc_opts o;
    mmpc_default_opts(&o);
    o.device = device;
    m->check(m->lib->create_from_json(ss.str().c_str(), &o, &m->h), "mmpc_create");
    mmpc_model_info info;
    m->check(m->lib->get_model_info(m->h, &info), "mmpc_get_model_info");
    m->nx = info.num_x;
    m->nu = info.num_u;
    m->N = info.num_shooting_nodes;
    m->NV = info.num_v;
    m->step = info.step_size;
    m->B = B;
    if (m_Q.size() != static_cast<size_t>(m->nx) || m_R.size() != static_cast<size_t>(m->nu) ||
        m_Rm.size() != static_cast<size_t>(m->nu))
        throw std::invalid_argument("BatchModelControl: Q, R, Rm must have num_x, num_u, num_u entries");
    if (device >= 0) HIPC(hipSetDevice(device));
    HIPC(hipGetDevice(&m->dev));
    const size_t nx = m->nx, nu = m->nu, N = m->N, NV = m->NV, b = static_cast<size_t>(B);
    m->off_up = b * nx;
    m->off_tr = m->off_up + b * nu;
    m->off_w = m->off_tr + b * N * nx;
    m->off_lb = m->off_w + nx + 2 * nu;
    m->off_ub = m->off_lb + nu;
    m->in_doubles = m->off_ub + nu;
    HIPC(hipStreamCreateWithFlags(&m->compute, hipStreamNonBlocking));
    HIPC(hipStreamCreateWithFlags(&m->copy, hipStreamNonBlocking));
    HIPC(hipMalloc(reinterpret_cast<void**>(&m->d_V), b * NV * sizeof(double)));
    HIPC(hipMemset(m->d_V, 0, b * NV * sizeof(double)));  // v_init = 0 (ModelControl.cpp:29-50)
    HIPC(hipMalloc(reinterpret_cast<void**>(&m->d_tmp), b * NV * sizeof(double)));
    for (int s = 0; s < 2; ++s) {
        HIPC(hipMalloc(reinterpret_cast<void**>(&m->d_in[s]), m->in_doubles * sizeof(double)));
        HIPC(hipHostMalloc(reinterpret_cast<void**>(&m->h_in[s]), m->in_doubles * sizeof(double), hipHostMallocDefault));
        HIPC(hipMalloc(reinterpret_cast<void**>(&m->d_Vout[s]), b * NV * sizeof(double)));
        HIPC(hipMalloc(reinterpret_cast<void**>(&m->d_st[s]), b * sizeof(int32_t)));
        HIPC(hipMalloc(reinterpret_cast<void**>(&m->d_it[s]), b * sizeof(int32_t)));
        HIPC(hipHostMalloc(reinterpret_cast<void**>(&m->h_V[s]), b * NV * sizeof(double), hipHostMallocDefault));
        HIPC(hipHostMalloc(reinterpret_cast<void**>(&m->h_st[s]), b * sizeof(int32_t), hipHostMallocDefault));
        HIPC(hipHostMalloc(reinterpret_cast<void**>(&m->h_it[s]), b * sizeof(int32_t), hipHostMallocDefault));
        HIPC(hipEventCreateWithFlags(&m->h2d_done[s], hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&m->solved[s], hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&m->d2h_done[s], hipEventDisableTiming));
    }
    // the Riccati solvers' workspace up front: solves never allocate (and never synchronise) inside the loop
    m->check(m->lib->reserve_workspace(m->h, B, nullptr), "mmpc_reserve_workspace");
    m_out_V.assign(b * NV, 0.0);
    m_out_status.assign(b, -1);
    m_out_iters.assign(b, 0);
}

BatchModelControl::~BatchModelControl() {
    stop_calc();
    if (!m) return;
    (void)hipSetDevice(m->dev);
    if (m->compute) (void)hipStreamSynchronize(m->compute);
    if (m->copy) (void)hipStreamSynchronize(m->copy);
    for (int s = 0; s < 2; ++s) {
        (void)hipFree(m->d_in[s]);
        (void)hipHostFree(m->h_in[s]);
        (void)hipFree(m->d_Vout[s]);
        (void)hipFree(m->d_st[s]);
        (void)hipFree(m->d_it[s]);
        (void)hipHostFree(m->h_V[s]);
        (void)hipHostFree(m->h_st[s]);
        (void)hipHostFree(m->h_it[s]);
        if (m->h2d_done[s]) (void)hipEventDestroy(m->h2d_done[s]);
        if (m->solved[s]) (void)hipEventDestroy(m->solved[s]);
        if (m->d2h_done[s]) (void)hipEventDestroy(m->d2h_done[s]);
    }
    (void)hipFree(m->d_V);
    (void)hipFree(m->d_tmp);
    if (m->h) m->lib->destroy(m->h);
    if (m->compute) (void)hipStreamDestroy(m->compute);
    if (m->copy) (void)hipStreamDestroy(m->copy);
}

void BatchModelControl::enqueue_tick(int slot, mahi::util::Time time, const double* states, const double* controls,
                                     const double* trajs) {
    Impl& I = *m;
    HIPC(hipSetDevice(I.dev));
    if (I.pending[slot]) publish(slot);  // the slot's pinned buffers are free again
    const size_t nx = I.nx, nu = I.nu, N = I.N, NV = I.NV, b = static_cast<size_t>(I.B);
    double* in = I.h_in[slot];
    std::memcpy(in, states, b * nx * sizeof(double));
    std::memcpy(in + I.off_up, controls, b * nu * sizeof(double));
    std::memcpy(in + I.off_tr, trajs, b * N * nx * sizeof(double));
    {
        std::lock_guard<std::mutex> lg(m_weights_mutex);  // ModelControl.cpp:120-122
        std::copy(m_Q.begin(), m_Q.end(), in + I.off_w);
        std::copy(m_R.begin(), m_R.end(), in + I.off_w + nx);
        std::copy(m_Rm.begin(), m_Rm.end(), in + I.off_w + nx + nu);
    }
    bool finite = false;
    {
        std::lock_guard<std::mutex> lg(m_control_limits_mutex);  // ModelControl.cpp:148-154
        for (size_t c = 0; c < nu; ++c) {
            const double lo = c < model_parameters.u_min.size() ? model_parameters.u_min[c] : -10e30;
            const double hi = c < model_parameters.u_max.size() ? model_parameters.u_max[c] : 10e30;
            in[I.off_lb + c] = lo;
            in[I.off_ub + c] = hi;
            finite |= lo > -1e19 || hi < 1e19;  // IPOPT: |bound| >= 1e19 is infinite
        }
    }
    I.bounded[slot] = finite;
    double* d = I.d_in[slot];
    HIPC(hipMemcpyAsync(d, in, I.in_doubles * sizeof(double), hipMemcpyHostToDevice, I.copy));
    HIPC(hipEventRecord(I.h2d_done[slot], I.copy));
    HIPC(hipStreamWaitEvent(I.compute, I.h2d_done[slot], 0));
    if (m_shift && I.have_prev) {  // warm start moved k stages earlier (the tail keeps its old values)
        const double dt = time.as_seconds() - I.prev_time.as_seconds();
        const int64_t k = std::min<int64_t>(I.N, std::max<int64_t>(0, std::llround(dt / I.step)));
        if (k > 0) {
            const size_t sh = static_cast<size_t>(k) * (nx + nu), w = (NV - sh) * sizeof(double);
            HIPC(hipMemcpy2DAsync(I.d_tmp, NV * sizeof(double), I.d_V + sh, NV * sizeof(double), w, b,
                                  hipMemcpyDeviceToDevice, I.compute));
            HIPC(hipMemcpy2DAsync(I.d_V, NV * sizeof(double), I.d_tmp, NV * sizeof(double), w, b,
                                  hipMemcpyDeviceToDevice, I.compute));
        }
    }
    I.have_prev = true;
    I.prev_time = time;
    I.check(I.lib->solve_batch(I.h, I.B, d, d + I.off_up, d + I.off_tr, d + I.off_w, 0,
                               finite ? d + I.off_lb : nullptr, finite ? d + I.off_ub : nullptr, I.d_V, I.d_st[slot],
                               I.d_it[slot], nullptr, I.compute),
            "mmpc_solve_batch");
    // the next solve updates d_V in place: download from a per-slot copy
    HIPC(hipMemcpyAsync(I.d_Vout[slot], I.d_V, b * NV * sizeof(double), hipMemcpyDeviceToDevice, I.compute));
    HIPC(hipEventRecord(I.solved[slot], I.compute));
    HIPC(hipStreamWaitEvent(I.copy, I.solved[slot], 0));
    HIPC(hipMemcpyAsync(I.h_V[slot], I.d_Vout[slot], b * NV * sizeof(double), hipMemcpyDeviceToHost, I.copy));
    HIPC(hipMemcpyAsync(I.h_st[slot], I.d_st[slot], b * sizeof(int32_t), hipMemcpyDeviceToHost, I.copy));
    HIPC(hipMemcpyAsync(I.h_it[slot], I.d_it[slot], b * sizeof(int32_t), hipMemcpyDeviceToHost, I.copy));
    HIPC(hipEventRecord(I.d2h_done[slot], I.copy));
    I.pending[slot] = true;
    I.pend_time[slot] = time;
}

void BatchModelControl::publish(int slot) {
    Impl& I = *m;
    if (!I.pending[slot]) return;
    HIPC(hipEventSynchronize(I.d2h_done[slot]));
    const size_t b = static_cast<size_t>(I.B);
    {
        std::lock_guard<std::mutex> lg(m_output_mutex);  // ModelControl.cpp:174-190
        std::memcpy(m_out_V.data(), I.h_V[slot], b * I.NV * sizeof(double));
        for (size_t i = 0; i < b; ++i) {
            m_out_status[i] = I.h_st[slot][i];
            m_out_iters[i] = I.h_it[slot][i];
        }
        m_out_time = I.pend_time[slot];
    }
    m_tick_ms_sum += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - I.pend_t0[slot]).count();
    I.pending[slot] = false;
    ++m_ticks;
}

void BatchModelControl::calc_u(mahi::util::Time time, const std::vector<double>& states,
                               const std::vector<double>& controls, const std::vector<double>& trajs) {
    const size_t b = static_cast<size_t>(m_B);
    if (states.size() != b * m->nx || controls.size() != b * m->nu || trajs.size() != b * m->N * m->nx)
        throw std::invalid_argument("BatchModelControl::calc_u: states/controls/trajs size mismatch");
    std::lock_guard<std::mutex> lg(m_solve_mutex);
    const int slot = m->next_slot;
    m->next_slot ^= 1;
    m->pend_t0[slot] = std::chrono::steady_clock::now();
    enqueue_tick(slot, time, states.data(), controls.data(), trajs.data());
    publish(slot ^ 1);
    publish(slot);
}

void BatchModelControl::set_state(mahi::util::Time time, const std::vector<double>& states,
                                  const std::vector<double>& controls, const std::vector<double>& trajs) {
    const size_t b = static_cast<size_t>(m_B);
    if (states.size() != b * m->nx || controls.size() != b * m->nu || trajs.size() != b * m->N * m->nx)
        throw std::invalid_argument("BatchModelControl::set_state: states/controls/trajs size mismatch");
    {
        std::lock_guard<std::mutex> lg(m_state_mutex);
        m_time = time;
        m_states = states;
        m_controls = controls;
        m_trajs = trajs;
        ++m_state_version;
    }
    m_state_cv.notify_one();
}

void BatchModelControl::worker() {
    uint64_t seen = 0;
    std::vector<double> s, c, tr;
    while (!m_stop) {
        mahi::util::Time t;
        {
            std::unique_lock<std::mutex> lk(m_state_mutex);
            m_state_cv.wait_for(lk, std::chrono::milliseconds(1), [&] { return m_stop || m_state_version != seen; });
            if (m_stop) break;
            if (m_state_version == seen) continue;
            seen = m_state_version;
            t = m_time;
            s = m_states;
            c = m_controls;
            tr = m_trajs;
        }
        std::lock_guard<std::mutex> lg(m_solve_mutex);
        const int slot = m->next_slot;
        m->next_slot ^= 1;
        m->pend_t0[slot] = std::chrono::steady_clock::now();
        enqueue_tick(slot, t, s.data(), c.data(), tr.data());
        // the previous tick's results are published while this tick's solve is queued behind it on the GPU
        publish(slot ^ 1);
    }
    std::lock_guard<std::mutex> lg(m_solve_mutex);
    publish(m->next_slot ^ 1);
    publish(m->next_slot);
}

void BatchModelControl::start_calc() {
    stop_calc();
    m_stop = false;
    m_thread = std::thread([this] { worker(); });
}

void BatchModelControl::stop_calc() {
    m_stop = true;
    m_state_cv.notify_all();
    if (m_thread.joinable()) m_thread.join();
}

BatchModelControl::ControlResult BatchModelControl::control_at_time(int64_t b, mahi::util::Time time) {
    if (b < 0 || b >= m_B) throw std::out_of_range("control_at_time: instance index");
    std::lock_guard<std::mutex> lg(m_output_mutex);
    if (m_ticks == 0) throw std::logic_error("control_at_time before the first solve");
    const size_t nx = m->nx, nu = m->nu, N = m->N;
    // ModelControl.cpp:192-197: the last stage whose time is before `time` (the first one if none)
    size_t i = 0;
    while (i < N && mahi::util::seconds(m_out_time.as_seconds() + m->step * i) < time) i++;
    const size_t k = i == 0 ? 0 : i - 1;
    const double* v = m_out_V.data() + static_cast<size_t>(b) * m->NV + k * (nx + nu);
    return ControlResult(mahi::util::seconds(m_out_time.as_seconds() + m->step * k), std::vector<double>(v, v + nx),
                         std::vector<double>(v + nx, v + nx + nu));
}

std::vector<double> BatchModelControl::controls_at_time(mahi::util::Time time) {
    std::vector<double> out;
    out.reserve(static_cast<size_t>(m_B) * m->nu);
    for (int64_t b = 0; b < m_B; ++b) {
        const ControlResult r = control_at_time(b, time);
        out.insert(out.end(), r.u.begin(), r.u.end());
    }
    return out;
}

std::vector<double> BatchModelControl::solution(int64_t b) {
    if (b < 0 || b >= m_B) throw std::out_of_range("solution: instance index");
    std::lock_guard<std::mutex> lg(m_output_mutex);
    const double* v = m_out_V.data() + static_cast<size_t>(b) * m->NV;
    return std::vector<double>(v, v + m->NV);
}

std::vector<int> BatchModelControl::last_status() {
    std::lock_guard<std::mutex> lg(m_output_mutex);
    return m_out_status;
}

std::vector<int> BatchModelControl::last_iterations() {
    std::lock_guard<std::mutex> lg(m_output_mutex);
    return m_out_iters;
}

mahi::util::Time BatchModelControl::last_solve_time() {
    std::lock_guard<std::mutex> lg(m_output_mutex);
    return m_out_time;
}

double BatchModelControl::mean_tick_ms() const { return m_ticks ? m_tick_ms_sum / m_ticks : 0.0; }

void BatchModelControl::update_weights(std::vector<double> Q, std::vector<double> R, std::vector<double> Rm) {
    std::lock_guard<std::mutex> lg(m_weights_mutex);
    if (!Q.empty()) {
        if (Q.size() != m_Q.size()) throw std::invalid_argument("update_weights: Q size");
        m_Q = Q;
    }
    if (!R.empty()) {
        if (R.size() != m_R.size()) throw std::invalid_argument("update_weights: R size");
        m_R = R;
    }
    if (!Rm.empty()) {
        if (Rm.size() != m_Rm.size()) throw std::invalid_argument("update_weights: Rm size");
        m_Rm = Rm;
    }
}

void BatchModelControl::update_control_limits(std::vector<double> u_min, std::vector<double> u_max) {
    std::lock_guard<std::mutex> lg(m_control_limits_mutex);
    model_parameters.u_min = u_min;
    model_parameters.u_max = u_max;
}

}  // namespace mpc
}  // namespace mahi
