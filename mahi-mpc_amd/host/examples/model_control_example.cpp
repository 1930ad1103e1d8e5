// Closed-loop cfg#1 through the drop-in C++ API: the reference's examples/model_control_example.cpp:8-154
// with the thread example's weights (thread_model_control_example.cpp:24-25) and an explicit Rm.
// ModelGenerator writes the model file (ex_model_generate.cpp:59-71 with N from the command line), then
// calc_u runs every 5th tick (model_control_example.cpp:74-76) and the Euler plant uses the device
// linearisation's x_dot through <name>_get_x_dot_init of the generated <name>_linear_functions.so
// (model_control_example.cpp:46,81-86).  Prints one CSV line per tick:
//   t, q0..q3, T0, T1, status, iterations
// With a 5th argument "thread" it runs the reference's threaded loop instead
// (thread_model_control_example.cpp:47-120, with Rm given): set_state at t = 0, start_calc, then a 1 kHz
// real-time plant that calls set_state every tick and applies control_at_time while ModelControl's worker thread
// solves from the latest snapshot; stop_calc at the end.  Prints
//   thread,ticks,last_status,max_abs_control,max_abs_err_q_second_half,all_finite
#include <Mahi/Mpc.hpp>
#include <Mahi/Util.hpp>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <vector>

#include "../../../include/mmpc.h"

using namespace mahi::mpc;

int main(int argc, char** argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 20;
    const double sim_seconds = argc > 2 ? std::atof(argv[2]) : 0.2;
    const bool linear = argc > 3 && argv[3][0] == 'l';
    // optional 4th argument: the path (without .json) of a model generated beforehand from SX expressions
    // (ex_model_generate): ModelControl then loads its own solver library through the JSON's dll_filepath
    const std::string model_path = argc > 4 && std::string(argv[4]) != "-" ? argv[4] : "";
    const bool threaded = argc > 5 && std::string(argv[5]) == "thread";
    std::string name = linear ? "linear_double_pendulum" : "nonlinear_double_pendulum";
    if (model_path.empty()) {
        ModelParameters mp(name, 4, 2, mahi::util::milliseconds(2), N, linear);
        ModelGenerator gen(mp, "two_link_arm");
        gen.create_model();
        gen.generate_c_code();
        gen.compile_model();
    } else {
        name = model_path;
    }

    ModelControl mc(name, {10, 1, 5, 5}, {5, 5}, {0.01, 0.01});
    if (mc.model_parameters.num_shooting_nodes != N) {
        std::fprintf(stderr, "model %s has N = %d\n", name.c_str(), mc.model_parameters.num_shooting_nodes);
        return 2;
    }
    const std::string ext_name = mc.model_parameters.name;
    const int nx = mc.model_parameters.num_x;
    const double h = mc.model_parameters.step_size.as_seconds();
    std::vector<double> state(4, 0.0), control(2, 0.0);
    // plant model through the generated CasADi external, as model_control_example.cpp:46
    auto ext_x_dot_init = external(ext_name + "_get_x_dot_init", name + "_linear_functions.so");
    const double PI = 3.14159265358979323846, sin_amp = 1.0, sin_freq = 1.0;
    auto make_traj = [&](double t0) {
        std::vector<double> traj;
        double tt = t0;
        for (int i = 0; i < N; i++) {  // model_control_example.cpp:58-68
            for (int j = 0; j < nx; j++) {
                if (j < nx / 2) traj.push_back(((j % 2 == 0) ? 1.0 : -1.0) * sin_amp * std::sin(2 * PI * sin_freq * tt));
                else traj.push_back((((j - nx / 2) % 2 == 0) ? 1.0 : -1.0) * sin_amp * 2 * PI * sin_freq * std::cos(2 * PI * sin_freq * tt));
            }
            tt += h;
        }
        return traj;
    };
    if (threaded) {   // thread_model_control_example.cpp:53-120
        mc.set_state(mahi::util::seconds(0), state, control, make_traj(0.0));
        mc.start_calc();
        mahi::util::sleep(mahi::util::milliseconds(100));   // thread_model_control_example.cpp:73
        // the reference reads an empty result vector if the worker's first solve is still running (SURVEY
        // Appendix A.9); here control_at_time throws then, so wait for the first published solve (the first one
        // also loads the kernels' code object)
        for (int i = 0; i < 1000; ++i) {
            try {
                mc.control_at_time(mahi::util::seconds(0));
                break;
            } catch (const std::logic_error&) {
                mahi::util::sleep(mahi::util::milliseconds(10));
            }
        }
        const mahi::util::Time sim_rate = mahi::util::microseconds(1000);
        mahi::util::Timer sim_clock(sim_rate);
        double t = 0.0, umax = 0.0, err2 = 0.0;
        long ticks = 0;
        bool finite = true;
        while (t < sim_seconds) {
            mc.set_state(mahi::util::seconds(t), state, control, make_traj(t));
            control = mc.control_at_time(mahi::util::seconds(t)).u;
            std::vector<double> xd(ext_x_dot_init({state, control})[0]);
            for (int i = 0; i < 4; i++) state[i] += xd[i] * sim_rate.as_seconds();
            for (double c : control) {
                umax = std::fmax(umax, std::fabs(c));
                finite = finite && std::isfinite(c);
            }
            if (t > 0.5 * sim_seconds) {   // q tracking error in the second half (targets as traj row 0)
                const double r0 = sin_amp * std::sin(2 * PI * sin_freq * t);
                err2 = std::fmax(err2, std::fmax(std::fabs(state[0] - r0), std::fabs(state[1] + r0)));
            }
            ++ticks;
            t = sim_clock.wait().as_seconds();
        }
        mc.stop_calc();
        std::printf("thread,%ld,%d,%.6g,%.6g,%d\n", ticks, mc.last_status(), umax, err2, finite ? 1 : 0);
        return finite ? 0 : 3;
    }
    double t = 0.0;
    int cycle = 0;
    while (t < sim_seconds - 1e-12) {
        const std::vector<double> traj = make_traj(t);
        if (cycle % 5 == 0) mc.calc_u(mahi::util::seconds(t), state, control, traj);
        control = mc.control_at_time(mahi::util::seconds(t)).u;
        std::vector<double> xd(ext_x_dot_init({state, control})[0]);  // model_control_example.cpp:81-82
        std::printf("%.6f,%.17g,%.17g,%.17g,%.17g,%.17g,%.17g,%d,%d\n", t, state[0], state[1], state[2], state[3],
                    control[0], control[1], mc.last_status(), mc.last_iterations());
        for (int i = 0; i < 4; i++) state[i] += xd[i] * h;
        t += h;
        cycle++;
    }
    return 0;
}
