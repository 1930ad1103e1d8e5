// B closed loops of the 2-link arm through BatchModelControl: the reference's
// model_control_example.cpp:8-154 for B plants at once.  Instance b starts at x0_b (deterministic in b) and
// tracks the reference's sinusoid (model_control_example.cpp:58-68) delayed by phase_b = 0.1 b; the plant is
// the Euler step of the model's <name>_get_x_dot_init external (model_control_example.cpp:81-86).
//
//   batch_control_example <model (path without .json)> <B> <sim_seconds> sync|async [shift]
// sync : calc_u every 5th tick (model_control_example.cpp:74-76), one GPU solve for all B instances; prints
//        "t,b,q0..q3,T0,T1,status,iters" for instances b < 8 every tick, then "final,b,q0..q3" for all b
// async: start_calc(); the main thread runs the plants in real time (2 ms ticks), calls set_state every tick and
//        applies controls_at_time(t); prints "async,ticks_published,mean_tick_ms,converged,max_abs_state"
#include <Mahi/Mpc.hpp>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

using namespace mahi::mpc;

static std::vector<double> targets(int nx, int N, double h, double t, double phase) {
    const double PI = 3.14159265358979323846;
    std::vector<double> traj;
    double tt = t;
    for (int i = 0; i < N; i++) {  // model_control_example.cpp:58-68, delayed by `phase`
        for (int j = 0; j < nx; j++) {
            if (j < nx / 2) traj.push_back(((j % 2 == 0) ? 1.0 : -1.0) * std::sin(2 * PI * (tt - phase)));
            else traj.push_back((((j - nx / 2) % 2 == 0) ? 1.0 : -1.0) * 2 * PI * std::cos(2 * PI * (tt - phase)));
        }
        tt += h;
    }
    return traj;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: batch_control_example model B sim_seconds sync|async [shift]\n");
        return 2;
    }
    const std::string model = argv[1];
    const int64_t B = std::atoll(argv[2]);
    const double sim_seconds = std::atof(argv[3]);
    const bool async = !std::strcmp(argv[4], "async");
    const bool shift = argc > 5 && !std::strcmp(argv[5], "shift");

    BatchModelControl bc(model, B, {10, 1, 5, 5}, {5, 5}, {0.01, 0.01});
    bc.set_warm_start_shift(shift);
    const int nx = bc.model_parameters.num_x, nu = bc.model_parameters.num_u, N = bc.model_parameters.num_shooting_nodes;
    const double h = bc.model_parameters.step_size.as_seconds();
    auto ext = external(bc.model_parameters.name + "_get_x_dot_init", model + "_linear_functions.so");

    std::vector<double> state(B * nx), control(B * nu, 0.0);
    for (int64_t b = 0; b < B; ++b)
        for (int j = 0; j < nx; ++j) state[b * nx + j] = 0.05 * std::sin(1.3 * b + 0.7 * j);
    auto all_targets = [&](double t) {
        std::vector<double> tr;
        tr.reserve(B * N * nx);
        for (int64_t b = 0; b < B; ++b) {
            const std::vector<double> r = targets(nx, N, h, t, 0.1 * b);
            tr.insert(tr.end(), r.begin(), r.end());
        }
        return tr;
    };
    auto plant_step = [&]() {
        for (int64_t b = 0; b < B; ++b) {
            std::vector<double> x(state.begin() + b * nx, state.begin() + (b + 1) * nx);
            std::vector<double> u(control.begin() + b * nu, control.begin() + (b + 1) * nu);
            const std::vector<double> xd = ext({x, u})[0];
            for (int j = 0; j < nx; ++j) state[b * nx + j] += xd[j] * h;
        }
    };

    if (!async) {
        const int ticks = static_cast<int>(std::lround(sim_seconds / h));
        for (int cycle = 0; cycle < ticks; ++cycle) {
            const double t = cycle * h;
            if (cycle % 5 == 0) bc.calc_u(mahi::util::seconds(t), state, control, all_targets(t));
            control = bc.controls_at_time(mahi::util::seconds(t));
            const std::vector<int> st = bc.last_status(), it = bc.last_iterations();
            for (int64_t b = 0; b < std::min<int64_t>(B, 8); ++b) {
                std::printf("%.6f,%lld", t, static_cast<long long>(b));
                for (int j = 0; j < nx; ++j) std::printf(",%.17g", state[b * nx + j]);
                for (int j = 0; j < nu; ++j) std::printf(",%.17g", control[b * nu + j]);
                std::printf(",%d,%d\n", st[b], it[b]);
            }
            plant_step();
        }
        for (int64_t b = 0; b < B; ++b) {
            std::printf("final,%lld", static_cast<long long>(b));
            for (int j = 0; j < nx; ++j) std::printf(",%.17g", state[b * nx + j]);
            std::printf("\n");
        }
        return 0;
    }

    bc.set_state(mahi::util::seconds(0.0), state, control, all_targets(0.0));
    bc.start_calc();
    const auto t0 = std::chrono::steady_clock::now();
    int converged_ticks = 0, seen_ticks = 0;
    double max_abs = 0.0;
    for (int cycle = 0;; ++cycle) {
        const double t = cycle * h;
        if (t >= sim_seconds) break;
        std::this_thread::sleep_until(t0 + std::chrono::microseconds(static_cast<int64_t>(t * 1e6)));
        if (bc.ticks_published() > 0) {
            control = bc.controls_at_time(mahi::util::seconds(t));
            const std::vector<int> st = bc.last_status();
            ++seen_ticks;
            bool all = true;
            for (int s : st) all &= s == 0;
            converged_ticks += all;
        }
        plant_step();
        for (double v : state) max_abs = std::max(max_abs, std::fabs(v));
        bc.set_state(mahi::util::seconds(t + h), state, control, all_targets(t + h));
    }
    bc.stop_calc();
    std::printf("async,%lld,%.4f,%d,%d,%.6g\n", static_cast<long long>(bc.ticks_published()), bc.mean_tick_ms(),
                converged_ticks, seen_ticks, max_abs);
    return 0;
}
