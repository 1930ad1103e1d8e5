// CPU-only self test of the host mirror (no GPU call is made): ModelParameters defaults and JSON round trip
// (ModelParameters.cpp:7-72), ModelGenerator's <name>.json artefact, ModelControl construction and its API
// errors.  Exit code 0 = pass; prints the failing check otherwise.
#include <Mahi/Mpc.hpp>

#include <cmath>
#include <cstdio>
#include <stdexcept>
#include <utility>

#include "../../../include/mmpc.h"

using namespace mahi::mpc;

#define CHECK(c)                                                  \
    do {                                                          \
        if (!(c)) {                                               \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                             \
        }                                                         \
    } while (0)

int main() {
    ModelParameters mp("selftest_double_pendulum", 4, 2, mahi::util::milliseconds(2), 25, false);
    CHECK(mp.timespan.as_microseconds() == 50000);
    CHECK(mp.x_min.size() == 4 && mp.x_min[0] == -10e30 && mp.u_max[1] == 10e30);
    ModelParameters rt = model_parameters_from_json_string(to_json_string(mp));
    CHECK(rt.name == mp.name && rt.num_x == 4 && rt.num_u == 2 && rt.num_shooting_nodes == 25);
    CHECK(rt.step_size == mp.step_size && rt.timespan == mp.timespan && !rt.is_linear);
    CHECK(std::isinf(rt.x_min[0]) && rt.x_min[0] < 0 && std::isinf(rt.x_max[3]));  // +-10e30 -> +-inf on load
    CHECK(rt.u_min[0] == -10e30 && rt.u_max[0] == 10e30);                         // u bounds stay
    ModelGenerator gen(mp, "two_link_arm");
    gen.create_model();
    gen.generate_c_code();
    gen.compile_model();
    mmpc_handle* h = nullptr;
    CHECK(mmpc_create("selftest_double_pendulum.json", nullptr, &h) == MMPC_OK);
    mmpc_model_info info;
    CHECK(mmpc_get_model_info(h, &info) == MMPC_OK && info.num_shooting_nodes == 25 && info.num_v == 154);
    mmpc_destroy(h);
    // CasADi-external linear functions (ModelGenerator.cpp:45-53,241-251): metadata only, no GPU call
    for (const char* fn : {"_get_A", "_get_B", "_get_x_dot_init"}) {
        External e = external(std::string("selftest_double_pendulum") + fn, "selftest_double_pendulum_linear_functions.so");
        CHECK(e.n_in() == 2 && e.n_out() == 1);
        CHECK(e.size_in(0) == std::make_pair(4LL, 1LL) && e.size_in(1) == std::make_pair(2LL, 1LL));
    }
    CHECK(external("selftest_double_pendulum_get_A", "selftest_double_pendulum_linear_functions.so").size_out(0) ==
          std::make_pair(4LL, 4LL));
    CHECK(external("selftest_double_pendulum_get_B", "selftest_double_pendulum_linear_functions.so").size_out(0) ==
          std::make_pair(4LL, 2LL));
    {
        ModelGenerator exo(ModelParameters("selftest_exo", 8, 4, mahi::util::milliseconds(2), 50, false), "exo_arm");
        exo.create_model();
        exo.compile_model();
        External e = external("selftest_exo_get_B", "selftest_exo_linear_functions.so");
        CHECK(e.size_in(0) == std::make_pair(8LL, 1LL) && e.size_out(0) == std::make_pair(8LL, 4LL));
        bool bad_size = false;
        try {
            e({std::vector<double>(8, 0.0), std::vector<double>(3, 0.0)});
        } catch (const std::invalid_argument&) {
            bad_size = true;
        }
        CHECK(bad_size);
    }
    bool threw = false;
    try {
        ModelGenerator bad(ModelParameters("bad", 8, 4, mahi::util::milliseconds(2), 10, false), "two_link_arm");
        bad.create_model();
    } catch (const std::invalid_argument&) {
        threw = true;
    }
    CHECK(threw);
    ModelControl mc("selftest_double_pendulum", {10, 1, 5, 5}, {5, 5});  // Rm omitted, as thread_..._example.cpp:29
    CHECK(mc.model_parameters.num_shooting_nodes == 25);
    threw = false;
    try {
        mc.control_at_time(mahi::util::seconds(0.0));
    } catch (const std::logic_error&) {
        threw = true;
    }
    CHECK(threw);
    threw = false;
    try {  // p of the wrong length in the reference -> API error before any GPU work
        mc.calc_u(mahi::util::seconds(0.0), {0, 0, 0, 0}, {0, 0}, std::vector<double>(100, 0.0));
    } catch (const std::invalid_argument&) {
        threw = true;
    }
    CHECK(threw);
    std::printf("host selftest ok\n");
    return 0;
}
