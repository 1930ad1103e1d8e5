// ModelControl::calc_u_batch through the drop-in C++ API with control limits (update_control_limits,
// ModelControl.cpp:205-209, enforced as calc_u enforces them, ModelControl.cpp:148-154).  The model is the
// reference's double pendulum (ex_model_generate.cpp:59-71, built-in two_link_arm kernels, N from argv[1]); the
// limits are argv[2] (|u_i| <= limit); instances come from stdin, one per line:
//   x0[4] u_prev[2] traj[N*4]
// and each solution is printed as one line: status, then V[NV] (reference layout).
#include <Mahi/Mpc.hpp>

#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <vector>

using namespace mahi::mpc;

int main(int argc, char** argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 30;
    const double lim = argc > 2 ? std::atof(argv[2]) : 2.0;
    const std::string name = "calc_u_batch_double_pendulum";
    {
        ModelParameters mp(name, 4, 2, mahi::util::milliseconds(2), N, false);
        ModelGenerator gen(mp, "two_link_arm");
        gen.create_model();
        gen.generate_c_code();
        gen.compile_model();
    }
    ModelControl mc(name, {10, 1, 5, 5}, {5, 5}, {0.01, 0.01});
    mc.update_control_limits({-lim, -lim}, {lim, lim});
    std::vector<std::vector<double>> states, controls, trajs;
    std::vector<double> row(4 + 2 + 4 * N);
    while (true) {
        for (double& v : row)
            if (!(std::cin >> v)) goto done;
        states.emplace_back(row.begin(), row.begin() + 4);
        controls.emplace_back(row.begin() + 4, row.begin() + 6);
        trajs.emplace_back(row.begin() + 6, row.end());
    }
done:
    std::vector<int> status;
    const auto V = mc.calc_u_batch(states, controls, trajs, &status);
    for (size_t b = 0; b < V.size(); ++b) {
        std::printf("%d", status[b]);
        for (double v : V[b]) std::printf(" %.17g", v);
        std::printf("\n");
    }
    return 0;
}
