// SX-defined models beyond the reference's double pendulum, generated through the same ModelGenerator calls
// (create_model / generate_c_code / compile_model) -- used by the tests to exercise the three kinematic
// structures the kernels handle (sqp_lane.h a_mul):
//   cart_pole       x = [p, th, p_dot, th_dot], u = [F]       second order, nq = 2 (tanh friction, division)
//   unicycle        x = [px, py, th, v],        u = [a, w]    first order,  nq = 0 (sqrt drag)
//   motor_pendulum  x = [th, om, i],            u = [V]       mixed,        nq = 1, na = 2 (exp, sq)
// The same equations are restated in sympy in tests/test_sx_models.py.
//   sx_model_zoo <model> <N> [linear]      writes <model>{,_model.h,_linear_functions.{c,so},.so,.json} in the cwd
#include <Mahi/Mpc.hpp>

#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

using namespace casadi;
using namespace mahi::mpc;

int main(int argc, char* argv[]) {
    if (argc < 3) {
        std::cerr << "usage: sx_model_zoo cart_pole|unicycle|motor_pendulum N [linear]" << std::endl;
        return 2;
    }
    const std::string which = argv[1];
    const int N = std::atoi(argv[2]);
    const bool linear = argc > 3 && !std::strcmp(argv[3], "linear");
    SX x, x_dot, u;
    if (which == "cart_pole") {
        const double mc = 1.0, mp = 0.1, l = 0.5, g = 9.81, fr = 0.2;
        SX p = SX::sym("p"), th = SX::sym("th"), p_dot = SX::sym("p_dot"), th_dot = SX::sym("th_dot");
        SX F = SX::sym("F");
        SX tmp = (F - fr * tanh(5 * p_dot) + mp * l * th_dot * th_dot * sin(th)) / (mc + mp);
        SX th_ddot = (g * sin(th) - cos(th) * tmp) / (l * (4.0 / 3.0 - mp * cos(th) * cos(th) / (mc + mp)));
        SX p_ddot = tmp - mp * l * th_ddot * cos(th) / (mc + mp);
        x = SX::vertcat({p, th, p_dot, th_dot});
        x_dot = SX::vertcat({p_dot, th_dot, p_ddot, th_ddot});
        u = F;
    } else if (which == "unicycle") {
        SX px = SX::sym("px"), py = SX::sym("py"), th = SX::sym("th"), v = SX::sym("v");
        SX a = SX::sym("a"), w = SX::sym("w");
        x = SX::vertcat({px, py, th, v});
        x_dot = SX::vertcat({v * cos(th), v * sin(th), w, a - 0.05 * v * sqrt(1 + v * v)});
        u = SX::vertcat({a, w});
    } else if (which == "motor_pendulum") {
        const double J = 0.01, b = 0.1, K = 0.05, R = 1.0, Lm = 0.5, m = 0.2, g = 9.81, l = 0.3;
        SX th = SX::sym("th"), om = SX::sym("om"), i = SX::sym("i"), V = SX::sym("V");
        SX om_dot = (K * i - b * om - m * g * l * sin(th)) / J;
        SX i_dot = (V - R * (1 + 0.1 * exp(-sq(i))) * i - K * om) / Lm;
        x = SX::vertcat({th, om, i});
        x_dot = SX::vertcat({om, om_dot, i_dot});
        u = V;
    } else {
        std::cerr << "unknown model " << which << std::endl;
        return 2;
    }
    const std::string name = (linear ? "linear_" : "") + which;
    ModelParameters mp(name, x.size1(), u.size1(), mahi::util::milliseconds(10), N, linear);
    ModelGenerator gen(mp, x, x_dot, u);
    gen.create_model();
    gen.generate_c_code();
    gen.compile_model();
    std::cout << name << ": nq = " << gen.kinematic_rows() << std::endl;
    return 0;
}
