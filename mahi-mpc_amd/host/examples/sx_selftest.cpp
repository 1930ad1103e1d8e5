// Self-test of the SX front end (Mahi/Mpc/SX.hpp), run by tests/test_sx_models.py on the CPU:
// derivative rules of every elementary operation against central differences, constant folding and algebraic
// simplification, common-subexpression elimination in emitted code, Function evaluation by name, matrix helpers
// and the error paths the reference's CasADi calls would raise (free symbols, non-symbolic jacobian variables).
#include <Mahi/Mpc/SX.hpp>

#include <cmath>
#include <cstdio>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

using namespace casadi;

static int g_fail = 0;
#define CHECK(cond, msg)                                          \
    do {                                                          \
        if (!(cond)) {                                            \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, msg); \
            ++g_fail;                                             \
        }                                                         \
    } while (0)

template <class F>
static bool throws(F&& f) {
    try {
        f();
    } catch (const std::exception&) {
        return true;
    }
    return false;
}

int main() {
    SX x = SX::sym("x"), y = SX::sym("y");
    SX v = SX::vertcat({x, y});
    // expressions over (x, y) in the region x in (0.2, 0.8), y in (0.5, 1.5)
    std::vector<std::pair<std::string, SX>> cases = {
        {"sin", sin(x * y)},        {"cos", cos(x + 2 * y)},      {"tan", tan(x) * y},
        {"exp", exp(-x * y)},       {"log", log(x + y)},          {"sqrt", sqrt(x * y + 1)},
        {"tanh", tanh(3 * x - y)},  {"sinh", sinh(x - y)},        {"cosh", cosh(x * y)},
        {"atan", atan(x / y)},      {"asin", asin(x * 0.9)},      {"acos", acos(x * y * 0.5)},
        {"atan2", atan2(y, x)},     {"fabs", fabs(x - 2 * y)},    {"sq", sq(x - y)},
        {"pow_const", pow(x, 3.5)}, {"pow_var", pow(y, x)},       {"div", (x - y) / (x * x + y)},
        {"neg", -(x * y)},          {"fmin", fmin(x, y * y)},     {"fmax", fmax(x * 3, y)},
        {"mix", sin(x) * cos(y) / (1 + sq(x)) - exp(y) * sqrt(x)}};
    const double x0 = 0.37, y0 = 0.91, eps = 1e-6;
    for (auto& c : cases) {
        Function f("f", {v}, {c.second, jacobian(c.second, v)});
        auto at = [&](double a, double b) { return f(std::vector<DM>{DM({a, b})}); };
        const auto r = at(x0, y0);
        const double fx = (at(x0 + eps, y0)[0](0) - at(x0 - eps, y0)[0](0)) / (2 * eps);
        const double fy = (at(x0, y0 + eps)[0](0) - at(x0, y0 - eps)[0](0)) / (2 * eps);
        const double jx = r[1](0), jy = r[1](1);
        const double tol = 1e-6 * (1 + std::fabs(fx) + std::fabs(fy));
        if (std::fabs(fx - jx) > tol || std::fabs(fy - jy) > tol) {
            std::printf("FAIL derivative of %s: fd (%.12g, %.12g) vs jacobian (%.12g, %.12g)\n", c.first.c_str(), fx,
                        fy, jx, jy);
            ++g_fail;
        }
    }
    // values: a few closed forms
    {
        Function f("f", {x, y}, {sin(x) * y + pow(x, 2.0), atan2(y, x)}, {"x", "y"}, {"a", "b"});
        auto out = f(DMDict{{"x", DM(0.5)}, {"y", DM(2.0)}});
        CHECK(std::fabs(out["a"](0) - (std::sin(0.5) * 2.0 + 0.25)) < 1e-15, "value a");
        CHECK(std::fabs(out["b"](0) - std::atan2(2.0, 0.5)) < 1e-15, "value b");
    }
    // simplification and constant folding
    {
        CHECK((x * 0.0).is_constant() && (x * 0.0).to_double() == 0.0, "x*0");
        CHECK((x + 0.0).nonzeros()[0] == x.nonzeros()[0], "x+0");
        CHECK((x * 1.0).nonzeros()[0] == x.nonzeros()[0], "x*1");
        CHECK((x - x).is_constant(), "x-x");
        CHECK((SX(2.0) * 3.0 + 1.0).to_double() == 7.0, "constant folding");
        SX J = jacobian(SX::vertcat({x * y, x}), v);
        CHECK(J.size1() == 2 && J.size2() == 2, "jacobian dims");
        CHECK(J(1, 0).is_constant() && J(1, 0).to_double() == 1.0, "d x / d x");
        CHECK(J(1, 1).is_constant() && J(1, 1).to_double() == 0.0, "d x / d y");
    }
    // common-subexpression elimination: sin(x) appears once however often it is used
    {
        SX e = sin(x) * sin(x) + sin(x) * y + cos(sin(x));
        std::map<const mahi::mpc::sx::Node*, std::string> in = {{x.nonzeros()[0].get(), "x"}, {y.nonzeros()[0].get(), "y"}};
        const auto cb = mahi::mpc::emit_code(e.nonzeros(), in);
        size_t cnt = 0, pos = 0;
        while ((pos = cb.body.find("sin(x)", pos)) != std::string::npos) ++cnt, ++pos;
        CHECK(cnt == 1, "sin(x) emitted once");
        CHECK(cb.n_ops <= 6, "op count after CSE");
    }
    // matrices
    {
        SX A = SX::sym("A", 2, 3), B = SX::sym("B", 3, 2);
        SX C = mtimes(A, B);
        CHECK(C.size1() == 2 && C.size2() == 2, "mtimes dims");
        Function f("f", {A, B}, {C});
        auto r = f(std::vector<DM>{DM({1, 2, 3, 4, 5, 6}), DM({1, 0, 0, 0, 1, 0})});  // column-major
        // A = [[1,3,5],[2,4,6]], B = [[1,0],[0,1],[0,0]] -> C = [[1,3],[2,4]]
        CHECK(r[0](0) == 1 && r[0](1) == 2 && r[0](2) == 3 && r[0](3) == 4, "mtimes values");
        CHECK(SX::eye(3)(1, 1).to_double() == 1.0 && SX::eye(3)(0, 1).to_double() == 0.0, "eye");
        CHECK(A.T().size1() == 3 && A.T()(2, 1).nonzeros()[0] == A(1, 2).nonzeros()[0], "transpose");
        SX s = substitute(x * y + y, x, SX(2.0));
        Function g("g", {y}, {s});
        CHECK(g(std::vector<DM>{DM(3.0)})[0](0) == 9.0, "substitute");
    }
    // error paths
    {
        SX z = SX::sym("z");
        CHECK(throws([&] { Function("f", {x}, {x + z}); }), "free symbol rejected");
        CHECK(throws([&] { jacobian(x * y, x * 2.0); }), "non-symbolic jacobian variable rejected");
        CHECK(throws([&] { SX::vertcat({SX::sym("a", 2, 2), SX::sym("b", 2, 3)}); }), "vertcat dims");
        CHECK(throws([&] { mtimes(SX::sym("a", 2, 2), SX::sym("b", 3, 1)); }), "mtimes dims");
        CHECK(throws([&] { Function("f", {SX::vertcat({x, x})}, {x}); }), "repeated input symbol");
    }
    if (g_fail) {
        std::printf("sx_selftest: %d failure(s)\n", g_fail);
        return 1;
    }
    std::printf("sx_selftest ok (%zu derivative cases)\n", cases.size());
    return 0;
}
