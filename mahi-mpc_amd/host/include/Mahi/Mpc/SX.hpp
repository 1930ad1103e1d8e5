// Mahi/Mpc/SX.hpp -- the symbolic expression type the reference's model definitions are written in.
//
// The reference builds its dynamics as casadi::SX scalar expression graphs (examples/ex_model_generate.cpp:28-43,
// model_generate_example.cpp:25-47), differentiates them with jacobian() (ModelGenerator.cpp:45-46) and
// code-generates C from them (ModelGenerator.cpp:232-259).  This is the build's own implementation of the part of
// that API the reference uses: scalar/vector/matrix expression graphs with shared sub-expressions, the elementary
// functions, forward-mode symbolic Jacobians, host evaluation (Function) and straight-line code emission with
// common-subexpression elimination (used by ModelGenerator to emit the device model and the CasADi-ABI
// <name>_linear_functions.c).  It is host code: nothing here runs on the GPU.
#pragma once
#include <cstdint>
#include <limits>
#include <map>
#include <memory>
#include <ostream>
#include <string>
#include <vector>

namespace mahi {
namespace mpc {

namespace sx {
enum class Op : uint8_t {
    Const, Sym, Add, Sub, Mul, Div, Neg, Sin, Cos, Tan, Exp, Log, Sqrt, Pow, Tanh, Sinh, Cosh, Atan, Asin, Acos,
    Atan2, Fabs, Sign, Sq
};
struct Node;
using NodeP = std::shared_ptr<const Node>;
struct Node {
    Op op;
    double val = 0.0;   // Const
    std::string name;   // Sym
    NodeP a, b;         // operands
    uint64_t id;        // creation order (unique)
};
NodeP constant(double v);
NodeP symbol(const std::string& name);
NodeP unary(Op op, const NodeP& a);
NodeP binary(Op op, const NodeP& a, const NodeP& b);
bool is_const(const NodeP& n, double v);
}  // namespace sx

class SX {
public:
    SX() {}                       // 0 x 0
    SX(double v);                 // 1 x 1 constant (implicit, as casadi::SX)
    SX(int n1, int n2);           // n1 x n2 zeros
    SX(const std::vector<double>& v);  // column of constants

    static SX sym(const std::string& name, int n1 = 1, int n2 = 1);
    static SX zeros(int n1, int n2 = 1);
    static SX ones(int n1, int n2 = 1);
    static SX eye(int n);
    static SX vertcat(const std::vector<SX>& v);
    static SX horzcat(const std::vector<SX>& v);

    int size1() const { return m_n1; }
    int size2() const { return m_n2; }
    int numel() const { return m_n1 * m_n2; }
    bool is_empty() const { return numel() == 0; }
    bool is_scalar() const { return numel() == 1; }
    bool is_column() const { return m_n2 == 1; }
    // every element a distinct free symbol (what Function inputs and ModelGenerator's x, u must be)
    bool is_symbolic() const;
    bool is_constant() const;
    double to_double() const;  // scalar constant only

    SX operator()(int i) const;         // element i (column-major), 0-based as casadi
    SX operator()(int i, int j) const;  // element (i, j)
    void set(int i, const SX& v);       // element i = scalar v
    SX T() const;

    SX& operator+=(const SX& o);
    SX& operator-=(const SX& o);
    SX& operator*=(const SX& o);
    SX& operator/=(const SX& o);

    const std::vector<sx::NodeP>& nonzeros() const { return m_e; }
    static SX from_nodes(int n1, int n2, std::vector<sx::NodeP> e);

private:
    int m_n1 = 0, m_n2 = 0;
    std::vector<sx::NodeP> m_e;  // column-major
};

// elementwise arithmetic; a 1x1 operand broadcasts
SX operator+(const SX& a, const SX& b);
SX operator-(const SX& a, const SX& b);
SX operator*(const SX& a, const SX& b);  // elementwise (casadi: use mtimes for matrix products)
SX operator/(const SX& a, const SX& b);
SX operator-(const SX& a);
SX operator+(const SX& a);

SX sin(const SX& x);
SX cos(const SX& x);
SX tan(const SX& x);
SX exp(const SX& x);
SX log(const SX& x);
SX sqrt(const SX& x);
SX pow(const SX& x, const SX& y);
SX tanh(const SX& x);
SX sinh(const SX& x);
SX cosh(const SX& x);
SX atan(const SX& x);
SX asin(const SX& x);
SX acos(const SX& x);
SX atan2(const SX& y, const SX& x);
SX fabs(const SX& x);
SX abs(const SX& x);
SX sign(const SX& x);
SX sq(const SX& x);
SX fmin(const SX& a, const SX& b);
SX fmax(const SX& a, const SX& b);

SX mtimes(const SX& a, const SX& b);
SX dot(const SX& a, const SX& b);
SX sum1(const SX& a);  // column sums -> 1 x n2
// d f / d x: (numel f) x (numel x), x purely symbolic (ModelGenerator.cpp:45-46)
SX jacobian(const SX& f, const SX& x);
// replace the symbols of `v` by the expressions `vdef` in `ex`
SX substitute(const SX& ex, const SX& v, const SX& vdef);

std::ostream& operator<<(std::ostream& os, const SX& x);

const double inf = std::numeric_limits<double>::infinity();

// Numeric column vector returned by Function calls (the reference converts casadi::DM to std::vector<double>,
// ModelControl.cpp:127-133, examples/ex_model_control.cpp:77-79,105-108).
class DM {
public:
    DM() {}
    DM(double v) : m_v(1, v) {}
    DM(const std::vector<double>& v) : m_v(v) {}
    DM(std::initializer_list<double> v) : m_v(v) {}
    operator std::vector<double>() const { return m_v; }
    const std::vector<double>& nonzeros() const { return m_v; }
    int size1() const { return static_cast<int>(m_v.size()); }
    double operator()(int i) const { return m_v.at(static_cast<size_t>(i)); }

private:
    std::vector<double> m_v;
};
DM operator+(const DM& a, const DM& b);
DM operator-(const DM& a, const DM& b);
DM operator*(const DM& a, const DM& b);  // elementwise, 1x1 broadcasts
DM operator/(const DM& a, const DM& b);
using DMDict = std::map<std::string, DM>;
using SXDict = DMDict;  // Function calls here are numeric: the reference only calls them with numbers

// Straight-line code of a set of scalar expressions (common-subexpression eliminated, one temporary per
// distinct operation), in C that compiles both as host C and as HIP device code.
struct CodeBlock {
    std::string body;                 // statements "const double tN = ...;"
    std::vector<std::string> values;  // one C expression per requested output
    int n_ops = 0;                    // arithmetic/elementary operations emitted
};
// inputs: symbol node -> C lvalue text (e.g. "x[2]"); throws if an expression uses an unmapped symbol.
// reciprocal_divisors: quotients sharing a divisor multiply by its reciprocal, computed once (within 1.5 ulp).
CodeBlock emit_code(const std::vector<sx::NodeP>& outputs, const std::map<const sx::Node*, std::string>& inputs,
                    const std::string& tmp_prefix = "t", const std::string& indent = "    ",
                    bool reciprocal_divisors = false);

class Function {
public:
    Function() {}
    Function(const std::string& name, const std::vector<SX>& in, const std::vector<SX>& out,
             const std::vector<std::string>& name_in = {}, const std::vector<std::string>& name_out = {});
    const std::string& name() const { return m_name; }
    int n_in() const { return static_cast<int>(m_in.size()); }
    int n_out() const { return static_cast<int>(m_out.size()); }
    const SX& sx_in(int i) const { return m_in.at(static_cast<size_t>(i)); }
    const SX& sx_out(int i) const { return m_out.at(static_cast<size_t>(i)); }
    const std::string& name_in(int i) const { return m_name_in.at(static_cast<size_t>(i)); }
    const std::string& name_out(int i) const { return m_name_out.at(static_cast<size_t>(i)); }
    // host evaluation (dense column-major values)
    std::vector<DM> operator()(const std::vector<DM>& args) const;
    DMDict operator()(const DMDict& args) const;
    // C source of this function with the CasADi external ABI (src/codegen_usage.cpp:61-146)
    std::string generate_external_c() const;

private:
    std::string m_name;
    std::vector<SX> m_in, m_out;
    std::vector<std::string> m_name_in, m_name_out;
};

}  // namespace mpc
}  // namespace mahi

// Source compatibility with the reference's model definitions, which say `using namespace casadi;` and
// spell casadi::SX / casadi::Function / casadi::inf (examples/ex_model_generate.cpp:4,28-43).
namespace casadi {
using mahi::mpc::DM;
using mahi::mpc::DMDict;
using mahi::mpc::Function;
using mahi::mpc::inf;
using mahi::mpc::SX;
using mahi::mpc::SXDict;
// casadi's stream operator for std::vector ("[a, b, c]"), which the reference's examples reach through
// `using namespace casadi;` (model_control_example.cpp:104 writes `file << time_result`)
template <class T>
std::ostream& operator<<(std::ostream& os, const std::vector<T>& v) {
    os << "[";
    for (size_t i = 0; i < v.size(); ++i) os << (i ? ", " : "") << v[i];
    return os << "]";
}
}  // namespace casadi
