// SX.cpp -- expression graphs, symbolic Jacobians, host evaluation and C emission (see Mahi/Mpc/SX.hpp).
#include <Mahi/Mpc/SX.hpp>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <sstream>
#include <stdexcept>
#include <tuple>
#include <unordered_map>
#include <unordered_set>

namespace mahi {
namespace mpc {

namespace sx {
namespace {
std::atomic<uint64_t> g_next_id{1};

NodeP make(Op op, double val, std::string name, NodeP a, NodeP b) {
    auto n = std::make_shared<Node>();
    n->op = op;
    n->val = val;
    n->name = std::move(name);
    n->a = std::move(a);
    n->b = std::move(b);
    n->id = g_next_id++;
    return n;
}

double apply1(Op op, double a) {
    switch (op) {
        case Op::Neg: return -a;
        case Op::Sin: return std::sin(a);
        case Op::Cos: return std::cos(a);
        case Op::Tan: return std::tan(a);
        case Op::Exp: return std::exp(a);
        case Op::Log: return std::log(a);
        case Op::Sqrt: return std::sqrt(a);
        case Op::Tanh: return std::tanh(a);
        case Op::Sinh: return std::sinh(a);
        case Op::Cosh: return std::cosh(a);
        case Op::Atan: return std::atan(a);
        case Op::Asin: return std::asin(a);
        case Op::Acos: return std::acos(a);
        case Op::Fabs: return std::fabs(a);
        case Op::Sign: return a > 0.0 ? 1.0 : (a < 0.0 ? -1.0 : (a == a ? 0.0 : a));
        case Op::Sq: return a * a;
        default: throw std::logic_error("sx: not a unary op");
    }
}
double apply2(Op op, double a, double b) {
    switch (op) {
        case Op::Add: return a + b;
        case Op::Sub: return a - b;
        case Op::Mul: return a * b;
        case Op::Div: return a / b;
        case Op::Pow: return std::pow(a, b);
        case Op::Atan2: return std::atan2(a, b);
        default: throw std::logic_error("sx: not a binary op");
    }
}
bool is_unary(Op op) { return op >= Op::Neg && op != Op::Pow && op != Op::Atan2; }
}  // namespace

bool is_const(const NodeP& n, double v) { return n->op == Op::Const && n->val == v; }

NodeP constant(double v) {
    static const NodeP zero = make(Op::Const, 0.0, "", nullptr, nullptr);
    static const NodeP one = make(Op::Const, 1.0, "", nullptr, nullptr);
    if (v == 0.0 && !std::signbit(v)) return zero;
    if (v == 1.0) return one;
    return make(Op::Const, v, "", nullptr, nullptr);
}

NodeP symbol(const std::string& name) { return make(Op::Sym, 0.0, name, nullptr, nullptr); }

NodeP unary(Op op, const NodeP& a) {
    if (a->op == Op::Const) return constant(apply1(op, a->val));
    if (op == Op::Neg && a->op == Op::Neg) return a->a;
    if (op == Op::Sq && a->op == Op::Neg) return unary(Op::Sq, a->a);
    return make(op, 0.0, "", a, nullptr);
}

NodeP binary(Op op, const NodeP& a, const NodeP& b) {
    if (a->op == Op::Const && b->op == Op::Const) return constant(apply2(op, a->val, b->val));
    switch (op) {
        case Op::Add:
            if (is_const(a, 0.0)) return b;
            if (is_const(b, 0.0)) return a;
            if (b->op == Op::Neg) return binary(Op::Sub, a, b->a);
            break;
        case Op::Sub:
            if (is_const(b, 0.0)) return a;
            if (is_const(a, 0.0)) return unary(Op::Neg, b);
            if (a == b) return constant(0.0);
            if (b->op == Op::Neg) return binary(Op::Add, a, b->a);
            break;
        case Op::Mul:
            if (is_const(a, 0.0) || is_const(b, 0.0)) return constant(0.0);
            if (is_const(a, 1.0)) return b;
            if (is_const(b, 1.0)) return a;
            if (is_const(a, -1.0)) return unary(Op::Neg, b);
            if (is_const(b, -1.0)) return unary(Op::Neg, a);
            if (a == b) return unary(Op::Sq, a);
            break;
        case Op::Div:
            if (is_const(a, 0.0)) return constant(0.0);
            if (is_const(b, 1.0)) return a;
            if (is_const(b, -1.0)) return unary(Op::Neg, a);
            break;
        case Op::Pow:
            if (is_const(b, 1.0)) return a;
            if (is_const(b, 0.0)) return constant(1.0);
            if (is_const(b, 2.0)) return unary(Op::Sq, a);
            break;
        default: break;
    }
    return make(op, 0.0, "", a, b);
}

namespace {
// children-first order of every node reachable from `roots` (iterative: expression chains can be long)
std::vector<const Node*> topo_order(const std::vector<NodeP>& roots) {
    std::vector<const Node*> order;
    std::unordered_set<const Node*> seen;
    std::vector<std::pair<const Node*, int>> stack;
    for (const NodeP& r : roots) {
        if (!r || seen.count(r.get())) continue;
        stack.push_back({r.get(), 0});
        while (!stack.empty()) {
            auto& top = stack.back();
            const Node* n = top.first;
            if (top.second == 0) {
                top.second = 1;
                if (seen.count(n)) {
                    stack.pop_back();
                    continue;
                }
                if (n->b && !seen.count(n->b.get())) stack.push_back({n->b.get(), 0});
                if (n->a && !seen.count(n->a.get())) stack.push_back({n->a.get(), 0});
            } else {
                stack.pop_back();
                if (seen.insert(n).second) order.push_back(n);
            }
        }
    }
    return order;
}
}  // namespace
}  // namespace sx

using sx::NodeP;
using sx::Op;

// ------------------------------------------------------------------------------------------------ SX
SX::SX(double v) : m_n1(1), m_n2(1), m_e{sx::constant(v)} {}
SX::SX(int n1, int n2) : m_n1(n1), m_n2(n2), m_e(static_cast<size_t>(n1) * n2, sx::constant(0.0)) {
    if (n1 < 0 || n2 < 0) throw std::invalid_argument("SX: negative dimension");
}
SX::SX(const std::vector<double>& v) : m_n1(static_cast<int>(v.size())), m_n2(1) {
    for (double d : v) m_e.push_back(sx::constant(d));
}

SX SX::from_nodes(int n1, int n2, std::vector<NodeP> e) {
    if (static_cast<size_t>(n1) * n2 != e.size()) throw std::invalid_argument("SX: size mismatch");
    SX r;
    r.m_n1 = n1;
    r.m_n2 = n2;
    r.m_e = std::move(e);
    return r;
}

SX SX::sym(const std::string& name, int n1, int n2) {
    if (n1 < 0 || n2 < 0) throw std::invalid_argument("SX::sym: negative dimension");
    std::vector<NodeP> e;
    if (n1 * n2 == 1) {
        e.push_back(sx::symbol(name));
    } else {
        for (int j = 0; j < n2; ++j)
            for (int i = 0; i < n1; ++i)
                e.push_back(sx::symbol(n2 == 1 ? name + "_" + std::to_string(i)
                                               : name + "_" + std::to_string(i + j * n1)));
    }
    return from_nodes(n1, n2, std::move(e));
}
SX SX::zeros(int n1, int n2) { return SX(n1, n2); }
SX SX::ones(int n1, int n2) { return from_nodes(n1, n2, std::vector<NodeP>(static_cast<size_t>(n1) * n2, sx::constant(1.0))); }
SX SX::eye(int n) {
    SX r(n, n);
    for (int i = 0; i < n; ++i) r.m_e[static_cast<size_t>(i) * n + i] = sx::constant(1.0);
    return r;
}
SX SX::vertcat(const std::vector<SX>& v) {
    int n2 = -1, n1 = 0;
    for (const SX& x : v) {
        if (x.is_empty()) continue;
        if (n2 >= 0 && x.m_n2 != n2) throw std::invalid_argument("vertcat: column counts differ");
        n2 = x.m_n2;
        n1 += x.m_n1;
    }
    if (n2 < 0) return SX();
    std::vector<NodeP> e(static_cast<size_t>(n1) * n2);
    int r0 = 0;
    for (const SX& x : v) {
        if (x.is_empty()) continue;
        for (int j = 0; j < n2; ++j)
            for (int i = 0; i < x.m_n1; ++i) e[static_cast<size_t>(j) * n1 + r0 + i] = x.m_e[static_cast<size_t>(j) * x.m_n1 + i];
        r0 += x.m_n1;
    }
    return from_nodes(n1, n2, std::move(e));
}
SX SX::horzcat(const std::vector<SX>& v) {
    std::vector<SX> t;
    for (const SX& x : v) t.push_back(x.T());
    return vertcat(t).T();
}

bool SX::is_symbolic() const {
    std::unordered_set<const sx::Node*> s;
    for (const NodeP& n : m_e)
        if (n->op != Op::Sym || !s.insert(n.get()).second) return false;
    return true;
}
bool SX::is_constant() const {
    for (const NodeP& n : m_e)
        if (n->op != Op::Const) return false;
    return true;
}
double SX::to_double() const {
    if (!is_scalar() || m_e[0]->op != Op::Const) throw std::invalid_argument("SX::to_double: not a scalar constant");
    return m_e[0]->val;
}

SX SX::operator()(int i) const {
    if (i < 0 || i >= numel()) throw std::out_of_range("SX: index out of range");
    return from_nodes(1, 1, {m_e[static_cast<size_t>(i)]});
}
SX SX::operator()(int i, int j) const {
    if (i < 0 || i >= m_n1 || j < 0 || j >= m_n2) throw std::out_of_range("SX: index out of range");
    return from_nodes(1, 1, {m_e[static_cast<size_t>(j) * m_n1 + i]});
}
void SX::set(int i, const SX& v) {
    if (i < 0 || i >= numel()) throw std::out_of_range("SX: index out of range");
    if (!v.is_scalar()) throw std::invalid_argument("SX::set: scalar expected");
    m_e[static_cast<size_t>(i)] = v.m_e[0];
}
SX SX::T() const {
    std::vector<NodeP> e(m_e.size());
    for (int j = 0; j < m_n2; ++j)
        for (int i = 0; i < m_n1; ++i) e[static_cast<size_t>(i) * m_n2 + j] = m_e[static_cast<size_t>(j) * m_n1 + i];
    return from_nodes(m_n2, m_n1, std::move(e));
}
SX& SX::operator+=(const SX& o) { return *this = *this + o; }
SX& SX::operator-=(const SX& o) { return *this = *this - o; }
SX& SX::operator*=(const SX& o) { return *this = *this * o; }
SX& SX::operator/=(const SX& o) { return *this = *this / o; }

namespace {
SX elementwise(Op op, const SX& a, const SX& b) {
    const auto& ea = a.nonzeros();
    const auto& eb = b.nonzeros();
    if (a.is_scalar() && !b.is_scalar()) {
        std::vector<NodeP> e;
        for (const NodeP& n : eb) e.push_back(sx::binary(op, ea[0], n));
        return SX::from_nodes(b.size1(), b.size2(), std::move(e));
    }
    if (b.is_scalar() && !a.is_scalar()) {
        std::vector<NodeP> e;
        for (const NodeP& n : ea) e.push_back(sx::binary(op, n, eb[0]));
        return SX::from_nodes(a.size1(), a.size2(), std::move(e));
    }
    if (a.size1() != b.size1() || a.size2() != b.size2()) throw std::invalid_argument("SX: dimension mismatch");
    std::vector<NodeP> e;
    for (size_t i = 0; i < ea.size(); ++i) e.push_back(sx::binary(op, ea[i], eb[i]));
    return SX::from_nodes(a.size1(), a.size2(), std::move(e));
}
SX elementwise1(Op op, const SX& a) {
    std::vector<NodeP> e;
    for (const NodeP& n : a.nonzeros()) e.push_back(sx::unary(op, n));
    return SX::from_nodes(a.size1(), a.size2(), std::move(e));
}
}  // namespace

SX operator+(const SX& a, const SX& b) { return elementwise(Op::Add, a, b); }
SX operator-(const SX& a, const SX& b) { return elementwise(Op::Sub, a, b); }
SX operator*(const SX& a, const SX& b) { return elementwise(Op::Mul, a, b); }
SX operator/(const SX& a, const SX& b) { return elementwise(Op::Div, a, b); }
SX operator-(const SX& a) { return elementwise1(Op::Neg, a); }
SX operator+(const SX& a) { return a; }
SX sin(const SX& x) { return elementwise1(Op::Sin, x); }
SX cos(const SX& x) { return elementwise1(Op::Cos, x); }
SX tan(const SX& x) { return elementwise1(Op::Tan, x); }
SX exp(const SX& x) { return elementwise1(Op::Exp, x); }
SX log(const SX& x) { return elementwise1(Op::Log, x); }
SX sqrt(const SX& x) { return elementwise1(Op::Sqrt, x); }
SX pow(const SX& x, const SX& y) { return elementwise(Op::Pow, x, y); }
SX tanh(const SX& x) { return elementwise1(Op::Tanh, x); }
SX sinh(const SX& x) { return elementwise1(Op::Sinh, x); }
SX cosh(const SX& x) { return elementwise1(Op::Cosh, x); }
SX atan(const SX& x) { return elementwise1(Op::Atan, x); }
SX asin(const SX& x) { return elementwise1(Op::Asin, x); }
SX acos(const SX& x) { return elementwise1(Op::Acos, x); }
SX atan2(const SX& y, const SX& x) { return elementwise(Op::Atan2, y, x); }
SX fabs(const SX& x) { return elementwise1(Op::Fabs, x); }
SX abs(const SX& x) { return elementwise1(Op::Fabs, x); }
SX sign(const SX& x) { return elementwise1(Op::Sign, x); }
SX sq(const SX& x) { return elementwise1(Op::Sq, x); }
// min/max through |a - b| keeps the graph arithmetic (derivative: the active branch, the mean at a tie)
SX fmin(const SX& a, const SX& b) { return (a + b - fabs(a - b)) * 0.5; }
SX fmax(const SX& a, const SX& b) { return (a + b + fabs(a - b)) * 0.5; }

SX mtimes(const SX& a, const SX& b) {
    if (a.size2() != b.size1()) throw std::invalid_argument("mtimes: inner dimensions differ");
    const int n = a.size1(), m = b.size2(), k = a.size2();
    std::vector<NodeP> e(static_cast<size_t>(n) * m);
    for (int j = 0; j < m; ++j)
        for (int i = 0; i < n; ++i) {
            NodeP acc = sx::constant(0.0);
            for (int l = 0; l < k; ++l)
                acc = sx::binary(Op::Add, acc,
                                 sx::binary(Op::Mul, a.nonzeros()[static_cast<size_t>(l) * n + i],
                                            b.nonzeros()[static_cast<size_t>(j) * k + l]));
            e[static_cast<size_t>(j) * n + i] = acc;
        }
    return SX::from_nodes(n, m, std::move(e));
}
SX dot(const SX& a, const SX& b) {
    if (a.numel() != b.numel()) throw std::invalid_argument("dot: sizes differ");
    NodeP acc = sx::constant(0.0);
    for (int i = 0; i < a.numel(); ++i) acc = sx::binary(Op::Add, acc, sx::binary(Op::Mul, a.nonzeros()[i], b.nonzeros()[i]));
    return SX::from_nodes(1, 1, {acc});
}
SX sum1(const SX& a) {
    std::vector<NodeP> e;
    for (int j = 0; j < a.size2(); ++j) {
        NodeP acc = sx::constant(0.0);
        for (int i = 0; i < a.size1(); ++i) acc = sx::binary(Op::Add, acc, a.nonzeros()[static_cast<size_t>(j) * a.size1() + i]);
        e.push_back(acc);
    }
    return SX::from_nodes(1, a.size2(), std::move(e));
}

namespace {
// derivative of node n given the derivatives of its operands (forward mode)
NodeP deriv_rule(const sx::Node* n, const NodeP& self, const NodeP& da, const NodeP& db) {
    using namespace sx;
    const NodeP& a = n->a;
    const NodeP& b = n->b;
    const bool za = !da || is_const(da, 0.0), zb = !db || is_const(db, 0.0);
    if (za && zb) return constant(0.0);
    const NodeP zero = constant(0.0);
    switch (n->op) {
        case Op::Add: return binary(Op::Add, za ? zero : da, zb ? zero : db);
        case Op::Sub: return binary(Op::Sub, za ? zero : da, zb ? zero : db);
        case Op::Mul:
            return binary(Op::Add, za ? zero : binary(Op::Mul, da, b), zb ? zero : binary(Op::Mul, a, db));
        case Op::Div:  // (da - (a/b) db) / b
            return binary(Op::Div, binary(Op::Sub, za ? zero : da, zb ? zero : binary(Op::Mul, self, db)), b);
        case Op::Neg: return unary(Op::Neg, da);
        case Op::Sin: return binary(Op::Mul, unary(Op::Cos, a), da);
        case Op::Cos: return unary(Op::Neg, binary(Op::Mul, unary(Op::Sin, a), da));
        case Op::Tan: return binary(Op::Mul, binary(Op::Add, constant(1.0), unary(Op::Sq, self)), da);
        case Op::Exp: return binary(Op::Mul, self, da);
        case Op::Log: return binary(Op::Div, da, a);
        case Op::Sqrt: return binary(Op::Div, da, binary(Op::Mul, constant(2.0), self));
        case Op::Pow:
            if (b->op == Op::Const)  // c a^(c-1) da
                return binary(Op::Mul, binary(Op::Mul, b, binary(Op::Pow, a, constant(b->val - 1.0))), da);
            // a^b (b' log a + b a'/a)
            return binary(Op::Mul, self,
                          binary(Op::Add, zb ? zero : binary(Op::Mul, db, unary(Op::Log, a)),
                                 za ? zero : binary(Op::Div, binary(Op::Mul, b, da), a)));
        case Op::Tanh: return binary(Op::Mul, binary(Op::Sub, constant(1.0), unary(Op::Sq, self)), da);
        case Op::Sinh: return binary(Op::Mul, unary(Op::Cosh, a), da);
        case Op::Cosh: return binary(Op::Mul, unary(Op::Sinh, a), da);
        case Op::Atan: return binary(Op::Div, da, binary(Op::Add, constant(1.0), unary(Op::Sq, a)));
        case Op::Asin: return binary(Op::Div, da, unary(Op::Sqrt, binary(Op::Sub, constant(1.0), unary(Op::Sq, a))));
        case Op::Acos:
            return unary(Op::Neg, binary(Op::Div, da, unary(Op::Sqrt, binary(Op::Sub, constant(1.0), unary(Op::Sq, a)))));
        case Op::Atan2:  // atan2(a, b): (b da - a db) / (a^2 + b^2)
            return binary(Op::Div,
                          binary(Op::Sub, za ? zero : binary(Op::Mul, b, da), zb ? zero : binary(Op::Mul, a, db)),
                          binary(Op::Add, unary(Op::Sq, a), unary(Op::Sq, b)));
        case Op::Fabs: return binary(Op::Mul, unary(Op::Sign, a), da);
        case Op::Sign: return constant(0.0);
        case Op::Sq: return binary(Op::Mul, binary(Op::Mul, constant(2.0), a), da);
        default: throw std::logic_error("jacobian: unexpected op");
    }
}
}  // namespace

SX jacobian(const SX& f, const SX& x) {
    if (!x.is_symbolic()) throw std::invalid_argument("jacobian: x must be purely symbolic");
    const int nf = f.numel(), nxv = x.numel();
    const std::vector<const sx::Node*> order = sx::topo_order(f.nonzeros());
    std::unordered_map<const sx::Node*, NodeP> owner;  // raw pointer -> shared pointer (for "self")
    for (const NodeP& r : f.nonzeros()) owner[r.get()] = r;
    for (const sx::Node* n : order) {
        if (n->a) owner[n->a.get()] = n->a;
        if (n->b) owner[n->b.get()] = n->b;
    }
    std::vector<NodeP> e(static_cast<size_t>(nf) * nxv);
    std::unordered_map<const sx::Node*, NodeP> d;
    for (int j = 0; j < nxv; ++j) {
        const sx::Node* var = x.nonzeros()[static_cast<size_t>(j)].get();
        d.clear();
        for (const sx::Node* n : order) {
            NodeP dn;
            if (n->op == Op::Const) dn = nullptr;
            else if (n->op == Op::Sym) dn = (n == var) ? sx::constant(1.0) : nullptr;
            else {
                NodeP da = n->a ? d[n->a.get()] : nullptr, db = n->b ? d[n->b.get()] : nullptr;
                if ((!da || sx::is_const(da, 0.0)) && (!db || sx::is_const(db, 0.0))) dn = nullptr;
                else dn = deriv_rule(n, owner[n], da, db);
            }
            d[n] = dn;
        }
        for (int i = 0; i < nf; ++i) {
            const NodeP& dn = d[f.nonzeros()[static_cast<size_t>(i)].get()];
            e[static_cast<size_t>(j) * nf + i] = dn ? dn : sx::constant(0.0);
        }
    }
    return SX::from_nodes(nf, nxv, std::move(e));
}

SX substitute(const SX& ex, const SX& v, const SX& vdef) {
    if (!v.is_symbolic() || v.numel() != vdef.numel()) throw std::invalid_argument("substitute: bad arguments");
    std::unordered_map<const sx::Node*, NodeP> m;
    for (int i = 0; i < v.numel(); ++i) m[v.nonzeros()[i].get()] = vdef.nonzeros()[i];
    const auto order = sx::topo_order(ex.nonzeros());
    for (const sx::Node* n : order) {
        if (m.count(n)) continue;
        if (n->op == Op::Const || n->op == Op::Sym) continue;
        const NodeP a = m.count(n->a.get()) ? m[n->a.get()] : n->a;
        if (sx::is_unary(n->op)) {
            if (a != n->a) m[n] = sx::unary(n->op, a);
        } else {
            const NodeP b = m.count(n->b.get()) ? m[n->b.get()] : n->b;
            if (a != n->a || b != n->b) m[n] = sx::binary(n->op, a, b);
        }
    }
    std::vector<NodeP> e;
    for (const NodeP& r : ex.nonzeros()) e.push_back(m.count(r.get()) ? m[r.get()] : r);
    return SX::from_nodes(ex.size1(), ex.size2(), std::move(e));
}

namespace {
const char* op_name(Op op) {
    switch (op) {
        case Op::Sin: return "sin";
        case Op::Cos: return "cos";
        case Op::Tan: return "tan";
        case Op::Exp: return "exp";
        case Op::Log: return "log";
        case Op::Sqrt: return "sqrt";
        case Op::Pow: return "pow";
        case Op::Tanh: return "tanh";
        case Op::Sinh: return "sinh";
        case Op::Cosh: return "cosh";
        case Op::Atan: return "atan";
        case Op::Asin: return "asin";
        case Op::Acos: return "acos";
        case Op::Atan2: return "atan2";
        case Op::Fabs: return "fabs";
        default: return nullptr;
    }
}
std::string literal(double v) {
    if (std::isnan(v)) return "__builtin_nan(\"\")";
    if (std::isinf(v)) return v > 0 ? "__builtin_inf()" : "(-__builtin_inf())";
    char buf[40];
    std::snprintf(buf, sizeof(buf), "%.17g", v);
    std::string s = buf;
    if (s.find_first_of(".eE") == std::string::npos) s += ".0";
    return v < 0 ? "(" + s + ")" : s;
}
std::string expr_text(Op op, const std::string& a, const std::string& b) {
    switch (op) {
        case Op::Add: return a + " + " + b;
        case Op::Sub: return a + " - " + b;
        case Op::Mul: return a + " * " + b;
        case Op::Div: return a + " / " + b;
        case Op::Neg: return "-" + a;
        case Op::Sq: return a + " * " + a;
        case Op::Sign: return "(" + a + " > 0.0 ? 1.0 : (" + a + " < 0.0 ? -1.0 : 0.0))";
        default: break;
    }
    const char* f = op_name(op);
    if (!f) throw std::logic_error("emit: unexpected op");
    return std::string(f) + (b.empty() ? "(" + a + ")" : "(" + a + ", " + b + ")");
}
}  // namespace

CodeBlock emit_code(const std::vector<NodeP>& outputs, const std::map<const sx::Node*, std::string>& inputs,
                    const std::string& tmp_prefix, const std::string& indent, bool reciprocal_divisors) {
    CodeBlock cb;
    std::ostringstream body;
    std::unordered_map<const sx::Node*, std::string> text;  // node -> operand text
    std::map<std::tuple<int, std::string, std::string>, std::string> cse;
    int ntmp = 0;
    const std::vector<const sx::Node*> order = sx::topo_order(outputs);
    // reciprocal_divisors: a divisor shared by several quotients is inverted once (1 ulp per quotient; an fp64
    // division is ~10 GPU instructions, a multiply one)
    std::unordered_map<const sx::Node*, int> ndiv;
    std::unordered_map<const sx::Node*, std::string> recip;
    if (reciprocal_divisors)
        for (const sx::Node* n : order)
            if (n->op == Op::Div) ++ndiv[n->b.get()];
    for (const sx::Node* n : order) {
        if (n->op == Op::Const) {
            text[n] = literal(n->val);
            continue;
        }
        if (n->op == Op::Sym) {
            auto it = inputs.find(n);
            if (it == inputs.end()) throw std::invalid_argument("emit: expression uses the free symbol \"" + n->name + "\"");
            text[n] = it->second;
            continue;
        }
        std::string a = text.at(n->a.get()), b = n->b ? text.at(n->b.get()) : std::string();
        Op op = n->op;
        if (op == Op::Div && reciprocal_divisors && ndiv[n->b.get()] >= 2) {
            auto r = recip.find(n->b.get());
            if (r == recip.end()) {
                const std::string t = tmp_prefix + std::to_string(ntmp++);
                body << indent << "const double " << t << " = 1.0 / " << b << ";\n";
                ++cb.n_ops;
                r = recip.emplace(n->b.get(), t).first;
            }
            op = Op::Mul;
            b = r->second;
        }
        if ((op == Op::Add || op == Op::Mul) && b < a) std::swap(a, b);  // commutative: canonical order
        const auto key = std::make_tuple(static_cast<int>(op), a, b);
        auto it = cse.find(key);
        if (it != cse.end()) {
            text[n] = it->second;
            continue;
        }
        const std::string t = tmp_prefix + std::to_string(ntmp++);
        body << indent << "const double " << t << " = " << expr_text(op, a, b) << ";\n";
        ++cb.n_ops;
        cse[key] = t;
        text[n] = t;
    }
    cb.body = body.str();
    for (const NodeP& o : outputs) cb.values.push_back(text.at(o.get()));
    return cb;
}

std::ostream& operator<<(std::ostream& os, const SX& x) {
    std::map<const sx::Node*, std::string> in;
    for (const sx::Node* n : sx::topo_order(x.nonzeros()))
        if (n->op == Op::Sym) in[n] = n->name;
    const CodeBlock cb = emit_code(x.nonzeros(), in, "@", "  ");
    os << "SX(" << x.size1() << "x" << x.size2() << ")";
    if (!cb.body.empty()) os << "\n" << cb.body;
    os << "[";
    for (size_t i = 0; i < cb.values.size(); ++i) os << (i ? ", " : "") << cb.values[i];
    return os << "]";
}

// ------------------------------------------------------------------------------------------------ DM
namespace {
DM dm_op(const DM& a, const DM& b, Op op) {
    const auto& x = a.nonzeros();
    const auto& y = b.nonzeros();
    std::vector<double> r;
    if (x.size() == 1 && y.size() != 1) {
        for (double v : y) r.push_back(sx::apply2(op, x[0], v));
    } else if (y.size() == 1 && x.size() != 1) {
        for (double v : x) r.push_back(sx::apply2(op, v, y[0]));
    } else {
        if (x.size() != y.size()) throw std::invalid_argument("DM: dimension mismatch");
        for (size_t i = 0; i < x.size(); ++i) r.push_back(sx::apply2(op, x[i], y[i]));
    }
    return DM(r);
}
}  // namespace
DM operator+(const DM& a, const DM& b) { return dm_op(a, b, Op::Add); }
DM operator-(const DM& a, const DM& b) { return dm_op(a, b, Op::Sub); }
DM operator*(const DM& a, const DM& b) { return dm_op(a, b, Op::Mul); }
DM operator/(const DM& a, const DM& b) { return dm_op(a, b, Op::Div); }

// ------------------------------------------------------------------------------------------------ Function
Function::Function(const std::string& name, const std::vector<SX>& in, const std::vector<SX>& out,
                   const std::vector<std::string>& name_in, const std::vector<std::string>& name_out)
    : m_name(name), m_in(in), m_out(out), m_name_in(name_in), m_name_out(name_out) {
    std::unordered_set<const sx::Node*> syms;
    for (const SX& x : in) {
        if (!x.is_symbolic()) throw std::invalid_argument("Function " + name + ": inputs must be purely symbolic");
        for (const NodeP& n : x.nonzeros())
            if (!syms.insert(n.get()).second) throw std::invalid_argument("Function " + name + ": repeated input symbol");
    }
    for (size_t i = m_name_in.size(); i < in.size(); ++i) m_name_in.push_back("i" + std::to_string(i));
    for (size_t i = m_name_out.size(); i < out.size(); ++i) m_name_out.push_back("o" + std::to_string(i));
    if (m_name_in.size() != in.size() || m_name_out.size() != out.size())
        throw std::invalid_argument("Function " + name + ": wrong number of names");
    std::vector<NodeP> outs;
    for (const SX& o : out) outs.insert(outs.end(), o.nonzeros().begin(), o.nonzeros().end());
    for (const sx::Node* n : sx::topo_order(outs))
        if (n->op == Op::Sym && !syms.count(n))
            throw std::invalid_argument("Function " + name + ": output depends on the free symbol \"" + n->name + "\"");
}

std::vector<DM> Function::operator()(const std::vector<DM>& args) const {
    if (args.size() != m_in.size()) throw std::invalid_argument("Function " + m_name + ": wrong number of inputs");
    std::unordered_map<const sx::Node*, double> val;
    for (size_t i = 0; i < args.size(); ++i) {
        const auto& v = args[i].nonzeros();
        if (static_cast<int>(v.size()) != m_in[i].numel())
            throw std::invalid_argument("Function " + m_name + ": input " + m_name_in[i] + " has the wrong size");
        for (size_t k = 0; k < v.size(); ++k) val[m_in[i].nonzeros()[k].get()] = v[k];
    }
    std::vector<NodeP> outs;
    for (const SX& o : m_out) outs.insert(outs.end(), o.nonzeros().begin(), o.nonzeros().end());
    for (const sx::Node* n : sx::topo_order(outs)) {
        if (n->op == Op::Const) val[n] = n->val;
        else if (n->op == Op::Sym) continue;
        else if (sx::is_unary(n->op)) val[n] = sx::apply1(n->op, val.at(n->a.get()));
        else val[n] = sx::apply2(n->op, val.at(n->a.get()), val.at(n->b.get()));
    }
    std::vector<DM> res;
    for (const SX& o : m_out) {
        std::vector<double> v;
        for (const NodeP& n : o.nonzeros()) v.push_back(val.at(n.get()));
        res.emplace_back(v);
    }
    return res;
}

DMDict Function::operator()(const DMDict& args) const {
    std::vector<DM> a;
    for (size_t i = 0; i < m_in.size(); ++i) {
        auto it = args.find(m_name_in[i]);
        a.push_back(it != args.end() ? it->second : DM(std::vector<double>(static_cast<size_t>(m_in[i].numel()), 0.0)));
    }
    const std::vector<DM> r = (*this)(a);
    DMDict out;
    for (size_t i = 0; i < r.size(); ++i) out[m_name_out[i]] = r[i];
    return out;
}

std::string Function::generate_external_c() const {
    std::map<const sx::Node*, std::string> in;
    std::ostringstream f;
    const std::string& fn = m_name;
    std::vector<NodeP> outs;
    for (const SX& o : m_out) outs.insert(outs.end(), o.nonzeros().begin(), o.nonzeros().end());
    // inputs are read into locals first (a NULL arg means zeros, as in CasADi-generated code)
    std::ostringstream pre;
    for (size_t i = 0; i < m_in.size(); ++i)
        for (int k = 0; k < m_in[i].numel(); ++k) {
            const std::string v = "a" + std::to_string(i) + "_" + std::to_string(k);
            pre << "    const casadi_real " << v << " = arg[" << i << "] ? arg[" << i << "][" << k << "] : 0.0;\n";
            in[m_in[i].nonzeros()[static_cast<size_t>(k)].get()] = v;
        }
    const CodeBlock cb = emit_code(outs, in, "t");
    auto pattern = [](const SX& x) {
        std::ostringstream o;
        o << "{" << x.size1() << ", " << x.size2();
        for (int c = 0; c <= x.size2(); ++c) o << ", " << c * x.size1();
        for (int c = 0; c < x.size2(); ++c)
            for (int r = 0; r < x.size1(); ++r) o << ", " << r;
        o << "}";
        return o.str();
    };
    for (size_t i = 0; i < m_in.size(); ++i) f << "static const casadi_int " << fn << "_s_in" << i << "[] = " << pattern(m_in[i]) << ";\n";
    for (size_t i = 0; i < m_out.size(); ++i) f << "static const casadi_int " << fn << "_s_out" << i << "[] = " << pattern(m_out[i]) << ";\n";
    f << "int " << fn << "(const casadi_real** arg, casadi_real** res, casadi_int* iw, casadi_real* w, int mem) {\n"
      << "    (void)iw; (void)w; (void)mem;\n"
      << pre.str() << cb.body;
    size_t k = 0;
    for (size_t i = 0; i < m_out.size(); ++i) {
        f << "    if (res[" << i << "]) {\n";
        for (int e = 0; e < m_out[i].numel(); ++e, ++k) f << "        res[" << i << "][" << e << "] = " << cb.values[k] << ";\n";
        f << "    }\n";
    }
    f << "    return 0;\n}\n";
    f << "int " << fn << "_alloc_mem(void) { return 0; }\n"
      << "int " << fn << "_init_mem(int mem) { (void)mem; return 0; }\n"
      << "void " << fn << "_free_mem(int mem) { (void)mem; }\n"
      << "int " << fn << "_checkout(void) { return 0; }\n"
      << "void " << fn << "_release(int mem) { (void)mem; }\n"
      << "void " << fn << "_incref(void) {}\n"
      << "void " << fn << "_decref(void) {}\n"
      << "casadi_int " << fn << "_n_in(void) { return " << m_in.size() << "; }\n"
      << "casadi_int " << fn << "_n_out(void) { return " << m_out.size() << "; }\n"
      << "casadi_real " << fn << "_default_in(casadi_int i) { (void)i; return 0; }\n";
    f << "const char* " << fn << "_name_in(casadi_int i) {\n    switch (i) {\n";
    for (size_t i = 0; i < m_in.size(); ++i) f << "        case " << i << ": return \"" << m_name_in[i] << "\";\n";
    f << "        default: return 0;\n    }\n}\n";
    f << "const char* " << fn << "_name_out(casadi_int i) {\n    switch (i) {\n";
    for (size_t i = 0; i < m_out.size(); ++i) f << "        case " << i << ": return \"" << m_name_out[i] << "\";\n";
    f << "        default: return 0;\n    }\n}\n";
    f << "const casadi_int* " << fn << "_sparsity_in(casadi_int i) {\n    switch (i) {\n";
    for (size_t i = 0; i < m_in.size(); ++i) f << "        case " << i << ": return " << fn << "_s_in" << i << ";\n";
    f << "        default: return 0;\n    }\n}\n";
    f << "const casadi_int* " << fn << "_sparsity_out(casadi_int i) {\n    switch (i) {\n";
    for (size_t i = 0; i < m_out.size(); ++i) f << "        case " << i << ": return " << fn << "_s_out" << i << ";\n";
    f << "        default: return 0;\n    }\n}\n";
    f << "int " << fn << "_work(casadi_int* sz_arg, casadi_int* sz_res, casadi_int* sz_iw, casadi_int* sz_w) {\n"
      << "    if (sz_arg) *sz_arg = " << m_in.size() << ";\n    if (sz_res) *sz_res = " << m_out.size() << ";\n"
      << "    if (sz_iw) *sz_iw = 0;\n    if (sz_w) *sz_w = 0;\n    return 0;\n}\n";
    return f.str();
}

}  // namespace mpc
}  // namespace mahi
