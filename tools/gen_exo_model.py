#!/usr/bin/env python3
"""Generate the exo mass-matrix code and its known-answer fixture (run in the build container only).

The reference's only exo dynamics artefact is the symbolic 4x4 mass matrix M(q) printed by CasADi in
src/inverseTest.cpp:59-74.  This script

  1. parses the ten upper-triangle entries M00..M33 of that file (as math, with sympy),
  2. substitutes the build-defined inertial parameters of tests/golden/exo_params.json (exact rationals),
  3. rewrites each entry as a polynomial in c_i = cos q_i, s_i = sin q_i (i = 1..3; M does not depend on q0),
     where the printout's symbols q1..q3 are joints 1..3 of the 0-based state [q0..q3, qd0..qd3]
     (util/testCorrectEquations.py:16-23); q0 is the base joint,
  4. emits
       mahi-mpc_amd/csrc/exo_model_gen.h  device functions mass_upper / dmass_upper<J> (sums of monomials over
                                          a table of trig powers, derivatives symbolic)
       oracle/exo_model_gen.h             C function      exo_mass_and_grad(q, M[16], dM[4][16])
                                          with the partial derivatives taken symbolically (independent of
                                          the device's forward-mode duals)
       tests/golden/exo_mass_kat.json     M(q) at fixed q evaluated from the *unexpanded* parsed expressions
                                          with 40-digit mpmath -- the pin for both generated forms.

/root/reference exists only in this container; the generated files are committed and nothing reads the
reference at build or run time.  Re-run after changing exo_params.json:
    python tools/gen_exo_model.py
"""
from __future__ import annotations

import json
import os
import re
import sys

import mpmath
import sympy as sp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src/inverseTest.cpp"
UPPER = ["M00", "M01", "M02", "M03", "M11", "M12", "M13", "M22", "M23", "M33"]
IDX = [(0, 0), (0, 1), (0, 2), (0, 3), (1, 1), (1, 2), (1, 3), (2, 2), (2, 3), (3, 3)]


def load_entries():
    text = open(REF).read()
    ents = dict(re.findall(r"casadi::SX (M\d\d) = (.*?);", text))
    q = sp.symbols("q1 q2 q3 q4")
    params = {}
    for base in ["Icxx", "Icyy", "Iczz", "Icxy", "Icxz", "Icyz", "Pcx", "Pcy", "Pcz", "m"]:
        for i in range(4):
            params[f"{base}{i}"] = sp.Symbol(f"{base}{i}")
    loc = dict(params)
    loc.update({"q1": q[0], "q2": q[1], "q3": q[2], "q4": q[3], "cos": sp.cos, "sin": sp.sin,
                "pow": lambda a, b: a ** b, "Rational": sp.Rational})
    out = {}
    for k in UPPER:
        e = re.sub(r"(\d+\.\d+(?:E[+-]\d+)?)", r"Rational('\1')", ents[k])
        out[k] = sp.sympify(e, locals=loc)
    # symmetry of the printout
    for a in range(4):
        for b in range(a):
            e = re.sub(r"(\d+\.\d+(?:E[+-]\d+)?)", r"Rational('\1')", ents[f"M{a}{b}"])
            lower = sp.sympify(e, locals=loc)
            assert sp.simplify(lower - out[f"M{b}{a}"]) == 0, f"M{a}{b} != M{b}{a}"
    return out, q, params


def param_subs(params, pj):
    subs = {}
    for base in ["Icxx", "Icyy", "Iczz", "Icxy", "Icxz", "Icyz", "Pcx", "Pcy", "Pcz", "m"]:
        for i in range(4):
            subs[params[f"{base}{i}"]] = sp.Rational(pj[base][i])
    return subs


class TPrinter:
    """Prints a sympy polynomial expression over a generic scalar type (only +, -, *, double literals)."""

    def __init__(self, num_fmt):
        self.num_fmt = num_fmt

    def p(self, e):
        if e.is_Symbol:
            return str(e)
        if e.is_Number:
            return self.num_fmt(float(e))
        if e.is_Add:
            terms = [self.p(a) for a in e.args]
            s = terms[0]
            for t in terms[1:]:
                s = f"{s} - {t[1:]}" if t.startswith("-") else f"{s} + {t}"
            return f"({s})"
        if e.is_Mul:
            coef, rest = e.as_coeff_Mul()
            factors = []
            for f in sp.Mul.make_args(rest):
                if f.is_Pow:
                    base, ex = f.args
                    assert ex.is_Integer and ex > 0, f
                    factors += [self.p(base)] * int(ex)
                else:
                    factors.append(self.p(f))
            body = " * ".join(factors)
            if coef == 1:
                return body
            if coef == -1:
                return f"-({body})" if len(factors) > 1 else f"-{body}"
            return f"{self.num_fmt(float(coef))} * {body}"
        if e.is_Pow:
            base, ex = e.args
            assert ex.is_Integer and ex > 0, e
            return "(" + " * ".join([self.p(base)] * int(ex)) + ")"
        raise ValueError(f"unsupported node {e!r}")


def lit(x):
    r = repr(float(x))
    return r if ("e" in r or "." in r or "inf" in r) else r + ".0"


def main():
    pj = json.load(open(os.path.join(REPO, "tests", "golden", "exo_params.json")))
    ents, q, params = load_entries()
    subs = param_subs(params, pj)
    c = sp.symbols("c1 c2 c3")
    s = sp.symbols("s1 s2 s3")
    trig = {}
    for i in range(3):
        trig[sp.cos(q[i])] = c[i]
        trig[sp.sin(q[i])] = s[i]
    polys = []
    for k in UPPER:
        e = sp.expand_trig(ents[k].subs(subs))
        e = sp.expand(e.subs(trig))
        assert not e.has(sp.sin) and not e.has(sp.cos), k
        polys.append(e)
    nterms = sum(len(sp.Add.make_args(p)) for p in polys)

    # ---- device code: M and dM/dq_j as sums of monomials over a table of trig powers ----
    # (no cross-entry CSE: every output is an independent fma chain, so few values are live at once)
    gens = list(c) + list(s)
    names = ["c1", "c2", "c3", "s1", "s2", "s3"]
    dpolys = []
    for j in range(3):
        dpolys.append([sp.expand(-s[j] * sp.diff(pe, c[j]) + c[j] * sp.diff(pe, s[j])) for pe in polys])
    used = set()

    coefs = []
    cindex = {}

    def cref(v):
        # every non-trivial coefficient lives in one __constant__ table: f64 literals cannot be encoded in
        # VALU instructions, and as immediates the compiler hoists all of them out of the solver loops
        # and spills them; table entries are scalar-loaded at their point of use
        if v not in cindex:
            cindex[v] = len(coefs)
            coefs.append(v)
        return f"K[{cindex[v]}]"

    # Horner form (round 4): the expanded monomial sums cost one product chain per monomial; nested in the variable
    # order that prints the fewest operations (sympy horner over a set of orders) the same polynomials take ~30 %
    # fewer FP64 operations.  Every nesting level is one fma(variable, inner, rest) with the coefficients from the
    # constant table.
    import itertools
    from sympy.polys.polyfuncs import horner

    def hp(e):
        """(code, op count) of a Horner-form expression: Add -> fma chain, Mul -> products, constants from the table"""
        if e.is_Number:
            return cref(float(e)), 0
        if e.is_Symbol:
            return str(e), 0
        if e.is_Pow:
            base, ex = e.args
            assert base.is_Symbol and ex.is_Integer and 2 <= ex, e
            v = str(base)
            used.add((v, 2))
            fs = [f"{v}_2"] * (int(ex) // 2) + [v] * (int(ex) % 2)
            return (fs[0] if len(fs) == 1 else "(" + " * ".join(fs) + ")"), len(fs) - 1
        if e.is_Mul:
            coef, rest = e.as_coeff_Mul()
            fs = [hp(f) for f in sp.Mul.make_args(rest)]
            codes = [c if not c.startswith("fma") and " + " not in c else f"({c})" for c, _ in fs]
            if coef != 1:
                codes.insert(0, cref(float(coef)))
            return " * ".join(codes), sum(c for _, c in fs) + len(codes) - 1
        if e.is_Add:
            const = sum((t for t in e.args if t.is_Number), sp.Integer(0))
            acc, cost = (cref(float(const)), 0) if const != 0 else (None, 0)
            for t in sorted((t for t in e.args if not t.is_Number), key=lambda t: 0 if t.is_Mul else 1):
                coef, r = t.as_coeff_Mul()
                fs = list(sp.Mul.make_args(r))
                if coef == 1 and len(fs) == 1:          # a plain term: add it
                    c, cc = hp(fs[0])
                    acc, cost = (c, cost + cc) if acc is None else (f"{acc} + {c}", cost + cc + 1)
                    continue
                if coef != 1:                            # K * (rest)
                    a_code, a_cost = cref(float(coef)), 0
                    b_code, b_cost = hp(sp.Mul(*fs))
                else:                                    # first factor * (rest)
                    a_code, a_cost = hp(fs[0])
                    b_code, b_cost = hp(sp.Mul(*fs[1:]))
                if b_code.startswith("fma") or " + " in b_code:
                    b_code = b_code if b_code.startswith("fma") else f"({b_code})"
                if acc is None:
                    acc, cost = f"{a_code} * {b_code}", cost + a_cost + b_cost + 1
                else:
                    acc, cost = f"fma({a_code}, {b_code}, {acc})", cost + a_cost + b_cost + 2
            return acc, cost
        raise ValueError(f"unsupported node {e!r}")

    # variable orders tried: the joints in any order, each joint's c before or after its s (48), and all c before
    # all s / all s before all c in any joint order (12)
    orders = []
    for perm in itertools.permutations(range(3)):
        for flips in itertools.product([0, 1], repeat=3):
            o = []
            for i, f in zip(perm, flips):
                o += [c[i], s[i]] if f == 0 else [s[i], c[i]]
            orders.append(tuple(o))
        orders.append(tuple([c[i] for i in perm] + [s[i] for i in perm]))
        orders.append(tuple([s[i] for i in perm] + [c[i] for i in perm]))

    def emit_horner(pe):
        best = None
        saved = (list(coefs), dict(cindex), set(used))
        for order in orders:
            coefs[:] = saved[0]
            cindex.clear()
            cindex.update(saved[1])
            used.clear()
            used.update(saved[2])
            code, cost = hp(horner(pe, *order))
            if best is None or cost < best[1]:
                best = (code, cost, list(coefs), dict(cindex), set(used))
        coefs[:] = best[2]
        cindex.clear()
        cindex.update(best[3])
        used.clear()
        used.update(best[4])
        return best[0], best[1]

    mlines, nmono = [], 0
    hcost = [0, 0]
    for i, pe in enumerate(polys):
        e, hc = emit_horner(pe)
        hcost[0] += hc
        n = len(sp.Poly(pe, *gens).terms())
        nmono += n
        mlines.append(f"    M[{i}] = {e};")
    dlines, ndmono = [], 0
    for j in range(3):
        dlines.append(f"    if (J == {j + 1}) {{")
        for i, pe in enumerate(dpolys[j]):
            e, hc = emit_horner(pe)
            hcost[1] += hc
            n = len(sp.Poly(pe, *gens).terms())
            ndmono += n
            dlines.append(f"        dM[{i}] = {e};")
        dlines.append("    }")
    # second derivatives d^2 M / dq_I dq_J (1 <= I <= J <= 3) for the exact Lagrangian Hessian of the exo
    # (round 4: mmpc_opts.hessian = EXACT on the exo model)
    pairs = [(a, b) for a in range(3) for b in range(a, 3)]
    d2polys = {}
    for a, b in pairs:
        d2polys[(a, b)] = [sp.expand(-s[a] * sp.diff(pe, c[a]) + c[a] * sp.diff(pe, s[a])) for pe in dpolys[b]]
    d2lines, nd2mono = [], 0
    for a, b in pairs:
        d2lines.append(f"    if (I == {a + 1} && J == {b + 1}) {{")
        for i, pe in enumerate(d2polys[(a, b)]):
            e, _ = emit_horner(pe)
            n = len(sp.Poly(pe, *gens).terms()) if pe != 0 else 0
            nd2mono += n
            d2lines.append(f"        d2M[{i}] = {e};")
        d2lines.append("    }")
    pw = []
    for v, e in sorted(used):
        pw.append(f"        {v}_{e} = " + " * ".join([v] * e) + ";")
    pw_decl = ", ".join(f"{v}_{e}" for v, e in sorted(used))
    unpack = ", ".join(f"{v}_{e} = t.{v}_{e}" for v, e in sorted(used))
    dev = f"""// exo_model_gen.h -- GENERATED by tools/gen_exo_model.py; do not edit.
//
// Mass matrix M(q) of the 4-DoF exo, restated from the CasADi printout of src/inverseTest.cpp:59-74
// with the build-defined inertial parameters of tests/golden/exo_params.json substituted (NOT
// reference-pinned values; the reference ships none), as polynomials in c_i = cos q_i, s_i = sin q_i
// (i = 1..3; M does not depend on q0): {nmono} monomials for M, {ndmono} for dM/dq_1..3 (symbolic
// derivatives).  Outputs are the upper triangle M00 M01 M02 M03 M11 M12 M13 M22 M23 M33.
#pragma once

namespace mmpc {{
namespace exo {{

constexpr double kGravityGain[4] = {{{", ".join(lit(sp.Rational(v)) for v in pj["gravity_gain"])}}};
constexpr double kDamping[4] = {{{", ".join(lit(sp.Rational(v)) for v in pj["damping"])}}};

// the {len(coefs)} distinct polynomial coefficients
__constant__ double kCoef[{len(coefs)}] = {{{", ".join(lit(v) for v in coefs)}}};

// table pointer made opaque per call: the loads stay at their uses (no loop-invariant hoisting).  Typed constant
// (address space 4), so the loads are scalar s_load: an opaque generic pointer becomes flat_load, and every use of
// a flat load waits for all outstanding vector-memory and LDS operations of the wave.
using cdouble = __attribute__((address_space(4))) const double;
__device__ __forceinline__ cdouble* coef_table() {{
    cdouble* K = (cdouble*)kCoef;
    asm volatile("" : "+s"(K));
    return K;
}}

struct TrigPowers {{
    double c1, c2, c3, s1, s2, s3;
    double {pw_decl};
    __device__ __forceinline__ TrigPowers(double c1_, double c2_, double c3_, double s1_, double s2_, double s3_)
        : c1(c1_), c2(c2_), c3(c3_), s1(s1_), s2(s2_), s3(s3_) {{
{chr(10).join(pw)}
    }}
}};

__device__ __forceinline__ void mass_upper(const TrigPowers& t, double* M) {{
    cdouble* const K = coef_table();
    [[maybe_unused]] const double c1 = t.c1, c2 = t.c2, c3 = t.c3, s1 = t.s1, s2 = t.s2, s3 = t.s3;
    [[maybe_unused]] const double {unpack};
{chr(10).join(mlines)}
}}

// dM/dq_J (J = 1..3), upper triangle
template <int J>
__device__ __forceinline__ void dmass_upper(const TrigPowers& t, double* dM) {{
    cdouble* const K = coef_table();
    [[maybe_unused]] const double c1 = t.c1, c2 = t.c2, c3 = t.c3, s1 = t.s1, s2 = t.s2, s3 = t.s3;
    [[maybe_unused]] const double {unpack};
{chr(10).join(dlines)}
}}

// d^2 M / dq_I dq_J (1 <= I <= J <= 3), upper triangle ({nd2mono} monomials; the exact exo Hessian)
template <int I, int J>
__device__ __forceinline__ void d2mass_upper(const TrigPowers& t, double* d2M) {{
    static_assert(1 <= I && I <= J && J <= 3, "I <= J in 1..3");
    cdouble* const K = coef_table();
    [[maybe_unused]] const double c1 = t.c1, c2 = t.c2, c3 = t.c3, s1 = t.s1, s2 = t.s2, s3 = t.s3;
    [[maybe_unused]] const double {unpack};
{chr(10).join(d2lines)}
}}

}}  // namespace exo
}}  // namespace mmpc
"""
    open(os.path.join(REPO, "mahi-mpc_amd", "csrc", "exo_model_gen.h"), "w").write(dev)
    repl = []
    P = TPrinter(lit)

    # ---- oracle: M and dM/dq_j by symbolic differentiation ----
    exprs = []
    for pexpr in polys:
        exprs.append(pexpr)
    for j in range(3):
        for pexpr in polys:
            d = -s[j] * sp.diff(pexpr, c[j]) + c[j] * sp.diff(pexpr, s[j])
            exprs.append(sp.expand(d))
    for a, b in pairs:
        exprs.extend(d2polys[(a, b)])
    repl2, red2 = sp.cse(exprs, symbols=sp.numbered_symbols("t"), optimizations="basic")
    ol = []
    for sym, ex in repl2:
        ol.append(f"    const double {sym} = {P.p(ex)};")
    for i, ex in enumerate(red2):
        ol.append(f"    up[{i}] = {P.p(ex)};")
    orc = f"""/* exo_model_gen.h -- GENERATED by tools/gen_exo_model.py; do not edit.
 *
 * TEST INFRASTRUCTURE (oracle).  M(q) of src/inverseTest.cpp:59-74 with the build-defined parameters of
 * tests/golden/exo_params.json, and its partial derivatives dM/dq_j taken symbolically (sympy), i.e.
 * independently of the device's forward-mode dual numbers.
 */
#ifndef MMPC_EXO_MODEL_GEN_H
#define MMPC_EXO_MODEL_GEN_H
#include <math.h>

static const double EXO_GRAVITY_GAIN[4] = {{{", ".join(lit(sp.Rational(v)) for v in pj["gravity_gain"])}}};
static const double EXO_DAMPING[4] = {{{", ".join(lit(sp.Rational(v)) for v in pj["damping"])}}};

/* M[16] row-major, dM[j][16] = dM/dq_j (dM[0] = 0: M does not depend on q0); d2M (may be NULL) [4][4][16] =
 * d^2 M / dq_i dq_j (zero where i or j is 0) */
static void exo_mass_derivs(const double* q, double* M, double dM[4][16], double d2M[4][4][16]) {{
    const double c1 = cos(q[1]), s1 = sin(q[1]), c2 = cos(q[2]), s2 = sin(q[2]), c3 = cos(q[3]), s3 = sin(q[3]);
    double up[{10 + 30 + 60}];
{chr(10).join(ol)}
    static const int ia[10] = {{0, 0, 0, 0, 1, 1, 1, 2, 2, 3}}, ib[10] = {{0, 1, 2, 3, 1, 2, 3, 2, 3, 3}};
    static const int pa[6] = {{1, 1, 1, 2, 2, 3}}, pb[6] = {{1, 2, 3, 2, 3, 3}};
    for (int j = 0; j < 16; ++j) dM[0][j] = 0.0;
    if (d2M)
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b)
                for (int j = 0; j < 16; ++j) d2M[a][b][j] = 0.0;
    for (int t = 0; t < 10; ++t) {{
        M[ia[t] * 4 + ib[t]] = M[ib[t] * 4 + ia[t]] = up[t];
        for (int j = 0; j < 3; ++j) dM[j + 1][ia[t] * 4 + ib[t]] = dM[j + 1][ib[t] * 4 + ia[t]] = up[10 + 10 * j + t];
        if (d2M)
            for (int p = 0; p < 6; ++p) {{
                const double v = up[40 + 10 * p + t];
                d2M[pa[p]][pb[p]][ia[t] * 4 + ib[t]] = d2M[pa[p]][pb[p]][ib[t] * 4 + ia[t]] = v;
                d2M[pb[p]][pa[p]][ia[t] * 4 + ib[t]] = d2M[pb[p]][pa[p]][ib[t] * 4 + ia[t]] = v;
            }}
    }}
}}
static void exo_mass_and_grad(const double* q, double* M, double dM[4][16]) {{ exo_mass_derivs(q, M, dM, NULL); }}
#endif
"""
    open(os.path.join(REPO, "oracle", "exo_model_gen.h"), "w").write(orc)

    # ---- known-answer fixture from the unexpanded expressions (40 digits) ----
    mpmath.mp.dps = 40
    pts = [[0.0, 0.0, 0.0, 0.0], [0.1, 0.3, -0.2, 0.4], [-0.5, 0.5, 0.5, -0.5], [1.0, -1.2, 0.7, 2.0],
           [0.0, 3.0, -2.5, 1.5], [0.2, 1.5707963267948966, 0.0, -1.5707963267948966]]
    import random
    rng = random.Random(20250213)
    for _ in range(6):
        pts.append([rng.uniform(-3.14, 3.14) for _ in range(4)])
    kat = []
    for qq in pts:
        # printout symbol q_k (k = 1..3) is joint k of the 0-based state [q0..q3] (q0 = base joint, on which
        # M of a serial chain cannot depend; q4 is declared but unused at inverseTest.cpp:11)
        vals = {q[i]: sp.Float(repr(qq[i + 1]), 40) for i in range(3)}
        M = [[0.0] * 4 for _ in range(4)]
        for (a, b), k in zip(IDX, UPPER):
            v = sp.N(ents[k].subs(subs).subs(vals), 40)
            M[a][b] = M[b][a] = float(v)
        kat.append({"q": qq, "M": M})
    # positive definiteness over a grid (the parameters must be physically consistent)
    import numpy as np
    f = sp.lambdify((c, s), polys, "numpy")
    worst = np.inf
    for _ in range(2000):
        qq = np.array([rng.uniform(-np.pi, np.pi) for _ in range(3)])
        up = f(np.cos(qq), np.sin(qq))
        Mn = np.zeros((4, 4))
        for (a, b), v in zip(IDX, up):
            Mn[a, b] = Mn[b, a] = v
        worst = min(worst, np.linalg.eigvalsh(Mn)[0])
    assert worst > 0, f"M(q) not positive definite (min eig {worst})"
    json.dump({"source": "src/inverseTest.cpp:59-74 (CasADi printout of M(q)), parameters tests/golden/exo_params.json",
               "method": "sympy parse of the printed expressions, evaluated with 40-digit mpmath, no expansion",
               "min_eigenvalue_over_2000_random_q": worst, "monomials": nterms, "cases": kat},
              open(os.path.join(REPO, "tests", "golden", "exo_mass_kat.json"), "w"), indent=1)
    print(f"monomials {nterms} (M) / {ndmono} (dM) / {nd2mono} (d2M), oracle cse temps {len(repl2)}, min eig {worst:.3e}")
    print(f"device Horner operation counts: M {hcost[0]}, dM {hcost[1]}")


if __name__ == "__main__":
    if not os.path.exists(REF):
        sys.exit(f"{REF} not found: the generator runs only in the build container")
    main()
