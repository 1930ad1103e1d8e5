"""CPU: the exo polynomials the device evaluates (mahi-mpc_amd/csrc/exo_model_gen.h, generated in Horner form by
tools/gen_exo_model.py in round 4) against the oracle's independent restatement of M(q) (oracle_exo_mass: the
expanded polynomial under sympy CSE, pinned to the inverseTest.cpp:59-74 printout by tests/golden/exo_mass_kat.json).

The device expressions are read from the header and evaluated in Python (fma as a*b + c): M(q) must equal the
oracle's to roundoff, dM/dq_j its central differences, d^2M/dq_i dq_j its second central differences."""
import math
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "mahi-mpc_amd", "csrc", "exo_model_gen.h")
UPPER = [(0, 0), (0, 1), (0, 2), (0, 3), (1, 1), (1, 2), (1, 3), (2, 2), (2, 3), (3, 3)]


def _parse():
    text = open(HDR).read()
    K = [float(v) for v in re.search(r"kCoef\[\d+\] = \{(.*?)\};", text, re.S).group(1).split(",")]
    body = lambda fn: text[text.index(fn):text.index("\n}\n", text.index(fn))]
    M = dict((int(i), e) for i, e in re.findall(r"^\s+M\[(\d+)\] = (.*);$", body("void mass_upper"), re.M))
    dM, cur = {}, None
    for line in body("void dmass_upper").splitlines():
        m = re.match(r"\s+if \(J == (\d)\) \{", line)
        if m:
            cur = int(m.group(1))
        m = re.match(r"\s+dM\[(\d+)\] = (.*);$", line)
        if m:
            dM[(cur, int(m.group(1)))] = m.group(2)
    d2M, cur = {}, None
    for line in body("void d2mass_upper").splitlines():
        m = re.match(r"\s+if \(I == (\d) && J == (\d)\) \{", line)
        if m:
            cur = (int(m.group(1)), int(m.group(2)))
        m = re.match(r"\s+d2M\[(\d+)\] = (.*);$", line)
        if m:
            d2M[cur + (int(m.group(1)),)] = m.group(2)
    return K, M, dM, d2M


def _env(K, q):
    env = {"K": K, "fma": lambda a, b, c: a * b + c}
    for i in range(1, 4):
        c, s = math.cos(q[i]), math.sin(q[i])
        env.update({f"c{i}": c, f"s{i}": s, f"c{i}_2": c * c, f"s{i}_2": s * s})
    return env


def _sym(vals):
    A = np.zeros((4, 4))
    for (a, b), v in zip(UPPER, vals):
        A[a, b] = A[b, a] = v
    return A


@pytest.fixture(scope="module")
def polys():
    K, M, dM, d2M = _parse()
    assert sorted(M) == list(range(10)) and len(dM) == 30 and len(d2M) == 60
    return K, {k: compile(v, "M", "eval") for k, v in M.items()}, {k: compile(v, "dM", "eval") for k, v in dM.items()}, \
        {k: compile(v, "d2M", "eval") for k, v in d2M.items()}


def _qs(n=60):
    rng = np.random.default_rng(11)
    return [np.concatenate([[0.3], rng.uniform(-3.1, 3.1, 3)]) for _ in range(n)]


def test_mass_matrix_equals_oracle(polys, oracle):
    K, M, _, _ = polys
    for q in _qs():
        dev = _sym([eval(M[i], _env(K, q)) for i in range(10)])
        ref = oracle.exo_mass(q).reshape(4, 4)
        assert np.abs(dev - ref).max() <= 1e-15 * max(1.0, np.abs(ref).max()) * 8


def test_mass_derivatives_match_differences(polys, oracle):
    K, _, dM, d2M = polys
    h1, h2 = 1e-5, 1e-4
    Mo = lambda q: oracle.exo_mass(q).reshape(4, 4)
    for q in _qs(25):
        for j in range(1, 4):
            e = np.zeros(4)
            e[j] = 1.0
            fd = (Mo(q + h1 * e) - Mo(q - h1 * e)) / (2 * h1)
            dev = _sym([eval(dM[(j, i)], _env(K, q)) for i in range(10)])
            assert np.abs(dev - fd).max() <= 1e-8, (j, np.abs(dev - fd).max())
        for a in range(1, 4):
            for b in range(a, 4):
                ea, eb = np.eye(4)[a], np.eye(4)[b]
                fd2 = (Mo(q + h2 * (ea + eb)) - Mo(q + h2 * (ea - eb)) - Mo(q - h2 * (ea - eb)) + Mo(q - h2 * (ea + eb))) / (4 * h2 * h2)
                dev = _sym([eval(d2M[(a, b, i)], _env(K, q)) for i in range(10)])
                assert np.abs(dev - fd2).max() <= 2e-6, (a, b, np.abs(dev - fd2).max())
