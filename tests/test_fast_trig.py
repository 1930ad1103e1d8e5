"""CPU: mahi-mpc_amd/csrc/fast_trig.h (the reduced-range fp64 sincos of the model evaluations: FMA Cody-Waite
reduction by pi/2 in three parts + the fdlibm kernels) compiled for the host, against libm (Python's math.sin /
math.cos).  The device models (ExoArm, TwoLinkFast) call this function; their parity with the oracle, which uses
libm, is in the GPU suite and in tests/test_sx_models.py."""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mahi-mpc_amd", "csrc")

SRC = r"""
#include <math.h>
#include "fast_trig.h"
extern "C" void fast_sincos_batch(const double* x, double* s, double* c, long n) {
    for (long i = 0; i < n; ++i) mmpc::sincos_fast(mmpc::trig_table(), x[i], s + i, c + i);
}
"""


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("fast_trig")
    src = d / "ft.cpp"
    src.write_text(SRC)
    so = d / "ft.so"
    # -ffp-contract=off: the host build rounds every product, the device build may contract; both stay within 1 ulp
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-ffp-contract=off", "-I", CSRC, str(src), "-o", str(so)],
                   check=True)
    return ctypes.CDLL(str(so))


def _run(lib, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    s, c = np.empty_like(x), np.empty_like(x)
    P = ctypes.POINTER(ctypes.c_double)
    lib.fast_sincos_batch(x.ctypes.data_as(P), s.ctypes.data_as(P), c.ctypes.data_as(P), ctypes.c_long(len(x)))
    return s, c


def _ulps(v, ref):
    return np.abs(v - ref) / np.spacing(np.maximum(np.abs(ref), np.finfo(float).tiny))


@pytest.mark.parametrize("half_range", [4.0, 50.0, 1e3, 1.6e6])
def test_within_one_ulp_of_libm(lib, half_range):
    x = np.random.default_rng(7).uniform(-half_range, half_range, 50000)
    s, c = _run(lib, x)
    rs = np.array([math.sin(v) for v in x])
    rc = np.array([math.cos(v) for v in x])
    assert _ulps(s, rs).max() <= 1.0 and _ulps(c, rc).max() <= 1.0
    assert np.abs(s - rs).max() <= 1.2e-16 and np.abs(c - rc).max() <= 1.2e-16


def test_multiples_of_half_pi(lib):
    """the zeros of sin / cos: the three-part reduction keeps the tiny results accurate relative to themselves"""
    x = np.arange(-100000, 100001) * (math.pi / 2)
    s, c = _run(lib, x)
    rs = np.array([math.sin(v) for v in x])
    rc = np.array([math.cos(v) for v in x])
    assert _ulps(s, rs).max() <= 1.0 and _ulps(c, rc).max() <= 1.0


def test_special_values(lib):
    s, c = _run(lib, np.array([np.nan, np.inf, -np.inf, 0.0, 1e-300, -1e-300]))
    assert np.isnan(s[:3]).all() and np.isnan(c[:3]).all()
    assert s[3] == 0.0 and c[3] == 1.0
    assert s[4] == 1e-300 and s[5] == -1e-300 and c[4] == 1.0
