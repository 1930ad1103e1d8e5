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


def _build(d, extra=()):
    src = d / "ft.cpp"
    src.write_text(SRC)
    so = d / "ft.so"
    # -ffp-contract=off: the host build rounds every product, the device build may contract; both stay within 1 ulp
    subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-ffp-contract=off", *extra, "-I", CSRC, str(src), "-o", str(so)],
                   check=True)
    return ctypes.CDLL(str(so))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    return _build(tmp_path_factory.mktemp("fast_trig"))


@pytest.fixture(scope="module")
def devpath(tmp_path_factory):
    """the device code path compiled for the host (no libm fallback), under UBSan that aborts on any report"""
    return _build(tmp_path_factory.mktemp("fast_trig_dev"),
                  ("-DMMPC_TRIG_DEVICE_PATH_ON_HOST", "-fsanitize=undefined", "-fno-sanitize-recover=all"))


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


def test_huge_arguments_device_path_well_defined(devpath):
    """a diverging iterate (|x| beyond 2^20 pi/2, up to 1e300): the device path returns NaN for both (the solver then
    reports the instance non-finite) and never performs an out-of-range int conversion (UBSan would abort)"""
    x = np.array([1647099.34, -2.0e6, 2.0 ** 31 * math.pi, -(2.0 ** 40) * 3.0, 1e15, -1e200, 1e300])
    s, c = _run(devpath, x)
    assert np.isnan(s).all() and np.isnan(c).all()
    # up to the limit the device path is the one the default build uses
    y = np.concatenate([np.random.default_rng(3).uniform(-1.6e6, 1.6e6, 2000), [1647099.32, -1647099.32]])
    sd, cd = _run(devpath, y)
    assert _ulps(sd, np.sin(y)).max() <= 1.0 and _ulps(cd, np.cos(y)).max() <= 1.0


def test_huge_arguments_host_build_uses_libm(lib):
    x = np.array([2.0e6, -3.3e9, 1e15, -1e200, 1e300])
    s, c = _run(lib, x)
    assert np.array_equal(s, np.array([math.sin(v) for v in x])) and np.array_equal(c, np.array([math.cos(v) for v in x]))


@pytest.fixture(scope="module")
def host_ubsan(tmp_path_factory):
    """the host build (libm beyond the reduced range) under UBSan with the float-to-int check, aborting on any report"""
    return _build(tmp_path_factory.mktemp("fast_trig_host_ubsan"),
                  ("-fsanitize=undefined,float-cast-overflow", "-fno-sanitize-recover=all"))


def test_nan_and_inf_take_the_libm_path_on_the_host(host_ubsan):
    """NaN compared false against the range limit and reached the quadrant's int conversion (undefined on the
    host); the guard is now !(|x| <= limit), so NaN and +-inf take the libm path (UBSan would abort otherwise)"""
    x = np.array([np.nan, -np.nan, np.inf, -np.inf, 0.5, 2.0e6])
    s, c = _run(host_ubsan, x)
    assert np.isnan(s[:4]).all() and np.isnan(c[:4]).all()
    assert s[4] == math.sin(0.5) or _ulps(s[4:5], np.array([math.sin(0.5)])).max() <= 1.0
    assert s[5] == math.sin(2.0e6) and c[5] == math.cos(2.0e6)
