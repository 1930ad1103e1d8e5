"""ASan + UBSan builds of the CPU-side code (sanitizer runs of the host code; GPU sanitizers are not
available on the pool): the oracle over every solve variant (oracle/sanitize_check.c), the SX engine's self-test and
the JSON / ModelParameters parsers under 20k byte-mutated inputs (mahi-mpc_amd/host/sanitize/json_fuzz.cpp).  Any
out-of-bounds access, leak or undefined behaviour aborts the binary (-fno-sanitize-recover=all)."""
import os
import subprocess

import pytest

from conftest import ROOT

ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


def _build(target_dir, target):
    r = subprocess.run(["make", "-s", "-C", target_dir, target], capture_output=True, text=True, timeout=600)
    if r.returncode != 0 and "sanitize" in r.stderr and "cannot find" in r.stderr:
        pytest.skip("sanitizer runtime not installed")
    assert r.returncode == 0, r.stderr[-2000:]


def test_oracle_under_asan_ubsan():
    _build(os.path.join(ROOT, "oracle"), "sanitize")
    r = subprocess.run([os.path.join(ROOT, "oracle", "sanitize_check")], capture_output=True, text=True, timeout=600,
                       env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "oracle sanitize ok" in r.stdout


@pytest.mark.parametrize("exe,ok", [("sx_selftest_san", "sx_selftest ok"), ("json_fuzz_san", "json_fuzz ok")])
def test_host_code_under_asan_ubsan(exe, ok):
    host = os.path.join(ROOT, "mahi-mpc_amd", "host")
    _build(host, os.path.join("bin", exe))
    r = subprocess.run([os.path.join(host, "bin", exe)], capture_output=True, text=True, timeout=600, env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert ok in r.stdout
