"""CPU: the C++ mirror of the reference API (mahi-mpc_amd/host) builds with g++ and its host-only behaviour
holds: ModelParameters defaults and JSON round trip, ModelGenerator's <name>.json, ModelControl's API errors
(mahi-mpc_amd/host/examples/host_selftest.cpp; no GPU call is made)."""
import os
import subprocess

from conftest import ROOT

HOST = os.path.join(ROOT, "mahi-mpc_amd", "host")


def test_host_mirror_selftest(tmp_path):
    subprocess.run(["make", "-s", "-C", HOST], check=True)
    out = subprocess.run([os.path.join(HOST, "bin", "host_selftest")], cwd=tmp_path, capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "host selftest ok" in out.stdout
    assert (tmp_path / "selftest_double_pendulum.json").exists()


def test_host_headers_mirror_reference_api():
    """every public member of the reference ModelControl/ModelGenerator/ModelParameters headers exists here"""
    mc = open(os.path.join(HOST, "include", "Mahi", "Mpc", "ModelControl.hpp")).read()
    for name in ["calc_u(", "load_model(", "control_at_time(", "start_calc(", "stop_calc(", "set_state(",
                 "update_weights(", "update_control_limits(", "model_parameters;", "control_results;",
                 "struct ControlResult"]:
        assert name in mc, name
    mg = open(os.path.join(HOST, "include", "Mahi", "Mpc", "ModelGenerator.hpp")).read()
    for name in ["create_model(", "generate_c_code(", "compile_model(", "save_param_file("]:
        assert name in mg, name
    mp = open(os.path.join(HOST, "include", "Mahi", "Mpc", "ModelParameters.hpp")).read()
    for name in ["name;", "timespan;", "step_size;", "num_x", "num_u", "num_shooting_nodes", "x_min;", "u_min;",
                 "x_max;", "u_max;", "dll_filepath;", "is_linear"]:
        assert name in mp, name
