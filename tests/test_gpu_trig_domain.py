"""GPU: an iterate whose joint angle lies beyond the domain of the device's reduced-range sin / cos (|q| > 2^20 pi/2 =
1.6e6 rad, mahi-mpc_amd/csrc/fast_trig.h) gets the same status as in the oracle, which applies that domain to its model
evaluations (oracle/mmpc_oracle.c kTrigDomain): non-finite, on every KKT solver and both built-in
models.  The other instances of the same batch (angles inside the domain) converge on both sides, to the oracle's V*
within 1e-10 relative.  The out-of-domain angle enters through the warm start V (init_states AS_GIVEN, the reference's
later ticks, ModelControl.cpp:160-161), at stage 5 for instances 0..3."""
import numpy as np
import pytest

from conftest import WEIGHTS_CFG

pytestmark = pytest.mark.gpu

WX = [10.0] * 4 + [1.0] * 4 + [1.0] * 4 + [0.01] * 4


@pytest.mark.parametrize("model,solver", [("two_link_arm", "condensed"), ("two_link_arm", "group"),
                                          ("two_link_arm", "lane"), ("exo_arm", "lane"), ("exo_arm", "group")])
def test_angle_beyond_trig_domain_same_status_as_oracle(model, solver, tmp_path, mmpc_mod, oracle):
    exo = model == "exo_arm"
    nx, nu, N = (8, 4, 20) if exo else (4, 2, 30)
    B = 8
    ks = {"condensed": mmpc_mod.KKT_CONDENSED, "group": mmpc_mod.KKT_RICCATI_GROUP, "lane": mmpc_mod.KKT_RICCATI}[solver]
    path = mmpc_mod.write_model_json(str(tmp_path / f"{model}.json"), model, nx, nu, 2000, N, model=model)
    s = mmpc_mod.Solver(path, kkt_solver=ks, init_states=mmpc_mod.INIT_AS_GIVEN)
    om = oracle.EXO if exo else oracle.TWO_LINK
    x0, up, tr = oracle.synth(20250213, 0, B, N, 0.002, model=om)
    w = np.array(WX if exo else WEIGHTS_CFG)
    nd = nx + nu
    V = np.zeros((B, s.NV))
    for k in range(N + 1):
        V[:, k * nd:k * nd + nx] = x0          # warm start: x_k = x_0
    V[:4, 5 * nd] = [2.0e6, -3.0e6, 1e12, 1647099.34]   # joint 0 at stage 5, each beyond 2^20 pi/2
    g = s.solve_batch_host(x0, up, tr, w, V=V)
    o = oracle.solve_batch(N, 0.002, x0, up, tr, w, V=V, model=om, init_states=mmpc_mod.INIT_AS_GIVEN, solver=s,
                           kkt=oracle.KKT_RICCATI if solver != "condensed" else oracle.KKT_DENSE)
    ST_NONFINITE = 3
    assert (g["status"][:4] == ST_NONFINITE).all(), g["status"]
    assert np.array_equal(g["status"], o["status"]), (g["status"], o["status"])
    assert (g["status"][4:] == 0).all()
    same = g["iters"][4:] == o["iters"][4:]
    assert same.all(), (g["iters"], o["iters"])
    rel = np.abs(g["V"][4:] - o["V"][4:]).max(1) / np.abs(o["V"][4:]).max(1)
    assert rel.max() <= 1e-10, rel
    s.close()
