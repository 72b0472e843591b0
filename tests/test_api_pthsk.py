"""pt_hs_k through the shyft.api surface (api/boostpython/pt_hs_k.cpp; shyft/api/pt_hs_k).

CPU: parameter / state names, defaults and the get/set contract (pt_hs_k.h:64-143).
GPU: the region scenario of test_region_model_stacks.py (build_model, dummy environment, states, run_cells)
with a PTHSKModel; the API model's discharge equals the C-ABI region run on the interpolated forcing, and
a frozen variant builds snow that the hbv_snow statistics report.
"""
import numpy as np
import pytest


def test_parameter_contract():
    from shyft_amd.api import pt_hs_k
    p = pt_hs_k.PTHSKParameter()
    assert p.size() == 18
    assert p.get_name(4) == "hs.lw" and p.get_name(17) == "msp.reservoir_direct_response_fraction"
    assert p.get(0) == pytest.approx(-2.439) and p.get(12) == pytest.approx(1.26)
    v = [float(p.get(i)) for i in range(p.size())]
    v[5] = 0.7
    p.set(v)
    assert p.hs.tx == pytest.approx(0.7)
    with pytest.raises(RuntimeError, match="set size missmatch"):
        p.set(v[:-1])
    assert len(p.to_vector()) == 18 + 17  # + the hbv_snow distribution row
    s = pt_hs_k.PTHSKState()
    assert s.kirchner.q == pytest.approx(0.1) and s.snow.swe == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("frozen", [False, True])
def test_pthsk_model_run_matches_capi(frozen):
    from shyft_amd import api
    from shyft_amd.api import pt_hs_k
    from shyft_amd.region import HipRegion, PT_HS_K, COLLECT_DISCHARGE
    from tests.test_api_region_model import build_model, dummy_env, interpolation_parameter, constant_source
    n = 20
    model = build_model(pt_hs_k.PTHSKModel, pt_hs_k.PTHSKParameter, n)
    assert model.size() == n
    cal = api.Calendar()
    ta = api.TimeAxisFixedDeltaT(cal.time(2015, 1, 1, 0, 0, 0), api.deltahours(1), 240)
    model.initialize_cell_environment(ta)
    env = dummy_env(ta, model.get_cells()[n // 2].geo.mid_point())
    if frozen:
        env.temperature = api.TemperatureSourceVector()
        env.temperature.append(constant_source(api.TemperatureSource, model.get_cells()[n // 2].geo.mid_point(),
                                               api.UtcPeriod(*ta.total_period()), -5.0))
    model.interpolate(interpolation_parameter(), env)
    s0 = pt_hs_k.PTHSKStateVector()
    for _ in range(n):
        si = pt_hs_k.PTHSKState()
        si.kirchner.q = 40.0
        s0.append(si)
    model.set_states(s0)
    model.set_state_collection(-1, True)
    model.run_cells()
    cids = api.IntVector()
    q = model.statistics.discharge(cids).values.to_numpy()
    assert np.all(np.isfinite(q)) and q[0] > 0
    swe = model.hbv_snow_state.swe(cids).values.to_numpy()
    assert swe.size == ta.size() + 1
    if frozen:
        assert swe[-1] > 100.0  # 5 mm/h of snow for 10 days, on the snow storage fraction
    else:
        assert swe.max() == 0.0
    assert model.kirchner_state.discharge_value(cids, 3) > 0.0
    # the same region through the C ABI directly
    r = HipRegion(PT_HS_K, n)
    geo = np.zeros((n, 11))
    for i in range(n):
        geo[i] = [500 + 1000.0 * i, 500.0, 500.0 * i / n, 1e6, 1, 0.9, 0.01, 0.05, 0.19, 0.30, 0.45]
    r.set_geo(geo)
    r.set_parameters(np.array(pt_hs_k.PTHSKParameter().to_vector()))
    r.set_time_axis(ta.start * 10**6, 3600 * 10**6, 240)
    r.set_collection(COLLECT_DISCHARGE)
    st = np.tile(np.array(pt_hs_k.PTHSKState().to_vector()), (n, 1))
    st[:, -1] = 40.0
    r.set_state(st)
    for v in range(5):
        r.set_forcing(v, 0, np.stack([model.cells[i].env_ts.__getattr__(api.FORCING[v]).to_numpy()
                                      for i in range(n)], axis=1))
    r.run_cells()
    assert np.allclose(r.get_series(0, 0, 240).sum(axis=1), q, rtol=1e-13, atol=0)
    r.close()
