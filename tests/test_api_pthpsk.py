"""pt_hps_k through the shyft.api surface (api/boostpython/pt_hps_k.cpp; shyft/api/pt_hps_k).

CPU: parameter / state names, defaults and the get/set contract (pt_hps_k.h:62-159).
GPU: the region scenario of test_region_model_stacks.py (build_model, dummy environment, states, run_cells)
with a PTHPSKModel; the API model's discharge equals the C-ABI region run on the interpolated forcing, a frozen
variant builds snow that the hbv_physical_snow statistics report, and the cell-identified state round-trips.
"""
import numpy as np
import pytest


def test_parameter_contract():
    from shyft_amd.api import pt_hps_k
    p = pt_hps_k.PTHPSKParameter()
    assert p.size() == 24
    assert p.get_name(4) == "hps.lw" and p.get_name(23) == "msp.reservoir_direct_response_fraction"
    assert p.hps.max_albedo == pytest.approx(0.9) and p.gm.direct_response == 0.0
    v = [float(p.get(i)) for i in range(p.size())]
    v[5] = 0.7
    p.set(v)
    assert p.hps.tx == pytest.approx(0.7)
    with pytest.raises(RuntimeError, match="set size missmatch"):
        p.set(v[:-1])
    p.gm.direct_response = 0.3
    assert len(p.to_vector()) == 24 + 1 + 17 and p.to_vector()[24] == 0.3
    s = pt_hps_k.PTHPSKState()
    assert s.kirchner.q == pytest.approx(0.1) and s.hps.surface_heat == 30000.0


@pytest.mark.gpu
@pytest.mark.parametrize("frozen", [False, True])
def test_pthpsk_model_run_matches_capi(frozen):
    from shyft_amd import api
    from shyft_amd.api import pt_hps_k
    from shyft_amd.region import HipRegion, PT_HPS_K, COLLECT_DISCHARGE
    from tests.test_api_region_model import build_model, dummy_env, interpolation_parameter, constant_source
    n = 20
    model = build_model(pt_hps_k.PTHPSKModel, pt_hps_k.PTHPSKParameter, n)
    cal = api.Calendar()
    ta = api.TimeAxisFixedDeltaT(cal.time(2015, 1, 1, 0, 0, 0), api.deltahours(1), 240)
    model.initialize_cell_environment(ta)
    env = dummy_env(ta, model.get_cells()[n // 2].geo.mid_point())
    if frozen:
        env.temperature = api.TemperatureSourceVector()
        env.temperature.append(constant_source(api.TemperatureSource, model.get_cells()[n // 2].geo.mid_point(),
                                               api.UtcPeriod(*ta.total_period()), -5.0))
    model.interpolate(interpolation_parameter(), env)
    s0 = pt_hps_k.PTHPSKStateVector()
    for _ in range(n):
        si = pt_hps_k.PTHPSKState()
        si.kirchner.q = 40.0
        s0.append(si)
    model.set_states(s0)
    model.set_state_collection(-1, True)
    model.run_cells()
    cids = api.IntVector()
    q = model.statistics.discharge(cids).values.to_numpy()
    assert np.all(np.isfinite(q)) and q[0] > 0
    swe = model.hbv_physical_snow_state.swe(cids).values.to_numpy()
    assert swe.size == ta.size() + 1
    if frozen:
        assert swe[-1] > 100.0
    else:
        assert swe.max() == 0.0
    states = model.state.extract_state(cids)
    assert len(model.state.apply_state(pt_hps_k.deserialize_from_bytes(states.serialize_to_bytes()), cids)) == 0
    r = HipRegion(PT_HPS_K, n)
    geo = np.zeros((n, 11))
    for i in range(n):
        geo[i] = [500 + 1000.0 * i, 500.0, 500.0 * i / n, 1e6, 1, 0.9, 0.01, 0.05, 0.19, 0.30, 0.45]
    r.set_geo(geo)
    r.set_parameters(np.array(pt_hps_k.PTHPSKParameter().to_vector()))
    r.set_time_axis(ta.start * 10**6, 3600 * 10**6, 240)
    r.set_collection(COLLECT_DISCHARGE)
    st = np.tile(np.array(pt_hps_k.PTHPSKState().to_vector()), (n, 1))
    st[:, -1] = 40.0
    r.set_state(st)
    for v in range(5):
        r.set_forcing(v, 0, np.stack([model.cells[i].env_ts.__getattr__(api.FORCING[v]).to_numpy()
                                      for i in range(n)], axis=1))
    r.run_cells()
    assert np.allclose(r.get_series(0, 0, 240).sum(axis=1), q, rtol=1e-13, atol=0)
    r.close()
