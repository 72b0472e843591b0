"""The reference's Python region-model scenario run through shyft_amd.api on the GPU.

Follows shyft/tests/api/test_region_model_stacks.py:14-30 (build_model), :46-55
(create_dummy_region_environment), :91-112 (area statistics), :114-310
(test_model_initialize_and_run: interpolation, is_cell_env_ts_ok, set_states,
state collection, run_cells, the statistics KATs -110.6998 / -16.7138 / 107.3981 /
0.189214067680088 / 0.9995599424191931, opt-model clone, stepwise 10 x 24 runs,
illegal cids, rasters, river network out(8) = 28.06, adjust_q) and :424-479 (hbv).
The KAT values are the reference's own; everything here goes through the C++ host
class and the C ABI (no oracle involved).
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def build_model(model_t, parameter_t, n, num_catchments=1):
    from shyft_amd import api
    gcds = api.GeoCellDataVector()
    for i in range(n):
        gp = api.GeoPoint(500 + 1000.0 * i, 500.0, 500.0 * i / n)
        ltf = api.LandTypeFractions(0.01, 0.05, 0.19, 0.3, 0.45)
        g = api.GeoCellData(gp, 1000 * 1000, 1 if num_catchments == 1 else 1 + i % num_catchments, 0.9, ltf)
        g.land_type_fractions_info().set_fractions(glacier=0.01, lake=0.05, reservoir=0.19, forest=0.3)
        gcds.append(g)
    return model_t(gcds, parameter_t())


def constant_source(src_t, gp, period, value):
    from shyft_amd import api
    tv = api.UtcTimeVector([period.start])
    vv = api.DoubleVector([value])
    return src_t(gp, api.TsFactory().create_time_point_ts(period, tv, vv, api.POINT_AVERAGE_VALUE))


def dummy_env(ta, gp):
    from shyft_amd import api
    p = api.UtcPeriod(*ta.total_period())
    re = api.ARegionEnvironment()
    re.precipitation.append(constant_source(api.PrecipitationSource, gp, p, 5.0))
    re.temperature.append(constant_source(api.TemperatureSource, gp, p, 10.0))
    re.wind_speed.append(constant_source(api.WindSpeedSource, gp, p, 2.0))
    re.rel_hum.append(constant_source(api.RelHumSource, gp, p, 0.7))
    re.radiation = api.RadiationSourceVector()
    re.radiation.append(constant_source(api.RadiationSource, gp, p, 300.0))
    return re


def interpolation_parameter():
    from shyft_amd import api
    ip = api.InterpolationParameter()
    ip.temperature_idw.default_temp_gradient = -0.005
    ip.temperature_idw.gradient_by_equation = True
    ip.temperature_idw.max_members = 6
    ip.temperature_idw.max_distance = 20000
    assert ip.temperature_idw.zscale == pytest.approx(1.0)
    ip.temperature_idw.zscale = 0.5
    ip.temperature_idw.distance_measure_factor = 1.0
    ip.use_idw_for_temperature = True
    assert ip.precipitation.scale_factor == pytest.approx(1.02)
    return ip


def test_model_area_functions():
    from shyft_amd import api
    from shyft_amd.api import pt_gs_k
    m = build_model(pt_gs_k.PTGSKModel, pt_gs_k.PTGSKParameter, 20)
    cids = api.IntVector()
    st = m.statistics
    total = st.total_area(cids)
    assert st.snow_storage_area(cids) == pytest.approx(total - st.lake_area(cids) - st.reservoir_area(cids))
    assert total == pytest.approx(st.forest_area(cids) + st.glacier_area(cids) + st.lake_area(cids) +
                                  st.reservoir_area(cids) + st.unspecified_area(cids))
    assert abs(st.elevation(cids) - 475 / 2.0) < 1e-3
    cids.append(3)
    with pytest.raises(RuntimeError):
        st.total_area(cids)


def test_model_initialize_and_run():
    from shyft_amd import api
    from shyft_amd.api import pt_gs_k
    n = 20
    model = build_model(pt_gs_k.PTGSKModel, pt_gs_k.PTGSKParameter, n)
    assert model.size() == n
    assert model.ncore >= 1
    model.ncore = 4
    assert model.ncore == 4
    rp = model.get_region_parameter()
    rp.gs.snow_cv_forest_factor = 0.1
    rp.gs.snow_cv_altitude_factor = 0.0001
    assert rp.gs.effective_snow_cv(1.0, 0.0) == pytest.approx(rp.gs.snow_cv + 0.1)
    assert rp.gs.effective_snow_cv(1.0, 1000.0) == pytest.approx(rp.gs.snow_cv + 0.1 + 0.1)
    cal = api.Calendar()
    ta = api.TimeAxisFixedDeltaT(cal.time(2015, 1, 1, 0, 0, 0), api.deltahours(1), 240)
    ip = interpolation_parameter()
    model.initialize_cell_environment(ta)
    model.interpolate(ip, dummy_env(ta, model.get_cells()[n // 2].geo.mid_point()))
    assert model.interpolation_parameter.use_idw_for_temperature
    assert model.interpolation_parameter.temperature_idw.zscale == pytest.approx(0.5)
    c0 = model.cells[0]
    for x in (c0.env_ts.temperature, c0.env_ts.precipitation, c0.env_ts.rel_hum, c0.env_ts.radiation,
              c0.env_ts.wind_speed):
        assert model.is_cell_env_ts_ok()
        vx = x.value(0)
        x.set(0, float("nan"))
        assert not model.is_cell_env_ts_ok()
        x.set(0, vx)
        assert model.is_cell_env_ts_ok()

    s0 = pt_gs_k.PTGSKStateVector()
    for _ in range(n):
        si = pt_gs_k.PTGSKState()
        si.kirchner.q = 40.0
        s0.append(si)
    model.set_states(s0)
    model.set_state_collection(-1, True)
    model2 = pt_gs_k.PTGSKModel(model)
    opt_model = pt_gs_k.create_opt_model_clone(model)
    model.run_cells()
    cids = api.IntVector()
    sum_discharge = model.statistics.discharge(cids)
    sum_discharge_value = model.statistics.discharge_value(cids, 0)
    assert model.statistics.charge_value(cids, 0) == pytest.approx(-110.6998, abs=0.5e-2)
    cell_charge = model.statistics.charge_value(api.IntVector([0, 1, 3]), 0, ix_type=api.stat_scope.cell)
    assert cell_charge == pytest.approx(-16.7138, abs=0.5e-2)
    s126 = model.statistics.charge(api.IntVector([1, 2, 6]), ix_type=api.stat_scope.cell).values.to_numpy().sum()
    assert s126 == pytest.approx(107.3981, abs=0.5e-2)
    ae_output = model.actual_evaptranspiration_response.output(cids)
    ae_pot_ratio = model.actual_evaptranspiration_response.pot_ratio(cids)
    assert ae_output.values.to_numpy().max() == pytest.approx(0.189214067680088, abs=0.5e-7)
    assert ae_pot_ratio.values.to_numpy().min() == pytest.approx(0.9995599424191931, abs=0.5e-7)
    assert ae_pot_ratio.values.to_numpy().max() == pytest.approx(1.0, abs=0.5e-7)
    opt_model.run_cells()
    assert opt_model.statistics.discharge_value(cids, 0) == pytest.approx(sum_discharge_value, abs=0.5e-3)
    assert sum_discharge_value >= 130.0
    # the reference asserts the clone SHARES the region env (apoint_ts shared impl): a set on one shows on the other
    opt_model.region_env.temperature[0].ts.set(0, 23.2)
    assert not abs(model.region_env.temperature[0].ts.value(0) - opt_model.region_env.temperature[0].ts.value(0)) > 0.5

    # stepwise 10 x 24 runs equal the full run
    model.set_states(s0)
    assert len(s0) == len(model.initial_state)
    for collect in (False, True):
        model2.set_state_collection(-1, collect)
        model2.set_states(s0)
        for section in range(10):
            model2.run_cells(use_ncore=0, start_step=section * 24, n_steps=24)
            assert model2.statistics.discharge(cids).size() == sum_discharge.size()
    diff = sum_discharge.values.to_numpy() - model2.statistics.discharge(cids).values.to_numpy()
    assert (diff * diff).max() == pytest.approx(0.0, abs=0.5e-4)
    with pytest.raises(RuntimeError):
        model.statistics.discharge(api.IntVector([0, 4, 5]))

    assert model.statistics.temperature(cids).size() == ta.size()
    assert model.statistics.precipitation(cids) is not None
    for t in range(ta.size()):
        assert len(model.statistics.precipitation(cids, t)) == n
    assert model.gamma_snow_response.sca_value(cids, 1) >= 0.0
    assert model.gamma_snow_response.sca(cids) is not None
    assert model.gamma_snow_state.albedo(cids) is not None
    copy_model = model.__class__(model)
    copy_model.run_cells()

    # routing: one river 3000 m downstream at 1/3.6 m/s, UHG alpha 7 (test_region_model_stacks.py:287-301)
    model.river_network.add(api.River(1, api.RoutingInfo(0, 3000.0), api.UHGParameter(1 / 3.60, 7.0, 0.0)))
    model.connect_catchment_to_river(1, 1)
    assert model.has_routing()
    out = model.river_output_flow_m3s(1)
    local = model.river_local_inflow_m3s(1)
    up = model.river_upstream_inflow_m3s(1)
    assert out.value(8) == pytest.approx(28.061248025828114, abs=0.5)
    # no cell UHG (routing distance 0): local inflow equals the cells' summed discharge; no upstream rivers
    assert np.allclose(local.values.to_numpy(), sum_discharge.values.to_numpy(), rtol=1e-12, atol=1e-12)
    assert np.all(up.values.to_numpy() == 0.0)
    model.connect_catchment_to_river(1, 0)
    assert not model.has_routing()

    q_0 = model.cells[0].state.kirchner.q
    model.adjust_q(2.0, cids)
    assert model.cells[0].state.kirchner.q == pytest.approx(q_0 * 2.0)
    model.revert_to_initial_state()
    model.run_cells(0, 10, 2)
    # state tuning to a wanted flow (test_region_model_stacks.py:316-333)
    q_avg = (model.statistics.discharge_value(cids, 10) + model.statistics.discharge_value(cids, 11)) / 2.0
    x = 0.7
    model.revert_to_initial_state()
    s_before = [s.kirchner.q for s in model.current_state]
    r = model.adjust_state_to_target_flow(x * q_avg, cids, start_step=10, scale_range=3.0, scale_eps=1e-3,
                                          max_iter=350, n_steps=2)
    assert len(r.diagnostics) == 0
    assert r.q_r == pytest.approx(q_avg * x, abs=0.5e-2)
    assert r.q_0 == pytest.approx(q_avg, abs=0.5e-2)
    # the state left behind is the tuned one: a uniform scale of every selected cell's q
    s_after = [s.kirchner.q for s in model.current_state]
    ratio = np.array(s_after) / np.array(s_before)
    assert np.allclose(ratio, ratio[0], rtol=1e-12) and 1 / 3 < ratio[0] < 3
    model.run_cells(0, 10, 2)
    q_tuned = (model.statistics.discharge_value(cids, 10) + model.statistics.discharge_value(cids, 11)) / 2.0
    assert q_tuned == pytest.approx(r.q_r, rel=1e-12)
    r = model.adjust_state_to_target_flow(float("nan"), cids, start_step=10, scale_range=3.0, scale_eps=1e-3,
                                          max_iter=300, n_steps=2)
    assert len(r.diagnostics) > 0
    model.cells[0].env_ts.temperature.set(10, float("nan"))
    r = model.adjust_state_to_target_flow(30.0, cids, start_step=10, scale_range=3.0, scale_eps=1e-3, max_iter=300,
                                          n_steps=2)
    assert len(r.diagnostics) > 0


def test_run_cells_argument_errors():
    from shyft_amd import api
    from shyft_amd.api import pt_gs_k
    m = build_model(pt_gs_k.PTGSKOptModel, pt_gs_k.PTGSKParameter, 4)
    with pytest.raises(RuntimeError, match="invalid time_axis"):
        m.run_cells()
    ta = api.TimeAxisFixedDeltaT(api.Calendar().time(2015, 1, 1), api.deltahours(1), 24)
    m.initialize_cell_environment(ta)
    with pytest.raises(RuntimeError, match="start_step must in range"):
        m.run_cells(0, 24, 0)
    with pytest.raises(RuntimeError, match="start_step\\+n_steps must be within"):
        m.run_cells(0, 10, 20)
    with pytest.raises(RuntimeError, match="more than 100 time"):
        m.run_cells(1000 * m.ncore)
    with pytest.raises(RuntimeError):
        m.set_catchment_calculation_filter(api.IntVector([7]))


def test_hbv_model_discharge():
    """test_region_model_stacks.py:424-479: hbv_stack, tank uz = lz = 40, discharge_value(0) >= 32."""
    from shyft_amd import api
    from shyft_amd.api import hbv_stack
    n = 20
    model = build_model(hbv_stack.HbvModel, hbv_stack.HbvParameter, n)
    cal = api.Calendar()
    ta = api.TimeAxisFixedDeltaT(cal.time(2015, 1, 1, 0, 0, 0), api.deltahours(1), 240)
    model.initialize_cell_environment(ta)
    model.interpolate(interpolation_parameter(), dummy_env(ta, model.get_cells()[n // 2].geo.mid_point()))
    s0 = hbv_stack.HbvStateVector()
    for _ in range(n):
        si = hbv_stack.HbvState()
        si.tank.uz = 40.0
        si.tank.lz = 40.0
        s0.append(si)
    model.set_states(s0)
    model.set_state_collection(-1, True)
    model.run_cells()
    cids = api.IntVector()
    assert model.statistics.discharge_value(cids, 0) >= 32.0
    assert model.hbv_snow_state.swe(cids).size() == ta.size() + 1
    assert math.isfinite(model.hbv_tank_state.uz_value(cids, 10))


def test_pt_ss_k_model_init_and_run():
    """test_region_model_stacks.py:71-78 (pt_ss_k model init) plus a run through the same dummy environment:
    the API model's discharge equals the C-ABI region run on the interpolated forcing (oracle-checked kernel)."""
    from shyft_amd import api
    from shyft_amd.api import pt_ss_k
    n = 20
    model = build_model(pt_ss_k.PTSSKModel, pt_ss_k.PTSSKParameter, n)
    assert model.size() == n
    assert model.skaugen_snow_response is not None and model.skaugen_snow_state is not None
    cal = api.Calendar()
    ta = api.TimeAxisFixedDeltaT(cal.time(2015, 1, 1, 0, 0, 0), api.deltahours(1), 240)
    model.initialize_cell_environment(ta)
    model.interpolate(interpolation_parameter(), dummy_env(ta, model.get_cells()[n // 2].geo.mid_point()))
    s0 = pt_ss_k.PTSSKStateVector()
    for _ in range(n):
        si = pt_ss_k.PTSSKState()
        si.kirchner.q = 40.0
        s0.append(si)
    model.set_states(s0)
    model.set_state_collection(-1, True)
    model.run_cells()
    cids = api.IntVector()
    q = model.statistics.discharge(cids).values.to_numpy()
    assert np.all(np.isfinite(q)) and q[0] > 0
    # 10 degC rain-on-bare-ground: no snow state appears
    assert model.skaugen_snow_state.swe(cids).values.to_numpy().max() == 0.0
    assert model.skaugen_snow_response.outflow_value(cids, 5) >= 0.0
    # the same region through the C ABI directly
    from shyft_amd.region import HipRegion, PT_SS_K, COLLECT_DISCHARGE
    r = HipRegion(PT_SS_K, n)
    geo = np.zeros((n, 11))
    for i in range(n):
        geo[i] = [500 + 1000.0 * i, 500.0, 500.0 * i / n, 1e6, 1, 0.9, 0.01, 0.05, 0.19, 0.30, 0.45]
    r.set_geo(geo)
    r.set_parameters(np.array(pt_ss_k.PTSSKParameter().to_vector()))
    r.set_time_axis(ta.start * 10**6, 3600 * 10**6, 240)
    r.set_collection(COLLECT_DISCHARGE)
    st = np.tile(np.array(pt_ss_k.PTSSKState().to_vector()), (n, 1))
    st[:, 7] = 40.0
    r.set_state(st)
    for v in range(5):
        r.set_forcing(v, 0, np.stack([model.cells[i].env_ts.__getattr__(api.FORCING[v]).to_numpy()
                                      for i in range(n)], axis=1))
    r.run_cells()
    assert np.allclose(r.get_series(0, 0, 240).sum(axis=1), q, rtol=1e-13, atol=0)


def test_routing_counts_filtered_out_cells():
    """routing::model::local_inflow (routing.h:345-350) sums every cell routed to the river, whatever the
    catchment calculation filter says: a filtered-out cell contributes the response it holds from the last
    run that included it (its collector series are not touched by a run that skips it)."""
    from shyft_amd import api
    from shyft_amd.api import pt_gs_k
    n = 20
    model = build_model(pt_gs_k.PTGSKModel, pt_gs_k.PTGSKParameter, n, num_catchments=2)
    ta = api.TimeAxisFixedDeltaT(api.Calendar().time(2015, 1, 1, 0, 0, 0), api.deltahours(1), 48)
    model.initialize_cell_environment(ta)
    model.interpolate(interpolation_parameter(), dummy_env(ta, model.get_cells()[n // 2].geo.mid_point()))
    s0 = pt_gs_k.PTGSKStateVector()
    for _ in range(n):
        si = pt_gs_k.PTGSKState()
        si.kirchner.q = 40.0
        s0.append(si)
    model.set_states(s0)
    model.run_cells()
    all_cids = api.IntVector()
    q_all = model.statistics.discharge(all_cids).values.to_numpy()
    q2_first = model.statistics.discharge(api.IntVector([2])).values.to_numpy()
    model.river_network.add(api.River(1, api.RoutingInfo(0, 0.0), api.UHGParameter(1 / 3.60, 7.0, 0.0)))
    model.connect_catchment_to_river(1, 1)
    model.connect_catchment_to_river(2, 1)
    # second run of catchment 1 only, from a different state: catchment 2 keeps its first-run series
    model.set_catchment_calculation_filter(api.IntVector([1]))
    s1 = pt_gs_k.PTGSKStateVector()
    for _ in range(n):
        si = pt_gs_k.PTGSKState()
        si.kirchner.q = 5.0
        s1.append(si)
    model.set_states(s1)
    model.run_cells()
    q1_second = model.statistics.discharge(api.IntVector([1])).values.to_numpy()
    local = model.river_local_inflow_m3s(1).values.to_numpy()
    assert not np.allclose(q1_second + q2_first, q_all)
    assert np.allclose(local, q1_second + q2_first, rtol=1e-12, atol=1e-12)
