"""End-to-end region KATs of the reference's Python API test
(shyft/tests/api/test_region_model_stacks.py:14-30, 46-55, 145-261, 424-479):
a 20-cell region, interpolation of a single constant source at cell 10's
mid-point, 240 hourly steps from 2015-01-01Z, then run_cells and the
catchment statistics. Run on the CPU oracle and on the HIP path (-m gpu)."""
import numpy as np
import pytest

from shyft_amd import synthetic
from tests import oracle_lib

HOUR = 3600 * 10**6
N, T = 20, 240
ENGINES = ["oracle", pytest.param("hip", marks=pytest.mark.gpu)]
# api.InterpolationParameter() as modified by the test (:165-183); rows are the C-ABI idw_param vector
# (max_members, max_distance, distance_measure_factor, zscale, default_temp_gradient, by_equation, scale_factor)
IDW = {
    0: [6, 20000.0, 1.0, 0.5, -0.005, 1.0, 1.02],    # temperature_idw (single source -> copied)
    1: [20, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],  # precipitation_parameter() (inverse_distance.h:66-70)
    2: [10, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],  # wind_speed: idw::parameter() (:43-46)
    3: [10, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],  # rel_hum
    4: [10, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],  # radiation
}
SOURCE_VALUE = {0: 10.0, 1: 5.0, 2: 2.0, 3: 0.7, 4: 300.0}  # create_dummy_region_environment (:46-55)
ORACLE_KIND = {1: 1, 2: 3, 3: 4, 4: 2}  # forcing var -> oracle idw kind (precipitation, wind, rel_hum, radiation)


def region_geo(n=N):
    """build_model (:14-30): x = 500 + 1000 i, y = 500, z = 500 i / n, area 1e6, cid 1, slope 0.9,
    fractions glacier 0.01 lake 0.05 reservoir 0.19 forest 0.30."""
    geo = np.zeros((n, 11))
    for i in range(n):
        geo[i] = [500 + 1000.0 * i, 500.0, 500.0 * i / n, 1e6, 1, 0.9, 0.01, 0.05, 0.19, 0.30, 0.45]
    return geo


def source_xyz(geo):
    return np.atleast_2d(geo[N // 2, :3]).copy()


def region_forcing(geo, T_=T):
    """env_ts of every cell after interpolate() with the oracle's IDW (temperature: single source copy,
    region_model.h:470-481)."""
    from tests.test_idw import oracle_idw
    n = geo.shape[0]
    f = np.empty((5, T_, n))
    f[0] = SOURCE_VALUE[0]
    src = source_xyz(geo)
    for var in (1, 2, 3, 4):
        vals = np.full((T_, 1), SOURCE_VALUE[var])
        f[var] = oracle_idw(ORACLE_KIND[var], src, vals, geo[:, :3], IDW[var], dst_slope=geo[:, 5])
    return f


def ptgsk_region_parameters():
    p = synthetic.default_ptgsk_parameters()
    p[17] = 0.1     # gs.snow_cv_forest_factor (:157-160)
    p[18] = 0.0001  # gs.snow_cv_altitude_factor
    return p


def _hip_region(stack, geo, params, state, collect_state):
    from shyft_amd.region import HipRegion, COLLECT_ALL
    r = HipRegion(stack, N)
    r.set_geo(geo)
    r.set_parameters(np.atleast_2d(params))
    r.set_time_axis(synthetic.T0_2015_US, HOUR, T)
    r.set_collection(COLLECT_ALL, collect_state)
    src = source_xyz(geo)
    for var in range(5):
        r.interpolate(var, src, np.full((T, 1), SOURCE_VALUE[var]), 0, IDW[var])
    r.set_state(state)
    return r


def run_ptgsk(engine, stepwise=False):
    geo = region_geo()
    st = synthetic.default_ptgsk_state(N, q=40.0)
    if engine == "oracle":
        f = region_forcing(geo)
        if not stepwise:
            return oracle_lib.ptgsk_run(geo, ptgsk_region_parameters(), st, synthetic.T0_2015_US, HOUR, f, full=True,
                                        collect_state=True)
        out = None
        for section in range(10):
            r = oracle_lib.ptgsk_run(geo, ptgsk_region_parameters(), st, synthetic.T0_2015_US, HOUR, f, section * 24, 24,
                                     full=True, collect_state=True)
            st = r["state"]
            out = r if out is None else out
            out["full"][:, section * 24:(section + 1) * 24] = r["full"][:, section * 24:(section + 1) * 24]
        return out
    from shyft_amd.region import PT_GS_K
    r = _hip_region(PT_GS_K, geo, ptgsk_region_parameters(), st, True)
    try:
        if stepwise:
            for section in range(10):
                r.run_cells(0, section * 24, 24)
        else:
            r.run_cells()
        return {"full": np.stack([r.get_series(k, 0, T) for k in range(8)]),
                "state_series": np.stack([r.get_state_series(k, 0, T + 1) for k in range(9)])}
    finally:
        r.close()


@pytest.fixture(scope="module", params=ENGINES)
def ptgsk(request):
    return request.param, run_ptgsk(request.param)


def places(a, b, n):
    """unittest assertAlmostEqual(a, b, places=n): round(a - b, n) == 0"""
    return round(a - b, n) == 0


def test_ptgsk_charge_kats(ptgsk):
    _, r = ptgsk
    charge = r["full"][1]                                         # [T][N]
    assert places(charge[0].sum(), -110.6998, 2)                  # charge_value(all, 0)
    assert places(charge[0, [0, 1, 3]].sum(), -16.7138, 2)        # charge_value(cells [0,1,3], 0)
    assert places(charge[:, [1, 2, 6]].sum(axis=1).sum(), 107.3981, 2)
    assert r["full"][0][0].sum() >= 130.0                         # discharge_value(all, 0)


def test_ptgsk_ae_kats(ptgsk):
    _, r = ptgsk
    ae = r["full"][6].mean(axis=1)  # area-weighted average over equal areas
    assert places(ae.max(), 0.189214067680088, 7)
    # pot_ratio over the state axis: calc_pot_ratio(m3s_to_mmh(kirchner_discharge), ae_scale_factor) (api.h:1527-1541)
    q = r["state_series"][0] / (1e6 / 3.6e6)
    ratio = (1.0 - np.exp(-q * 3.0 / 1.5)).mean(axis=1)
    assert places(ratio.min(), 0.9995599424191931, 7)
    assert places(ratio.max(), 1.0, 7)


@pytest.mark.parametrize("engine", ENGINES)
def test_ptgsk_stepwise_equals_full(engine):
    full = run_ptgsk(engine)["full"][0].sum(axis=1)
    step = run_ptgsk(engine, stepwise=True)["full"][0].sum(axis=1)
    assert places(((full - step) ** 2).max(), 0.0, 4)


@pytest.mark.parametrize("engine", ENGINES)
def test_hbv_region_discharge_kat(engine):
    """test_hbv_model_initialize_and_run (:424-479): tank uz = lz = 40, discharge_value(all, 0) >= 32."""
    geo = region_geo()
    st = np.stack([oracle_lib.hbv_snow_state(uz=40.0, lz=40.0) for _ in range(N)])
    if engine == "oracle":
        q0 = oracle_lib.hbv_run(geo, synthetic.default_hbv_parameters(), st, synthetic.T0_2015_US, HOUR,
                                region_forcing(geo))["main"][0, 0].sum()
    else:
        from shyft_amd.region import HBV_STACK
        r = _hip_region(HBV_STACK, geo, synthetic.default_hbv_parameters(), st, False)
        try:
            r.run_cells()
            q0 = r.get_series(0, 0, T)[0].sum()
        finally:
            r.close()
    assert q0 >= 32.0
