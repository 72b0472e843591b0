"""pt_hs_k (Priestley-Taylor + hbv_snow + kirchner, core/pt_hs_k.h:199-283).

CPU: the oracle restatement against the reference's known answers in test/pt_hs_k_test.cpp
(test_call_stack :42-92, pt_hs_k_lake_reservoir_response :93-154, doctest Approx semantics
|a - b| < eps * (1 + max(|a|, |b|))).

GPU: the HIP kernel (kernels/pthsk.hip) against the oracle, bit for bit: both evaluate the same
expressions in the same order with the same deterministic exp/pow (detmath), and share the hbv_snow
and kirchner device code with the hbv_stack and pt_gs_k kernels. Cases: the synthetic region over a
winter and the melt, two ragged parameter sets with a user snow distribution, stepwise == full, the
reference KATs through the device.
"""
import numpy as np
import pytest

from shyft_amd import synthetic
from tests import engines, oracle_lib

HOUR = synthetic.HOUR_US
T0_2014_08_01 = 1406851200 * 10**6


def approx(a, b, eps):  # doctest::Approx(b).epsilon(eps) == a
    return abs(a - b) < eps * (1.0 + max(abs(a), abs(b)))


def mmh_to_m3s(mmh, area):
    return area * mmh / (1000.0 * 3600.0)


def _lake_reservoir_case():
    """pt_hs_k_lake_reservoir_response (pt_hs_k_test.cpp:93-130): freezing cold, 3 mm/h precipitation except
    step 0, 0.2 lake, 0.3 reservoir, 0.5 unspecified, kirchner q 1 mm/h, default hbv_snow state."""
    n = 50
    geo = np.array([[1000.0, 1000.0, 100.0, 1e6, 0.0, 0.9, 0.0, 0.2, 0.3, 0.0, 0.5]])
    f = np.zeros((5, n, 1))
    f[0] = -15.0
    f[1] = 3.0
    f[1, 0] = 0.0
    f[2] = 2.0
    f[3] = 0.8
    f[4] = 300.0
    st = synthetic.default_pthsk_state(1, q=1.0)
    return geo, f, st


def _check_lake_reservoir(engine):
    geo, f, st = _lake_reservoir_case()
    p = synthetic.default_pthsk_parameters()
    q3 = mmh_to_m3s(3.0, 1e6)
    p[17] = 0.0  # msp.reservoir_direct_response_fraction: all reservoir water through kirchner
    r = engines.run_pthsk(engine, geo, p, st, T0_2014_08_01, HOUR, f, collect_state=True)
    q = r["full"][0, :, 0]
    assert approx(q[0], 0.266, 0.01)
    assert approx(q[-1], 0.5 * q3, 0.01)
    p[17] = 1.0  # reservoir direct to the outlet, lake through kirchner
    r = engines.run_pthsk(engine, geo, p, st, T0_2014_08_01, HOUR, f, collect_state=True)
    q = r["full"][0, :, 0]
    assert approx(q[0], 0.266 * 0.7, 0.01)
    assert approx(q[1], 0.266 + 0.3 * 0.5 * q3, 0.05)
    sc_swe = r["state_series"][2, :, 0]   # state collector snow_swe (scaled by the snow storage fraction)
    rc_swe = r["full"][3, :, 0]           # response snow_swe
    assert approx(sc_swe[0], 0.0, 0.0001) and approx(sc_swe[1], 0.0, 0.0001) and approx(sc_swe[2], 1.5, 0.0001)
    assert approx(rc_swe[0], 0.0, 0.0001) and approx(rc_swe[1], 1.5, 0.0001) and approx(rc_swe[2], 3.0, 0.0001)
    assert approx(q[-1], 0.2 * q3 * (1.0 - 0.3) + 0.3 * q3, 0.01)


def test_oracle_lake_reservoir_response_kat():
    _check_lake_reservoir("oracle")


def test_oracle_call_stack():
    """test_call_stack (pt_hs_k_test.cpp:42-92): a non-normalised even distribution, state swe 10 / sca 0.5
    distributed at run start, three summer days; the collected snow swe is finite and >= 0."""
    n, T = 4, 72
    geo = synthetic.geo11(n)
    f = synthetic.forcing(n, 24 * 212, T, z=geo[:, 2])  # Aug 1
    st = synthetic.default_pthsk_state(n, q=5.0, swe=10.0, sca=0.5)
    d = oracle_lib.hbv_dist_row([1.0] * 5, [0.0, 0.25, 0.5, 0.75, 1.0])
    r = engines.run_pthsk("oracle", geo, synthetic.default_pthsk_parameters(), st, T0_2014_08_01, HOUR, f,
                          snow_dist=d)
    swe = r["full"][3]
    assert np.isfinite(swe).all() and (swe >= 0).all()


def _case(n, T, step0=0, seed=3):
    geo = synthetic.geo11(n, n_catchments=4)
    rng = np.random.default_rng(seed)
    geo[:, 6] = rng.choice([0.0, 0.05, 0.3], n)      # glacier
    geo[:, 7] = rng.choice([0.0, 0.05], n)           # lake
    geo[:, 8] = rng.choice([0.0, 0.19], n)           # reservoir
    geo[:, 10] = 1.0 - geo[:, 6:10].sum(axis=1)
    f = synthetic.forcing(n, step0, T, z=geo[:, 2])
    return geo, f


def _assert_same(a, b, keys):
    for k in keys:
        x, y = a[k], b[k]
        assert x.shape == y.shape, k
        same = (x == y) | (np.isnan(x) & np.isnan(y))
        if not same.all():
            idx = np.argwhere(~same)[0]
            raise AssertionError(f"{k} differs first at {tuple(idx)}: {x[tuple(idx)]!r} vs {y[tuple(idx)]!r} "
                                 f"({(~same).sum()} values)")


def test_oracle_stepwise_equals_full():
    n, T = 40, 96
    geo, f = _case(n, T, step0=24 * 60)
    st = synthetic.default_pthsk_state(n)
    p = synthetic.default_pthsk_parameters()
    full = oracle_lib.pthsk_run(geo, p, st, synthetic.T0_2015_US, HOUR, f, full=True)
    s = st.copy()
    out = np.full_like(full["full"], np.nan)
    for k in range(4):
        r = oracle_lib.pthsk_run(geo, p, s, synthetic.T0_2015_US, HOUR, f, 24 * k, 24, full=True)
        out[:, 24 * k:24 * (k + 1)] = r["full"][:, 24 * k:24 * (k + 1)]
        s = r["state"]
    assert np.array_equal(out, full["full"])
    assert np.array_equal(s, full["state"])


@pytest.mark.gpu
def test_device_lake_reservoir_response_kat():
    _check_lake_reservoir("hip")


@pytest.mark.gpu
def test_pthsk_synthetic_winter_to_melt_bitexact():
    n, T = 777, 24 * 120  # Jan 1 .. Apr 30: snow build-up, melt season
    geo, f = _case(n, T)
    st = synthetic.default_pthsk_state(n)
    p = synthetic.default_pthsk_parameters()
    ref = engines.run_pthsk("oracle", geo, p, st, synthetic.T0_2015_US, HOUR, f, collect_state=True)
    got = engines.run_pthsk("hip", geo, p, st, synthetic.T0_2015_US, HOUR, f, collect_state=True)
    assert np.nanmax(ref["state_series"][2]) > 10.0  # snow did accumulate
    _assert_same(got, ref, ["full", "state", "state_series"])


@pytest.mark.gpu
def test_pthsk_two_sets_custom_distribution_bitexact():
    n, T = 333, 24 * 40
    geo, f = _case(n, T, step0=24 * 50, seed=9)  # late Feb - early Apr
    p0 = synthetic.default_pthsk_parameters()
    p1 = p0.copy()
    p1[[0, 1, 3, 5, 6, 8, 10]] = [-2.2, 0.9, 1.2, 0.5, 2.5, 0.3, 1.1]  # c1 c2 ae_scale tx cx cfr p_corr
    i1 = [0.0, 0.2, 0.5, 0.8, 1.0]
    d0 = oracle_lib.hbv_dist_row([1.0] * 5, [0.0, 0.25, 0.5, 0.75, 1.0])
    d1 = oracle_lib.hbv_dist_row(oracle_lib.hbv_normalize([0.5, 0.8, 1.0, 1.3, 1.5], i1), i1)
    ix = (np.arange(n) * 7 % 3 == 0).astype(np.int32)
    st = synthetic.default_pthsk_state(n, q=2.0, swe=60.0, sca=0.8)  # undistributed: distributed at run start
    args = (geo, np.stack([p0, p1]), st, synthetic.T0_2015_US, HOUR, f)
    ref = engines.run_pthsk("oracle", *args, set_ix=ix, snow_dist=np.stack([d0, d1]), collect_state=True)
    got = engines.run_pthsk("hip", *args, set_ix=ix, snow_dist=np.stack([d0, d1]), collect_state=True)
    _assert_same(got, ref, ["full", "state", "state_series"])


@pytest.mark.gpu
def test_pthsk_stepwise_equals_full_on_gpu():
    from shyft_amd.region import HipRegion, PT_HS_K, COLLECT_ALL
    n, T = 256, 24 * 10
    geo, f = _case(n, T, step0=24 * 75)
    p = synthetic.default_pthsk_parameters()
    st = synthetic.default_pthsk_state(n)
    full = engines.run_pthsk("hip", geo, p, st, synthetic.T0_2015_US, HOUR, f)
    r = HipRegion(PT_HS_K, n)
    try:
        r.set_geo(geo)
        r.set_parameters(p)
        r.set_time_axis(synthetic.T0_2015_US, HOUR, T)
        r.set_collection(COLLECT_ALL)
        r.set_state(st)
        for v in range(5):
            r.set_forcing(v, 0, f[v])
        for k in range(10):
            r.run_cells(0, 24 * k, 24)
        got = np.stack([r.get_series(k, 0, T) for k in range(8)])
        assert np.array_equal(got, full["full"])
        assert np.array_equal(r.get_state(), full["state"])
    finally:
        r.close()


@pytest.mark.gpu
def test_pthsk_stale_bins_beyond_the_state_count_read_as_zero():
    """The state carries nb bins (the reference's vectors); slots nb..7 of the flat row are padding and come back 0."""
    n, T = 150, 24 * 20
    geo, f = _case(n, T, step0=24 * 60, seed=4)
    st = synthetic.default_pthsk_state(n, q=2.0)
    st[:, 0:2] = 0.0
    st[:, 2] = 5.0
    st[:, 3:19] = 0.0
    st[:, 8:11] = st[:, 16:19] = 1.5
    args = (geo, synthetic.default_pthsk_parameters(), st, synthetic.T0_2015_US, HOUR, f)
    ref = engines.run_pthsk("oracle", *args)
    got = engines.run_pthsk("hip", *args)
    _assert_same(got, ref, ["full", "state"])
    assert (got["state"][:, [8, 9, 10, 16, 17, 18]] == 0.0).all()
