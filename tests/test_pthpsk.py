"""pt_hps_k (Priestley-Taylor + hbv_physical_snow + kirchner, core/pt_hps_k.h:203-300).

CPU: the oracle restatement against the reference's known answers: test/hbv_physical_snow_test.cpp
(mass balance at reset, build-up, tx, rain without snow, melt without precipitation; 1e-8) and
test/pt_hps_k_test.cpp (test_call_stack :43-83, pt_hps_k_lake_reservoir_response :84-157; doctest Approx
|a - b| < eps * (1 + max(|a|, |b|))).

GPU: the HIP kernel (kernels/pthpsk.hip) against the oracle, bit for bit (same expressions, same order,
detmath elementary functions): the synthetic region over a winter and the melt, two ragged parameter sets
with a user snow distribution, iso_pot_energy on, stepwise == full, the KATs through the device.
"""
import numpy as np
import pytest

from shyft_amd import synthetic
from tests import engines, oracle_lib
from tests.test_pthsk import approx, mmh_to_m3s, _lake_reservoir_case, _assert_same, T0_2014_08_01

HOUR = synthetic.HOUR_US
S5 = [1.0] * 5
A5 = [0.0, 0.25, 0.5, 0.75, 1.0]
P12 = [0.0, 0.1, 0.5, 2.0, 1.0, 30.0, 0.9, 0.6, 5.0, 5.0, 5.0, 0.0]  # hbv_physical_snow::parameter() defaults


def _hps_state(swe, sca, nb=5):
    st = np.zeros(36)
    st[0], st[1], st[2], st[3] = swe, sca, 0.0, nb
    st[4 + 16:4 + 16 + nb] = 0.6       # albedo
    st[4 + 24:4 + 24 + nb] = 1752.56396484375  # iso_pot_energy
    return st


@pytest.mark.parametrize("prec,T,sca,swe", [
    (0.04, 1.0, 1.0, 0.05),    # mass_balance_at_snowpack_reset (:21-48)
    (0.15, -1.0, 0.6, 0.2),    # mass_balance_at_snowpack_buildup (:49-79)
    (0.15, 0.0, 0.6, 0.2),     #   ... at T = tx
    (0.15, 0.0, 0.0, 0.0),     # mass_balance_rain_no_snow (:80-106)
    (0.0, 3.0, 0.5, 10.0),     # mass_balance_melt_no_precip (:107-131)
])
def test_hbv_physical_snow_mass_balance(prec, T, sca, swe):
    d = oracle_lib.hbv_dist_row(oracle_lib.hbv_normalize(S5, A5), A5)
    st = _hps_state(swe, sca)
    out, r_sca, _ = oracle_lib.hps_step(st, P12, d, 1, HOUR, T, 10.0, prec, 2.0, 0.7)
    assert abs((prec + swe) - (st[0] + out)) <= 1e-8
    if sca == 0.0 and swe == 0.0:
        assert abs(st[1]) <= 1e-8 and abs(st[0]) <= 1e-8


def _check_lake_reservoir(engine):
    geo, f, _ = _lake_reservoir_case()
    st = synthetic.default_pthpsk_state(1, q=1.0)
    p = synthetic.default_pthpsk_parameters()
    q3 = mmh_to_m3s(3.0, 1e6)
    p[23] = 0.0  # msp.reservoir_direct_response_fraction
    r = engines.run_pthpsk(engine, geo, p, st, T0_2014_08_01, HOUR, f, collect_state=True)
    q = r["full"][0, :, 0]
    assert approx(q[0], 0.266, 0.01)
    assert approx(q[-1], 0.5 * q3, 0.01)
    p[23] = 1.0
    r = engines.run_pthpsk(engine, geo, p, st, T0_2014_08_01, HOUR, f, collect_state=True)
    q = r["full"][0, :, 0]
    assert approx(q[0], 0.266 * 0.7, 0.01)
    assert approx(q[1], 0.266 + 0.3 * 0.5 * q3, 0.05)
    sc_swe = r["state_series"][2, :, 0]
    rc_swe = r["full"][3, :, 0]
    assert approx(sc_swe[0], 0.0, 0.0001) and approx(sc_swe[1], 0.0, 0.0001) and approx(sc_swe[2], 1.5, 0.0001)
    assert approx(rc_swe[0], 0.0, 0.0001) and approx(rc_swe[1], 1.5, 0.0001) and approx(rc_swe[2], 3.0, 0.0001)
    assert approx(q[-1], 0.2 * q3 * (1.0 - 0.3) + 0.3 * q3, 0.01)


def test_oracle_lake_reservoir_response_kat():
    _check_lake_reservoir("oracle")


def test_oracle_call_stack():
    """test_call_stack (pt_hps_k_test.cpp:43-83): hps state albedo 0.4 x5, swe 10, sca 0.5, kirchner q 5,
    three August days; the collected snow swe is finite and >= 0."""
    n, T = 4, 72
    geo = synthetic.geo11(n)
    f = synthetic.forcing(n, 24 * 212, T, z=geo[:, 2])
    st = synthetic.default_pthpsk_state(n, q=5.0, swe=10.0, sca=0.5)
    st[:, 3] = 5
    st[:, 4 + 16:4 + 21] = 0.4
    r = engines.run_pthpsk("oracle", geo, synthetic.default_pthpsk_parameters(), st, T0_2014_08_01, HOUR, f)
    swe = r["full"][3]
    assert np.isfinite(swe).all() and (swe >= 0).all()


def _case(n, T, step0=0, seed=3):
    from tests.test_pthsk import _case as c
    return c(n, T, step0, seed)


def test_oracle_stepwise_equals_full():
    n, T = 40, 96
    geo, f = _case(n, T, step0=24 * 60)
    st = synthetic.default_pthpsk_state(n)
    p = synthetic.default_pthpsk_parameters()
    full = oracle_lib.pthpsk_run(geo, p, st, synthetic.T0_2015_US, HOUR, f, full=True)
    s = st.copy()
    out = np.full_like(full["full"], np.nan)
    for k in range(4):
        r = oracle_lib.pthpsk_run(geo, p, s, synthetic.T0_2015_US, HOUR, f, 24 * k, 24, full=True)
        out[:, 24 * k:24 * (k + 1)] = r["full"][:, 24 * k:24 * (k + 1)]
        s = r["state"]
    assert np.array_equal(out, full["full"])
    assert np.array_equal(s, full["state"])


@pytest.mark.gpu
def test_device_lake_reservoir_response_kat():
    _check_lake_reservoir("hip")


@pytest.mark.gpu
def test_pthpsk_synthetic_winter_to_melt_bitexact():
    n, T = 777, 24 * 120
    geo, f = _case(n, T)
    st = synthetic.default_pthpsk_state(n)
    p = synthetic.default_pthpsk_parameters()
    ref = engines.run_pthpsk("oracle", geo, p, st, synthetic.T0_2015_US, HOUR, f, collect_state=True)
    got = engines.run_pthpsk("hip", geo, p, st, synthetic.T0_2015_US, HOUR, f, collect_state=True)
    assert np.nanmax(ref["state_series"][2]) > 10.0  # snow did accumulate
    _assert_same(got, ref, ["full", "state", "state_series"])


@pytest.mark.gpu
def test_pthpsk_two_sets_custom_distribution_iso_bitexact():
    """Two ragged parameter sets: the default 5 bins and 8 even bins (all registers in use), iso_pot_energy
    and gm.direct_response on the second. (A snowpack handed in undistributed, or a skewed distribution, makes
    the reference's hbv_physical_snow throw "Negative outflow" -- see the next test.)"""
    n, T = 333, 24 * 40
    geo, f = _case(n, T, step0=24 * 50, seed=9)
    p0 = synthetic.default_pthpsk_parameters()
    p1 = p0.copy()
    p1[[0, 3, 5, 6, 7, 10, 15, 17]] = [-2.2, 1.2, 0.5, 0.3, 3.0, 0.85, 1.0, 1.1]  # c1 ae tx cfr wind max_alb iso p_corr
    i1 = list(np.linspace(0.0, 1.0, 8))
    d0 = oracle_lib.hbv_dist_row(oracle_lib.hbv_normalize(S5, A5), A5)
    d1 = oracle_lib.hbv_dist_row(oracle_lib.hbv_normalize([1.0] * 8, i1), i1)
    ix = (np.arange(n) * 7 % 3 == 0).astype(np.int32)
    st = synthetic.default_pthpsk_state(n, q=2.0)
    args = (geo, np.stack([p0, p1]), st, synthetic.T0_2015_US, HOUR, f)
    kw = dict(set_ix=ix, gm_direct=[0.0, 0.4], snow_dist=np.stack([d0, d1]), collect_state=True)
    ref = engines.run_pthpsk("oracle", *args, **kw)
    got = engines.run_pthpsk("hip", *args, **kw)
    assert np.nanmax(ref["state_series"][2]) > 10.0
    _assert_same(got, ref, ["full", "state", "state_series"])


@pytest.mark.gpu
def test_pthpsk_negative_outflow_raises_like_the_reference():
    from shyft_amd._native import ShyftHipError
    n, T = 64, 24 * 40
    geo, f = _case(n, T, step0=24 * 50, seed=9)
    i1 = [0.0, 0.2, 0.5, 0.8, 1.0]
    d = oracle_lib.hbv_dist_row(oracle_lib.hbv_normalize([0.5, 0.8, 1.0, 1.3, 1.5], i1), i1)
    st = synthetic.default_pthpsk_state(n, q=2.0)
    args = (geo, synthetic.default_pthpsk_parameters(), st, synthetic.T0_2015_US, HOUR, f)
    with pytest.raises(RuntimeError, match="Negative outflow"):
        engines.run_pthpsk("oracle", *args, snow_dist=d)
    with pytest.raises(ShyftHipError, match="Negative outflow"):
        engines.run_pthpsk("hip", *args, snow_dist=d)


@pytest.mark.gpu
def test_pthpsk_stepwise_equals_full_on_gpu():
    from shyft_amd.region import HipRegion, PT_HPS_K, COLLECT_ALL
    n, T = 256, 24 * 10
    geo, f = _case(n, T, step0=24 * 75)
    p = synthetic.default_pthpsk_parameters()
    st = synthetic.default_pthpsk_state(n)
    full = engines.run_pthpsk("hip", geo, p, st, synthetic.T0_2015_US, HOUR, f)
    r = HipRegion(PT_HPS_K, n)
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
def test_pthpsk_stale_bins_beyond_the_state_count_read_as_zero():
    """Slots nb..7 of the sp, sw, albedo and iso_pot_energy rows are padding and come back 0 (pthpsk.hpp state)."""
    n, T = 150, 24 * 20
    geo, f = _case(n, T, step0=24 * 60, seed=4)
    st = synthetic.default_pthpsk_state(n, q=2.0)
    st[:, 0:2] = 0.0
    st[:, 3] = 5.0
    st[:, 4:36] = 0.0
    stale = [c for b in (4, 12, 20, 28) for c in range(b + 5, b + 8)]
    st[:, stale] = 1.5
    args = (geo, synthetic.default_pthpsk_parameters(), st, synthetic.T0_2015_US, HOUR, f)
    ref = engines.run_pthpsk("oracle", *args)
    got = engines.run_pthpsk("hip", *args)
    _assert_same(got, ref, ["full", "state"])
    assert (got["state"][:, stale] == 0.0).all()
