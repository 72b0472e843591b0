"""pt_ss_k (Skaugen snow): the HIP kernel against the CPU oracle, bit for bit.

Both sides evaluate Skaugen's routine (core/skaugen.h) with the same expressions in
the same order, unsigned 64-bit unit counts, half-even lrint and the same detmath
gamma pdf/cdf, so every response series, the state-collector series and the end
state must be identical. The cases run the synthetic region from Jan 1 through the
spring melt, where partial melts send lanes through sca_rel_red (Brent + bisection
on two gamma densities); 0 < sca < 1 in the collected state shows that path ran."""
import numpy as np
import pytest

from shyft_amd import synthetic
from tests import engines, oracle_lib

HOUR = synthetic.HOUR_US


def _case(n, T, step0=0, seed=5):
    geo = synthetic.geo11(n, n_catchments=4)
    rng = np.random.default_rng(seed)
    geo[:, 6] = rng.choice([0.0, 0.05, 0.3], n)   # glacier
    geo[:, 7] = rng.choice([0.0, 0.05], n)        # lake
    geo[:, 8] = rng.choice([0.0, 0.19], n)        # reservoir
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
    geo, f = _case(n, T, step0=24 * 90)
    st = synthetic.default_ptssk_state(n)
    p = synthetic.default_ptssk_parameters()
    full = oracle_lib.ptssk_run(geo, p, st, synthetic.T0_2015_US, HOUR, f, full=True)
    s = st.copy()
    out = np.full_like(full["full"], np.nan)
    for k in range(4):
        r = oracle_lib.ptssk_run(geo, p, s, synthetic.T0_2015_US, HOUR, f, 24 * k, 24, full=True)
        out[:, 24 * k:24 * (k + 1)] = r["full"][:, 24 * k:24 * (k + 1)]
        s = r["state"]
    assert np.array_equal(out, full["full"])
    assert np.array_equal(s, full["state"])


def test_oracle_partial_melt_path_and_libm_distance():
    """The winter-to-melt case reaches partial snow cover (the sca_rel_red path), and the oracle built with
    the host libm (as the reference) stays close to the detmath build on the yearly discharge."""
    n, T = 64, 24 * 150
    geo, f = _case(n, T)
    st = synthetic.default_ptssk_state(n)
    p = synthetic.default_ptssk_parameters()
    a = oracle_lib.ptssk_run(geo, p, st, synthetic.T0_2015_US, HOUR, f, full=True, collect_state=True)
    sca = a["state_series"][1]
    assert ((sca > 0.0) & (sca < 1.0)).sum() > 100
    b = oracle_lib.ptssk_run(geo, p, st, synthetic.T0_2015_US, HOUR, f, full=True, variant="libm")
    qa, qb = a["main"][0].sum(axis=0), b["main"][0].sum(axis=0)
    assert np.allclose(qa, qb, rtol=1e-3), np.max(np.abs(qa / qb - 1))


@pytest.mark.gpu
def test_ptssk_winter_to_melt_bitexact():
    n, T = 777, 24 * 150  # Jan 1 .. May 30: accumulation, partial melts, melt-out
    geo, f = _case(n, T)
    st = synthetic.default_ptssk_state(n)
    p = synthetic.default_ptssk_parameters()
    ref = engines.run_ptssk("oracle", geo, p, st, synthetic.T0_2015_US, HOUR, f, collect_state=True)
    got = engines.run_ptssk("hip", geo, p, st, synthetic.T0_2015_US, HOUR, f, collect_state=True)
    _assert_same(ref, got, ("full", "state", "state_series"))
    sca = ref["state_series"][1]
    assert ((sca > 0.0) & (sca < 1.0)).sum() > 1000


@pytest.mark.gpu
def test_ptssk_ragged_parameter_sets_and_stepwise():
    n, T = 333, 24 * 20
    geo, f = _case(n, T, step0=24 * 95, seed=9)
    st = synthetic.default_ptssk_state(n)
    p0 = synthetic.default_ptssk_parameters()
    p1 = p0.copy()
    p1[6] = 0.2     # ss.unit_size
    p1[9] = 3.5     # ss.cx
    p1[20] = 0.3    # msp.reservoir_direct_response_fraction
    p1[19] = 0.5    # gm.direct_response
    ix = (np.arange(n) % 3 == 0).astype(np.int32)
    params = np.stack([p0, p1])
    ref = engines.run_ptssk("oracle", geo, params, st, synthetic.T0_2015_US, HOUR, f, set_ix=ix, collect_state=True)
    got = engines.run_ptssk("hip", geo, params, st, synthetic.T0_2015_US, HOUR, f, set_ix=ix, collect_state=True)
    _assert_same(ref, got, ("full", "state", "state_series"))
    # a partial run (start_step, n_steps) on both engines
    ref = engines.run_ptssk("oracle", geo, params, st, synthetic.T0_2015_US, HOUR, f, 48, 100, set_ix=ix)
    got = engines.run_ptssk("hip", geo, params, st, synthetic.T0_2015_US, HOUR, f, 48, 100, set_ix=ix)
    _assert_same(ref, got, ("full", "state"))


@pytest.mark.gpu
def test_ptssk_odd_start_step_and_single_steps_in_melt():
    """run_cells from an ODD start_step and one step at a time in April (partial melts queue sca_rel_red
    jobs): the rotating job counters start at zero whatever the first step."""
    n, T = 300, 24 * 4
    step0 = 24 * 100
    geo, f = _case(n, T, step0=step0, seed=11)
    st = synthetic.default_ptssk_state(n)
    p = synthetic.default_ptssk_parameters()
    # a snow pack to melt: run the oracle through the winter first
    geo_w, f_w = _case(n, step0, seed=11)
    st = oracle_lib.ptssk_run(geo_w, p, st, synthetic.T0_2015_US, HOUR, f_w, full=False)["state"]
    t0 = synthetic.T0_2015_US + step0 * HOUR
    ref = engines.run_ptssk("oracle", geo, p, st, t0, HOUR, f, 13, 59, collect_state=False)
    got = engines.run_ptssk("hip", geo, p, st, t0, HOUR, f, 13, 59, collect_state=False)
    assert np.array_equal(ref["full"][:, 13:72], got["full"][:, 13:72])
    assert np.array_equal(ref["state"], got["state"])
    from shyft_amd.region import HipRegion, PT_SS_K, COLLECT_ALL
    r = HipRegion(PT_SS_K, n)
    try:
        r.set_geo(geo)
        r.set_parameters(np.atleast_2d(p))
        r.set_time_axis(t0, HOUR, T)
        r.set_collection(COLLECT_ALL)
        r.set_state(st)
        for v in range(5):
            r.set_forcing(v, 0, f[v])
        for i in range(13, 72):
            r.run_cells(0, i, 1)
        s = np.stack([r.get_series(k, 13, 59) for k in range(8)])
        assert np.array_equal(s, ref["full"][:, 13:72])
        assert np.array_equal(r.get_state(), ref["state"])
    finally:
        r.close()


@pytest.mark.gpu
def test_ptssk_year_every_job_group_size_bitexact():
    """A whole year (spring and autumn melts) of 2048 cells: steps with a few sca_rel_red jobs per workgroup give each
    job a group of 4 or 2 lanes (grouped lgammas, opening evaluations, cdfs, and 2 bisection levels per round), busy
    steps one lane per job, and the bisection takes its midpoints' signs without the pdf divisions where they are
    certain (device/ptssk_dev.h). Every series and the end state must equal the oracle's."""
    n, T = 2048, 8760
    geo, f = _case(n, T, seed=13)
    st = synthetic.default_ptssk_state(n)
    p = synthetic.default_ptssk_parameters()
    ref = engines.run_ptssk("oracle", geo, p, st, synthetic.T0_2015_US, HOUR, f)
    got = engines.run_ptssk("hip", geo, p, st, synthetic.T0_2015_US, HOUR, f)
    _assert_same(ref, got, ("full", "state"))
    swe = ref["full"][3]
    autumn = slice(24 * 243, 24 * 334)   # Sep - Nov: few partial melts per step
    assert (swe[autumn] > 0).any() and (swe[:24 * 150] > 0).any()
