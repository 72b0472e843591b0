"""hbv_stack: the HIP kernel against the CPU oracle, bit for bit.

Both sides evaluate the same expressions in the same order (contraction off)
with the same deterministic pow/exp (detmath), so every response series, the
state series and the end state must be identical. Cases: the synthetic region
over a winter and the spring melt, a user snow distribution with 7 bins, two
ragged parameter sets, pre-distributed states, stepwise == full, the
catchment calculation filter."""
import numpy as np
import pytest

from shyft_amd import synthetic
from tests import engines, oracle_lib

HOUR = synthetic.HOUR_US


def _case(n, T, step0=0, seed=3):
    geo = synthetic.geo11(n, n_catchments=4)
    rng = np.random.default_rng(seed)
    geo[:, 6] = rng.choice([0.0, 0.05, 0.3], n)      # glacier
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
    st = synthetic.default_hbv_state(n)
    p = synthetic.default_hbv_parameters()
    full = oracle_lib.hbv_run(geo, p, st, synthetic.T0_2015_US, HOUR, f, full=True)
    s = st.copy()
    out = np.full_like(full["full"], np.nan)
    for k in range(4):
        r = oracle_lib.hbv_run(geo, p, s, synthetic.T0_2015_US, HOUR, f, 24 * k, 24, full=True)
        out[:, 24 * k:24 * (k + 1)] = r["full"][:, 24 * k:24 * (k + 1)]
        s = r["state"]
    assert np.array_equal(out, full["full"])
    assert np.array_equal(s, full["state"])


@pytest.mark.gpu
def test_hbv_synthetic_winter_to_melt_bitexact():
    n, T = 777, 24 * 120  # Jan 1 .. Apr 30: snow build-up, melt season
    geo, f = _case(n, T)
    st = synthetic.default_hbv_state(n)
    p = synthetic.default_hbv_parameters()
    ref = engines.run_hbv("oracle", geo, p, st, synthetic.T0_2015_US, HOUR, f, collect_state=True)
    got = engines.run_hbv("hip", geo, p, st, synthetic.T0_2015_US, HOUR, f, collect_state=True)
    assert np.nanmax(ref["state_series"][0]) > 10.0  # snow did accumulate
    _assert_same(got, ref, ["full", "state", "state_series"])
    # the discharge collector alone (no state series, one 5-bin parameter set): the LEAN kernel instance
    lean = engines.run_hbv("hip", geo, p, st, synthetic.T0_2015_US, HOUR, f, full=False)
    _assert_same(lean, ref, ["main", "state"])


@pytest.mark.gpu
@pytest.mark.parametrize("s1,i1,predistributed", [
    ([1.0] * 8, list(np.linspace(0.0, 1.0, 8)), True),                   # 8 bins (all registers in use)
    ([0.5, 0.8, 1.0, 1.3, 1.5], [0.0, 0.2, 0.5, 0.8, 1.0], False),       # skewed 5-bin distribution
])
def test_hbv_custom_distribution_two_sets_bitexact(s1, i1, predistributed):
    """(Several skewed distributions make hbv_snow throw "Negative outflow" in the reference
    itself, see the next test; these two run clean.)"""
    n, T = 333, 24 * 40
    geo, f = _case(n, T, step0=24 * 50, seed=9)  # late Feb - early Apr
    p0 = synthetic.default_hbv_parameters()
    p1 = p0.copy()
    p1[[0, 1, 2, 9, 10, 12, 13]] = [250.0, 1.7, 120.0, 0.5, 2.5, 0.3, 1.1]  # fc beta lp tx cx cfr p_corr
    d0 = oracle_lib.hbv_dist_row([1.0, 1.0, 1.0, 1.0, 1.0], [0.0, 0.25, 0.5, 0.75, 1.0])
    d1 = oracle_lib.hbv_dist_row(oracle_lib.hbv_normalize(s1, i1), i1)
    ix = (np.arange(n) * 7 % 3 == 0).astype(np.int32)  # ragged interleave of the two sets
    st = synthetic.default_hbv_state(n)
    st[:, 0], st[:, 1] = 60.0, 0.8  # undistributed swe/sca: distributed at run start
    if predistributed:
        st[::5, 5] = 5.0            # some cells claim 5 distributed (all-zero) bins: kept unless the count differs
    args = (geo, np.stack([p0, p1]), st, synthetic.T0_2015_US, HOUR, f)
    ref = engines.run_hbv("oracle", *args, set_ix=ix, snow_dist=np.stack([d0, d1]), collect_state=True)
    got = engines.run_hbv("hip", *args, set_ix=ix, snow_dist=np.stack([d0, d1]), collect_state=True)
    _assert_same(got, ref, ["full", "state", "state_series"])


@pytest.mark.gpu
def test_hbv_five_bin_kernel_keeps_and_clears_upper_bins_like_the_oracle():
    """One parameter set with the default 5 bins and no state series runs the 5-bin kernel instance: state bins 5..7
    must come out as the oracle's padded state vector: zero, whether the bins were redistributed or kept."""
    n, T = 300, 24 * 30
    geo, f = _case(n, T, step0=24 * 60, seed=5)
    p = synthetic.default_hbv_parameters()
    st = synthetic.default_hbv_state(n)
    st[:, 0], st[:, 1] = 40.0, 0.9
    st[::3, 5] = 8.0                    # claims 8 bins: redistributed to 5, bins 5..7 cleared
    st[::3, 6:22] = 2.5
    st[1::3, 0:2] = 0.0                 # snow-free, 5 distributed (empty) bins kept; stale bins 5..7
    st[1::3, 5] = 5.0
    st[1::3, 6:22] = 0.0
    st[1::3, 11:14] = st[1::3, 19:22] = 1.5
    ref = engines.run_hbv("oracle", geo, p, st, synthetic.T0_2015_US, HOUR, f)
    got = engines.run_hbv("hip", geo, p, st, synthetic.T0_2015_US, HOUR, f)
    _assert_same(got, ref, ["full", "state"])
    assert (got["state"][:, [11, 12, 13, 19, 20, 21]] == 0.0).all()
    got8 = engines.run_hbv("hip", geo, p, st, synthetic.T0_2015_US, HOUR, f, collect_state=True)  # 8-bin instance
    _assert_same(got8, ref, ["full", "state"])


@pytest.mark.gpu
def test_hbv_stepwise_equals_full_on_gpu():
    from shyft_amd.region import HipRegion, HBV_STACK, COLLECT_ALL
    n, T = 256, 24 * 10
    geo, f = _case(n, T, step0=24 * 75)
    p = synthetic.default_hbv_parameters()
    st = synthetic.default_hbv_state(n)
    full = engines.run_hbv("hip", geo, p, st, synthetic.T0_2015_US, HOUR, f)
    r = HipRegion(HBV_STACK, n)
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
        got = np.stack([r.get_series(k, 0, T) for k in range(9)])
        assert np.array_equal(got, full["full"])
        assert np.array_equal(r.get_state(), full["state"])
    finally:
        r.close()


@pytest.mark.gpu
def test_hbv_catchment_filter_runs_only_selected_cells():
    from shyft_amd.region import HipRegion, HBV_STACK, COLLECT_DISCHARGE
    n, T = 200, 48
    geo, f = _case(n, T)
    r = HipRegion(HBV_STACK, n)
    try:
        r.set_geo(geo)
        r.set_parameters(synthetic.default_hbv_parameters())
        r.set_time_axis(synthetic.T0_2015_US, HOUR, T)
        r.set_collection(COLLECT_DISCHARGE)
        r.set_state(synthetic.default_hbv_state(n))
        for v in range(5):
            r.set_forcing(v, 0, f[v])
        cid = int(geo[0, 4])
        r.set_catchment_filter([cid])
        r.run_cells()
        q = r.get_series(0, 0, T)
        sel = geo[:, 4] == cid
        assert np.isfinite(q[:, sel]).all() and np.isnan(q[:, ~sel]).all()
        ref = engines.run_hbv("oracle", geo[sel], synthetic.default_hbv_parameters(),
                              synthetic.default_hbv_state(int(sel.sum())), synthetic.T0_2015_US, HOUR, f[:, :, sel])
        assert np.array_equal(q[:, sel], ref["main"][0])
    finally:
        r.close()


@pytest.mark.gpu
def test_hbv_negative_outflow_raises_like_the_reference():
    """An un-normalised distribution (mean > 1) makes the bins hold more water than fell:
    hbv_snow::step throws "Negative outflow" (hbv_snow.h:259-263); run_cells must fail too."""
    from shyft_amd._native import ShyftHipError
    n, T = 64, 24 * 30
    geo, f = _case(n, T, step0=24 * 20)
    p = synthetic.default_hbv_parameters()
    d = oracle_lib.hbv_dist_row([1.0, 1.0, 3.0, 3.0, 3.0], [0.0, 0.25, 0.5, 0.75, 1.0])
    st = synthetic.default_hbv_state(n)
    st[:, 0], st[:, 1] = 60.0, 0.8
    with pytest.raises(RuntimeError, match="Negative outflow"):
        engines.run_hbv("oracle", geo, p, st, synthetic.T0_2015_US, HOUR, f, snow_dist=d)
    with pytest.raises(ShyftHipError, match="Negative outflow"):
        engines.run_hbv("hip", geo, p, st, synthetic.T0_2015_US, HOUR, f, snow_dist=d)
