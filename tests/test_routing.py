"""routing::uhg river aggregation (core/routing.h:239-421, region_model.h:909-949).

CPU: the oracle's UHG (make_uhg_from_gamma with a restated gamma quantile/pdf) against
scipy and against the host layer's UHG; the oracle reproduces the reference's river KAT
out(8) = 28.06 of test_region_model_stacks.py:287-301 on the oracle region run.
GPU: the engine's (river, UHG)-group sums + level-wise device convolution against the
oracle's literal per-cell convolution on a 4-river network with several UHGs per river
(tolerance 1e-12 relative: the engine adds the same terms in a different order)."""
import numpy as np
import pytest

from shyft_amd import synthetic
from tests import oracle_lib

HOUR = synthetic.HOUR_US


def test_oracle_uhg_vs_scipy_and_host():
    ss = pytest.importorskip("scipy.stats")
    from shyft_amd import api
    for n, a, b in [(3, 7.0, 0.0), (12, 2.5, 0.0), (30, 7.0, 0.005), (2, 1.2, 0.0), (1, 7.0, 0.0)]:
        w = oracle_lib.make_uhg(n, a, b)
        if n > 1:
            x = np.arange(n) * ss.gamma(a).ppf(0.99) / n
            y = np.maximum(0.0, ss.gamma(a).pdf(x) + b)
            assert np.allclose(w, y / y.sum(), rtol=1e-12, atol=1e-15)
        assert np.allclose(w, api.make_uhg_from_gamma(n, a, b), rtol=1e-13, atol=1e-16)


def test_oracle_river_kat():
    """test_region_model_stacks.py:287-301: river 1 (3000 m, 1/3.6 m/s, alpha 7), all cells routed to it
    with routing distance 0: river_output_flow_m3s(1).value(8) == 28.06 (0 decimals)."""
    from tests.test_region_kat import run_ptgsk
    r = run_ptgsk("oracle")
    q = r["main"][0]  # [T][N] avg_discharge
    N = q.shape[1]
    vab = np.tile([1.0, 7.0, 0.0], (N, 1))  # PTGSKParameter().routing
    local, up, out = oracle_lib.route(q, HOUR, np.ones(N, np.int64), np.zeros(N), vab, [(1, 0, 3000.0, 1 / 3.6, 7.0, 0.0)], 1)
    assert abs(out[8] - 28.061248025828114) < 0.5
    assert np.allclose(local, q.sum(axis=1), rtol=1e-14)
    assert np.all(up == 0.0)


RIVERS = [(1, 0, 8000.0, 1.0, 3.0, 0.0), (2, 1, 20000.0, 1.5, 7.0, 0.0), (3, 1, 3000.0, 0.5, 5.0, 0.001),
          (4, 2, 6000.0, 2.0, 2.0, 0.0)]


@pytest.mark.gpu
def test_device_routing_matches_oracle_network():
    from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_DISCHARGE, route
    from shyft_amd import api
    n, T = 3000, 24 * 20
    geo = synthetic.geo11(n, n_catchments=8)
    p0 = synthetic.default_ptgsk_parameters()
    p1 = p0.copy()
    p1[25:28] = (0.7, 4.0, 0.0)  # routing velocity alpha beta of the second set
    ix = (np.arange(n) % 5 == 0).astype(np.int32)
    rng = np.random.default_rng(11)
    cell_rid = 1 + (geo[:, 4].astype(np.int64) - 1) % 4          # catchment -> river 1..4
    cell_rid[rng.random(n) < 0.05] = 0                             # some cells not routed
    cell_dist = rng.choice([0.0, 1500.0, 5000.0, 12000.0], n)
    r = HipRegion(PT_GS_K, n)
    r.set_geo(geo)
    r.set_parameters(np.stack([p0, p1]), ix)
    r.set_time_axis(synthetic.T0_2015_US, HOUR, T)
    r.set_collection(COLLECT_DISCHARGE)
    r.set_state(synthetic.default_ptgsk_state(n))
    r.synthetic_forcing(synthetic.SEED, 0, T)
    r.run_cells()
    q = r.get_series(0, 0, T)
    # groups: (river, uhg steps, alpha, beta)
    params = np.stack([p0, p1])
    keys, group_of, group_uhgs, group_river = {}, np.full(n, -1, np.int32), [], []
    for i in range(n):
        if cell_rid[i] <= 0:
            continue
        v, a, b = params[ix[i], 25:28]
        steps = int((cell_dist[i] / v) / 3600.0 + 0.5)
        k = (cell_rid[i], steps, a, b)
        if k not in keys:
            keys[k] = len(group_uhgs)
            group_uhgs.append(api.make_uhg_from_gamma(steps, a, b))
            group_river.append(cell_rid[i] - 1)
        group_of[i] = keys[k]
    r.set_routing_groups(group_of, len(group_uhgs))
    sums = r.routing_group_sums(0, T)
    river_uhgs = [api.make_uhg_from_gamma(int((d / v) / 3600.0 + 0.5), a, b) for (_, _, d, v, a, b) in RIVERS]
    river_down = [ds - 1 for (_, ds, *_rest) in RIVERS]
    local, up, out = route(sums, group_uhgs, group_river, river_uhgs, river_down)
    vab = params[ix, 25:28]
    for k, (rid, *_rest) in enumerate(RIVERS):
        ol, ou, oo = oracle_lib.route(q, HOUR, cell_rid, cell_dist, vab, RIVERS, rid)
        assert np.allclose(local[k], ol, rtol=1e-12, atol=1e-12), rid
        assert np.allclose(up[k], ou, rtol=1e-12, atol=1e-12), rid
        assert np.allclose(out[k], oo, rtol=1e-12, atol=1e-12), rid
    assert out[0].sum() > 0 and up[0].sum() > 0
