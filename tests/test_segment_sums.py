"""Catchment and routing-group sums (region_model::catchment_discharges, core/region_model.h:873-885; routing.h's
per-group local inflow) bit for bit against a numpy restatement of the device reduction order: each of the 256 lanes
of a workgroup sums its cells k = b + lane, b + lane + 256, ... in order, then a 64-lane xor butterfly per wavefront
and the four wavefront partials added in order (kernels/stats.hip). Both index paths are covered: segments that are
the identity permutation (catchments as contiguous cell ranges: the index array is not read) and interleaved ones."""
import numpy as np
import pytest

from shyft_amd import synthetic

pytestmark = pytest.mark.gpu

RB = 256


def device_order_sum(vals):
    """The segment-sum kernel's reduction of one segment's values (in segment order)."""
    acc = [0.0] * RB
    for k, v in enumerate(vals.tolist()):
        acc[k % RB] += v
    w = np.array(acc).reshape(RB // 64, 64)
    lanes = np.arange(64)
    off = 32
    while off:
        w = w + w[:, lanes ^ off]
        off >>= 1
    part = w[:, 0]
    r = part[0]
    for p in part[1:]:
        r = r + p
    return r


def expected(series, groups, order):
    """[group][step] sums; groups[i] = the group of cell i; order = the groups in output order."""
    out = np.empty((len(order), series.shape[0]))
    for gi, g in enumerate(order):
        cells = np.flatnonzero(groups == g)  # segment order: cell order
        for t in range(series.shape[0]):
            out[gi, t] = device_order_sum(series[t, cells])
    return out


@pytest.fixture(scope="module", params=["contiguous", "interleaved"])
def region(request):
    from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_DISCHARGE
    n, T = 4099, 36
    geo = synthetic.geo11(n, n_catchments=3)
    if request.param == "interleaved":
        geo[:, 4] = np.random.default_rng(5).choice([3, 1, 2], n)
    r = HipRegion(PT_GS_K, n)
    r.set_geo(geo)
    r.set_parameters(synthetic.default_ptgsk_parameters())
    r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, T)
    r.set_collection(COLLECT_DISCHARGE)
    r.set_state(synthetic.default_ptgsk_state(n))
    r.synthetic_forcing(synthetic.SEED, 0, T)
    r.run_cells()
    yield r, geo, r.get_series(0, 0, T), request.param
    r.close()


def test_catchment_sums_bit_exact_in_device_order(region):
    r, geo, series, _ = region
    got = r.catchment_sums(0, 0, series.shape[0])
    want = expected(series, geo[:, 4].astype(int), [int(c) for c in r.catchment_ids()])
    assert np.array_equal(got, want)


def test_routing_group_sums_bit_exact_in_device_order(region):
    r, geo, series, layout = region
    n = len(geo)
    if layout == "contiguous":
        groups = (np.arange(n) * 4) // n          # every cell in a group, ranges in cell order: the identity
    else:
        groups = np.random.default_rng(9).integers(-1, 4, n)   # interleaved, some cells routed nowhere
    r.set_routing_groups(groups, 4)
    got = r.routing_group_sums(0, series.shape[0])
    assert np.array_equal(got, expected(series, groups, [0, 1, 2, 3]))
