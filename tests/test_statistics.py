"""Catchment statistics on the GPU (cell_statistics, core/cell_model.h:194-406;
region_model::catchment_discharges, core/region_model.h:873-885) against numpy
sums over the same per-cell series. The GPU reduces in a fixed tree order,
the reference sums sequentially in cell order: tolerance 1e-13 relative."""
import numpy as np
import pytest

from shyft_amd import synthetic
from shyft_amd._native import ShyftHipError

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def run():
    from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_ALL
    n, T = 333, 120
    geo = synthetic.geo11(n, n_catchments=3)
    rng = np.random.default_rng(2)
    geo[:, 4] = rng.choice([7, 11, 42], n)      # interleaved catchments, first-appearance order
    geo[:, 3] = rng.uniform(0.5e6, 2e6, n)       # unequal areas for the weighted averages
    f = synthetic.forcing(n, 4000, T)
    r = HipRegion(PT_GS_K, n)
    r.set_geo(geo)
    r.set_parameters(synthetic.default_ptgsk_parameters())
    r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, T)
    r.set_collection(COLLECT_ALL)
    r.set_state(synthetic.default_ptgsk_state(n))
    for v in range(5):
        r.set_forcing(v, 0, f[v])
    r.run_cells()
    series = np.stack([r.get_series(k, 0, T) for k in range(8)])
    yield r, geo, series
    r.close()


def _close(a, b):
    return np.allclose(a, b, rtol=1e-13, atol=1e-13 * np.abs(b).max())


def test_catchment_ids_first_appearance_order(run):
    r, geo, _ = run
    cids = []
    for c in geo[:, 4].astype(int):
        if c not in cids:
            cids.append(c)
    assert list(r.catchment_ids()) == cids
    assert r.number_of_catchments() == 3


def test_sum_and_average_by_catchment(run):
    from shyft_amd.region import SCOPE_CATCHMENT
    r, geo, series = run
    for ids in ([], [7], [11, 42], [42, 7, 11]):
        sel = np.isin(geo[:, 4], ids) if ids else np.ones(len(geo), bool)
        got = r.statistics(0, ids, SCOPE_CATCHMENT)
        assert _close(got, series[0][:, sel].sum(axis=1))
        w = geo[sel, 3]
        got = r.statistics(2, ids, SCOPE_CATCHMENT, weighted=True)
        assert _close(got, (series[2][:, sel] * w).sum(axis=1) * (1 / w.sum()))


def test_sum_by_cell_index(run):
    from shyft_amd.region import SCOPE_CELL_IX
    r, geo, series = run
    got = r.statistics(1, [0, 1, 3], SCOPE_CELL_IX, step0=5, n=10)
    assert _close(got, series[1][5:15, [0, 1, 3]].sum(axis=1))


def test_unknown_ids_raise_like_the_reference(run):
    from shyft_amd.region import SCOPE_CATCHMENT, SCOPE_CELL_IX
    r, _, _ = run
    with pytest.raises(ShyftHipError, match="one or more supplied catchment_indexes does not exist:3"):
        r.statistics(0, [7, 3], SCOPE_CATCHMENT)
    with pytest.raises(ShyftHipError, match="is ouside valid range"):
        r.statistics(0, [10_000], SCOPE_CELL_IX)


def test_catchment_sums_all_catchments(run):
    r, geo, series = run
    got = r.catchment_sums(0, 0, series.shape[1])
    for row, c in zip(got, r.catchment_ids()):
        assert _close(row, series[0][:, geo[:, 4] == c].sum(axis=1))


def test_catchment_sums_torch_device_single_rank(run):
    import torch
    from shyft_amd import distributed
    r, geo, series = run
    cids = sorted(int(c) for c in r.catchment_ids())
    tot = distributed.catchment_sums(r, 0, 0, series.shape[1], cids, device=torch.device("cuda", 0)).cpu().numpy()
    for row, c in zip(tot, cids):
        assert _close(row, series[0][:, geo[:, 4] == c].sum(axis=1))
