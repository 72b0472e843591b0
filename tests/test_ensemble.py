"""Parameter ensembles (shyft_hip_ensemble_run): n_members parameter vectors evaluated in one launch must give,
member by member, exactly what the region gives when run alone with that parameter vector from the same state
(model_calibration.h:830-857: set parameters -> revert state -> run_cells -> catchment sums).

Parity bar: BIT-EXACT for the plain catchment sums (same kernel arithmetic per lane and the same fixed-order
reduction over each catchment's cells); area-weighted snow sums within 1e-13 relative of the per-cell series
reduced on the host (numpy summation order differs). The region's own state is left untouched."""
import numpy as np
import pytest

from shyft_amd import synthetic
from shyft_amd.region import (COLLECT_DISCHARGE, COLLECT_DISCHARGE_SNOW, HBV_STACK, PT_GS_K, PT_SS_K, HipRegion)

pytestmark = pytest.mark.gpu

HOUR = synthetic.HOUR_US


def _members(base, n, idx_scale, seed=11):
    """n perturbations of the base vector: parameter i scaled by U(1-s, 1+s) for (i, s) in idx_scale."""
    rng = np.random.default_rng(seed)
    p = np.tile(base, (n, 1))
    for i, s in idx_scale:
        p[1:, i] *= rng.uniform(1 - s, 1 + s, n - 1)  # member 0 keeps the base vector
    return p


def _region(stack, n_cells, n_steps, params, state, n_catchments=5):
    geo = synthetic.geo11(n_cells, n_catchments=n_catchments)
    r = HipRegion(stack, n_cells)
    r.set_geo(geo)
    r.set_parameters(np.atleast_2d(params))
    r.set_time_axis(synthetic.T0_2015_US, HOUR, n_steps)
    r.set_collection(COLLECT_DISCHARGE_SNOW)
    r.set_state(state)
    f = synthetic.forcing(n_cells, 0, n_steps)
    for v in range(5):
        r.set_forcing(v, 0, f[v])
    return r, geo


def _check(stack, base, state, idx_scale, n_cells=300, n_steps=24 * 40, n_members=6, filt=None, snow=True):
    r, geo = _region(stack, n_cells, n_steps, base, state)
    try:
        if filt is not None:
            r.set_catchment_filter(filt)
        members = _members(base, n_members, idx_scale)
        s0 = r.get_state().copy()
        r.ensemble_run(members, 0, 0, COLLECT_DISCHARGE_SNOW if snow else COLLECT_DISCHARGE)
        assert np.array_equal(r.get_state(), s0), "ensemble run modified the region state"
        q = r.ensemble_sums(0, 0, n_steps)
        charge = r.ensemble_sums(1, 0, n_steps)
        sca_w = r.ensemble_sums(2, 0, n_steps, area_weighted=True) if snow else None
        cids = r.catchment_ids()
        area = geo[:, 3]
        cell_cid = geo[:, 4].astype(np.int64)
        for m in range(n_members):
            r.set_parameters(members[m:m + 1])
            r.set_state(s0)
            r.run_cells(0, 0, 0)
            ref_q = r.catchment_sums(0, 0, n_steps)
            ref_c = r.catchment_sums(1, 0, n_steps)
            calc = np.array([filt is None or cid in filt for cid in cids])
            assert np.array_equal(q[m][calc], ref_q[calc]), f"member {m}: discharge sums differ"
            assert np.array_equal(charge[m][calc], ref_c[calc]), f"member {m}: charge sums differ"
            if snow:
                sca = r.get_series(2, 0, n_steps)
                for c, cid in enumerate(cids):
                    sel = cell_cid == cid
                    if filt is not None and cid not in filt:
                        assert np.all(sca_w[m, c] == 0.0)
                        continue
                    host = (sca[:, sel] * area[sel]).sum(axis=1)
                    np.testing.assert_allclose(sca_w[m, c], host, rtol=1e-13, atol=1e-9)
        if filt is not None:
            for c, cid in enumerate(cids):
                if cid not in filt:
                    assert np.all(q[:, c] == 0.0)
        # the members really differ (the ensemble is not n copies of one run)
        assert not np.array_equal(q[0], q[-1])
    finally:
        r.close()


def test_ensemble_ptgsk_bitexact():
    base = synthetic.default_ptgsk_parameters()
    # kirchner c1 c2, gs tx, snow_cv, p_corr, ae scale
    _check(PT_GS_K, base, synthetic.default_ptgsk_state(300), [(0, 0.2), (1, 0.05), (4, 0.5), (14, 0.3), (16, 0.2),
                                                                 (3, 0.3)])


def test_ensemble_ptgsk_filtered_discharge_only():
    base = synthetic.default_ptgsk_parameters()
    _check(PT_GS_K, base, synthetic.default_ptgsk_state(300), [(0, 0.2), (1, 0.05)], n_members=3, filt=[2, 4],
           snow=False)


def test_ensemble_hbv_bitexact():
    base = synthetic.default_hbv_parameters()
    _check(HBV_STACK, base, synthetic.default_hbv_state(300), [(0, 0.3), (1, 0.3), (3, 0.3), (7, 0.5)], n_members=4,
           n_steps=24 * 20)


def test_ensemble_ptssk_bitexact():
    base = synthetic.default_ptssk_parameters()
    _check(PT_SS_K, base, synthetic.default_ptssk_state(200), [(0, 0.2), (1, 0.05), (8, 0.5)], n_cells=200,
           n_members=4, n_steps=24 * 20)


def test_ensemble_errors():
    base = synthetic.default_ptgsk_parameters()
    r, _ = _region(PT_GS_K, 10, 48, base, synthetic.default_ptgsk_state(10))
    try:
        with pytest.raises(RuntimeError, match="no ensemble run"):
            r.ens_members = 1
            r.ensemble_sums(0, 0, 48)
        with pytest.raises(RuntimeError, match="size missmatch"):
            r.ensemble_run(np.zeros((2, 5)))
        with pytest.raises(RuntimeError, match="outside"):
            r.ensemble_run(np.tile(base, (2, 1)), 40, 20)
        r.ensemble_run(np.tile(base, (2, 1)), 10, 20, COLLECT_DISCHARGE)
        with pytest.raises(RuntimeError, match="outside the last ensemble run"):
            r.ensemble_sums(0, 0, 20)
        with pytest.raises(RuntimeError, match="not collected"):
            r.ensemble_sums(2, 10, 20)
        assert r.ensemble_sums(0, 10, 20).shape == (2, r.number_of_catchments(), 20)
    finally:
        r.close()
