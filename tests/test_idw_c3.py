"""BASELINE configs[2] (C3) parity: inverse-distance interpolation from S = 500 stations, and the chained
IDW -> pt_gs_k run, device against the oracle, bit for bit.

Two gather kernels exist and every test asserts which one ran (shyft_hip_interpolation_path):
- the wavefront-union gather, taken when every wavefront's 64 cells draw their neighbours from at most 64
  stations. On the C3 station grid (45 km spacing scaled to the region) that holds from ~65K grid-ordered cells
  up (the bench's 1M-cell region: unions of 26-30), not at 1500 cells, where a wavefront spans 1.7 grid rows of a
  39 km wide region and its union covers most of the 500 stations;
- the row-tile gather (SHYFT_IDW_TILE=1 forces it; a region whose unions overflow falls back to it). At 500
  stations the temperature tile holds 5 rows (32 KB budget minus the station coordinates), so a 730-row chunk runs
  ~146 tiles with their barriers and per-tile finite-row flags. Above ~1365 sources a row set no longer fits and
  the kernel reads rows from global memory (lds_rows = 0); the reference's own 70 x 70 = 4900-source scenario
  (test/inverse_distance_test.cpp:396-450, "test_performance") covers that path.
"""
import math
import os
import sys

import numpy as np
import pytest

from tests.test_idw import IDW_PARAMS, oracle_idw

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HOUR = 3600 * 10**6


def c3_region(n_cells, rows, step0=0, nan_frac=0.03, seed=11):
    """The bench's C3 layout scaled to n_cells: synthetic grid cells, 500 stations on the 22 x 23 grid
    covering the region (bench.station_network), station values from the device generator's host twin
    (bench.station_values), plus missing observations in a random subset of the rows."""
    import bench
    from shyft_amd import synthetic
    geo = synthetic.geo11(n_cells)
    xyz = bench.station_network(n_cells)
    vals = bench.station_values(xyz, step0, rows)                   # [5][rows][S]
    rng = np.random.default_rng(seed)
    bad_rows = rng.uniform(size=rows) < 0.2
    miss = (rng.uniform(size=vals.shape) < nan_frac) & bad_rows[None, :, None]
    vals = np.where(miss, np.nan, vals)
    return geo, xyz, vals


def _device_interpolate(geo, xyz, vals, var, prm, splits, path=None):
    """Interpolate var over the rows of vals in the calls [0, s1), [s1, s2), ... on a fresh region; `path`, if
    given, is the gather every call must have run ("wave" / "tile")."""
    from shyft_amd import synthetic
    from shyft_amd.region import HipRegion, PT_GS_K
    T, N = vals.shape[0], geo.shape[0]
    r = HipRegion(PT_GS_K, N)
    try:
        r.set_geo(geo)
        r.set_parameters(synthetic.default_ptgsk_parameters())
        r.set_time_axis(synthetic.T0_2015_US, HOUR, T)
        assert r.interpolation_path(var) == "none"
        b = 0
        for e in list(splits) + [T]:
            r.interpolate(var, xyz, vals[b:e], b, prm)
            if path is not None:
                assert r.interpolation_path(var) == path, f"rows [{b},{e}): ran {r.interpolation_path(var)}"
            b = e
        return r.get_forcing(var, 0, T)
    finally:
        r.close()


def _same(got, exp):
    same = (got == exp) | (np.isnan(got) & np.isnan(exp))
    return same.all(), f"{(~same).sum()} of {same.size} differ; max abs {np.nanmax(np.abs(got - exp))}"


C3_PARAMS = {   # bench.IDW_DEFAULTS (inverse_distance.h:38-74 defaults) per forcing variable
    0: [20, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],
    1: [20, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],
    2: [10, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],
    3: [10, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],
    4: [10, 200000.0, 2.0, 1.0, -0.006, 0.0, 1.02],
}


def test_c3_station_network_shape():
    """The test region is the bench's: 500 stations, values from the same generator, NaNs only where planted."""
    geo, xyz, vals = c3_region(1500, 50)
    assert xyz.shape == (500, 3) and vals.shape == (5, 50, 500)
    assert xyz[:, 0].max() == pytest.approx(math.ceil(math.sqrt(1500)) * 1000.0)
    assert np.isnan(vals).any() and np.isfinite(vals).mean() > 0.99


def _wave_unions(geo, xyz, K, max_distance=200000.0):
    """numpy restatement of the neighbour selection (distance order; the C3 case has no weight ties that could
    reorder members) -> the size of each 64-cell wavefront's station union."""
    d2 = ((geo[:, None, 0] - xyz[None, :, 0]) ** 2 + (geo[:, None, 1] - xyz[None, :, 1]) ** 2 +
          (geo[:, None, 2] - xyz[None, :, 2]) ** 2)
    d2 = np.where(d2 <= max_distance ** 2, d2, np.inf)
    nb = np.argsort(d2, axis=1, kind="stable")[:, :K]
    return [np.unique(nb[b:b + 64]).size for b in range(0, geo.shape[0], 64)]


# C3 parity regions: 1500 cells (every wavefront union overflows 64 stations -> row tiles) and 65,536 cells (the
# largest union is ~52 -> the wavefront-union gather), both with the bench's station grid scaled to the region
C3_TILE_CELLS, C3_WAVE_CELLS = 1500, 1 << 16
C3_ROWS = 730


def test_c3_wave_union_geometry():
    """The two test regions are on the intended side of the 64-station limit (checked on the host, the same
    neighbour rule as the kernels): at 65,536 grid-ordered cells every union of K = 20 fits, at 1500 cells
    none does -- so the device assertions on the path below test what they claim to test."""
    g, x, _ = c3_region(C3_WAVE_CELLS, 1)
    sel = np.arange(0, C3_WAVE_CELLS, 97 * 64)          # every 97th wavefront (the full 65K x 500 distance
    rows = np.concatenate([np.arange(b, b + 64) for b in sel])   # matrix is 0.26 GB)
    assert max(_wave_unions(g[rows], x, 20)) <= 64
    g, x, _ = c3_region(C3_TILE_CELLS, 1)
    assert min(_wave_unions(g, x, 20)) > 64


_ORACLE_CACHE = {}


def _c3_case(n_cells, var, by_equation):
    key = (n_cells, var, by_equation)
    if key not in _ORACLE_CACHE:
        geo, xyz, vals = c3_region(n_cells, C3_ROWS)
        prm = list(C3_PARAMS[var])
        prm[5] = 1.0 if by_equation else 0.0
        v = np.ascontiguousarray(vals[var])
        exp = oracle_idw(IDW_PARAMS[var][0], xyz, v, geo[:, :3], prm, dst_slope=geo[:, 5])
        assert np.isfinite(exp).all()   # 500 stations within 200 km: every cell always has a valid neighbour
        _ORACLE_CACHE.clear()           # one region at a time (65K x 730 doubles per entry)
        _ORACLE_CACHE[key] = (geo, xyz, v, prm, exp)
    return _ORACLE_CACHE[key]


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["wave", "tile"])
@pytest.mark.parametrize("var,by_equation", [(0, False), (0, True), (1, False), (2, False), (3, False), (4, False)])
def test_c3_idw_500_stations_730_rows_bitexact(var, by_equation, path, monkeypatch):
    """S = 500, 730 rows in one call plus a 2-call split (the neighbour table is reused), against the oracle's
    run_interpolation (inverse_distance.h:142-250), on the 65,536-cell C3 region: the wavefront-union gather
    (asserted: every wavefront's neighbours fit one 64-station list) and, with SHYFT_IDW_TILE=1, the multi-tile
    LDS loop (asserted) over the same cells."""
    if path == "tile":
        monkeypatch.setenv("SHYFT_IDW_TILE", "1")
    geo, xyz, v, prm, exp = _c3_case(C3_WAVE_CELLS, var, by_equation)
    ok, msg = _same(_device_interpolate(geo, xyz, v, var, prm, [], path=path), exp)
    assert ok, msg
    ok, msg = _same(_device_interpolate(geo, xyz, v, var, prm, [333], path=path), exp)
    assert ok, msg


@pytest.mark.gpu
@pytest.mark.parametrize("var,by_equation", [(0, False), (0, True), (1, False), (4, False)])
def test_c3_small_region_overflowing_unions_take_tiles_bitexact(var, by_equation):
    """1500 cells: every wavefront union exceeds 64 stations, so the launch falls back to the row tiles without
    being told to (asserted), and is bit-exact there too."""
    geo, xyz, v, prm, exp = _c3_case(C3_TILE_CELLS, var, by_equation)
    ok, msg = _same(_device_interpolate(geo, xyz, v, var, prm, [333], path="tile"), exp)
    assert ok, msg


def reference_performance_scenario(n=72):
    """inverse_distance_test.cpp:396-450: 70 x 70 temperature sources 3 km apart, z = (i + j) 500 / 140,
    constant series 10 - 0.1 x/1000 - 0.6/100 z; 55 x 55 cells (mocks.h:417-427 GenerateTestGrid: x, y = 500 +
    1000 i, z = 100 + (x + y) 700/110); Parameter(2 * 3000, 4): max_distance 6 km, 4 neighbours."""
    s_n, s_dxy = 70, 3000.0
    i, j = np.meshgrid(np.arange(s_n), np.arange(s_n), indexing="ij")
    xyz = np.stack([s_dxy * i.ravel(), s_dxy * j.ravel(), (i + j).ravel() * 500.0 / (s_n + s_n)], 1)
    v = 10.0 - xyz[:, 0] * 0.1 / 1000.0 - 0.6 / 100.0 * xyz[:, 2]
    vals = np.tile(v, (n, 1))
    nx = ny = 55
    dz = (800.0 - 100.0) / (nx + ny)
    cx, cy = np.meshgrid(np.arange(nx), np.arange(ny), indexing="ij")
    geo = np.zeros((nx * ny, 11))
    geo[:, 0] = 500.0 + cx.ravel() * 1000
    geo[:, 1] = 500.0 + cy.ravel() * 1000
    geo[:, 2] = 100.0 + (cx + cy).ravel() * dz
    geo[:, 3] = 1e6
    geo[:, 4] = 1
    geo[:, 5] = 0.9
    geo[:, 10] = 1.0
    prm = [4, 2 * s_dxy, 2.0, 1.0, -0.006, 0.0, 1.02]
    return geo, xyz, vals, prm


def test_reference_4900_source_scenario_oracle():
    """The oracle on the reference's performance scenario: finite everywhere (every cell has sources within
    6 km), and the temperature stays inside the sources' range adjusted by the gradient."""
    from tests.test_idw import TEMPERATURE
    geo, xyz, vals, prm = reference_performance_scenario(8)
    out = oracle_idw(TEMPERATURE, xyz, vals, geo[:, :3], prm)
    assert np.isfinite(out).all()
    assert np.all(out == out[0])           # constant source series -> constant cell series
    assert -1.0 < out.min() and out.max() < 10.0   # 10 - 0.1 x/km over 55 km, -0.006 C/m over <= 800 m


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["wave", "tile"])
@pytest.mark.parametrize("with_nan", [False, True])
def test_reference_4900_source_scenario_bitexact(with_nan, path, monkeypatch):
    """4900 sources: the wavefront-union gather, and (SHYFT_IDW_TILE=1) the tile kernel, where 3 x 4900 x 8 B of
    coordinates exceed the 32 KB LDS budget, so the gather reads rows from global memory (lds_rows = 0)."""
    if path == "tile":
        monkeypatch.setenv("SHYFT_IDW_TILE", "1")
    from tests.test_idw import TEMPERATURE
    geo, xyz, vals, prm = reference_performance_scenario(72)
    if with_nan:
        rng = np.random.default_rng(3)
        vals = np.where(rng.uniform(size=vals.shape) < 0.1, np.nan, vals)
    exp = oracle_idw(TEMPERATURE, xyz, vals, geo[:, :3], prm)
    ok, msg = _same(_device_interpolate(geo, xyz, vals, 0, prm, [30], path=path), exp)
    assert ok, msg


@pytest.mark.gpu
@pytest.mark.parametrize("var", [0, 1])
def test_c3_shuffled_cells_fall_back_to_tiles_bitexact(var):
    """Cells in random order: a wavefront's 64 cells are scattered over the region, their neighbour lists need
    more than 64 stations, so the union kernel reports the overflow and the gather keeps the row tiles."""
    geo, xyz, vals = c3_region(1500, 100)
    geo = geo[np.random.default_rng(5).permutation(geo.shape[0])]
    kind = IDW_PARAMS[var][0]
    prm = list(C3_PARAMS[var])
    v = np.ascontiguousarray(vals[var])
    exp = oracle_idw(kind, xyz, v, geo[:, :3], prm, dst_slope=geo[:, 5])
    ok, msg = _same(_device_interpolate(geo, xyz, v, var, prm, [], path="tile"), exp)
    assert ok, msg


@pytest.mark.gpu
def test_c3_chain_idw_then_pt_gs_k_bitexact():
    """run_interpolation (all five variables by IDW from the 500 stations, use_idw_for_temperature) followed by
    run_cells, against the same chain on the oracle: region_model::interpolate (region_model.h:397-555) feeding
    cell::run (pt_gs_k_cell_model.h:243-262). 65,536 cells, so every variable takes the wavefront-union gather
    (asserted); the interpolated forcing is compared for every cell, the pt_gs_k run on 1024 sampled cells (the
    oracle run on just those cells, from the oracle's own interpolated forcing)."""
    from shyft_amd import synthetic
    from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_ALL
    from tests import oracle_lib
    N, T = C3_WAVE_CELLS, C3_ROWS
    geo, xyz, vals = c3_region(N, T, nan_frac=0.01)
    idx = np.unique(np.concatenate([[0, N - 1], np.random.default_rng(2).choice(N, 1022, replace=False)]))
    p = synthetic.default_ptgsk_parameters()
    s = synthetic.default_ptgsk_state(N)
    r = HipRegion(PT_GS_K, N)
    f_idx = np.empty((5, T, idx.size))
    try:
        r.set_geo(geo)
        r.set_parameters(p)
        r.set_time_axis(synthetic.T0_2015_US, HOUR, T)
        r.set_collection(COLLECT_ALL)
        r.set_state(s)
        for var in range(5):
            r.interpolate(var, xyz, np.ascontiguousarray(vals[var]), 0, C3_PARAMS[var])
            assert r.interpolation_path(var) == "wave"
        for var in range(5):
            exp_f = oracle_idw(IDW_PARAMS[var][0], xyz, np.ascontiguousarray(vals[var]), geo[:, :3], C3_PARAMS[var],
                               dst_slope=geo[:, 5])
            ok, msg = _same(r.get_forcing(var, 0, T), exp_f)
            assert ok, f"forcing {var}: " + msg
            f_idx[var] = exp_f[:, idx]
            del exp_f
        r.run_cells(0, 0, T)
        got = np.stack([r.get_series(k, 0, T)[:, idx] for k in range(8)])
        st = r.get_state()[idx]
    finally:
        r.close()
    exp = oracle_lib.ptgsk_run(geo[idx], p, s[idx], synthetic.T0_2015_US, HOUR, f_idx, full=True)
    ok, msg = _same(got, exp["full"])
    assert ok, "series: " + msg
    assert np.array_equal(st, exp["state"])


@pytest.mark.gpu
def test_c3_fullsize_1m_cells_two_windows_sampled_bitexact():
    """configs[2] at full size: 1,048,576 cells, the bench's 500-station network, two 438-step windows (the bench's
    chunks) of run_interpolation (all five variables, asserted on the wavefront-union gather) then run_cells with the
    state carried in HBM; 512 sampled cells (first and last included) compared bit for bit with the oracle's IDW on
    just those cells (all 500 stations) and the oracle's pt_gs_k run over the same 876 steps."""
    import torch
    import bench
    from shyft_amd import synthetic
    from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_ALL
    from tests import oracle_lib
    N, W = 1 << 20, 438
    T = 2 * W
    geo = synthetic.geo11(N)
    xyz = bench.station_network(N)
    vals = bench.station_values(xyz, 0, T)                            # [5][T][500]
    rng = np.random.default_rng(19)
    vals = np.where((rng.uniform(size=vals.shape) < 0.01) & (rng.uniform(size=(1, T, 1)) < 0.2), np.nan, vals)
    idx = np.unique(np.concatenate([[0, N - 1], rng.choice(N, 510, replace=False)]))
    p = synthetic.default_ptgsk_parameters()
    dev = torch.device("cuda", 0)
    got = np.empty((8, T, idx.size))
    got_f = np.empty((5, T, idx.size))
    r = HipRegion(PT_GS_K, N, device=0)
    try:
        r.set_geo(geo)
        r.set_parameters(p)
        r.set_time_axis(synthetic.T0_2015_US, HOUR, T, W)
        r.set_collection(COLLECT_ALL)
        r.set_state(synthetic.default_ptgsk_state(N))
        buf = torch.empty((W, N), dtype=torch.float64, device=dev)
        cols = torch.from_numpy(idx).to(dev)
        for w0 in (0, W):
            r.move_window(w0, 0)
            for var in range(5):
                r.interpolate(var, xyz, np.ascontiguousarray(vals[var, w0:w0 + W]), w0, C3_PARAMS[var])
                assert r.interpolation_path(var) == "wave", f"variable {var}: {r.interpolation_path(var)}"
            r.run_cells(0, w0, W)
            for var in range(5):
                torch.cuda.synchronize(dev)
                r.get_forcing_device(var, w0, W, buf.data_ptr())
                got_f[var, w0:w0 + W] = buf.index_select(1, cols).cpu().numpy()
            for k in range(8):
                torch.cuda.synchronize(dev)
                r.get_series_device(k, w0, W, buf.data_ptr())
                got[k, w0:w0 + W] = buf.index_select(1, cols).cpu().numpy()
        state = r.get_state()[idx]
    finally:
        r.close()
    exp_f = np.stack([oracle_idw(IDW_PARAMS[v][0], xyz, np.ascontiguousarray(vals[v]), geo[idx, :3], C3_PARAMS[v],
                                 dst_slope=geo[idx, 5]) for v in range(5)])
    ok, msg = _same(got_f, exp_f)
    assert ok, "forcing: " + msg
    exp = oracle_lib.ptgsk_run(geo[idx], p, synthetic.default_ptgsk_state(idx.size), synthetic.T0_2015_US, HOUR, exp_f,
                               full=True, ncore=8)
    ok, msg = _same(got, exp["full"])
    assert ok, "series: " + msg
    assert np.array_equal(state, exp["state"])
