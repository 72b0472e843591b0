"""Bayesian temperature kriging (core/bayesian_kriging.h:280-402).

CPU: the oracle restatement (oracle/src/btk.hpp) against the reference's own known answers in
test/bayesian_kriging_test.cpp (covariance entries :219-220, interpolated temperatures :259-261), its
error texts, and an independent numpy statement of the same algebra (the reduced-operator branch with
missing sources included).

GPU: the device path (kernels/btk.hip through the C ABI: shyft_hip_btk, shyft_hip_interpolate_btk)
against the oracle. The device evaluates the reference's per-step products as one dense product per
valid-source pattern, so agreement is to floating-point reassociation: the tolerance is
1e-9 degC absolute on temperatures of O(10) degC.
"""
import ctypes as C
import math

import numpy as np
import pytest

from tests.oracle_lib import load

TOL = 1e-9  # degC, device vs oracle (summation order only)
_p = lambda a: a.ctypes.data_as(C.c_void_p)


def oracle_btk(src_xyz, src_values, prior, param, dst_xyz):
    L = load()
    L.oracle_btk_run.restype = C.c_int
    L.oracle_btk_run.argtypes = [C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t,
                                 C.c_void_p, C.c_void_p, C.c_char_p, C.c_size_t]
    xyz = np.ascontiguousarray(src_xyz, dtype=np.float64)
    v = np.ascontiguousarray(src_values, dtype=np.float64)
    g = np.ascontiguousarray(prior, dtype=np.float64)
    p = np.ascontiguousarray(param, dtype=np.float64)
    d = np.ascontiguousarray(dst_xyz, dtype=np.float64)
    T, S, D = v.shape[0], xyz.shape[0], d.shape[0]
    out = np.full((T, D), np.nan)
    err = C.create_string_buffer(512)
    if L.oracle_btk_run(S, _p(xyz), _p(v), T, _p(g), _p(p), D, _p(d), _p(out), err, 512) != 0:
        raise RuntimeError(err.value.decode())
    return out


def oracle_source_covariance(src_xyz, param):
    L = load()
    L.oracle_btk_source_covariance.restype = None
    L.oracle_btk_source_covariance.argtypes = [C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p]
    xyz = np.ascontiguousarray(src_xyz, dtype=np.float64)
    p = np.ascontiguousarray(param, dtype=np.float64)
    K = np.empty((xyz.shape[0], xyz.shape[0]))
    L.oracle_btk_source_covariance(xyz.shape[0], _p(xyz), _p(p), _p(K))
    return K


# the test Parameter of bayesian_kriging_test.cpp:59-85: gradient -0.006 (per step), gradient_sd 0.0025,
# sill 25, nugget 0.5, range 200 km, zscale 20
TEST_PARAM = [0.0025, 25.0, 0.5, 200000.0, 20.0]


def build_sources_and_dests(nsx, nsy, ndx, ndy):
    """build_sources_and_dests (bayesian_kriging_test.cpp:108-156) without randomisation: source
    temperature 10 + 2 * xy_dist(p0, p) / max_dist + 0.006 z, constant in time."""
    x_max, y_max = 100000.0, 1000000.0
    max_d = math.hypot(x_max, y_max)
    src, temps = [], []
    for i in range(nsx):
        x = i * x_max / (nsx - 1)
        for j in range(nsy):
            y = j * y_max / (nsy - 1)
            z = 500 * math.sin(x / x_max) + math.sin(y / y_max) / 2
            src.append((x, y, z))
            temps.append(10 + 2.0 * math.hypot(x, y) / max_d + z * (0.6 / 100))
    dst = []
    for i in range(ndx):
        x = i * x_max / (ndx - 1)
        for j in range(ndy):
            y = j * y_max / (ndy - 1)
            dst.append((x, y, 500 * (math.sin(x / x_max) + math.sin(y / y_max)) / 2))
    return np.array(src), np.array(temps), np.array(dst)


def test_covariance_matrix_kat():
    # test_build_covariance_matrices (bayesian_kriging_test.cpp:199-224)
    src, _, _ = build_sources_and_dests(3, 3, 15, 15)
    K = oracle_source_covariance(src, TEST_PARAM)
    assert K.shape == (9, 9)
    assert np.allclose(np.diag(K), 25.0 - 0.5, atol=1e-5)
    assert np.array_equal(K, K.T)
    assert K[0, 1] == pytest.approx(2.011082466, abs=1e-6)
    assert K[0, 2] == pytest.approx(0.165079701, abs=1e-6)


def test_interpolation_kat():
    # test_interpolation (bayesian_kriging_test.cpp:240-262): 3x3 sources, 9x9 destinations, one period
    src, temps, dst = build_sources_and_dests(3, 3, 9, 9)
    out = oracle_btk(src, temps[None, :], [-0.006], TEST_PARAM, dst)
    e_temp = [10.0, 11.9918, 12.3670, 12.1815, 10.5669, 12.2066]
    assert np.all(np.abs(out[0, :6] - e_temp) < 0.01), out[0, :6]


def numpy_btk(src_xyz, src_values, prior, param, dst_xyz):
    """The reference's algebra (bayesian_kriging.h:299-395) restated with numpy's dense inverse, per step,
    with the reduced operators for the valid sources of each step: an independent check of the oracle."""
    sd, sill, nug, rng, zs = param

    def cov(a, b):
        d = np.sqrt(((a[:, None, 0] - b[None, :, 0]) ** 2 + (a[:, None, 1] - b[None, :, 1]) ** 2 +
                     ((a[:, None, 2] - b[None, :, 2]) * zs) ** 2))
        return (sill - nug) * np.exp(-d / rng)

    K = cov(src_xyz, src_xyz)
    np.fill_diagonal(K, sill - nug)
    k = cov(src_xyz, dst_xyz)
    F = np.stack([np.ones(len(src_xyz)), src_xyz[:, 2]], 1)
    f = np.stack([np.ones(len(dst_xyz)), dst_xyz[:, 2]], 0)
    out = np.empty((src_values.shape[0], len(dst_xyz)))
    for t, row in enumerate(src_values):
        v = np.isfinite(row)
        Fr, Kinv, kr = F[v], np.linalg.inv(K[np.ix_(v, v)]), k[v]
        H_inv = Fr.T @ Kinv @ Fr
        G_inv = H_inv.copy()
        G_inv[1, 1] += 1 / (sd * sd)
        GH = np.linalg.inv(G_inv) @ H_inv
        BM = (f - Fr.T @ Kinv @ kr).T @ (np.eye(2) - GH)
        beta = np.linalg.inv(H_inv) @ Fr.T @ Kinv @ row[v]
        T_hat = f.T @ beta + kr.T @ Kinv @ (row[v] - Fr @ beta)
        out[t] = T_hat - BM @ (beta - np.array([0.0, prior[t]]))
    return out


def random_case(S=12, D=150, T=40, seed=3, missing=0.15):
    rng = np.random.default_rng(seed)
    src = np.stack([rng.uniform(0, 60000, S), rng.uniform(0, 60000, S), rng.uniform(0, 1500, S)], 1)
    dst = np.stack([rng.uniform(0, 60000, D), rng.uniform(0, 60000, D), rng.uniform(0, 2000, D)], 1)
    vals = 12.0 - 0.0065 * src[None, :, 2] + rng.normal(0, 1.5, (T, S))
    miss = rng.uniform(size=vals.shape) < missing
    miss[:5] = False            # full-set steps first, then reduced patterns, then the full set again
    miss[T - 3:] = False
    miss[:, 0] = False          # keep two sources at different heights in every step
    miss[:, 1] = False
    vals[miss] = np.nan
    prior = 1.18e-3 * np.sin(6.2831 / 365 * (np.arange(T) % 365 + 79.0)) - 5.48e-3
    return src, vals, prior, dst


def test_oracle_matches_numpy_algebra():
    src, vals, prior, dst = random_case()
    got = oracle_btk(src, vals, prior, [0.0025, 25.0, 0.5, 20000.0, 20.0], dst)
    ref = numpy_btk(src, vals, prior, [0.0025, 25.0, 0.5, 20000.0, 20.0], dst)
    assert np.max(np.abs(got - ref)) < 1e-8


def test_oracle_error_texts():
    src = np.array([[0.0, 0.0, 100.0], [1000.0, 0.0, 100.0], [0.0, 1000.0, 100.0]])
    with pytest.raises(RuntimeError, match="at least two sources at different heights"):
        oracle_btk(src, np.ones((2, 3)), [-0.006] * 2, TEST_PARAM, np.zeros((4, 3)))
    src[1, 2] = 300.0
    vals = np.ones((3, 3))
    vals[1] = np.nan
    with pytest.raises(RuntimeError, match="No valid sources for time period"):
        oracle_btk(src, vals, [-0.006] * 3, TEST_PARAM, np.zeros((4, 3)))


# ---- device ---------------------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_device_kat_and_oracle_parity():
    from shyft_amd.region import btk
    src, temps, dst = build_sources_and_dests(3, 3, 9, 9)
    out = btk(src, temps[None, :], [-0.006], TEST_PARAM, dst)
    assert np.all(np.abs(out[0, :6] - [10.0, 11.9918, 12.3670, 12.1815, 10.5669, 12.2066]) < 0.01)
    assert np.max(np.abs(out - oracle_btk(src, temps[None, :], [-0.006], TEST_PARAM, dst))) < TOL
    # missing sources: the reduced-operator patterns, interleaved with full-set steps
    src, vals, prior, dst = random_case(S=25, D=700, T=96)
    prm = [0.0025, 25.0, 0.5, 20000.0, 20.0]
    got = btk(src, vals, prior, prm, dst)
    assert np.max(np.abs(got - oracle_btk(src, vals, prior, prm, dst))) < TOL


@pytest.mark.gpu
def test_device_errors_and_single_source():
    from shyft_amd.region import btk
    src = np.array([[0.0, 0.0, 100.0], [1000.0, 0.0, 100.0], [0.0, 1000.0, 100.0]])
    with pytest.raises(RuntimeError, match="at least two sources at different heights"):
        btk(src, np.ones((2, 3)), [-0.006] * 2, TEST_PARAM, np.zeros((4, 3)))
    src[1, 2] = 300.0
    vals = np.ones((3, 3))
    vals[1] = np.nan
    with pytest.raises(RuntimeError, match="No valid sources for time period"):
        btk(src, vals, [-0.006] * 3, TEST_PARAM, np.zeros((4, 3)))
    one = btk(src[:1], np.array([[3.0], [4.0]]), [-0.006] * 2, TEST_PARAM, np.zeros((5, 3)))
    assert np.array_equal(one, np.array([[3.0] * 5, [4.0] * 5]))


@pytest.mark.gpu
def test_region_interpolate_btk_with_filter_and_day_of_year_prior():
    from shyft_amd import synthetic
    from shyft_amd.region import HipRegion, PT_GS_K, TEMPERATURE
    N, T = 600, 72
    src, vals, _, _ = random_case(S=18, D=1, T=T, seed=11)
    rng = np.random.default_rng(4)
    geo = np.zeros((N, 11))
    geo[:, 0] = rng.uniform(0, 60000, N)
    geo[:, 1] = rng.uniform(0, 60000, N)
    geo[:, 2] = rng.uniform(0, 2000, N)
    geo[:, 3] = 1e6
    geo[:, 4] = 1 + (np.arange(N) * 3) // N          # catchments 1, 2, 3
    geo[:, 5] = 0.9
    geo[:, 6:10] = (0.01, 0.05, 0.19, 0.30)
    geo[:, 10] = 0.45
    t0 = synthetic.T0_2015_US + 40 * 86400 * 1000000
    dt = 3600 * 1000000
    # bayesian_kriging::parameter::temperature_gradient: day of year of the period midpoint
    doy = np.array([(t0 + i * dt + dt // 2) // (86400 * 1000000) for i in range(T)])
    doy = (doy - synthetic.T0_2015_US // (86400 * 1000000)) + 1   # 2015: day 1 is Jan 1
    prior = 1.18e-3 * np.sin(6.2831 / 365 * (doy + 79.0)) - 5.48e-3
    prm = [0.0025, 25.0, 0.5, 20000.0, 20.0]
    r = HipRegion(PT_GS_K, N)
    r.set_geo(geo)
    r.set_parameters(synthetic.default_ptgsk_parameters())
    r.set_time_axis(t0, dt, T)
    r.set_catchment_filter([1, 3])
    r.interpolate_btk(src, vals[:30], 0, prm)          # prior from the region's time axis
    r.interpolate_btk(src, vals[30:], 30, prm, prior[30:])
    got = r.get_forcing(TEMPERATURE, 0, T)
    r.close()
    active = geo[:, 4] != 2
    assert np.isnan(got[:, ~active]).all()             # uncalculated cells keep the initial NaN fill
    ref = oracle_btk(src, vals, prior, prm, geo[active, :3])
    assert np.max(np.abs(got[:, active] - ref)) < TOL
