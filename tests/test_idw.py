"""Inverse-distance interpolation: the oracle against the reference's own tests
(test/inverse_distance_test.cpp), and the HIP kernels against the oracle (bit-exact)."""
import ctypes as C
import math

import numpy as np
import pytest

from tests import oracle_lib

TEMPERATURE, PRECIPITATION, RADIATION, WIND_SPEED, REL_HUM = range(5)  # oracle idw kinds
HOUR = 3600 * 10**6


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def oracle_idw(kind, src_xyz, src_values, dst_xyz, param, dst_slope=None):
    return oracle_lib.idw_run(kind, src_xyz, src_values, dst_xyz, param, dst_slope)


def mock_param(max_distance=200000.0, max_members=20, by_equation=False, default_gradient=-0.006):
    # shyfttest::idw::Parameter (test/mocks.h:455-466)
    return [max_members, max_distance, 2.0, 1.0, default_gradient, 1.0 if by_equation else 0.0, 1.02]


def test_sources(n, x, y, radius):
    # Source::GenerateTestSources (test/mocks.h:344-356)
    pi = 3.1415
    delta = 2.0 * pi / n
    out, angle = [], 0.0
    while angle < 2 * pi:
        xa, ya = x + radius * math.sin(angle), y + radius * math.cos(angle)
        za = (xa + ya) / 1000.0
        out.append((xa, ya, za, 10.0 + za * -0.006))
        angle += delta
    return out


test_sources.__test__ = False  # not a test


def dm(a, b, f=2.0, zscale=1.0):
    return ((a[0] - b[0]) ** 2 + (a[1] - b[1]) ** 2 + (a[2] - b[2]) ** 2 * zscale * zscale) ** (f / 2.0)


def grad_minmax(pts, default=-0.006):
    if len(pts) < 2:
        return default
    mn = mx = 0
    for i, p in enumerate(pts):
        if p[2] < pts[mn][2]:
            mn = i
        elif p[2] > pts[mx][2]:
            mx = i
    dz = pts[mx][2] - pts[mn][2]
    return (pts[mx][3] - pts[mn][3]) / dz if dz > 50.0 else default


def _run_case(n_sources, max_members, nan_index=None, far_index=None):
    src = test_sources(n_sources, 500.0, 500.0, 0.25 * 0.5 * 2 * 1000)
    dst = np.array([[500.0, 500.0, 100.0]])  # MCell::GenerateTestGrid(1, 1) (mocks.h:417-427)
    max_distance = 2.75 * 0.5 * 2 * 1000
    xyz = np.array([s[:3] for s in src])
    vals = np.array([[s[3] for s in src]])
    if nan_index is not None:
        vals[0, nan_index] = np.nan
    if far_index is not None:
        xyz[far_index] = (max_distance + 1000, max_distance + 1000, 300)
    out = oracle_idw(TEMPERATURE, xyz, vals, dst, mock_param(max_distance, max_members))[0, 0]
    used = [tuple(xyz[i]) + (vals[0, i],) for i in (0, 1)]
    g = grad_minmax(used)
    w = [1.0 / dm(u, dst[0]) for u in used]
    v = [w[i] * (used[i][3] + g * (dst[0][2] - used[i][2])) for i in range(2)]
    return out, (v[0] + v[1]) / (w[0] + w[1])


def test_one_source_one_dest():
    # inverse_distance_test.cpp:146-176
    src = test_sources(1, 500.0, 500.0, 250.0)
    xyz = np.array([s[:3] for s in src[:1]])
    out = oracle_idw(TEMPERATURE, xyz, np.array([[src[0][3]]]), np.array([[500.0, 500.0, 100.0]]),
                     mock_param(2750.0, 8))[0, 0]
    expected = src[0][3] + -0.006 * (100.0 - src[0][2])
    assert abs(out - expected) < 1e-7


@pytest.mark.parametrize("case", ["two_sources", "finite_only", "far_away", "max_members"])
def test_two_source_cases(case):
    # inverse_distance_test.cpp:177-329
    if case == "two_sources":
        out, exp = _run_case(2, 2)
    elif case == "finite_only":
        out, exp = _run_case(3, 3, nan_index=2)
    elif case == "far_away":
        out, exp = _run_case(3, 3, far_index=2)
    else:
        out, exp = _run_case(3, 2)
    assert abs(out - exp) < 1e-7


def test_nan_outside_defined_period():
    # inverse_distance_test.cpp:372-394: source 2 only defined on steps 1..2
    xyz = np.array([[0.0, 1000.0, 100.0], [1000.0, 0.0, 100.0]])
    vals = np.array([[10.0, np.nan], [10.0, 20.0], [10.0, 20.0], [10.0, np.nan]])
    out = oracle_idw(TEMPERATURE, xyz, vals, np.array([[500.0, 500.0, 100.0]]), mock_param(2000.0, 4))[:, 0]
    assert out == pytest.approx([10.0, 15.0, 15.0, 10.0], rel=1e-12)


def _gradient(pts, by_equation, default=-0.0065):
    L = oracle_lib.load()
    L.oracle_idw_temperature_gradient.restype = C.c_double
    L.oracle_idw_temperature_gradient.argtypes = [C.c_size_t, C.c_void_p, C.c_void_p, C.c_double, C.c_int]
    xyz = np.ascontiguousarray([p[:3] for p in pts], dtype=np.float64)
    t = np.ascontiguousarray([p[3] for p in pts], dtype=np.float64)
    return L.oracle_idw_temperature_gradient(len(pts), _p(xyz) if len(pts) else None, _p(t) if len(pts) else None,
                                             default, int(by_equation))


def test_temperature_gradient_model():
    # inverse_distance_test.cpp:457-495 (arma::solve path and its singular fallback)
    dT = np.array([0.001, 0.002, 0.001])
    P = [np.array(p) for p in ((0, 0, 10), (1000, 0, 110), (0, 1000, 110), (1000, 1000, 220))]
    t = [10.0 + float(dT @ (p - P[0])) for p in P]
    pts = [tuple(P[i]) + (t[i],) for i in range(4)]
    assert _gradient(pts[:1], True) == pytest.approx(-0.0065, abs=1e-6)
    assert _gradient(pts[:2], True) == pytest.approx((t[1] - t[0]) / (110 - 10), abs=1e-6)
    assert _gradient(pts[:3], True) == pytest.approx((t[1] - t[0]) / (110 - 10), abs=1e-6)
    assert _gradient(pts[:3] + [pts[2]], True) == pytest.approx((t[1] - t[0]) / (110 - 10), abs=1e-6)  # singular
    assert _gradient(pts, True) == pytest.approx(0.001, abs=1e-5)


def test_temperature_model_gradient_sequence():
    # inverse_distance_test.cpp:14-67 (min/max method)
    pts = [(1000, 1000, 100, 10.0)]
    assert _gradient(pts, False, -0.006) == pytest.approx(-0.006, abs=1e-9)
    pts.append((1000, 1000, 149, 10 - 0.005 * 59))
    assert _gradient(pts, False, -0.006) == pytest.approx(-0.006, abs=1e-9)  # dz < 50 m: default
    pts.append((2000, 2000, 200, 9.5))
    assert _gradient(pts, False, -0.006) == pytest.approx(-0.005, abs=1e-9)
    pts.append((3000, 3000, 300, 9.0))
    assert _gradient(pts, False, -0.006) == pytest.approx(-0.005, abs=1e-9)
    pts.append((4000, 4000, 500, 8.0))
    assert _gradient(pts, False, -0.006) == pytest.approx(-0.005, abs=1e-9)
    pts.append((4000, 4000, 600, 10 - 0.006 * (600 - 100)))
    assert _gradient(pts, False, -0.006) == pytest.approx(-0.006, abs=1e-9)


def test_precipitation_and_radiation_transforms():
    # inverse_distance_test.cpp:77-145: one source -> the transform of that source
    xyz = np.array([[1000.0, 1000.0, 100.0]])
    dst = np.array([[1500.0, 1500.0, 200.0]])
    p = mock_param(100 * 1000.0, 10)
    prec = oracle_idw(PRECIPITATION, xyz, np.array([[10.0]]), dst, p)[0, 0]
    assert prec == pytest.approx(10.0 * 1.02 ** ((200.0 - 100.0) / 100.0), rel=1e-12)
    rad = oracle_idw(RADIATION, xyz, np.array([[10.0]]), dst, p, dst_slope=[0.5])[0, 0]
    assert rad == pytest.approx(5.0, rel=1e-15)


def _c3_like(n_cells=700, n_sources=60, T=48, seed=5):
    rng = np.random.default_rng(seed)
    W = int(math.ceil(math.sqrt(n_cells)))
    i = np.arange(n_cells)
    geo = np.zeros((n_cells, 11))
    geo[:, 0] = 500.0 + 1000.0 * (i % W)
    geo[:, 1] = 500.0 + 1000.0 * (i // W)
    geo[:, 2] = rng.uniform(0, 2000, n_cells)
    geo[:, 3] = 1e6
    geo[:, 4] = 1 + (i * 3) // n_cells
    geo[:, 5] = rng.uniform(0.7, 1.0, n_cells)
    geo[:, 6:10] = (0.01, 0.05, 0.19, 0.30)
    geo[:, 10] = 0.45
    # stations on a coarse grid around the cells, plus two duplicates of the grid spacing (distance ties)
    g = int(math.ceil(math.sqrt(n_sources)))
    sx = (np.arange(n_sources) % g) * (W * 1000.0 / (g - 1))
    sy = (np.arange(n_sources) // g) * (W * 1000.0 / (g - 1))
    sz = rng.uniform(0, 2000, n_sources)
    xyz = np.stack([sx, sy, sz], 1)
    vals = rng.normal(5.0, 4.0, (T, n_sources))
    # missing observations in the even rows only: odd rows are all-finite (the kernel's precomputed-gradient
    # fast path), even rows take the general neighbour scan
    miss = rng.uniform(size=vals.shape) < 0.05
    miss[1::2] = False
    vals[miss] = np.nan
    return geo, xyz, vals


IDW_PARAMS = {
    # var (forcing index) -> (oracle kind, idw_param)
    0: (TEMPERATURE, [20, 15000.0, 2.0, 1.0, -0.006, 0.0, 1.02]),
    1: (PRECIPITATION, [20, 15000.0, 2.0, 0.5, -0.006, 0.0, 1.02]),
    2: (WIND_SPEED, [10, 15000.0, 2.0, 1.0, -0.006, 0.0, 1.02]),
    3: (REL_HUM, [10, 200000.0, 1.5, 1.0, -0.006, 0.0, 1.02]),
    4: (RADIATION, [10, 15000.0, 2.0, 1.0, -0.006, 0.0, 1.02]),
}


@pytest.mark.gpu
# gradient_by_equation applies to temperature only
@pytest.mark.parametrize("var,by_equation", [(0, False), (0, True), (1, False), (2, False), (3, False), (4, False)])
def test_idw_kernel_bitexact_vs_oracle(var, by_equation):
    from shyft_amd.region import HipRegion, PT_GS_K
    from shyft_amd import synthetic
    geo, xyz, vals = _c3_like()
    kind, prm = IDW_PARAMS[var]
    prm = list(prm)
    prm[5] = 1.0 if by_equation else 0.0
    T, N = vals.shape[0], geo.shape[0]
    expected = oracle_idw(kind, xyz, vals, geo[:, :3], prm, dst_slope=geo[:, 5])
    r = HipRegion(PT_GS_K, N)
    r.set_geo(geo)
    r.set_parameters(synthetic.default_ptgsk_parameters())
    r.set_time_axis(synthetic.T0_2015_US, HOUR, T)
    r.interpolate(var, xyz, vals[:20], 0, prm)   # two calls: the second reuses the neighbour table
    r.interpolate(var, xyz, vals[20:], 20, prm)
    got = r.get_forcing(var, 0, T)
    r.close()
    same = (got == expected) | (np.isnan(got) & np.isnan(expected))
    assert same.all(), f"{(~same).sum()} differ; max abs {np.nanmax(np.abs(got - expected))}"
