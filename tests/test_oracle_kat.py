"""Pin the CPU oracle against the reference's own known-answer tests.

Each test names the reference test it restates (file:line under /root/reference).
"""
import ctypes as C
import math

import numpy as np
import pytest

from shyft_amd import synthetic
from tests import oracle_lib

HOUR = 3600 * 10**6


def test_gamma_p_vs_scipy(oracle):
    sp = pytest.importorskip("scipy.special")
    rng = np.random.default_rng(1)
    for a in (0.1, 0.5, 1.0, 1.26, 2.0, 3.9, 6.25, 10.0, 50.0):
        for x in np.concatenate([rng.uniform(0, 3 * a + 20, 20), [1e-8, a, a + 1]]):
            assert oracle.oracle_gamma_p(a, x) == pytest.approx(sp.gammainc(a, x), rel=1e-12, abs=1e-300)


def test_calculate_snow_state(oracle):
    # gamma_snow_test.cpp:76-93
    swe, sca = C.c_double(), C.c_double()
    shape = 1.0 / (0.4 * 0.4)
    oracle.oracle_gs_calc_snow_state(shape, 0.4 / shape, 0.04, 0.0, 0.0, 0.1, 0.0, C.byref(swe), C.byref(sca))
    assert swe.value == pytest.approx(0.384, abs=1e-10)
    assert sca.value == pytest.approx(0.96, abs=1e-10)


def test_correct_lwc(oracle):
    # gamma_snow_test.cpp:95-115 ("as a result of using lower resolution, less accuracy")
    assert oracle.oracle_gs_corr_lwc(4.0, 6.0, 1.0, 5.0, 5.0, 2.0) == pytest.approx(3.8411, abs=1e-4)
    for args in ((1.0, 6.25, 0.005358, 0.5, 6.25, 0.005358), (0.0, 6.0, 1.0, 5.0, 5.0, 2.0),
                 (4.0, 6.0, 1.0, 0.0, 5.0, 2.0)):
        assert math.isfinite(oracle.oracle_gs_corr_lwc(*args))


def _gs_step(oracle, st, t, dt, p, T, rad, prec, ws, rh):
    st = np.asarray(st, dtype=np.float64).copy()
    resp = np.zeros(3)
    assert oracle.oracle_gs_step(st.ctypes.data, resp.ctypes.data, t, dt, p.ctypes.data, T, rad, prec, ws, rh, 0.0, 0.0) == 0
    return st, resp


def test_output_independent_of_timestep(oracle):
    # gamma_snow_test.cpp:204-237
    p = synthetic.default_ptgsk_parameters()
    s0 = np.array([0.0, 0.0, 0.0, 1.0 / (0.4 * 0.4), 0.0, -1.0, 0.0, 0.0])
    for temp in (10.0, -10.0):
        s1, out = s0, 0.0
        for i in range(3):
            s1, r1 = _gs_step(oracle, s1, i * HOUR, HOUR, p, temp, 10.0, 5.0, 2.0, 0.7)
            out += r1[2]
        s3, r3 = _gs_step(oracle, s0, 0, 3 * HOUR, p, temp, 10.0, 5.0, 2.0, 0.7)
        assert out / 3.0 == pytest.approx(r3[2], abs=1e-5)
        assert s1[1] == pytest.approx(s3[1], abs=1e-6)
        assert r1[1] == pytest.approx(r3[1], abs=1e-5)


def test_warm_winter_effect_runs(oracle):
    # gamma_snow_test.cpp:117-174: 100 days of warm weather on a wet spring pack must not fail
    p = synthetic.default_ptgsk_parameters()
    st = np.array([0.6, 3148.9609375, 0.0, 3.960848093032837, 1525.66064453125, 2753.03076171875, 1752.56396484375, 0.0])
    for i in range(24 * 100):
        st, r = _gs_step(oracle, st, HOUR * 24 * 232 + i * HOUR, HOUR, p, 7.99117956, 0.0, 0.0, 2.0, 0.70)
        assert np.all(np.isfinite(r))


def test_kirchner_single_solve(oracle):
    # kirchner_test.cpp:14-28
    q1, q2, a1, a2 = C.c_double(1.0), C.c_double(1.0), C.c_double(), C.c_double()
    oracle.oracle_kirchner_step(-2.439, 0.966, -0.1, 1e-7, 1e-8, 0, 10**6, C.byref(q1), C.byref(a1), 2.0, 0.5)
    oracle.oracle_kirchner_step(-2.439, 0.966, -0.1, 1e-7, 1e-8, 0, 10**6, C.byref(q2), C.byref(a2), 2.0, 0.5)
    assert q1.value == pytest.approx(q2.value, abs=1e-6)
    assert a1.value == pytest.approx(a2.value, abs=1e-6)


def test_kirchner_hard_case(oracle):
    # kirchner_test.cpp:48-66
    q, qa = C.c_double(2.29339), C.c_double()
    atol, rtol = 1.0e-2, 1.0e-4
    for _ in range(10):
        assert oracle.oracle_kirchner_step(-2.439, 0.966, -0.1, atol, rtol, 0, HOUR, C.byref(q), C.byref(qa), 5.93591,
                                           0.0) == 0
        atol /= 2.0
        rtol /= 2.0
    assert q.value < 100.0


def test_kirchner_solve_from_zero_q(oracle):
    # kirchner_test.cpp:29-46 (converges after ~2e5 hourly steps)
    q, qa = C.c_double(0.0), C.c_double(0.0)
    for _ in range(10_000_000):
        oracle.oracle_kirchner_step(-2.439, 0.966, -0.1, 1e-7, 1e-8, 0, HOUR, C.byref(q), C.byref(qa), 10.0, 0.0)
        if abs(q.value - 10.0) < 0.001 and abs(qa.value - 10.0) < 0.001:
            break
    assert q.value == pytest.approx(10.0, abs=0.001)
    assert qa.value == pytest.approx(10.0, abs=0.001)


def test_priestley_taylor_regression(oracle):
    # priestley_taylor_test.cpp:7-24
    pt = lambda T, r, rh: oracle.oracle_pt_pot_evap(0.2, 1.26, T, r, rh)
    assert pt(20.5, 445, 0.64) * 24.0 * 3600 == pytest.approx(11.0, abs=1.0)
    assert pt(-20, 200, 0.30) * 24 * 3600 == pytest.approx(0.0, abs=0.5)
    assert pt(0, 200, 0.30) * 24 * 3600 == pytest.approx(1.0, abs=0.5)
    for t in np.arange(0.0, 30.0, 0.5):
        assert pt(t, 400, 0.5) < pt(t + 0.5, 400, 0.5)
    for rh in np.arange(0.01, 1.0, 0.01):
        assert pt(15, 400, rh) < pt(15, 400, rh + 1.0)
    for r in np.arange(10.0, 900.0, 50.0):
        assert pt(15, r, 60) < pt(15, r + 50.0, 60)


def test_calendar(oracle):
    # calendar::day_of_year / trim(YEAR) (utctime_utilities.cpp:230-253)
    t = synthetic.T0_2015_US
    assert oracle.oracle_day_of_year(t) == 1
    assert oracle.oracle_day_of_year(t + 99 * 24 * HOUR) == 100
    assert oracle.oracle_trim_year(t + 200 * 24 * HOUR + 5) == t
    assert oracle.oracle_day_of_year(-1) == 365  # 1969-12-31
