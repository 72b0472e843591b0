"""detmath (the elementary-function library shared by the HIP kernels and the
oracle) against the host libm (glibc) and scipy."""
import numpy as np
import pytest

from tests import oracle_lib


def _ulps(a, b):
    a, b = np.asarray(a), np.asarray(b)
    sp = np.spacing(np.abs(b))
    return np.abs(a - b) / sp


@pytest.fixture(scope="module")
def libs():
    return oracle_lib.load("detmath"), oracle_lib.load("libm")


def _vec(f, *xs):
    return np.array([f(*v) for v in zip(*xs)])


def test_exp_log_pow_within_one_ulp_of_glibc(libs):
    dm, lm = libs
    rng = np.random.default_rng(7)
    x = rng.uniform(-745.0, 709.7, 20000)
    a, b = _vec(dm.oracle_exp, x), _vec(lm.oracle_exp, x)
    ok = b > 0
    assert _ulps(a[ok], b[ok]).max() <= 1.0
    y = np.exp(rng.uniform(-700, 700, 20000))
    assert _ulps(_vec(dm.oracle_log, y), _vec(lm.oracle_log, y)).max() <= 1.0
    px = np.exp(rng.uniform(-5, 6, 20000))
    py = rng.uniform(-20, 20, 20000)
    a, b = _vec(dm.oracle_pow, px, py), _vec(lm.oracle_pow, px, py)
    ok = np.isfinite(b) & (b > 0)
    assert _ulps(a[ok], b[ok]).max() <= 2.0
    # the exponents the method stacks use
    for xx, yy in ((273.15, 4.0), (2.0, -1.0 / 24 / 5.0), (0.85, 8.0), (0.3, 0.0687), (1.7, -1.0 / 3.0), (0.2, -0.2)):
        assert _ulps(dm.oracle_pow(xx, yy), lm.oracle_pow(xx, yy)) <= 1.0


def test_special_values(libs):
    dm, _ = libs
    assert dm.oracle_exp(0.0) == 1.0
    assert dm.oracle_log(1.0) == 0.0
    assert dm.oracle_exp(1000.0) == float("inf")
    assert dm.oracle_exp(-1000.0) == 0.0
    assert np.isnan(dm.oracle_log(-1.0))
    assert dm.oracle_log(0.0) == float("-inf")
    assert dm.oracle_pow(2.0, 0.0) == 1.0
    assert dm.oracle_pow(-2.0, 3.0) == -8.0
    assert np.isnan(dm.oracle_pow(-2.0, 0.5))
    assert dm.oracle_pow(0.0, -1.0) == float("inf")


def test_lgamma_against_scipy(libs):
    sp = pytest.importorskip("scipy.special")
    dm, _ = libs
    x = np.concatenate([np.exp(np.linspace(np.log(1e-6), np.log(1e3), 4000)), [0.5, 1.0, 1.26, 2.0, 6.25, 7.25]])
    a = _vec(dm.oracle_lgamma_fn, x)
    b = sp.gammaln(x)
    assert (np.abs(a - b) / np.maximum(np.abs(b), 1.0)).max() < 5e-15


def test_gamma_pq_against_scipy(libs):
    import ctypes as C
    sp = pytest.importorskip("scipy.special")
    dm, _ = libs
    rng = np.random.default_rng(11)
    a = np.exp(rng.uniform(np.log(0.05), np.log(300.0), 6000))
    x = a * rng.uniform(0.0, 3.0, a.size)
    x[:50] = a[:50] + 1.0  # branch boundary
    p, p1, pre = C.c_double(), C.c_double(), C.c_double()
    worst = 0.0
    for ai, xi in zip(a, x):
        dm.oracle_gamma_pq(ai, xi, C.byref(p), C.byref(p1), C.byref(pre))
        for got, want in ((p.value, sp.gammainc(ai, xi)), (p1.value, sp.gammainc(ai + 1, xi))):
            err = abs(got - want) / max(abs(want), 1e-300)
            # relative 1e-12, or absolute 1e-14 where P is tiny / its complement dominates
            worst = max(worst, min(err, abs(got - want) / 1e-2))
            assert err < 1e-12 or abs(got - want) < 1e-14, (ai, xi, got, want)
