"""pt_gs_k known-answer tests of the reference (test/pt_gs_k_test.cpp), run on
the CPU oracle (always) and on the HIP product path (-m gpu)."""
import numpy as np
import pytest

from shyft_amd import synthetic
from tests import engines
from tests.engines import geo_row, ltf

HOUR = 3600 * 10**6
T0_20140801 = 1406851200 * 10**6  # cal.time(2014, 8, 1)
AREA = 1000.0 * 1000.0
ENGINES = ["oracle", pytest.param("hip", marks=pytest.mark.gpu)]


def approx(a, b, eps):
    """doctest::Approx(b).epsilon(eps) == a: |a-b| < eps*(1 + max(|a|,|b|)) (scale 1.0)."""
    return abs(a - b) < eps * (1.0 + max(abs(a), abs(b)))


def mmh_to_m3s(v, area):
    return area * v * (1 / (3600.0 * 1000.0))


def forcing(T, temp, prec, rh, ws, rad):
    f = np.empty((5, T, 1))
    f[0], f[1], f[2], f[3], f[4] = temp, prec, ws, rh, rad
    return f


class Cell:
    """one pt_gs_k cell driven step by step (state carried between calls)"""

    def __init__(self, engine, geo, params, state, T=1):
        self.engine, self.geo, self.params, self.state, self.T = engine, geo, params.copy(), state.copy(), T

    def run(self, f):
        r = engines.run(self.engine, self.geo, self.params, self.state, T0_20140801, HOUR, f, full=True)
        self.state = r["state"][0].copy()
        return r["full"][:, :, 0]


def gs_default_state(lwc=0.0, acc_melt=-1.0):
    return np.array([0.4, lwc, 30000.0, 1.26, 0.0, acc_melt, 0.0, 0.0, 5.0])


@pytest.fixture(params=ENGINES)
def engine(request):
    return request.param


def _mass_balance_prefix(engine):
    # pt_gs_k_test.cpp:174-216: 10001 one-step runs, constant 3 mm/h rain at 15 degC
    params = synthetic.default_ptgsk_parameters()
    geo = geo_row(1000, 1000, 100)
    c = Cell(engine, geo, params, gs_default_state())
    f = forcing(1, 15.0, 3.0, 0.8, 2.0, 300.0)
    if engine == "hip":
        # the GPU path runs the 10001 steps in one launch on a 10001-step axis (same state recurrence)
        T = 10001
        fT = forcing(T, 15.0, 3.0, 0.8, 2.0, 300.0)
        r = engines.run(engine, geo, params, c.state, T0_20140801, HOUR, fT, full=True)
        c.state = r["state"][0].copy()
        # the KAT inspects the last step (the oracle's collectors hold step 0 of the last 1-step run)
        out = r["full"][:, -1, 0]
        return c, out, f
    out = None
    for _ in range(10001):
        out = c.run(f)[:, 0]
    return c, out, f


def test_mass_balance(engine):
    c, out, f = _mass_balance_prefix(engine)
    dt_s = 3600.0
    assert out[0] * dt_s * 1000 / AREA + out[6] == pytest.approx(3.0, abs=1e-7)
    assert out[4] * dt_s * 1000 / AREA == pytest.approx(3.0, abs=1e-7)


def test_direct_response_on_reservoir_only(engine):
    c, _, f = _mass_balance_prefix(engine)
    g = ltf(0.0, 0.5, 0.5, 0.0, 0.0)
    c.geo = geo_row(1000, 1000, 100, glacier=g[0], lake=g[1], reservoir=g[2], forest=g[3])
    c.state[8] = 1e-4
    c.state[1] = 0.0
    c.state[5] = -1
    out = c.run(f)
    assert approx(out[0, 0] * 3600 * 1000.0 / AREA, 0.5 * 3.0, 0.001)
    c.state[1] = 1.0
    c.state[5] = 300.0
    out = c.run(forcing(1, -10.0, 3.0, 0.8, 2.0, 300.0))
    assert out[2, 0] == pytest.approx(0.96, abs=0.01)
    assert approx(out[0, 0] * 3600 * 1000.0 / AREA, 0.5 * 3.0, 0.05)
    c.state[5] = 5.0
    c.state[7] = 3.0
    c.state[1] = 10.0
    fw = forcing(1, 10.0, 3.0, 0.8, 2.0, 300.0)
    for _ in range(5000):
        out = c.run(fw)
        if out[2, 0] < 0.1:
            break
    assert out[2, 0] == pytest.approx(0.0, abs=0.1)
    assert approx(out[0, 0], 0.5 * 0.8333, 0.001)


@pytest.mark.parametrize("which", ["glacier", "reservoir"])
def test_glacier_and_reservoir_direct_response(engine, which):
    c, _, f = _mass_balance_prefix(engine)
    if which == "glacier":
        g = ltf(0.5, 0.0, 0.0, 0.0, 0.5)
        knob = 29  # gm.direct_response
    else:
        g = ltf(0.0, 0.0, 0.5, 0.0, 0.5)
        knob = 30  # msp.reservoir_direct_response_fraction
    c.geo = geo_row(1000, 1000, 100, glacier=g[0], lake=g[1], reservoir=g[2], forest=g[3])
    c.state[8] = 1e-4
    c.state[1] = 0.0
    c.state[5] = -1
    c.params[knob] = 1.0
    out = c.run(f)
    expected = 0.5 * mmh_to_m3s(3.0, AREA) + (out[5, 0] if which == "glacier" else 0.0)
    assert approx(out[0, 0], expected, 0.001)
    c.params[knob] = 0.5
    out = c.run(f)
    expected = 0.5 * (0.5 * mmh_to_m3s(3.0, AREA) + (out[5, 0] if which == "glacier" else 0.0))
    assert approx(out[0, 0], expected, 0.001)
    c.params[knob] = 0.0
    out = c.run(f)
    assert approx(out[0, 0], 2.778e-5, 0.01e-5)


def test_lake_reservoir_response(engine):
    # pt_gs_k_test.cpp:300-353
    n = 50
    params = synthetic.default_ptgsk_parameters()
    g = ltf(0.0, 0.2, 0.3, 0.0, 0.5)
    geo = geo_row(1000, 1000, 100, glacier=g[0], lake=g[1], reservoir=g[2], forest=g[3])
    f = forcing(n, -15.0, 3.0, 0.8, 2.0, 300.0)
    f[1, 0, 0] = 0.0
    s0 = np.array([0.4, 100.0, 30000.0, 1.26, 0.0, 100.0, 0.0, 0.0, 1.0])
    params[30] = 0.0
    r = engines.run(engine, geo, params, s0, T0_20140801, HOUR, f, full=True)["full"][:, :, 0]
    assert approx(r[0, 0], 0.266, 0.01)
    assert approx(r[0, n - 1], 0.5 * mmh_to_m3s(3.0, AREA), 0.01)
    params[30] = 1.0
    r = engines.run(engine, geo, params, s0, T0_20140801, HOUR, f, full=True)["full"][:, :, 0]
    assert approx(r[0, 0], 0.266 * 0.7, 0.01)
    assert approx(r[3, 0], 0.0, 0.001)
    assert approx(r[3, 1], 1.548, 0.01)
    assert approx(r[3, 2], 3.048, 0.01)
    assert approx(r[0, 1], 0.266 + 0.3 * 0.5 * mmh_to_m3s(3.0, AREA), 0.05)
    expected_2 = 0.2 * mmh_to_m3s(3.0, AREA) * (1.0 - 0.3) + 0.3 * mmh_to_m3s(3.0, AREA)
    assert approx(r[0, n - 1], expected_2, 0.01)
