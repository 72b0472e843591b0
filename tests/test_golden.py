"""Golden fixtures (tests/golden/, written by tests/golden/make_golden.py from the KAT-pinned oracle).

CPU: the oracle reproduces every fixture bit for bit (the checker itself has not drifted).
GPU: the HIP kernels reproduce the same fixtures bit for bit through the C ABI."""
import os

import numpy as np
import pytest

from shyft_amd import synthetic
from tests import engines
from tests.golden import make_golden as mg

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STACKS = list(mg.STACKS)


def _load(stack):
    return np.load(os.path.join(HERE, f"{stack}_20x240.npz"))


def _check(engine, stack):
    g = _load(stack)
    geo, f = mg.case_inputs()
    assert np.array_equal(geo, g["geo"]) and np.array_equal(f, g["forcing"])  # inputs regenerate identically
    r = mg.run_case(engine, stack, g["geo"], g["params"], g["state0"], g["forcing"])
    assert np.array_equal(r["main"], g["main"], equal_nan=True), f"{stack}: series differ from the golden fixture"
    assert np.array_equal(np.asarray(r["state"]).reshape(g["state"].shape), g["state"], equal_nan=True), \
        f"{stack}: final state differs from the golden fixture"


@pytest.mark.parametrize("stack", STACKS)
def test_oracle_reproduces_golden(stack):
    _check("oracle", stack)


@pytest.mark.gpu
@pytest.mark.parametrize("stack", STACKS)
def test_hip_reproduces_golden(stack):
    _check("hip", stack)


def _c1(engine):
    g = np.load(os.path.join(HERE, "c1_sampled.npz"))
    geo, f = mg.c1_inputs()
    r = engines.run(engine, geo, synthetic.default_ptgsk_parameters(), synthetic.default_ptgsk_state(mg.C1_CELLS),
                    synthetic.T0_2015_US, synthetic.HOUR_US, f, full=False)
    assert np.array_equal(r["main"][0][:, list(g["cells"])], g["avg_discharge"])
    assert np.array_equal(r["state"], g["state"])


def test_oracle_reproduces_c1_sample():
    _c1("oracle")


@pytest.mark.gpu
def test_hip_reproduces_c1_sample():
    _c1("hip")
