"""GPU pt_gs_k (HIP kernel via the C ABI) vs the CPU oracle on the same seeded
synthetic region.

Parity bar: BIT-EXACT. The kernel evaluates the reference's expressions in the
reference's order with FP contraction off, and both sides take their
elementary functions from detmath (detmath/detmath.h), so every response,
state-series and final-state value must be identical to the oracle's.

The libm-vs-detmath effect (how far the reference build, which uses glibc,
can sit from this oracle) is bounded separately in test_oracle_variants.py.
"""
import ctypes as C

import numpy as np
import pytest

from shyft_amd import synthetic
from tests import engines, oracle_lib

pytestmark = pytest.mark.gpu

HOUR = synthetic.HOUR_US


def _region(n_cells, n_steps, step0=0, seed=synthetic.SEED):
    geo = synthetic.geo11(n_cells)
    f = synthetic.forcing(n_cells, step0, n_steps, seed)
    params = synthetic.default_ptgsk_parameters()
    state = synthetic.default_ptgsk_state(n_cells)
    return geo, f, params, state


def _assert_bitexact(gpu, cpu, what):
    same = (gpu == cpu) | (np.isnan(gpu) & np.isnan(cpu))
    if not same.all():
        i = np.argwhere(~same)[0]
        raise AssertionError(f"{what}: {int((~same).sum())} values differ; first at {tuple(i)}: "
                             f"gpu {gpu[tuple(i)]!r} cpu {cpu[tuple(i)]!r}")


def test_device_math_bitexact_with_host():
    from shyft_amd import _native
    L = _native.lib()
    dm = oracle_lib.load("detmath")
    rng = np.random.default_rng(3)
    x = np.ascontiguousarray(np.concatenate([rng.uniform(-745, 709, 4000), [0.0, -0.0, 1e-310]]))
    xp = np.ascontiguousarray(np.exp(rng.uniform(-700, 700, x.size)))
    y = np.ascontiguousarray(rng.uniform(-20, 20, x.size))
    a = np.ascontiguousarray(rng.uniform(0.05, 30, x.size))
    out = np.empty(x.size)
    cases = [(0, x, None, dm.oracle_exp), (1, xp, None, dm.oracle_log),
             (2, np.ascontiguousarray(np.exp(rng.uniform(-5, 6, x.size))), y, dm.oracle_pow),
             (3, a, None, dm.oracle_lgamma_fn), (4, a, np.ascontiguousarray(a * rng.uniform(0, 3, x.size)), dm.oracle_gamma_p)]
    for fn, xs, ys, host in cases:
        assert L.shyft_hip_math_selftest(fn, xs.ctypes.data_as(C.c_void_p),
                                         None if ys is None else ys.ctypes.data_as(C.c_void_p), xs.size,
                                         out.ctypes.data_as(C.c_void_p)) == 0
        ref = np.array([host(v) if ys is None else host(v, w) for v, w in zip(xs, xs if ys is None else ys)])
        _assert_bitexact(out, ref, f"math fn {fn}")


def test_ptgsk_c1_full_year_200_cells_bitexact():
    """config[0]: 200 synthetic cells x 8760 hourly steps, all 8 response series,
    the 9 state-collector series and the final state, bit for bit."""
    n, T = 200, 8760
    geo, f, params, state = _region(n, T)
    cpu = engines.run("oracle", geo, params, state, synthetic.T0_2015_US, HOUR, f, full=True, collect_state=True)
    gpu = engines.run("hip", geo, params, state, synthetic.T0_2015_US, HOUR, f, full=True, collect_state=True)
    names = ("avg_discharge", "charge_m3s", "snow_sca", "snow_swe", "snow_outflow", "glacier_melt", "ae", "pe")
    for k, nm in enumerate(names):
        _assert_bitexact(gpu["full"][k], cpu["full"][k], nm)
    for k in range(9):
        _assert_bitexact(gpu["state_series"][k], cpu["state_series"][k], f"state series {k}")
    _assert_bitexact(gpu["state"], cpu["state"], "final state")


def test_ptgsk_catchment_parameters_and_filter_bitexact():
    """two parameter sets (region + catchment override, region_model.h:287-319) on a ragged
    region (n not a multiple of the 256-lane workgroup), 1000 steps from mid-March."""
    n, T, step0 = 333, 1000, 1800
    geo, f, params, state = _region(n, T, step0)
    p2 = params.copy()
    p2[0] = -2.2      # kirchner.c1
    p2[14] = 0.6      # gs.snow_cv
    p2[17] = 0.1      # snow_cv_forest_factor
    p2[18] = 1e-4     # snow_cv_altitude_factor
    p2[23] = 1.0      # calculate_iso_pot_energy
    P = np.stack([params, p2])
    set_ix = (geo[:, 4] > 50).astype(np.int32)
    t0 = synthetic.T0_2015_US + step0 * HOUR
    cpu = engines.run("oracle", geo, P, state, t0, HOUR, f, set_ix=set_ix, full=True)
    gpu = engines.run("hip", geo, P, state, t0, HOUR, f, set_ix=set_ix, full=True)
    for k in range(8):
        _assert_bitexact(gpu["full"][k], cpu["full"][k], f"series {k}")
    _assert_bitexact(gpu["state"], cpu["state"], "final state")


def test_stepwise_equals_full_run():
    """run_cells(start_step, n_steps) chunks continue from the current state
    (test_region_model_stacks.py:248-261): 10 x 24 steps == one 240-step run, bitwise."""
    from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_DISCHARGE
    n, T = 150, 240
    geo, f, params, state = _region(n, T)
    outs = []
    for chunks in (1, 10):
        r = HipRegion(PT_GS_K, n)
        r.set_geo(geo)
        r.set_parameters(params)
        r.set_time_axis(synthetic.T0_2015_US, HOUR, T)
        r.set_collection(COLLECT_DISCHARGE)
        r.set_state(state)
        for v in range(5):
            r.set_forcing(v, 0, f[v])
        step = T // chunks
        for c in range(chunks):
            r.run_cells(0, c * step, step)
        outs.append((r.get_series(0, 0, T), r.get_state()))
        r.close()
    _assert_bitexact(outs[1][0], outs[0][0], "discharge")
    _assert_bitexact(outs[1][1], outs[0][1], "state")


def test_odd_start_step_and_single_steps_in_snowfall_bitexact():
    """run_cells from an ODD start_step and one step at a time, in January (Brent jobs on most steps): the
    workgroup's double-buffered job counter must start at zero for either parity of the first step."""
    n, T = 300, 24 * 6
    geo, f, params, state = _region(n, T)
    cpu = engines.run("oracle", geo, params, state, synthetic.T0_2015_US, HOUR, f, 37, 61, full=True)
    gpu = engines.run("hip", geo, params, state, synthetic.T0_2015_US, HOUR, f, 37, 61, full=True)
    for k in range(8):
        _assert_bitexact(gpu["full"][k][37:98], cpu["full"][k][37:98], f"series {k}")
    _assert_bitexact(gpu["state"], cpu["state"], "final state")
    from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_ALL
    r = HipRegion(PT_GS_K, n)
    try:
        r.set_geo(geo)
        r.set_parameters(params)
        r.set_time_axis(synthetic.T0_2015_US, HOUR, T)
        r.set_collection(COLLECT_ALL)
        r.set_state(state)
        for v in range(5):
            r.set_forcing(v, 0, f[v])
        for i in range(37, 98):
            r.run_cells(0, i, 1)
        got = np.stack([r.get_series(k, 37, 61) for k in range(8)])
        _assert_bitexact(got, cpu["full"][:, 37:98], "single-step series")
        _assert_bitexact(r.get_state(), cpu["state"], "single-step final state")
    finally:
        r.close()


def test_copy_state_then_set_state_on_source():
    """copy_state(dst, src) followed at once by set_state(src): the destination keeps the source's old state
    (the upload is ordered after the copy on the region streams)."""
    from shyft_amd.region import HipRegion, PT_GS_K
    n = 1 << 16
    geo, f, params, state = _region(n, 4)
    regs = [HipRegion(PT_GS_K, n) for _ in range(2)]
    try:
        for r in regs:
            r.set_geo(geo)
            r.set_parameters(params)
        src, dst = regs
        a = state.copy()
        a[:, 1] = np.arange(n) * 1e-3  # lwc
        b = state.copy()
        b[:, 1] = -1.0
        for _ in range(3):
            src.set_state(a)
            dst.copy_state_from(src)
            src.set_state(b)
            _assert_bitexact(dst.get_state(), a, "destination state")
            _assert_bitexact(src.get_state(), b, "source state")
    finally:
        for r in regs:
            r.close()


def test_use_ncore_check_uses_host_core_count():
    """region_model.h:579-584 through the raw C ABI: use_ncore above 100 x the host's hardware_concurrency is
    the reference's 'illegal parameter value' error; up to that it is accepted (and ignored by the GPU path)."""
    import os
    from shyft_amd.region import HipRegion, PT_GS_K
    n = 64
    geo, f, params, state = _region(n, 4)
    r = HipRegion(PT_GS_K, n)
    try:
        r.set_geo(geo)
        r.set_parameters(params)
        r.set_time_axis(synthetic.T0_2015_US, HOUR, 4)
        r.set_state(state)
        for v in range(5):
            r.set_forcing(v, 0, f[v])
        hi = os.cpu_count() or 4  # hardware_concurrency lies between the affinity set and the online CPUs
        lo = len(os.sched_getaffinity(0))
        with pytest.raises(RuntimeError, match="more than 100 time available physical cores"):
            r.run_cells(100 * hi + 1, 0, 4)
        r.run_cells(100 * lo, 0, 4)
    finally:
        r.close()
