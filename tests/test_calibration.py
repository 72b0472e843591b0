"""Calibration (core/model_calibration.h:404-899; expose.h:472-730) over the MI355X engine.

CPU tests: the goal functions against their formulas (time_series.h:2301-2450), the target specification
surface (test_calibration_types.py:316-420), and the search restatements on analytic functions
(sceua_optimizer.cpp, dream_optimizer.cpp, the bounded trust-region stand-in for dlib's find_min_bobyqa).
GPU tests: the reference's optimizer scenario test_region_model_stacks.py:350-422 with its KAT (optimize()
recovers kirchner c1/c2 to 4 decimals, goal <= 10), and the MI355X batching contract: goal values of an
ensemble launch are bit-identical to sequential evaluations, SCE-UA with batching on/off gives the same
trace. Parity of the search traces with the reference is unpinned (no runnable reference here); the
algorithms are pinned by their results on these cases."""
import math

import numpy as np
import pytest


def _api():
    from shyft_amd import api
    return api


# ------------------------------------------------------------------ goal functions (CPU)
def test_goal_functions_match_their_formulas():
    api = _api()
    rng = np.random.default_rng(3)
    o = rng.uniform(1, 10, 200)
    m = o + rng.normal(0, 0.5, 200)
    o[5] = np.nan
    m[7] = np.inf
    ok = np.isfinite(o) & np.isfinite(m)
    oo, mm = o[ok], m[ok]
    ns = np.sum((oo - mm) ** 2) / np.sum((oo - oo.mean()) ** 2)
    assert api.nash_sutcliffe_goal_function(list(o), list(m)) == pytest.approx(ns, rel=1e-12)
    rmse = math.sqrt(np.mean((oo - mm) ** 2)) / oo.mean()
    assert api.rmse_goal_function(list(o), list(m)) == pytest.approx(rmse, rel=1e-12)
    r = np.corrcoef(oo, mm)[0, 1]
    a = mm.mean() / oo.mean()
    b = mm.std(ddof=1) / oo.std(ddof=1)
    kg = math.sqrt((1.0 * (r - 1)) ** 2 + (2.0 * (a - 1)) ** 2 + (0.5 * (b - 1)) ** 2)
    assert api.kling_gupta_goal_function(list(o), list(m), 1.0, 2.0, 0.5) == pytest.approx(kg, rel=1e-10)
    # s_a = s_b = 0: only the correlation term (the optimizer KAT's setting)
    assert api.kling_gupta_goal_function(list(o), list(m), 1.0, 0.0, 0.0) == pytest.approx(1 - r, rel=1e-9)
    assert api.abs_diff_sum_goal_function(list(o), list(m)) == pytest.approx(np.sum(np.abs(oo - mm)), rel=1e-12)
    s = np.full(200, 2.0)
    s[9] = 0.0  # |scale| <= 1e-20 is skipped
    ok2 = ok.copy()
    ok2[9] = False
    assert api.abs_diff_sum_goal_function_scaled(list(o), list(m), list(s)) == pytest.approx(
        np.sum(np.abs(o[ok2] - m[ok2]) / 2.0), rel=1e-12)
    with pytest.raises(RuntimeError):
        api.nash_sutcliffe_goal_function([1.0, 2.0], [1.0])
    # perfect simulation: every criterion at its optimum 0
    assert api.nash_sutcliffe_goal_function(list(oo), list(oo)) == 0.0
    assert api.kling_gupta_goal_function(list(oo), list(oo), 1, 1, 1) == pytest.approx(0.0, abs=1e-7)


def test_target_specification_surface():
    """test_calibration_types.py:316-404: fields, enums, TsTransform averaging, copies."""
    api = _api()
    t = api.TargetSpecificationPts()
    t.scale_factor = 1.0
    for mode in (api.NASH_SUTCLIFFE, api.KLING_GUPTA, api.ABS_DIFF, api.RMSE):
        t.calc_mode = mode
    t.s_r, t.s_a, t.s_b = 1.0, 2.0, 3.0
    assert t.uid is not None
    t.uid = "test"
    assert t.uid == "test"
    cal = api.Calendar()
    start = cal.time(2015, 1, 1, 0, 0, 0)
    dt = api.deltahours(1)
    times = api.UtcTimeVector([start + 1 * dt, start + 3 * dt, start + 4 * dt])
    values = api.DoubleVector([1.0, 3.0, np.nan])
    tsp = api.TsFactory().create_time_point_ts(api.UtcPeriod(start, start + 24 * dt), times, values)
    tsa = api.TsTransform().to_average(start, dt, 24, tsp)
    cids = api.IntVector([0, 2, 3])
    t2 = api.TargetSpecificationPts(tsa, cids, 0.7, api.KLING_GUPTA, 1.0, 1.0, 1.0, api.SNOW_COVERED_AREA, "test_uid")
    assert t2.uid == "test_uid"
    t2.catchment_property = api.SNOW_WATER_EQUIVALENT
    assert t2.catchment_property == api.SNOW_WATER_EQUIVALENT
    t2.catchment_property = api.CELL_CHARGE
    assert list(t2.catchment_indexes) == [0, 2, 3]
    t.ts = api.TimeSeries(tsa)
    tv = api.TargetSpecificationVector()
    tv[:] = [t, t2]
    assert tv.size() == 2
    assert tv[0].ts.value(1) == pytest.approx(1.5)  # linear between points, averaged over [1h, 2h)
    assert tv[0].ts.value(2) == pytest.approx(2.5)
    assert math.isnan(tv[0].ts.value(3))  # strictly linear: the nan at 4h poisons [3h, 4h)
    tsa.set(1, 3.0)
    assert tv[0].ts.value(1) == pytest.approx(1.5)  # the target holds its own copy
    tv2 = api.TargetSpecificationVector(tv)
    tv2[0].scale_factor = 10.0
    assert tv[0].scale_factor == pytest.approx(1.0) and tv2[0].scale_factor == pytest.approx(10.0)
    # the river constructor
    t3 = api.TargetSpecificationPts(tsa, 7, 0.7, api.KLING_GUPTA, 1.0, 1.0, 1.0, "uid_r")
    assert t3.catchment_property == api.ROUTED_DISCHARGE and t3.river_id == 7 and t3.uid == "uid_r"
    assert t3._impl().ts.size() == 24


# ------------------------------------------------------------------ search restatements (CPU)
def _quad(x0):
    c = np.asarray(x0)
    w = np.arange(1, len(c) + 1, dtype=float)
    return lambda x: float(np.sum(w * (np.asarray(x) - c) ** 2))


def test_sceua_restatement_converges_and_is_deterministic():
    from shyft_amd.api import _api as A
    f = _quad([0.3, 0.7, 0.55])
    x1, y1, st1 = A._sceua_find_min(f, [0.9, 0.1, 0.5], 3000, 1e-4, 1e-6)
    x2, y2, st2 = A._sceua_find_min(f, [0.9, 0.1, 0.5], 3000, 1e-4, 1e-6)
    assert (x1, y1, st1) == (x2, y2, st2)  # default-seeded std::default_random_engine per call
    assert st1 in (1, 2, 3)  # fx / x convergence or max iterations
    assert y1 < 1e-4
    assert np.allclose(x1, [0.3, 0.7, 0.55], atol=0.02)


def test_dream_restatement_finds_the_mode():
    from shyft_amd.api import _api as A
    f = _quad([0.4, 0.6, 0.5, 0.45])
    x, g = A._dream_find_max(lambda v: -50.0 * f(v), [0.5] * 4, 1500)
    assert g <= 0.0
    assert np.allclose(x, [0.4, 0.6, 0.5, 0.45], atol=0.05)


def test_box_trust_region_bounded_minimisation():
    from shyft_amd.api import _api as A
    # interior minimum of a rotated, badly scaled quadratic
    def f(x):
        u, v = x[0] - 0.31, x[1] - 0.77
        return (u + v) ** 2 + 30.0 * (u - 0.5 * v) ** 2
    x, y, n = A._box_trust_region_min(f, [0.55, 0.58], 0.1, 1e-6, 1500)
    assert n <= 1500
    assert abs(x[0] - 0.31) < 1e-4 and abs(x[1] - 0.77) < 1e-4
    # minimum outside the box: lands on the bound
    x, y, n = A._box_trust_region_min(lambda x: (x[0] - 1.4) ** 2 + (x[1] - 0.2) ** 2, [0.5, 0.5], 0.1, 1e-6, 500)
    assert x[0] == pytest.approx(1.0, abs=1e-9) and x[1] == pytest.approx(0.2, abs=1e-4)


# ------------------------------------------------------------------ the optimizer on the device (GPU)
def _opt_scenario(num_cells=20):
    """test_region_model_stacks.py:350-398: 20 cells, 240 hourly steps, q0 = 40, KG target on catchment 1."""
    from tests.test_api_region_model import build_model, dummy_env
    api = _api()
    from shyft_amd.api import pt_gs_k
    model = build_model(pt_gs_k.PTGSKModel, pt_gs_k.PTGSKParameter, num_cells)
    cal = api.Calendar()
    t0 = cal.time(2015, 1, 1, 0, 0, 0)
    dt = api.deltahours(1)
    n = 240
    ta = api.TimeAxisFixedDeltaT(t0, dt, n)
    model.initialize_cell_environment(ta)
    model.interpolate(api.InterpolationParameter(), dummy_env(ta, model.get_cells()[num_cells // 2].geo.mid_point()))
    s0 = pt_gs_k.PTGSKStateVector()
    for _ in range(num_cells):
        si = pt_gs_k.PTGSKState()
        si.kirchner.q = 40.0
        s0.append(si)
    model.set_states(s0)
    model.run_cells()
    cids = api.IntVector.from_numpy([1])
    sum_discharge = model.statistics.discharge(cids)
    assert model.statistics.discharge_value(cids, 0) >= 130.0
    opt_model = pt_gs_k.create_opt_model_clone(model)
    opt_model.run_cells()
    opt_model.revert_to_initial_state()
    tsa = api.TsTransform().to_average(t0, dt, n, sum_discharge)
    return api, pt_gs_k, model, opt_model, tsa, cids


@pytest.mark.gpu
def test_optimizer_recovers_kirchner_parameters():
    """The reference KAT (test_region_model_stacks.py:380-422)."""
    api, pt_gs_k, model, opt_model, tsa, cids = _opt_scenario()
    model_type = pt_gs_k.PTGSKModel
    optimizer = pt_gs_k.PTGSKOptModel.optimizer_t(opt_model)
    t_spec_1 = api.TargetSpecificationPts(tsa, cids, 1.0, api.KLING_GUPTA, 1.0, 0.0, 0.0, api.DISCHARGE, "test_uid")
    target_spec = api.TargetSpecificationVector()
    target_spec.append(t_spec_1)
    upper_bound = model_type.parameter_t(model.get_region_parameter())
    lower_bound = model_type.parameter_t(model.get_region_parameter())
    upper_bound.kirchner.c1 = -1.9
    lower_bound.kirchner.c1 = -3.0
    upper_bound.kirchner.c2 = 0.99
    lower_bound.kirchner.c2 = 0.80
    optimizer.set_target_specification(target_spec, lower_bound, upper_bound)
    p0 = model_type.parameter_t(model.get_region_parameter())
    orig_c1, orig_c2 = p0.kirchner.c1, p0.kirchner.c2
    goal_f0 = optimizer.calculate_goal_function(p0)
    assert goal_f0 == pytest.approx(0.0, abs=1e-12)  # the target IS the simulation with p0
    p0.kirchner.c1 = -2.4
    p0.kirchner.c2 = 0.91
    opt_param = optimizer.optimize(p0, 1500, 0.1, 1e-5)
    goal_fx = optimizer.calculate_goal_function(opt_param)
    assert goal_fx <= 10.0
    assert round(orig_c1 - opt_param.kirchner.c1, 4) == 0  # assertAlmostEqual(..., 4)
    assert round(orig_c2 - opt_param.kirchner.c2, 4) == 0
    assert optimizer.trace_size > 3  # optimize() restarted the trace; it holds this search's evaluations
    assert min(optimizer.trace_goal_function_values) <= optimizer.trace_goal_function_value(0)
    global_opt_param = optimizer.optimize_global(p0, max_n_evaluations=1500, max_seconds=3.0, solver_eps=1e-5)
    assert global_opt_param is not None
    assert optimizer.calculate_goal_function(global_opt_param) <= goal_fx + 0.05


@pytest.mark.gpu
def test_batched_goal_functions_are_bit_identical_to_sequential():
    api, pt_gs_k, model, opt_model, tsa, cids = _opt_scenario()
    targets = api.TargetSpecificationVector()
    targets.append(api.TargetSpecificationPts(tsa, cids, 1.0, api.NASH_SUTCLIFFE, 1.0, 1.0, 1.0, api.DISCHARGE))
    targets.append(api.TargetSpecificationPts(tsa, cids, 0.5, api.KLING_GUPTA, 1.0, 2.0, 0.5, api.DISCHARGE))
    targets.append(api.TargetSpecificationPts(tsa, cids, 0.25, api.ABS_DIFF, 1.0, 1.0, 1.0, api.CELL_CHARGE))
    targets.append(api.TargetSpecificationPts(tsa, cids, 0.25, api.RMSE, 1.0, 1.0, 1.0, api.SNOW_WATER_EQUIVALENT))
    lo = pt_gs_k.PTGSKParameter(model.get_region_parameter())
    hi = pt_gs_k.PTGSKParameter(model.get_region_parameter())
    lo.kirchner.c1, hi.kirchner.c1 = -3.0, -1.9
    lo.kirchner.c2, hi.kirchner.c2 = 0.8, 0.99
    lo.gs.tx, hi.gs.tx = -2.0, 2.0
    o = pt_gs_k.PTGSKOptimizer(opt_model)
    o.set_target_specification(targets, lo, hi)
    rng = np.random.default_rng(5)
    ps = []
    for _ in range(9):
        p = pt_gs_k.PTGSKParameter(model.get_region_parameter())
        p.kirchner.c1 = rng.uniform(-3.0, -1.9)
        p.kirchner.c2 = rng.uniform(0.8, 0.99)
        p.gs.tx = rng.uniform(-2, 2)
        ps.append(p)
    batched = o.calculate_goal_functions(ps)
    assert o.trace_size == 9
    sequential = [o.calculate_goal_function(p) for p in ps]
    assert batched == sequential  # bit-identical
    assert all(np.isfinite(batched))


@pytest.mark.gpu
def test_sceua_batched_equals_sequential():
    api, pt_gs_k, model, opt_model, tsa, cids = _opt_scenario()
    targets = api.TargetSpecificationVector()
    targets.append(api.TargetSpecificationPts(tsa, cids, 1.0, api.NASH_SUTCLIFFE, 1.0, 1.0, 1.0, api.DISCHARGE))
    lo = pt_gs_k.PTGSKParameter(model.get_region_parameter())
    hi = pt_gs_k.PTGSKParameter(model.get_region_parameter())
    lo.kirchner.c1, hi.kirchner.c1 = -3.0, -1.9
    lo.kirchner.c2, hi.kirchner.c2 = 0.8, 0.99
    p0 = pt_gs_k.PTGSKParameter(model.get_region_parameter())
    p0.kirchner.c1, p0.kirchner.c2 = -2.2, 0.85
    runs = []
    for batch in (True, False):
        o = pt_gs_k.PTGSKOptimizer(opt_model)
        o.batch_evaluation = batch
        o.set_target_specification(targets, lo, hi)
        p = o.optimize_sceua(p0, 300, 1e-4, 1e-6)
        runs.append((p.to_vector(), o.trace_goal_function_values))
    assert runs[0][0] == runs[1][0]
    assert runs[0][1] == runs[1][1]
    assert min(runs[0][1]) < 1e-3
