"""Sharded regions (shyft_hip_region_create_sharded): one region_model whose cells are split into contiguous shards,
driven from one process -- the engine's multi-GPU path (core/region_model.h:972-1021 runs the whole region in one
process; catchment sums over all cells, core/cell_model.h:308-333; routing inflows, core/routing.h:344-383).

On a one-GPU box the shards share device 0, so the partial sums combine by device copies; with one shard per GPU the
same code all-gathers them with RCCL. Per-cell results never depend on the sharding (run_cells has no cross-cell
coupling): every series and state value must equal the unsharded region's bit for bit. A catchment (or routing
group) whose cells lie in one shard sums exactly as unsharded (the other shards' partials are +0.0); one that a shard
boundary cuts is reassociated (within 1e-12 relative)."""
import numpy as np
import pytest

from shyft_amd import synthetic

pytestmark = pytest.mark.gpu

HOUR = synthetic.HOUR_US
N, C, T = 4096, 100, 96          # cell 2048 starts catchment 51: two shards split at a catchment boundary


def _region(stack, devices, n=N, n_catch=C, T_=T, collect=None, state=None):
    import bench
    from shyft_amd.region import HipRegion, COLLECT_ALL, STACK_NSTATE
    sid = {"pt_gs_k": 1, "hbv_stack": 2, "pt_ss_k": 3}[stack]
    r = HipRegion(sid, n, devices=devices) if devices is not None else HipRegion(sid, n)
    r.set_geo(synthetic.geo11(n, n_catchments=n_catch))
    r.set_parameters(bench.stack_defaults(stack, 1)[0])
    r.set_time_axis(synthetic.T0_2015_US, HOUR, T_)
    r.set_collection(COLLECT_ALL if collect is None else collect)
    r.set_state(bench.stack_defaults(stack, n)[1] if state is None else state)
    return r


def _run(r, T_=T):
    r.synthetic_forcing(synthetic.SEED, 0, T_)
    r.run_cells(0, 0, T_)


def _same(a, b):
    return np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("stack", ["pt_gs_k", "hbv_stack", "pt_ss_k"])
def test_two_shards_on_one_device_equal_unsharded(stack):
    ref, sh = _region(stack, None), _region(stack, [0, 0])
    try:
        assert sh.shards() == [(0, 0, N // 2), (0, N // 2, N // 2)]
        assert sh.combine_path() == "copy" and ref.combine_path() == "none"
        _run(ref)
        _run(sh)
        ns = 9 if stack == "hbv_stack" else 8
        for k in range(ns):
            assert _same(sh.get_series(k, 0, T), ref.get_series(k, 0, T)), f"series {k}"
        assert _same(sh.get_state(), ref.get_state())
        for v in range(5):
            assert _same(sh.get_forcing(v, 0, T), ref.get_forcing(v, 0, T))
        assert np.array_equal(sh.catchment_ids(), ref.catchment_ids())
        assert _same(sh.catchment_sums(0, 0, T), ref.catchment_sums(0, 0, T))
        # a selection inside one shard reduces the same cells in the same order: exact; one that spans the shards
        # adds the shards' partial sums (reassociated)
        assert _same(sh.statistics(0, [1, 50]), ref.statistics(0, [1, 50]))
        assert _same(sh.statistics(0, [77, 100], weighted=True), ref.statistics(0, [77, 100], weighted=True))
        assert np.allclose(sh.statistics(0, [1, 50, 51, 100]), ref.statistics(0, [1, 50, 51, 100]), rtol=1e-12, atol=0)
        assert np.allclose(sh.statistics(0, [3, 77], weighted=True), ref.statistics(0, [3, 77], weighted=True),
                           rtol=1e-12, atol=0)
        from shyft_amd.region import SCOPE_CELL_IX
        cells = [0, 5, 2047, 2048, 4095]
        got = sh.statistics(0, cells, scope=SCOPE_CELL_IX)
        exp = ref.statistics(0, cells, scope=SCOPE_CELL_IX)
        assert np.allclose(got, exp, rtol=1e-12, atol=0)   # a cut selection: reassociated partial sums
    finally:
        ref.close()
        sh.close()


def test_three_shards_cut_catchments_within_reassociation():
    ref, sh = _region("pt_gs_k", None), _region("pt_gs_k", [0, 0, 0])
    try:
        _run(ref)
        _run(sh)
        assert _same(sh.get_series(0, 0, T), ref.get_series(0, 0, T))
        a, b = sh.catchment_sums(0, 0, T), ref.catchment_sums(0, 0, T)
        assert np.allclose(a, b, rtol=1e-12, atol=0)
        cut = {int(synthetic.geo11(N, n_catchments=C)[c0, 4]) for (_, c0, _) in sh.shards()[1:]}
        whole = [i for i, cid in enumerate(ref.catchment_ids()) if int(cid) not in cut]
        assert _same(a[whole], b[whole])                   # catchments inside one shard: exact
    finally:
        ref.close()
        sh.close()


def test_routing_group_sums_and_routed_river_equal_unsharded():
    from shyft_amd import api
    from shyft_amd.region import route
    ref, sh = _region("pt_ss_k", None), _region("pt_ss_k", [0, 0])
    try:
        _, _, group = synthetic.cell_routing(N, C)
        G = C * len(synthetic.ROUTE_DISTANCES)
        for r in (ref, sh):
            r.set_routing_groups(group, G)
            _run(r)
        a, b = sh.routing_group_sums(0, T), ref.routing_group_sums(0, T)
        assert _same(a, b)
        steps = [int(d / 3600.0 + 0.5) for d in synthetic.ROUTE_DISTANCES]
        guhg = [api.make_uhg_from_gamma(steps[k], 7.0, 0.0) for _ in range(C) for k in range(len(steps))]
        rivers = synthetic.river_network(C)
        ruhg = [api.make_uhg_from_gamma(int((d / v) / 3600.0 + 0.5), al, be) for (_, _, d, v, al, be) in rivers]
        down = [ds - 1 for (_, ds, *_rest) in rivers]
        gr = [g // len(steps) for g in range(G)]
        out_a = route(a, guhg, gr, ruhg, down)
        out_b = route(b, guhg, gr, ruhg, down)
        for x, y in zip(out_a, out_b):
            assert _same(x, y)
    finally:
        ref.close()
        sh.close()


def test_catchment_filter_idle_shard_and_interpolation():
    """A filter on catchments of the second shard only: the first shard is idle (not run, not interpolated); the
    calculated cells match the unsharded filtered region, the IDW forcing too (per-cell neighbour tables)."""
    import bench
    from tests.test_idw_c3 import C3_PARAMS
    ref, sh = _region("pt_gs_k", None), _region("pt_gs_k", [0, 0])
    try:
        xyz = bench.station_network(N)
        vals = bench.station_values(xyz, 0, T)
        for r in (ref, sh):
            r.set_catchment_filter([60, 61, 99])
            for v in range(5):
                r.interpolate(v, xyz, vals[v], 0, C3_PARAMS[v])
            r.run_cells(0, 0, T)
        cid = synthetic.geo11(N, n_catchments=C)[:, 4]
        on = np.isin(cid, [60, 61, 99])
        for v in range(5):
            a, b = sh.get_forcing(v, 0, T), ref.get_forcing(v, 0, T)
            assert _same(a[:, on], b[:, on])
        assert _same(sh.get_series(0, 0, T)[:, on], ref.get_series(0, 0, T)[:, on])
        assert _same(sh.catchment_sums(0, 0, T), ref.catchment_sums(0, 0, T))
        assert sh.interpolation_path(0) == ref.interpolation_path(0)
        with pytest.raises(RuntimeError, match="no cells have supplied cid"):
            sh.set_catchment_filter([12345])
    finally:
        ref.close()
        sh.close()


def test_ensemble_and_host_roundtrips():
    from shyft_amd.region import COLLECT_DISCHARGE
    import bench
    ref, sh = _region("pt_gs_k", None), _region("pt_gs_k", [0, 0])
    try:
        rng = np.random.default_rng(1)
        f = rng.uniform(0, 1, size=(T, N))
        for r in (ref, sh):
            _run(r)
            r.set_forcing(1, 0, f)          # host forcing split over the shards and back
        assert _same(sh.get_forcing(1, 0, T), f)
        p = np.tile(bench.stack_defaults("pt_gs_k", 1)[0], (3, 1))
        p[1, 0] -= 0.3                      # kirchner c1 of member 1
        ref.ensemble_run(p, 0, T, COLLECT_DISCHARGE)
        sh.ensemble_run(p, 0, T, COLLECT_DISCHARGE)
        assert _same(sh.ensemble_sums(0, 0, T), ref.ensemble_sums(0, 0, T))
    finally:
        ref.close()
        sh.close()


def test_api_model_with_devices():
    """PTGSKModel(..., devices=[0, 0]) behaves as the unsharded model through the reference's Python scenario
    (test_region_model_stacks.py:114-200: interpolate from a region environment, run_cells, the discharge
    statistics) and a deep clone (create_opt_model_clone) of it stays sharded."""
    from shyft_amd import api
    from shyft_amd.api import pt_gs_k
    from tests.test_api_region_model import build_model, dummy_env, interpolation_parameter

    def sharded(gcds, p):
        return pt_gs_k.PTGSKModel(gcds, p, devices=[0, 0])

    a = build_model(pt_gs_k.PTGSKModel, pt_gs_k.PTGSKParameter, 20, num_catchments=4)
    b = build_model(sharded, pt_gs_k.PTGSKParameter, 20, num_catchments=4)
    assert list(b.shard_devices) == [0, 0] and list(a.shard_devices) == [0]
    cal = api.Calendar()
    ta = api.TimeAxisFixedDeltaT(cal.time(2015, 1, 1, 0, 0, 0), api.deltahours(1), 240)
    for m in (a, b):
        m.initialize_cell_environment(ta)
        m.interpolate(interpolation_parameter(), dummy_env(ta, m.get_cells()[10].geo.mid_point()))
        m.set_state_collection(-1, True)
        m.run_cells()
    for cids in ([], [1], [2, 4]):
        qa = a.statistics.discharge(api.IntVector(cids))
        qb = b.statistics.discharge(api.IntVector(cids))
        assert np.allclose(qa.values.to_numpy(), qb.values.to_numpy(), rtol=1e-12, atol=0)  # cids interleave (i % 4)
    ea = a.statistics.charge(api.IntVector([1, 2, 17]), ix_type=api.stat_scope.cell).values.to_numpy()
    eb = b.statistics.charge(api.IntVector([1, 2, 17]), ix_type=api.stat_scope.cell).values.to_numpy()
    assert np.allclose(ea, eb, rtol=1e-12, atol=0)
    c = pt_gs_k.create_opt_model_clone(b)
    assert list(c.shard_devices) == [0, 0]
    c.run_cells()


# ---- the combine path's choice, self-check and fallbacks (shyft_hip_region_create_sharded_ex) ----
# On a one-GPU box RCCL_ALWAYS makes a one-shard region build a one-rank communicator, so ncclCommInitAll, the
# self-check's ncclAllGather and the run-time all-gathers execute on the hardware; the TEST_ flags inject the failures
# whose fallback must leave every result unchanged.

def _sums_vs_unsharded(sh, stack="pt_gs_k"):
    ref = _region(stack, None)
    try:
        _run(ref)
        _run(sh)
        assert _same(sh.catchment_sums(0, 0, T), ref.catchment_sums(0, 0, T))
        assert _same(sh.get_series(0, 0, T), ref.get_series(0, 0, T))
    finally:
        ref.close()


def _flagged(flags, devices=(0,)):
    from shyft_amd.region import HipRegion, COLLECT_ALL
    import bench
    r = HipRegion(1, N, devices=list(devices), shard_flags=flags)
    r.set_geo(synthetic.geo11(N, n_catchments=C))
    r.set_parameters(bench.stack_defaults("pt_gs_k", 1)[0])
    r.set_time_axis(synthetic.T0_2015_US, HOUR, T)
    r.set_collection(COLLECT_ALL)
    r.set_state(bench.stack_defaults("pt_gs_k", N)[1])
    return r


def test_rccl_one_rank_self_check_and_sums():
    from shyft_amd.region import SHARD_RCCL_ALWAYS
    sh = _flagged(SHARD_RCCL_ALWAYS)
    try:
        assert sh.combine_path() == "rccl", sh.combine_report()
        assert "self-check passed" in sh.combine_report()
        _sums_vs_unsharded(sh)
        assert sh.combine_path() == "rccl", sh.combine_report()     # no run-time fallback happened
        c = sh.__class__.__new__(sh.__class__)                       # a clone builds and checks its own communicator
        import ctypes as C
        h = C.c_void_p()
        assert sh._L.shyft_hip_region_clone(sh.h, C.byref(h)) == 0
        c._L, c.h, c.stack, c.n = sh._L, h, sh.stack, sh.n
        try:
            assert c.combine_path() == "rccl" and "self-check passed" in c.combine_report()
        finally:
            c.close()
    finally:
        sh.close()


def test_rccl_init_failure_falls_back_to_copies():
    from shyft_amd.region import SHARD_RCCL_ALWAYS, SHARD_TEST_FAIL_INIT
    sh = _flagged(SHARD_RCCL_ALWAYS | SHARD_TEST_FAIL_INIT)
    try:
        assert sh.combine_path() == "copy"
        assert "initialisation failed" in sh.combine_report() and "injected" in sh.combine_report()
        _sums_vs_unsharded(sh)
    finally:
        sh.close()


def test_rccl_self_check_mismatch_falls_back_to_copies():
    from shyft_amd.region import SHARD_RCCL_ALWAYS, SHARD_TEST_CORRUPT_CHECK
    sh = _flagged(SHARD_RCCL_ALWAYS | SHARD_TEST_CORRUPT_CHECK)
    try:
        assert sh.combine_path() == "copy"
        assert "self-check failed" in sh.combine_report()
        _sums_vs_unsharded(sh)
    finally:
        sh.close()


def test_rccl_gather_failure_at_run_time_falls_back_to_copies():
    from shyft_amd.region import SHARD_RCCL_ALWAYS, SHARD_TEST_FAIL_GATHER
    sh = _flagged(SHARD_RCCL_ALWAYS | SHARD_TEST_FAIL_GATHER)
    try:
        assert sh.combine_path() == "rccl" and "self-check passed" in sh.combine_report()
        _sums_vs_unsharded(sh)                                       # the first all-gather fails: copies, same sums
        assert sh.combine_path() == "copy"
        assert "failed at run time" in sh.combine_report()
    finally:
        sh.close()


def test_rccl_stalled_self_check_falls_back_to_copies(monkeypatch):
    """Every RCCL step has a deadline (non-blocking communicators, polled): a self-check all-gather that is not seen to
    complete (TEST_STALL_CHECK) is aborted at SHYFT_HIP_RCCL_DEADLINE_MS and the region runs on device copies, with
    the same sums and the reason in its report."""
    import time
    from shyft_amd.region import SHARD_RCCL_ALWAYS, SHARD_TEST_STALL_CHECK
    monkeypatch.setenv("SHYFT_HIP_RCCL_DEADLINE_MS", "1500")
    t0 = time.monotonic()
    sh = _flagged(SHARD_RCCL_ALWAYS | SHARD_TEST_STALL_CHECK)
    took = time.monotonic() - t0
    try:
        assert sh.combine_path() == "copy", sh.combine_report()
        rep = sh.combine_report()
        assert "did not complete within 1500 ms" in rep and "injected stall" in rep, rep
        assert took < 60, took
        _sums_vs_unsharded(sh)
        assert sh.combine_path() == "copy"
    finally:
        sh.close()


def test_shards_on_distinct_gpus_use_rccl():
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    sh = _region("pt_gs_k", [0, 1])
    try:
        assert sh.combine_path() == "rccl", sh.combine_report()
        _sums_vs_unsharded(sh)
        assert sh.combine_path() == "rccl"
    finally:
        sh.close()


def test_duplicate_catchments_in_filter_accepted_like_unsharded():
    ref, sh = _region("pt_gs_k", None), _region("pt_gs_k", [0, 0])
    try:
        for r in (ref, sh):
            r.set_catchment_filter([3, 3, 3, 60])
            _run(r)
        cid = synthetic.geo11(N, n_catchments=C)[:, 4]
        on = np.isin(cid, [3, 60])
        assert _same(sh.get_series(0, 0, T)[:, on], ref.get_series(0, 0, T)[:, on])
        assert _same(sh.catchment_sums(0, 0, T), ref.catchment_sums(0, 0, T))
    finally:
        ref.close()
        sh.close()


def test_shards_below_the_small_region_threshold_equal_unsharded():
    """262,144 cells = 1,024 workgroups of 256: the unsharded region runs the 4-wave 256-lane pt_gs_k instance, each of
    its two 131,072-cell shards (512 workgroups <= 2 per CU) the small-region 64-lane speculative instance. The
    per-cell arithmetic is the same, so every series must be bit-equal (January: Brent jobs on both paths)."""
    n, Tn = 1 << 18, 96
    ref, sh = _region("pt_gs_k", None, n=n, T_=Tn), _region("pt_gs_k", [0, 0], n=n, T_=Tn)
    try:
        for r in (ref, sh):
            r.synthetic_forcing(synthetic.SEED, 0, Tn)
            r.run_cells(0, 0, Tn)
        for k in range(8):
            assert _same(sh.get_series(k, 0, Tn), ref.get_series(k, 0, Tn)), f"series {k}"
        assert _same(sh.get_state(), ref.get_state())
    finally:
        ref.close()
        sh.close()


def test_sample_cells_equals_full_series():
    ref, sh = _region("pt_gs_k", None), _region("pt_gs_k", [0, 0, 0])
    try:
        _run(ref)
        _run(sh)
        cells = [0, 1, 1365, 1366, 2047, 2048, 4095, 7]
        full = ref.get_series(1, 0, T)
        for r in (ref, sh):
            assert _same(r.sample_cells(1, cells, 10, 40), full[10:50][:, cells])
            from shyft_amd.region import SERIES_FORCING
            assert _same(r.sample_cells(SERIES_FORCING + 0, cells, 0, T), ref.get_forcing(0, 0, T)[:, cells])
        with pytest.raises(RuntimeError, match="out of range"):
            sh.sample_cells(0, [N], 0, 1)
    finally:
        ref.close()
        sh.close()


# ---- SHYFT_HIP_SHARD_BALANCE_Z: shards dealt by elevation rank ("interleave or sort cells by z") ----

def _ramp_region(n, devices, flags=0, T_=438):
    """pt_gs_k region whose elevation ramps 0 -> 3000 m with the cell index (catchments at rising elevation, as in
    real regions), January: the high cells carry the snow and the corr_lwc Brent jobs, the low ones do not."""
    import bench
    from shyft_amd.region import HipRegion, COLLECT_DISCHARGE
    r = HipRegion(1, n, devices=devices, shard_flags=flags) if devices is not None else HipRegion(1, n)
    g = synthetic.geo11(n, n_catchments=C)
    g[:, 2] = np.linspace(0.0, 3000.0, n)
    r.set_geo(g)
    r.set_parameters(bench.stack_defaults("pt_gs_k", 1)[0])
    r.set_time_axis(synthetic.T0_2015_US, HOUR, T_)
    r.set_collection(COLLECT_DISCHARGE)
    r.set_state(bench.stack_defaults("pt_gs_k", n)[1])
    return r


def test_balance_z_spreads_snow_work_and_keeps_results():
    from shyft_amd.region import SHARD_BALANCE_Z, KNOB_SERIAL_SHARDS
    n, S, T_ = 1 << 19, 4, 438
    ref = _ramp_region(n, None, T_=T_)
    try:
        ref.synthetic_forcing(synthetic.SEED, 0, T_)
        ref.run_cells(0, 0, T_)
        exp = [ref.get_series(k, 0, T_) for k in range(2)]
        exp_state = ref.get_state()
        exp_sums = ref.catchment_sums(0, 0, T_)
    finally:
        ref.close()
    spread = {}
    for name, flags in (("contiguous", 0), ("balanced", SHARD_BALANCE_Z)):
        sh = _ramp_region(n, [0] * S, flags, T_)
        try:
            sh.set_test_knob(KNOB_SERIAL_SHARDS, 1)     # per-shard kernel times without the other shards beside
            sh.synthetic_forcing(synthetic.SEED, 0, T_)
            sh.run_cells(0, 0, T_)
            ms = sh.shard_run_ms()
            spread[name] = (max(ms) - min(ms)) / max(ms)
            for k in range(2):                         # per-cell results in the region's cell order: exact
                assert _same(sh.get_series(k, 0, T_), exp[k]), f"{name} series {k}"
            assert _same(sh.get_state(), exp_state)
            a = sh.catchment_sums(0, 0, T_)
            if flags:                                  # every catchment spans the shards: reassociated
                assert np.allclose(a, exp_sums, rtol=1e-12, atol=0)
                cells = [0, 1, n // 2, n - 1, 12345]
                assert _same(sh.sample_cells(0, cells, 0, T_), exp[0][:, cells])
                buf = np.empty(T_)
                from shyft_amd import _native
                import ctypes as C_
                assert sh._L.shyft_hip_cell_series(sh.h, 1, n - 1, 0, T_, buf.ctypes.data_as(C_.c_void_p), 0) == 0
                assert _same(buf, exp[1][:, n - 1])
                f = sh.get_forcing(1, 0, 4)            # forcing in region order; and back
                sh.set_forcing(1, 0, f)
                assert _same(sh.get_forcing(1, 0, 4), f)
            print(name, [round(x, 2) for x in ms], round(spread[name], 3))
        finally:
            sh.close()
    # the per-shard kernel times are reported, not asserted (wall-clock spread depends on the box): the
    # measured spread is in DESIGN.md (r05: 29.8 % contiguous, 1.7 % dealt by elevation)
    print("per-shard kernel time spread", spread)


def test_balance_z_refuses_per_cell_data_before_the_deal():
    """SHYFT_HIP_SHARD_BALANCE_Z deals the cells at the first set_geo: state, forcing, per-cell parameter indexes or
    routing groups given before it would land on the wrong cells, so they raise; after set_geo the same
    calls work."""
    from shyft_amd.region import HipRegion, SHARD_BALANCE_Z, PT_GS_K
    from shyft_amd._native import ShyftHipError
    import bench
    n = 4096
    r = HipRegion(PT_GS_K, n, devices=[0, 0], shard_flags=SHARD_BALANCE_Z)
    try:
        st = bench.stack_defaults("pt_gs_k", n)[1]
        with pytest.raises(ShyftHipError, match="dealt by elevation"):
            r.set_state(st)
        with pytest.raises(ShyftHipError, match="dealt by elevation"):
            r.set_routing_groups(np.zeros(n, dtype=np.int32), 1)
        r.set_geo(synthetic.geo11(n, n_catchments=C))
        r.set_state(st)
        assert np.array_equal(r.get_state(), st)
    finally:
        r.close()


def test_clone_failure_midway_cleans_up_and_leaves_the_source_usable():
    """a clone that fails at shard k > 0 (shards before it cloned, their streams created) must report
    the error and release what it built -- not crash in the clean-up -- and the source region keeps working."""
    import ctypes as C
    from shyft_amd.region import KNOB_CLONE_FAIL_AT
    sh = _flagged(0, devices=(0, 0, 0))
    try:
        s0 = sh.get_state()
        _run(sh)
        before = sh.catchment_sums(0, 0, T), sh.get_series(0, 0, T)
        for k in (2, 1, 0):
            sh.set_test_knob(KNOB_CLONE_FAIL_AT, k)
            h = C.c_void_p()
            assert sh._L.shyft_hip_region_clone(sh.h, C.byref(h)) != 0
            assert not h.value
            assert f"injected failure at shard {k}" in sh._L.shyft_hip_last_error(None).decode()
        # the knob disarms itself: the next clone builds, and the source still runs with unchanged results
        h = C.c_void_p()
        assert sh._L.shyft_hip_region_clone(sh.h, C.byref(h)) == 0 and h.value
        sh._L.shyft_hip_region_destroy(h)
        sh.set_state(s0)
        _run(sh)
        assert _same(sh.catchment_sums(0, 0, T), before[0]) and _same(sh.get_series(0, 0, T), before[1])
    finally:
        sh.close()


def test_clone_fail_knob_needs_a_sharded_region():
    from shyft_amd._native import ShyftHipError
    from shyft_amd.region import KNOB_CLONE_FAIL_AT
    r = _region("pt_gs_k", None)
    try:
        with pytest.raises(ShyftHipError, match="needs a sharded region"):
            r.set_test_knob(KNOB_CLONE_FAIL_AT, 1)
    finally:
        r.close()
