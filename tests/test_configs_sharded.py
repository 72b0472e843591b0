"""BASELINE configs[3] and configs[4] as stated, on one GPU through the engine's shards.

- configs[3]: hbv_stack, 4,194,304 cells x 8,760 hourly steps (the calendar year in 20 chunks of 438), the region in 8
  engine shards (shyft_hip_region_create_sharded on device 0 x 8), catchment sums per chunk;
- configs[4]: pt_ss_k + routing::uhg, 8,388,608 cells x 26,280 steps (3 years in 60 chunks of 438), 8 shards, catchment
  and routing-group sums per chunk, the river network convolved after the last chunk (about 200 GB resident).

Each region runs exactly as `bench.py --gpus 1 --shards 8 --total-cells N` runs it (bench.build_region, the device
forcing generator, the window moved per chunk). Checks:
- 512 sampled cells (first and last included) bit for bit against the CPU oracle over the whole horizon, and their
  final state;
- the same region unsharded (one region on device 0, run after the sharded one is closed): catchment sums, routing
  group sums and the routed river series bit-equal wherever no shard boundary cuts the catchment (for a river: none
  of its upstream network's catchments), within 1e-12 relative where one does (partials added in shard order).

The reference sums the whole region in one process (core/region_model.h:972-1021, core/cell_model.h:308-333,
core/routing.h:344-383); per-cell results never depend on the sharding."""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHUNK = 438
S = 8


def _progress(msg):
    # long GPU tests: a line per phase under gpurun_out/ (the box's hang detector watches it; pytest captures stdout)
    d = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, "progress.log"), "a") as f:
            f.write(f"{time.strftime('%H:%M:%S')} {msg}\n")


def _sample(n, k=512, seed=5):
    rng = np.random.default_rng(seed)
    return np.unique(np.concatenate([[0, n - 1], rng.choice(n, k - 2, replace=False)])).astype(np.int64)


def _cut_catchments(n, n_catch, n_shards):
    cid = lambda i: 1 + (i * n_catch) // n      # synthetic.geo11's catchment of cell i
    cut = set()
    for k in range(1, n_shards):
        b = n * k // n_shards
        if cid(b - 1) == cid(b):
            cut.add(cid(b))
    return cut


def _run(stack, n, n_catch, n_chunks, devices, idx, routing):
    import bench
    from shyft_amd import synthetic
    a = bench.parse(["--stack", stack, "--total-cells", str(n), "--catchments", str(n_catch), "--chunk", str(CHUNK),
                     "--steps", str(n_chunks)])
    L = bench.Layout(a, 1, 0, engine_gpus=1)
    T = CHUNK * n_chunks
    r = bench.build_region(stack, L, 0, CHUNK, T, devices)
    out = {}
    try:
        assert [x[2] for x in r.shards()] == ([n // S] * S if devices else [n])
        G = 0
        if routing:
            _, _, group = synthetic.cell_routing(n, n_catch)
            G = n_catch * len(synthetic.ROUTE_DISTANCES)
            r.set_routing_groups(group, G)
            out["groups"] = np.empty((G, T))
        r.set_state(bench.stack_defaults(stack, n)[1])
        out["sums"] = np.empty((n_catch, T))
        got = np.empty((2, T, idx.size))
        for c in range(n_chunks):
            w0 = c * CHUNK
            r.move_window(w0, 0)
            r.synthetic_forcing(synthetic.SEED, w0, CHUNK)
            r.run_cells(0, w0, CHUNK)
            out["sums"][:, w0:w0 + CHUNK] = r.catchment_sums(0, w0, CHUNK)
            if routing:
                out["groups"][:, w0:w0 + CHUNK] = r.routing_group_sums(w0, CHUNK)
            for s in range(2):
                got[s, w0:w0 + CHUNK] = r.sample_cells(s, idx, w0, CHUNK)
            if c % 10 == 9:
                _progress(f"{stack} {'sharded' if devices else 'unsharded'} chunk {c + 1}/{n_chunks}")
        out["sample"] = got
        out["state"] = r.get_state()[idx]
        out["combine"] = r.combine_path()
    finally:
        r.close()
    return out


def _oracle(stack, n, n_catch, idx, T):
    import bench
    from shyft_amd import synthetic
    from tests import oracle_lib
    geo = synthetic.geo11(n, n_catchments=n_catch)[idx]
    f = np.stack([synthetic.forcing(1, 0, T, cell_offset=int(i))[:, :, 0] for i in idx], axis=2)   # [5][T][n]
    params, state0 = bench.stack_defaults(stack, idx.size)
    run = {"hbv_stack": oracle_lib.hbv_run, "pt_ss_k": oracle_lib.ptssk_run}[stack]
    return run(geo, params, state0, synthetic.T0_2015_US, synthetic.HOUR_US, f, ncore=8)


def _same(a, b):
    return np.array_equal(a, b, equal_nan=True)


def _check_rows(a, b, exact_rows):
    """rows in exact_rows bit-equal, the others within 1e-12 relative (sharded vs unsharded sums)"""
    exact = np.zeros(a.shape[0], bool)
    exact[list(exact_rows)] = True
    assert _same(a[exact], b[exact]), f"{int((a[exact] != b[exact]).sum())} values of uncut rows differ"
    assert np.allclose(a[~exact], b[~exact], rtol=1e-12, atol=0)
    return int(exact.sum()), int((~exact).sum())


def _check(stack, n, n_catch, n_chunks, routing):
    T = CHUNK * n_chunks
    idx = _sample(n)
    _progress(f"{stack} {n} cells: sharded run")
    sh = _run(stack, n, n_catch, n_chunks, [0] * S, idx, routing)
    assert sh["combine"] == "copy"                                  # 8 shards on one device: device copies
    _progress(f"{stack}: oracle on {idx.size} cells")
    exp = _oracle(stack, n, n_catch, idx, T)
    same = (sh["sample"] == exp["main"]) | (np.isnan(sh["sample"]) & np.isnan(exp["main"]))
    assert same.all(), f"{stack}: {(~same).sum()} of {same.size} sampled values differ from the oracle"
    assert np.array_equal(sh["state"], exp["state"])
    assert np.isfinite(sh["sample"]).all() and (sh["sample"][0] > 0).any()
    _progress(f"{stack}: unsharded run")
    un = _run(stack, n, n_catch, n_chunks, None, idx, routing)
    assert _same(sh["sample"], un["sample"]) and _same(sh["state"], un["state"])
    cut = _cut_catchments(n, n_catch, S)
    assert 0 < len(cut) < n_catch
    whole = [c - 1 for c in range(1, n_catch + 1) if c not in cut]   # catchment_ids() = 1..C in cell order
    _check_rows(sh["sums"], un["sums"], whole)
    if routing:
        from shyft_amd import synthetic
        k = len(synthetic.ROUTE_DISTANCES)
        _check_rows(sh["groups"], un["groups"], [g for g in range(n_catch * k) if (g // k) + 1 not in cut])
        ro_sh, ro_un = _route(sh["groups"], n_catch), _route(un["groups"], n_catch)
        # river r's network: itself and everything upstream (downstream of river j is j // 2)
        rivers = synthetic.river_network(n_catch)
        up = {rid: [] for (rid, *_r) in rivers}
        for (rid, ds, *_r) in rivers:
            if ds > 0:
                up[ds].append(rid)

        def net(rid):
            out, todo = set(), [rid]
            while todo:
                x = todo.pop()
                out.add(x)
                todo += up[x]
            return out
        exact_rivers = [rid - 1 for (rid, *_r) in rivers if not (net(rid) & cut)]
        assert exact_rivers
        for a, b in zip(ro_sh, ro_un):
            _check_rows(a, b, exact_rivers)
        assert np.isfinite(ro_sh[2]).all() and (ro_sh[2] > 0).any()
    _progress(f"{stack}: done")


def _route(groups, n_catch):
    from shyft_amd import api, synthetic
    from shyft_amd.region import route
    steps = [int(d / 3600.0 + 0.5) for d in synthetic.ROUTE_DISTANCES]
    G = n_catch * len(steps)
    guhg = [api.make_uhg_from_gamma(steps[k], 7.0, 0.0) for _ in range(n_catch) for k in range(len(steps))]
    rivers = synthetic.river_network(n_catch)
    ruhg = [api.make_uhg_from_gamma(int((d / v) / 3600.0 + 0.5), al, be) for (_, _, d, v, al, be) in rivers]
    down = [ds - 1 for (_, ds, *_rest) in rivers]
    return route(groups, guhg, [g // len(steps) for g in range(G)], ruhg, down, device=0)


@pytest.mark.timeout(900)
def test_c4_hbv_stack_4m_cells_8_shards_calendar_year():
    _check("hbv_stack", 1 << 22, 100, 20, routing=False)


@pytest.mark.timeout(1200)
def test_c5_pt_ss_k_routing_8m_cells_8_shards_26280_steps():
    _check("pt_ss_k", 1 << 23, 100, 60, routing=True)
