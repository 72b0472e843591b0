"""Full-size (BASELINE configs[1]) correctness on a sample: a 1,048,576-cell pt_gs_k region runs two 730-step
windows on the device exactly as the bench does (device forcing generator, resident window moved between chunks,
state carried in HBM), and a fixed random sample of 512 cells -- the first and the last cell included -- is
compared bit for bit with the oracle run on just those cells over the same 1460 steps. This is the reference's
stepwise == full property (shyft/tests/api/test_region_model_stacks.py:248-261) at full scale, and it exercises
the size_t offsets of the [series][step][cell] layout beyond 2^32 elements (8 x 730 x 2^20 = 6.1e9).

The bench lines themselves are checked the same way (test_bench_workload_sampled_bitexact): each stack's bench
region and kernel instance (discharge collector, one parameter set -> the uniform / LEAN launch the bench times),
over the bench's horizon in the bench's chunks, 512 sampled cells against the oracle:
- configs[1] pt_gs_k: 1,048,576 cells, one calendar year in 20 chunks of 438 steps;
- configs[3] hbv_stack per GPU: 524,288 cells, the same year;
- configs[4] pt_ss_k per GPU: 1,048,576 cells, 26,280 steps (3 years) in 36 chunks of 730."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1 << 20
W = 730
HOUR = 3600 * 10**6


def _sample(n=512, seed=7):
    rng = np.random.default_rng(seed)
    idx = np.unique(np.concatenate([[0, N - 1], rng.choice(N, n - 2, replace=False)]))
    return idx


def test_full_region_two_windows_sampled_bitexact():
    import torch
    from shyft_amd import synthetic
    from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_ALL
    from tests import oracle_lib
    idx = _sample()
    p = synthetic.default_ptgsk_parameters()
    r = HipRegion(PT_GS_K, N, device=0)
    dev = torch.device("cuda", 0)
    got = np.empty((8, 2 * W, idx.size))
    try:
        r.set_geo(synthetic.geo11(N))
        r.set_parameters(p)
        r.set_time_axis(synthetic.T0_2015_US, HOUR, 2 * W, W)
        r.set_collection(COLLECT_ALL)
        r.set_state(synthetic.default_ptgsk_state(N))
        buf = torch.empty((W, N), dtype=torch.float64, device=dev)
        cols = torch.from_numpy(idx).to(dev)
        for w0 in (0, W):
            r.move_window(w0, 0)
            r.synthetic_forcing(synthetic.SEED, w0, W)
            r.run_cells(0, w0, W)
            for k in range(8):
                torch.cuda.synchronize(dev)
                r.get_series_device(k, w0, W, buf.data_ptr())
                got[k, w0:w0 + W] = buf.index_select(1, cols).cpu().numpy()
        state = r.get_state()[idx]
    finally:
        r.close()
    # the oracle on the sampled cells only: same geo rows, same generator bits (per-cell counter hash)
    geo = synthetic.geo11(N)[idx]
    f = np.stack([synthetic.forcing(1, 0, 2 * W, cell_offset=int(i))[:, :, 0] for i in idx], axis=2)  # [5][T][n]
    exp = oracle_lib.ptgsk_run(geo, p, synthetic.default_ptgsk_state(idx.size), synthetic.T0_2015_US, HOUR, f,
                               full=True)
    same = (got == exp["full"]) | (np.isnan(got) & np.isnan(exp["full"]))
    assert same.all(), f"{(~same).sum()} values differ"
    assert np.array_equal(state, exp["state"])
    assert np.isfinite(got).all() and (got[0] > 0).any()


BENCH_CASES = {   # stack: (cells, chunk, chunks)
    "pt_gs_k": (1 << 20, 438, 20),
    "hbv_stack": (1 << 19, 438, 20),
    "pt_ss_k": (1 << 20, 730, 36),
}


@pytest.mark.parametrize("stack", list(BENCH_CASES))
def test_bench_workload_sampled_bitexact(stack):
    import torch
    import bench
    from shyft_amd import synthetic
    from shyft_amd.region import COLLECT_DISCHARGE
    from tests import oracle_lib
    n, w, k = BENCH_CASES[stack]
    T = w * k
    rng = np.random.default_rng(11)
    idx = np.unique(np.concatenate([[0, n - 1], rng.choice(n, 510, replace=False)]))
    L = bench.Layout(bench.parse(["--stack", stack, "--cells", str(n)]), 1, 0)
    r = bench.build_region(stack, L, 0, w, T)          # the bench's region: geo, default parameters, collector
    params, state0 = bench.stack_defaults(stack, n)
    dev = torch.device("cuda", 0)
    got = np.empty((2, T, idx.size))
    try:
        r.set_state(state0)
        buf = torch.empty((w, n), dtype=torch.float64, device=dev)
        cols = torch.from_numpy(idx).to(dev)
        for c in range(k):
            w0 = c * w
            r.move_window(w0, 0)
            r.synthetic_forcing(synthetic.SEED, w0, w, cell_offset=L.off)
            r.run_cells(0, w0, w)
            for s in range(2):
                torch.cuda.synchronize(dev)
                r.get_series_device(s, w0, w, buf.data_ptr())
                got[s, w0:w0 + w] = buf.index_select(1, cols).cpu().numpy()
        state = r.get_state()[idx]
    finally:
        r.close()
    geo = synthetic.geo11(n)[idx]
    f = np.stack([synthetic.forcing(1, 0, T, cell_offset=int(i))[:, :, 0] for i in idx], axis=2)   # [5][T][n]
    run = {"pt_gs_k": oracle_lib.ptgsk_run, "hbv_stack": oracle_lib.hbv_run, "pt_ss_k": oracle_lib.ptssk_run}[stack]
    exp = run(geo, params, state0[idx], synthetic.T0_2015_US, HOUR, f, ncore=8)
    same = (got == exp["main"]) | (np.isnan(got) & np.isnan(exp["main"]))
    assert same.all(), f"{stack}: {(~same).sum()} of {same.size} values differ"
    assert np.array_equal(state, exp["state"])
    assert np.isfinite(got).all() and (got[0] > 0).any()
