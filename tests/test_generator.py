"""The device forcing generator (kernels/synth.hip) against its numpy statement
(shyft_amd/synthetic.forcing), bit for bit: even and odd cell counts, a window that starts mid-year and a cell offset
(a rank's or a shard's slice), and windows longer than the kernel's 64 row blocks (several rows per workgroup, each
row's step terms shared through LDS) and than one 256-row LDS batch."""
import numpy as np
import pytest

from shyft_amd import synthetic

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,T", [(1000, 30), (1001, 30), (4096, 30), (1001, 700), (257, 17000)])
def test_device_generator_matches_numpy(n, T):
    from shyft_amd.region import HipRegion, PT_GS_K
    off, step0 = 12345, 4000
    geo = synthetic.geo11(n, cell_offset=off, n_total=1 << 20)
    r = HipRegion(PT_GS_K, n)
    try:
        r.set_geo(geo)
        r.set_parameters(synthetic.default_ptgsk_parameters())
        r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, step0 + T)
        r.synthetic_forcing(synthetic.SEED, step0, T, cell_offset=off)
        want = synthetic.forcing(n, step0, T, cell_offset=off, z=geo[:, 2])
        for v in range(5):
            assert np.array_equal(r.get_forcing(v, step0, T), want[v]), f"variable {v}"
    finally:
        r.close()


@pytest.mark.parametrize("n_cus", [8, -1])
def test_prefetched_window_matches_numpy(n_cus):
    """The prefetch generator (synthetic_forcing_stream_kernel: grid-stride over cells, the window's rows in LDS
    batches of 256) writes the next window bit for bit as numpy states it; 300-row windows span two batches."""
    from shyft_amd.region import HipRegion, PT_GS_K
    n, off, W = 1001, 777, 300
    geo = synthetic.geo11(n, cell_offset=off, n_total=1 << 20)
    r = HipRegion(PT_GS_K, n)
    try:
        r.set_geo(geo)
        r.set_parameters(synthetic.default_ptgsk_parameters())
        r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, 4 * W, W)
        r.prefetch_synthetic_forcing(synthetic.SEED, 2 * W, cell_offset=off, n_cus=n_cus)
        r.swap_forcing_window(2 * W)
        want = synthetic.forcing(n, 2 * W, W, cell_offset=off, z=geo[:, 2])
        for v in range(5):
            assert np.array_equal(r.get_forcing(v, 2 * W, W), want[v]), f"variable {v}"
    finally:
        r.close()
