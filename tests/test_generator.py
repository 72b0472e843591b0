"""The device forcing generator (kernels/synth.hip) against its numpy statement
(shyft_amd/synthetic.forcing), bit for bit: even and odd cell counts, a window that starts mid-year and a cell offset
(a rank's or a shard's slice)."""
import numpy as np
import pytest

from shyft_amd import synthetic

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1000, 1001, 4096])
def test_device_generator_matches_numpy(n):
    from shyft_amd.region import HipRegion, PT_GS_K
    off, step0, T = 12345, 4000, 30
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
