"""The pt_gs_k Brent job queue under a forced interleaving (gamma_snow.h:425-435 corr_lwc, solved per workgroup
from an LDS queue, kernels/ptgsk.hip).

A 256-lane workgroup queues its lanes' corr_lwc jobs in LDS each step; after the solve every lane reads its result
from jres[slot] behind the step's second barrier. The first wavefront to leave that barrier may run on into the next
step and enqueue its jobs (slots from 0 again) while a slower wavefront has not read its result yet, so the results
must not share storage with the job arrays (round 4 briefly let them alias the z1 slots -- a race the GPU suite did
not catch, because wavefronts rarely drift that far apart). The test knob SHYFT_HIP_KNOB_BRENT_READ_DELAY makes every
wavefront but the first sleep before reading its results, which forces exactly that drift on every step; the run
must still equal the CPU oracle bit for bit (January: about one job per ten lanes per step)."""
import numpy as np
import pytest

from shyft_amd import synthetic

pytestmark = pytest.mark.gpu

N, T = 4096, 240


def _run(delay, instance=4):
    from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_ALL, KNOB_PTGSK_INSTANCE, KNOB_BRENT_READ_DELAY
    r = HipRegion(PT_GS_K, N, device=0)
    try:
        r.set_geo(synthetic.geo11(N, n_total=1 << 20))
        r.set_parameters(synthetic.default_ptgsk_parameters())
        r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, T)
        r.set_collection(COLLECT_ALL)
        r.set_state(synthetic.default_ptgsk_state(N))
        r.set_test_knob(KNOB_PTGSK_INSTANCE, instance)     # the 256-lane 4-wave instance (the bench's)
        r.set_test_knob(KNOB_BRENT_READ_DELAY, delay)
        r.synthetic_forcing(synthetic.SEED, 0, T)
        r.run_cells(0, 0, T)
        return np.stack([r.get_series(k, 0, T) for k in range(8)]), r.get_state()
    finally:
        r.close()


def test_delayed_result_reads_stay_bitexact():
    from tests import engines
    full, state = _run(delay=40)
    geo = synthetic.geo11(N, n_total=1 << 20)
    f = synthetic.forcing(N, 0, T)
    exp = engines.run("oracle", geo, synthetic.default_ptgsk_parameters(), synthetic.default_ptgsk_state(N),
                      synthetic.T0_2015_US, synthetic.HOUR_US, f, full=True)
    assert np.array_equal(full, exp["full"], equal_nan=True)
    assert np.array_equal(state, exp["state"])
    # the window has Brent jobs to interleave: snow on wet packs (lwc > 0 somewhere during the window)
    assert (full[3] > 0).any()


def test_knob_validation():
    from shyft_amd.region import HipRegion, PT_GS_K, KNOB_PTGSK_INSTANCE, KNOB_BRENT_READ_DELAY
    r = HipRegion(PT_GS_K, 64, device=0)
    try:
        with pytest.raises(RuntimeError, match="instance"):
            r.set_test_knob(KNOB_PTGSK_INSTANCE, 3)
        with pytest.raises(RuntimeError, match="delay"):
            r.set_test_knob(KNOB_BRENT_READ_DELAY, -1)
        with pytest.raises(RuntimeError, match="unknown knob"):
            r.set_test_knob(99, 0)
    finally:
        r.close()
