"""Per-phase time of the pt_ss_k kernel from a -DSHYFT_PROF build (s_memtime per wavefront, summed).

usage (GPU box): python tools/ptssk_phases.py lib.so [cells]
Runs the bench region from Jan 1 through 12 chunks of 730 steps and prints, per chunk, the kernel ms and the share of
wavefront time in: front (forcing + ss_front), queue (job queue + first barrier), jobs (sca_rel_red evaluation; ~0 on
wavefronts without jobs), wait (second barrier), back (ss_back, glacier), pt+kirchner (PT, AE, kirchner, stores); for
the solving wavefronts the cycles per job phase and the job lanes per solving wavefront-step; and inside the jobs the
share of each part (lgammas, opening evaluations, Brent + walk, bisection, final cdfs; s_memtime marks of the wavefronts
running jobs, device/ptssk_dev.h SS_JOB_MARK)."""
import ctypes as C
import os
import sys

sys.path.insert(0, ".")
os.environ["SHYFT_HIP_LIB"] = os.path.abspath(sys.argv[1])
from shyft_amd import synthetic  # noqa: E402
from shyft_amd.region import HipRegion, PT_SS_K, COLLECT_DISCHARGE  # noqa: E402
from shyft_amd import _native  # noqa: E402

N = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
L = _native.lib()
L.shyft_ptssk_prof_read.argtypes = [C.c_void_p]
buf = (C.c_ulonglong * 16)()
r = HipRegion(PT_SS_K, N, device=0)
r.set_geo(synthetic.geo11(N, n_catchments=100))
r.set_parameters(synthetic.default_ptssk_parameters())
r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, 8760, 730)
r.set_collection(COLLECT_DISCHARGE)
r.set_state(synthetic.default_ptssk_state(N))
L.shyft_ptssk_prof_read(buf)
names = ("front", "queue", "jobs", "wait", "back", "pt+kirchner")
for s in range(12):
    r.move_window(s * 730, 0)
    r.synthetic_forcing(synthetic.SEED, s * 730, 730)
    r.run_cells(0, s * 730, 730)
    L.shyft_ptssk_prof_read(buf)
    tot = sum(buf[k] for k in range(6)) or 1
    extra = ""
    if buf[9]:
        extra = f"  solver: {buf[8] / buf[9]:7.0f} cyc/job-phase, {buf[10] / buf[9]:4.1f} job lanes/wave"
        jt = sum(buf[11 + k] for k in range(5)) or 1
        extra += "  in job: " + " ".join(f"{n} {100.0 * buf[11 + k] / jt:4.1f}%" for k, n in
                                         enumerate(("lgamma", "open", "brent+walk", "bisect", "cdf")))
    print(f"chunk {s:2d} {r.last_run_ms():6.1f} ms  " +
          "  ".join(f"{n} {100.0 * buf[k] / tot:4.1f}%" for k, n in enumerate(names)) + extra, flush=True)
r.close()
