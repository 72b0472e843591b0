"""Run a stack's bench region in-process for K chunks of 730 steps from Jan 1 (for rocprofv3 passes).

usage (GPU box): python tools/run_chunks.py [lib.so|-] [cells] [chunks] [stack (pt_gs_k)]   ('-' = the in-tree library)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1 and sys.argv[1] != "-":
    os.environ["SHYFT_HIP_LIB"] = os.path.abspath(sys.argv[1])
from shyft_amd import synthetic  # noqa: E402
from shyft_amd.region import HipRegion, PT_GS_K, PT_SS_K, COLLECT_DISCHARGE  # noqa: E402

N = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
K = int(sys.argv[3]) if len(sys.argv) > 3 else 12
stack = sys.argv[4] if len(sys.argv) > 4 else "pt_gs_k"
sid, par, st = {"pt_gs_k": (PT_GS_K, synthetic.default_ptgsk_parameters, synthetic.default_ptgsk_state),
                "pt_ss_k": (PT_SS_K, synthetic.default_ptssk_parameters, synthetic.default_ptssk_state)}[stack]
r = HipRegion(sid, N, device=0)
r.set_geo(synthetic.geo11(N, n_catchments=100))
r.set_parameters(par())
r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, 8760, 730)
r.set_collection(COLLECT_DISCHARGE)
r.set_state(st(N))
for s in range(K):
    r.move_window(s * 730, 0)
    r.synthetic_forcing(synthetic.SEED, s * 730, 730)
    r.run_cells(0, s * 730, 730)
    print(f"chunk {s} {r.last_run_ms():.1f} ms", flush=True)
