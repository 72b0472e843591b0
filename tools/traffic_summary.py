"""Per-launch HBM-side bytes of ptgsk_run_kernel from tools/traffic_variants.sh's two rocprofv3 passes.

usage: python tools/traffic_summary.py <dir> <name> [stack]   (reads <dir>/<name>_FETCH_SIZE, <dir>/<name>_WRITE_SIZE)
FETCH_SIZE is scaled by the gfx950 correction the r06 bench passes calibrated (1.991: 8-byte-per-lane loads, the
catchment sums' known bytes; profiles/r06/pmc_*.json); WRITE_SIZE needs none. Algorithmic bytes: DESIGN.md §3.1
(56 B per cell-step + 144 B per cell per launch; pt_ss_k: 48 B + 128 B)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import counter_rows  # noqa: E402

FETCH_CORRECTION = 1.991
d, n = sys.argv[1], sys.argv[2]
stack = sys.argv[3] if len(sys.argv) > 3 else "pt_gs_k"
kern, state_b, step_b = {"pt_gs_k": ("ptgsk_run_kernel", 144.0, 56.0), "pt_ss_k": ("ptssk_run_kernel", 128.0, 48.0)}[stack]
f = counter_rows(os.path.join(d, f"{n}_FETCH_SIZE", "run_counter_collection.csv"), kern)
w = counter_rows(os.path.join(d, f"{n}_WRITE_SIZE", "run_counter_collection.csv"), kern)
tot_t = tot_a = 0.0
for k, ((_, fr, fm), (_, wr, wm)) in enumerate(zip(f, w)):
    steps = 730
    alg = fm["grid"] * (step_b * steps + state_b)
    fb = fr["FETCH_SIZE"] * 1024 * FETCH_CORRECTION
    wb = wr["WRITE_SIZE"] * 1024
    print(f"{n:12s} launch {k}: fetch {fb / 1e9:6.2f} GB  write {wb / 1e9:6.2f} GB  traffic/algorithmic "
          f"{(fb + wb) / alg:5.2f}  ({fm['duration_ns'] / 1e6:.1f} / {wm['duration_ns'] / 1e6:.1f} ms, scratch "
          f"{fm['scratch_bytes_per_lane']} B/lane)", flush=True)
    tot_t += fb + wb
    tot_a += alg
print(f"{n:12s} all launches: traffic/algorithmic {tot_t / tot_a:5.3f}", flush=True)
