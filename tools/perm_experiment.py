"""Divergence experiment: the same pt_gs_k cells and forcing, run in cell-index order and in elevation order.

usage (GPU box): python tools/perm_experiment.py [N] [chunks]
Region A is the bench region (cells in index order, device-generated forcing). Region B holds the same cells
permuted by elevation (stable argsort of z); its forcing window is region A's, column-permuted on the host.
Prints the per-chunk kernel ms of both and checks B's discharge equals A's after un-permuting."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from shyft_amd import synthetic  # noqa: E402
from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_DISCHARGE  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
chunk = 730
geo = synthetic.geo11(N, n_total=1 << 20)
perm = np.argsort(geo[:, 2], kind="stable")
regs = []
for g in (geo, geo[perm]):
    r = HipRegion(PT_GS_K, N, device=0)
    r.set_geo(np.ascontiguousarray(g))
    r.set_parameters(synthetic.default_ptgsk_parameters())
    r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, 8760, chunk)
    r.set_collection(COLLECT_DISCHARGE)
    r.set_state(synthetic.default_ptgsk_state(N))
    regs.append(r)
A, B = regs
for s in range(K):
    s0 = s * chunk
    A.move_window(s0, 0)
    A.synthetic_forcing(synthetic.SEED, s0, chunk)
    B.move_window(s0, 0)
    t = time.time()
    for v in range(5):
        f = A.get_forcing(v, s0, chunk)
        B.set_forcing(v, s0, np.ascontiguousarray(f[:, perm]))
    t = time.time() - t
    A.run_cells(0, s0, chunk)
    B.run_cells(0, s0, chunk)
    qa = A.get_series(0, s0, chunk)
    qb = B.get_series(0, s0, chunk)
    same = np.array_equal(qa[:, perm], qb)
    print(f"chunk {s}: index order {A.last_run_ms():7.1f} ms   elevation order {B.last_run_ms():7.1f} ms   "
          f"{'bit-exact' if same else 'DIFFERS'}   (forcing copy {t:.1f}s)", flush=True)
