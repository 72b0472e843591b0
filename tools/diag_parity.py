"""Diagnostic: GPU vs oracle max relative differences + a quick throughput probe."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from shyft_amd import synthetic  # noqa: E402
from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_DISCHARGE  # noqa: E402
from tests import engines  # noqa: E402

n, T = int(sys.argv[1]) if len(sys.argv) > 1 else 200, int(sys.argv[2]) if len(sys.argv) > 2 else 8760
geo = synthetic.geo11(n)
f = synthetic.forcing(n, 0, T)
p = synthetic.default_ptgsk_parameters()
s = synthetic.default_ptgsk_state(n)
t = time.time()
cpu = engines.run("oracle", geo, p, s, synthetic.T0_2015_US, synthetic.HOUR_US, f, full=True, collect_state=True)
print("oracle s", time.time() - t, "elapsed", cpu["elapsed_s"], flush=True)
t = time.time()
gpu = engines.run("hip", geo, p, s, synthetic.T0_2015_US, synthetic.HOUR_US, f, full=True, collect_state=True)
print("gpu s", time.time() - t, flush=True)
for k in range(8):
    a, b = gpu["full"][k], cpu["full"][k]
    d = np.abs(a - b)
    rel = d / np.maximum(np.abs(b), 1e-300)
    i = np.unravel_index(np.nanargmax(d), d.shape)
    print(f"series {k}: max abs {np.nanmax(d):.3e} max rel {np.nanmax(np.where(np.abs(b) > 1e-12, rel, 0)):.3e} "
          f"n_exact {np.mean(a == b):.4f} at {i} gpu {a[i]:.17g} cpu {b[i]:.17g}")
d = np.abs(gpu["state"] - cpu["state"])
print("final state max abs per field", d.max(axis=0))
# throughput probe
N = 1 << 20
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 168
r = HipRegion(PT_GS_K, N)
r.set_geo(synthetic.geo11(N))
r.set_parameters(p)
r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, 8760, steps)
r.set_collection(COLLECT_DISCHARGE)
r.set_state(synthetic.default_ptgsk_state(N))
r.synthetic_forcing(synthetic.SEED, 0, steps)
r.run_cells(0, 0, steps)
print(f"1M cells x {steps} steps: kernel {r.last_run_ms():.1f} ms -> {N*steps/(r.last_run_ms()*1e-3):.3e} cell-steps/s")
# check generator bit-exactness on a slice
fz = synthetic.forcing(N, 0, 3)
for v in range(5):
    g = r.get_forcing(v, 0, 3)
    print("synthetic var", v, "bit-exact:", np.array_equal(g, fz[v]))
