"""Time the pt_gs_k kernel for several library variants (one subprocess each)."""
import json
import os
import subprocess
import sys

CODE = r'''
import sys, json
sys.path.insert(0, ".")
import numpy as np
from shyft_amd import synthetic
from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_DISCHARGE
N = int(sys.argv[1]); chunk = int(sys.argv[2]); starts = [int(x) for x in sys.argv[3].split(",")]
r = HipRegion(PT_GS_K, N)
r.set_geo(synthetic.geo11(N, n_total=1 << 20))
r.set_parameters(synthetic.default_ptgsk_parameters())
r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, 8760, chunk)
r.set_collection(COLLECT_DISCHARGE)
res = {}
for s0 in starts:
    r.set_state(synthetic.default_ptgsk_state(N))
    # spin up state through the preceding months with coarse chunks is too slow; start cold at s0
    r.set_window(s0)
    r.synthetic_forcing(synthetic.SEED, s0, chunk)
    r.run_cells(0, s0, chunk)
    r.set_state(synthetic.default_ptgsk_state(N))
    r.run_cells(0, s0, chunk)
    res[s0] = N * chunk / (r.last_run_ms() * 1e-3)
print(json.dumps(res))
'''
variants = sys.argv[1:]
for v in variants:
    env = dict(os.environ)
    env["SHYFT_HIP_LIB"] = os.path.abspath(v)
    out = subprocess.run([sys.executable, "-c", CODE, str(1 << 18), "168", "0,2190,4380"], env=env,
                         capture_output=True, text=True, timeout=600)
    print(os.path.basename(v), out.stdout.strip() or out.stderr[-500:], flush=True)
