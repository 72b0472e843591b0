"""Time the device forcing generator (kernels/synth.hip) per library: one 1M-cell x 438-step window, as the bench
generates it before each run (shyft_hip_synthetic_forcing, which waits for the kernel), and a digest of the window.

usage (GPU box): python tools/synth_time.py lib1.so lib2.so ..."""
import hashlib
import json
import os
import subprocess
import sys

CODE = r'''
import sys, json, time, hashlib
sys.path.insert(0, ".")
from shyft_amd import synthetic
from shyft_amd.region import HipRegion, PT_GS_K
N, W, K = 1 << 20, 438, 12
r = HipRegion(PT_GS_K, N, device=0)
r.set_geo(synthetic.geo11(N, n_catchments=100))
r.set_parameters(synthetic.default_ptgsk_parameters())
r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, 8760, W)
ms = []
for k in range(K):
    r.move_window(k * W, 0)
    t = time.perf_counter()
    r.synthetic_forcing(synthetic.SEED, k * W, W)
    ms.append((time.perf_counter() - t) * 1e3)
h = hashlib.sha256()
for v in range(5):
    h.update(r.get_forcing(v, (K - 1) * W, 64).tobytes())
r.close()
print(json.dumps({"ms": ms, "digest": h.hexdigest()[:16]}))
'''

for lib in sys.argv[1:]:
    env = dict(os.environ, SHYFT_HIP_LIB=os.path.abspath(lib))
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=600)
    try:
        d = json.loads(out.stdout.strip().splitlines()[-1])
    except Exception:
        print(lib, "FAILED", out.stderr[-1500:], flush=True)
        sys.exit(1)
    ms = sorted(d["ms"][2:])
    print(f"{os.path.basename(lib):20s} median {ms[len(ms) // 2]:6.2f} ms  min {ms[0]:6.2f}  digest {d['digest']}", flush=True)
