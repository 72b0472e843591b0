"""Time pt_gs_k kernel variants on the bench workload and check they agree bit-for-bit.

usage (GPU box): python tools/ptgsk_variants.py [--cells N] [--chunks K] lib1.so lib2.so ...
Each library runs in its own subprocess (SHYFT_HIP_LIB): N cells from Jan 1 through K chunks of 730 steps with
the device generator (the bench's run_year), printing the per-chunk kernel ms, and a digest of a 4096-cell x
2920-step run (discharge + charge series and the final state, Jan-Apr: snow, Brent and kirchner paths). Every
variant's digest must equal the first library's (the first library is the parity-tested build)."""
import hashlib
import json
import os
import subprocess
import sys

CODE = r'''
import sys, json, hashlib
sys.path.insert(0, ".")
import numpy as np
from shyft_amd import synthetic
from shyft_amd.region import HipRegion, PT_GS_K, COLLECT_DISCHARGE
N = int(sys.argv[1]); K = int(sys.argv[2]); chunk = 730
r = HipRegion(PT_GS_K, N, device=0)
r.set_geo(synthetic.geo11(N, n_catchments=100))
r.set_parameters(synthetic.default_ptgsk_parameters())
r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, max(8760, K * chunk), chunk)
r.set_collection(COLLECT_DISCHARGE)
r.set_state(synthetic.default_ptgsk_state(N))
ms = []
for s in range(K):
    r.move_window(s * chunk, 0)
    r.synthetic_forcing(synthetic.SEED, s * chunk, chunk)
    r.run_cells(0, s * chunk, chunk)
    ms.append(r.last_run_ms())
r.close()
n, T = 4096, 2920
g = HipRegion(PT_GS_K, n, device=0)
g.set_geo(synthetic.geo11(n, n_total=1 << 20))
g.set_parameters(synthetic.default_ptgsk_parameters())
g.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, T)
g.set_collection(COLLECT_DISCHARGE)
g.set_state(synthetic.default_ptgsk_state(n))
g.synthetic_forcing(synthetic.SEED, 0, T)
g.run_cells(0, 0, T)
h = hashlib.sha256()
for s in range(2):
    h.update(g.get_series(s, 0, T).tobytes())
h.update(g.get_state().tobytes())
print(json.dumps({"ms": ms, "digest": h.hexdigest()[:16]}))
'''


def main():
    args = sys.argv[1:]
    cells, chunks = 1 << 20, 12
    while args and args[0].startswith("--"):
        k, v = args[0], int(args[1])
        args = args[2:]
        if k == "--cells":
            cells = v
        elif k == "--chunks":
            chunks = v
    ref = None
    for lib in args:
        env = dict(os.environ, SHYFT_HIP_LIB=os.path.abspath(lib))
        out = subprocess.run([sys.executable, "-c", CODE, str(cells), str(chunks)], env=env, capture_output=True,
                             text=True, timeout=600)
        try:
            d = json.loads(out.stdout.strip().splitlines()[-1])
        except Exception:
            print(os.path.basename(lib), "FAILED", out.stderr[-1500:], flush=True)
            continue
        if ref is None:
            ref = d["digest"]
        ms = d["ms"]
        print(f"{os.path.basename(lib):28s} mean {sum(ms) / len(ms):7.1f} ms  "
              f"{'bit-exact' if d['digest'] == ref else 'DIFFERS ' + d['digest']}  "
              + " ".join(f"{m:.0f}" for m in ms), flush=True)


if __name__ == "__main__":
    main()
