"""Time pt_gs_k kernel variants on the bench workload and check they agree bit-for-bit.

usage (GPU box): python tools/ptgsk_variants.py [--stack S] [--cells N] [--chunks K] lib1.so lib2.so ...
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
from shyft_amd.region import HipRegion, PT_GS_K, HBV_STACK, PT_SS_K, PT_HS_K, PT_HPS_K, COLLECT_DISCHARGE
import bench
N = int(sys.argv[1]); K = int(sys.argv[2]); chunk = 730; stack = sys.argv[3]
SID = {"pt_gs_k": PT_GS_K, "hbv_stack": HBV_STACK, "pt_ss_k": PT_SS_K, "pt_hs_k": PT_HS_K, "pt_hps_k": PT_HPS_K}[stack]
par, st0 = bench.stack_defaults(stack, N)
r = HipRegion(SID, N, device=0)
r.set_geo(synthetic.geo11(N, n_catchments=100))
r.set_parameters(par)
r.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, max(8760, K * chunk), chunk)
r.set_collection(COLLECT_DISCHARGE)
r.set_state(st0)
ms = []
for s in range(K):
    r.move_window(s * chunk, 0)
    r.synthetic_forcing(synthetic.SEED, s * chunk, chunk)
    r.run_cells(0, s * chunk, chunk)
    ms.append(r.last_run_ms())
h0 = hashlib.sha256(r.get_state().tobytes()).hexdigest()[:16]   # the large-region instance's own final state
r.close()
n, T = 4096, 2920
g = HipRegion(SID, n, device=0)
g.set_geo(synthetic.geo11(n, n_total=1 << 20))
g.set_parameters(par)
g.set_time_axis(synthetic.T0_2015_US, synthetic.HOUR_US, T)
g.set_collection(COLLECT_DISCHARGE)
g.set_state(bench.stack_defaults(stack, n)[1])
if stack == "pt_gs_k" and hasattr(g, "set_test_knob"):
    try:
        g.set_test_knob(1, 4)   # the large-region (256-lane) instance on the digest region too
    except Exception:
        pass
g.synthetic_forcing(synthetic.SEED, 0, T)
g.run_cells(0, 0, T)
h = hashlib.sha256()
for s in range(2):
    h.update(g.get_series(s, 0, T).tobytes())
h.update(g.get_state().tobytes())
print(json.dumps({"ms": ms, "digest": h.hexdigest()[:16] + "/" + h0}))
'''


def main():
    args = sys.argv[1:]
    cells, chunks, stack = 1 << 20, 12, "pt_gs_k"
    args = [x for x in args if x != "--keep-going"]
    while args and args[0].startswith("--"):
        k, v = args[0], args[1]
        args = args[2:]
        if k == "--cells":
            cells = int(v)
        elif k == "--chunks":
            chunks = int(v)
        elif k == "--stack":
            stack = v
    ref = None
    for spec in args:  # lib.so[:VAR=value[:VAR=value...]] -- environment settings for that run
        lib, *envs = spec.split(":")
        env = dict(os.environ, SHYFT_HIP_LIB=os.path.abspath(lib))
        env.update(kv.split("=", 1) for kv in envs)
        out = subprocess.run([sys.executable, "-c", CODE, str(cells), str(chunks), stack], env=env, capture_output=True,
                             text=True, timeout=600)
        try:
            d = json.loads(out.stdout.strip().splitlines()[-1])
        except Exception:
            print(spec, "FAILED", out.stderr[-1500:], flush=True)
            if "--keep-going" not in sys.argv:
                sys.exit(1)  # a fault leaves the GPU in an unknown state: run nothing more
            continue
        if ref is None:
            ref = d["digest"]
        ms = d["ms"]
        print(f"{os.path.basename(spec):28s} mean {sum(ms) / len(ms):7.1f} ms  "
              f"{'bit-exact' if d['digest'] == ref else 'DIFFERS ' + d['digest']}  "
              + " ".join(f"{m:.0f}" for m in ms), flush=True)


if __name__ == "__main__":
    main()
