"""Print GPU vs oracle state/response trajectories of one cell around a step."""
import sys

import numpy as np

sys.path.insert(0, ".")
from shyft_amd import synthetic  # noqa: E402
from tests import engines  # noqa: E402

cell, s0, s1 = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
n, T = cell + 1, s1 + 1
geo = synthetic.geo11(200)[:n]
f = synthetic.forcing(200, 0, T)[:, :, :n]
p = synthetic.default_ptgsk_parameters()
s = synthetic.default_ptgsk_state(n)
cpu = engines.run("oracle", geo, p, s, synthetic.T0_2015_US, synthetic.HOUR_US, f, full=True, collect_state=True)
gpu = engines.run("hip", geo, p, s, synthetic.T0_2015_US, synthetic.HOUR_US, f, full=True, collect_state=True)
np.set_printoptions(precision=17, linewidth=250)
for t in range(s0, s1):
    print("step", t, "forcing", f[:, t, cell])
    for k in range(9):
        a, b = gpu["state_series"][k, t, cell], cpu["state_series"][k, t, cell]
        print(f"  state{k}: gpu {a:.17g} cpu {b:.17g} {'' if a == b else '<-- diff %.3e' % (a - b)}")
    for k in range(8):
        a, b = gpu["full"][k, t, cell], cpu["full"][k, t, cell]
        print(f"  resp{k}: gpu {a:.17g} cpu {b:.17g} {'' if a == b else '<-- diff %.3e' % (a - b)}")
