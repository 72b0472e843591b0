"""Generate the golden fixtures under tests/golden/ (run from the repo root: python tests/golden/make_golden.py).

Each fixture is one small region run of one method stack on the CPU oracle (oracle/, detmath build): the inputs
(geo rows, parameter row, initial state, time axis, forcing) and the expected outputs (discharge and charge series
[2][T][N], final state [N][S]). tests/test_golden.py checks that the oracle still reproduces them bit for bit
(CPU) and that the HIP kernels do too (GPU), so a change to either side -- or to detmath, which both use -- shows
up as a fixture difference. The expected values are the oracle's, which is pinned to the reference by the
reference's own known-answer tests (tests/test_oracle_kat.py, test_kat_*.py, test_region_kat.py); after an
intended change to the shared arithmetic, regenerate with this script and say so in the commit.

Cases (20 cells x 240 hourly steps from 2015-01-01, synthetic region + generator of SURVEY.md §8d, cells with
mixed glacier / lake / reservoir fractions; winter start so the snow routines and gamma_snow's Brent run):
  pt_gs_k, hbv_stack, pt_ss_k, pt_hs_k, pt_hps_k
plus c1_sampled: BASELINE configs[0] (pt_gs_k, 200 cells x 8760 steps): the avg_discharge of 4 cells over the
whole year and the final state of all 200 (forcing regenerated from the generator, which tests/test_capi.py pins
to the device generator)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from shyft_amd import synthetic  # noqa: E402
from tests import engines  # noqa: E402

N, T = 20, 240
C1_CELLS, C1_SAMPLE = 200, (0, 57, 123, 199)

STACKS = {
    "pt_gs_k": (engines.run, synthetic.default_ptgsk_parameters, synthetic.default_ptgsk_state),
    "hbv_stack": (engines.run_hbv, synthetic.default_hbv_parameters, synthetic.default_hbv_state),
    "pt_ss_k": (engines.run_ptssk, synthetic.default_ptssk_parameters, synthetic.default_ptssk_state),
    "pt_hs_k": (engines.run_pthsk, synthetic.default_pthsk_parameters, synthetic.default_pthsk_state),
    "pt_hps_k": (engines.run_pthpsk, synthetic.default_pthpsk_parameters, synthetic.default_pthpsk_state),
}


def case_inputs(n=N, t=T):
    geo = synthetic.geo11(n, n_catchments=4)
    rng = np.random.default_rng(11)
    geo[:, 6] = rng.choice([0.0, 0.05, 0.3], n)   # glacier
    geo[:, 7] = rng.choice([0.0, 0.05], n)        # lake
    geo[:, 8] = rng.choice([0.0, 0.19], n)        # reservoir
    geo[:, 10] = 1.0 - geo[:, 6:10].sum(axis=1)
    f = synthetic.forcing(n, 0, t, z=geo[:, 2])
    return geo, f


def run_case(engine, stack, geo, params, state, forcing):
    fn = STACKS[stack][0]
    return fn(engine, geo, params, state, synthetic.T0_2015_US, synthetic.HOUR_US, forcing, full=False)


def c1_inputs():
    geo = synthetic.geo11(C1_CELLS, n_total=1 << 20)
    f = synthetic.forcing(C1_CELLS, 0, 8760)
    return geo, f


def main():
    for stack, (_, par, st) in STACKS.items():
        geo, f = case_inputs()
        p, s = par(), st(N)
        r = run_case("oracle", stack, geo, p, s, f)
        np.savez_compressed(os.path.join(HERE, f"{stack}_20x240.npz"), geo=geo, params=p, state0=s, forcing=f,
                            t0_us=synthetic.T0_2015_US, dt_us=synthetic.HOUR_US, main=r["main"], state=r["state"])
        print(stack, r["main"].shape, float(r["main"][0].sum()))
    geo, f = c1_inputs()
    r = engines.run("oracle", geo, synthetic.default_ptgsk_parameters(), synthetic.default_ptgsk_state(C1_CELLS),
                    synthetic.T0_2015_US, synthetic.HOUR_US, f, full=False)
    np.savez_compressed(os.path.join(HERE, "c1_sampled.npz"), cells=np.array(C1_SAMPLE),
                        avg_discharge=r["main"][0][:, list(C1_SAMPLE)], state=r["state"])
    print("c1_sampled", float(r["main"][0].sum()))


if __name__ == "__main__":
    main()
