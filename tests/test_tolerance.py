"""The stated fp64 tolerance (BASELINE north_star: discharge, SWE, soil state) of this engine against the reference
CPU region_model, on configs[0] (200 cells x 8760 hourly steps), for pt_gs_k, hbv_stack and pt_ss_k.

The HIP kernels equal the detmath oracle bit for bit (the -m gpu parity tests). The oracle differs from the reference
build only in (1) the elementary-function library (detmath here, glibc there) and (2) the incomplete gamma's
implementation inside boost's precision policy for gamma_snow (gamma_snow.h:189-201). tools/tolerance.py measures
the oracle against builds that swap each for the reference-side choice (host libm) or for the exact value
(full-precision gamma); the bounds below are those measurements rounded up, and are the numbers DESIGN.md states.
odeint's step sequence (kirchner.h:171-176) is the one further difference (parity unpinned): its per-step bound is
in test_oracle_bounds.py (5e-7 relative)."""
import pytest

from tools import tolerance

# stated tolerance: stack -> field -> (max |delta| in the field's unit, max |delta| / max|field|, yearly-total rel)
STATED = {
    "pt_gs_k": {"discharge_m3s": (2e-4, 3e-4, 1e-4), "snow_swe_mm": (0.15, 5e-4, 5e-6),
                "kirchner_q_mm_h": (1e-6, 1e-5, None), "snow_lwc_mm": (3.0, 3e-3, 1e-4)},
    "hbv_stack": {"discharge_m3s": (1e-12, 1e-12, 1e-12), "snow_swe_mm": (1e-12, 1e-12, 1e-12),
                  "soil_moisture_mm": (1e-10, 1e-12, 1e-12), "tank_uz_mm": (1e-12, 1e-12, 1e-12),
                  "tank_lz_mm": (1e-12, 1e-12, 1e-12)},
    "pt_ss_k": {"discharge_m3s": (1e-12, 1e-12, 1e-12), "snow_swe_mm": (1e-12, 1e-12, 1e-12),
                "kirchner_q_mm_h": (1e-12, 1e-12, None)},
}


@pytest.fixture(scope="module")
def measured():
    return tolerance.measure()


@pytest.mark.parametrize("stack", sorted(STATED))
def test_stated_tolerance(measured, stack):
    for variant, fields in measured[stack].items():
        for field, d in fields.items():
            abs_b, rel_b, yr_b = STATED[stack][field]
            assert d["max_abs"] <= abs_b, (stack, variant, field, d)
            assert d["max_rel_to_range"] <= rel_b, (stack, variant, field, d)
            if yr_b is not None and "yearly_total_max_rel" in d:
                assert d["yearly_total_max_rel"] <= yr_b, (stack, variant, field, d)
