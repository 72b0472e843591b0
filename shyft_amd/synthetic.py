"""Synthetic region + forcing, bit-identical to the device
generator in shyft_amd/csrc/include_internal/synth_hash.h.

Grid cells x = 500 + 1000*(i mod W), y = 500 + 1000*(i div W), W = ceil(sqrt(N)),
z = 2000*u(seed, 7, i, 0), area 1e6 m2, fractions glacier 0.01 / lake 0.05 /
reservoir 0.19 / forest 0.30 (test_region_model_stacks.py:25-26), slope 0.9,
cid = 1 + i*C//N (contiguous catchment blocks). Time axis 2015-01-01Z hourly.
"""
from __future__ import annotations

import math

import numpy as np

SEED = 20251015
T0_2015_US = 1420070400 * 1_000_000  # 2015-01-01T00:00:00Z
HOUR_US = 3600 * 1_000_000
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _sm64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _key(seed: int, cell: np.ndarray, step: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        c = np.asarray(cell, dtype=np.uint64) * np.uint64(0xD1B54A32D192ED03)
        return _sm64(_sm64(np.uint64(seed) ^ c) ^ np.asarray(step, dtype=np.uint64))


def _u(key: np.ndarray, var: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        v = np.uint64(var) * np.uint64(0xA24BAED4963EE407)
    return (_sm64(key ^ v) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def elevation(n_cells: int, seed: int = SEED, cell_offset: int = 0) -> np.ndarray:
    cells = np.arange(cell_offset, cell_offset + n_cells, dtype=np.uint64)
    return 2000.0 * _u(_key(seed, cells, np.zeros_like(cells)), 7)


def geo11(n_cells: int, n_catchments: int = 100, seed: int = SEED, cell_offset: int = 0,
          n_total: int | None = None) -> np.ndarray:
    """n_cells x 11 geo_cell_data_io rows of cells [cell_offset, cell_offset+n_cells) of an n_total-cell region."""
    n_total = n_total or (cell_offset + n_cells)
    i = np.arange(cell_offset, cell_offset + n_cells, dtype=np.int64)
    W = int(math.ceil(math.sqrt(n_total)))
    g = np.zeros((n_cells, 11), dtype=np.float64)
    g[:, 0] = 500.0 + 1000.0 * (i % W)
    g[:, 1] = 500.0 + 1000.0 * (i // W)
    g[:, 2] = elevation(n_cells, seed, cell_offset)
    g[:, 3] = 1.0e6
    g[:, 4] = 1 + (i * n_catchments) // n_total
    g[:, 5] = 0.9
    g[:, 6:10] = (0.01, 0.05, 0.19, 0.30)
    g[:, 10] = 1.0 - 0.01 - 0.05 - 0.19 - 0.30
    return g


def forcing(n_cells: int, step0: int, n_steps: int, seed: int = SEED, cell_offset: int = 0,
            z: np.ndarray | None = None) -> np.ndarray:
    """[5][n_steps][n_cells] temperature, precipitation, wind_speed, rel_hum, radiation."""
    if z is None:
        z = elevation(n_cells, seed, cell_offset)
    cells = np.arange(cell_offset, cell_offset + n_cells, dtype=np.uint64)[None, :]
    steps = np.arange(step0, step0 + n_steps, dtype=np.uint64)[:, None]
    key = _key(seed, cells, steps)
    f = (steps % np.uint64(8760)).astype(np.float64) / 8760.0
    g = f * (1.0 - f)
    b = 16.0 * g * g
    h = (steps % np.uint64(24)).astype(np.float64)
    dd = (h - 12.0) / 6.0
    di = 1.0 - dd * dd
    di = np.where(di < 0.0, 0.0, di)
    u0, u1, u2, u3, u5 = (_u(key, k) for k in (0, 1, 2, 3, 5))
    out = np.empty((5, n_steps, n_cells), dtype=np.float64)
    out[0] = 8.0 + 12.0 * (2.0 * b - 1.0) - 0.006 * z[None, :] + 4.0 * (u0 - 0.5)
    out[1] = np.where(u1 < 0.15, 3.0 * u5, 0.0)
    out[2] = 10.0 * u2
    out[3] = 0.5 + 0.5 * u3
    out[4] = np.broadcast_to(800.0 * di * (0.3 + 0.7 * b), (n_steps, n_cells))
    return out


def default_ptgsk_parameters() -> np.ndarray:
    """PTGSKParameter() defaults in the reference get/set order (core/pt_gs_k.h:77-112)."""
    return np.array([
        -2.439, 0.966, -0.10,            # kirchner c1 c2 c3 (kirchner.h:120-125)
        1.5,                             # ae.ae_scale_factor
        -0.5, 2.0, 0.1, 1.0,             # gs.tx wind_scale max_water wind_const (gamma_snow.h:46-65)
        5.0, 5.0, 30.0, 0.9, 0.6, 5.0,   # fast/slow albedo decay, surface_magnitude, max/min albedo, snowfall_reset_depth
        0.4, 0.4,                        # snow_cv, glacier_albedo
        1.0,                             # p_corr.scale_factor
        0.0, 0.0,                        # snow_cv_forest_factor, snow_cv_altitude_factor
        0.2, 1.26,                       # pt.albedo pt.alpha
        0.04, 100.0, 0.0,                # initial_bare_ground_fraction, winter_end_day_of_year, calculate_iso_pot_energy
        6.0,                             # gm.dtf
        1.0, 7.0, 0.0,                   # routing velocity alpha beta (routing.h:76)
        221.0,                           # gs.n_winter_days
        0.0,                             # gm.direct_response
        1.0,                             # msp.reservoir_direct_response_fraction
    ], dtype=np.float64)


def default_ptgsk_state(n_cells: int, q: float = 1.0) -> np.ndarray:
    """PTGSKState() defaults (gamma_snow.h:101-116) with kirchner.q = q."""
    s = np.empty((n_cells, 9), dtype=np.float64)
    s[:] = (0.4, 0.1, 30000.0, 1.26, 0.0, 0.0, 0.0, 0.0, q)
    return s


def default_hbv_parameters() -> np.ndarray:
    """HbvParameter() defaults in the reference get/set order (core/hbv_stack.h:82-109)."""
    return np.array([
        300.0, 2.0,                   # soil.fc soil.beta (hbv_soil.h:19-24)
        150.0,                        # ae.lp (hbv_actual_evapotranspiration.h:13-16)
        25.0, 0.5, 0.3, 0.8, 0.02,    # tank uz1 kuz2 kuz1 perc klz (hbv_tank.h:19-31)
        0.1, 0.0, 1.0, 0.0, 0.5,      # snow lw tx cx ts cfr (hbv_snow.h:49-53)
        1.0,                          # p_corr.scale_factor
        0.2, 1.26,                    # pt.albedo pt.alpha
        6.0,                          # gm.dtf
        1.0, 7.0, 0.0,                # routing velocity alpha beta
        0.0,                          # gm.direct_response
        1.0,                          # msp.reservoir_direct_response_fraction
    ], dtype=np.float64)


HBV_MAX_BINS = 8
HBV_NS = 6 + 2 * HBV_MAX_BINS  # swe sca sm uz lz n_bins sp[8] sw[8]


def default_hbv_state(n_cells: int, uz: float = 40.0, lz: float = 40.0) -> np.ndarray:
    """HbvState() (hbv_stack.h:181-190: snow swe = sca = 0 undistributed, soil sm 0) with tank uz, lz."""
    s = np.zeros((n_cells, HBV_NS), dtype=np.float64)
    s[:, 3] = uz
    s[:, 4] = lz
    return s


def default_ptssk_parameters() -> np.ndarray:
    """PTSSKParameter() defaults in the reference get/set order (core/pt_ss_k.h:78-101)."""
    return np.array([
        -2.439, 0.966, -0.10,                                # kirchner c1 c2 c3
        1.5,                                                 # ae.ae_scale_factor
        40.77, 113.0, 0.1, 0.1, 0.16, 2.5, 0.14, 0.01,       # ss alpha_0 d_range unit_size max_water_fraction tx cx ts cfr
        1.0,                                                 # p_corr.scale_factor
        0.2, 1.26,                                           # pt.albedo pt.alpha
        6.0,                                                 # gm.dtf
        1.0, 7.0, 0.0,                                       # routing velocity alpha beta
        0.0,                                                 # gm.direct_response
        1.0,                                                 # msp.reservoir_direct_response_fraction
    ], dtype=np.float64)


PTSSK_NS = 8  # nu alpha sca swe free_water residual num_units kirchner.q


# ---- synthetic river network for configs[4] (pt_ss_k + routing::uhg) --------------------------------------------------
# One river per catchment (river id = catchment id). River k drains into river k // 2 (a binary tree rooted at
# river 1), 4 km + 1 km*(k % 7) downstream, UHGParameter() defaults (velocity 1 m/s, alpha 7, beta 0,
# routing.h:70-76). Each cell routes to its catchment's river at 0 m or 7200 m (a 2-step cell UHG at the
# default routing velocity), chosen by the cell hash; cells sharing (river, distance class) are one routing group.
ROUTE_DISTANCES = (0.0, 7200.0)


def river_network(n_rivers: int):
    """[(id, downstream_id, distance, velocity, alpha, beta)] for rivers 1..n_rivers."""
    return [(k, k // 2, 4000.0 + 1000.0 * (k % 7), 1.0, 7.0, 0.0) for k in range(1, n_rivers + 1)]


def cell_routing(n_cells: int, n_catchments: int, seed: int = SEED, cell_offset: int = 0, n_total: int | None = None):
    """(river id [n], routing distance [n], global routing group [n]) of cells [cell_offset, cell_offset+n)."""
    n_total = n_total or (cell_offset + n_cells)
    i = np.arange(cell_offset, cell_offset + n_cells, dtype=np.int64)
    rid = 1 + (i * n_catchments) // n_total
    cells = np.arange(cell_offset, cell_offset + n_cells, dtype=np.uint64)
    klass = (_u(_key(seed, cells, np.zeros_like(cells)), 11) < 0.5).astype(np.int64)
    dist = np.asarray(ROUTE_DISTANCES)[klass]
    group = (rid - 1) * len(ROUTE_DISTANCES) + klass
    return rid, dist, group.astype(np.int32)


def default_ptssk_state(n_cells: int, q: float = 1.0) -> np.ndarray:
    """PTSSKState(): skaugen::state() (skaugen.h:122-124: nu 4.077, alpha 40.77, no snow) with kirchner.q = q."""
    s = np.zeros((n_cells, PTSSK_NS), dtype=np.float64)
    s[:, 0] = 4.077
    s[:, 1] = 40.77
    s[:, 7] = q
    return s


def default_pthsk_parameters() -> np.ndarray:
    """PTHSKParameter() defaults in the reference get/set order (core/pt_hs_k.h:66-88)."""
    return np.array([
        -2.439, 0.966, -0.10,            # kirchner c1 c2 c3 (kirchner.h:120-125)
        1.5,                             # ae.ae_scale_factor
        0.1, 0.0, 1.0, 0.0, 0.5,         # hs lw tx cx ts cfr (hbv_snow.h:49-53)
        6.0,                             # gm.dtf
        1.0,                             # p_corr.scale_factor
        0.2, 1.26,                       # pt.albedo pt.alpha
        1.0, 7.0, 0.0,                   # routing velocity alpha beta
        0.0,                             # gm.direct_response
        1.0,                             # msp.reservoir_direct_response_fraction
    ], dtype=np.float64)


PTHSK_NS = 3 + 2 * HBV_MAX_BINS + 1  # swe sca n_bins sp[8] sw[8] kirchner.q


def default_pthsk_state(n_cells: int, q: float = 1.0, swe: float = 0.0, sca: float = 0.0) -> np.ndarray:
    """PTHSKState(): hbv_snow::state(swe, sca) undistributed (hbv_snow.h:74-99) with kirchner.q = q."""
    s = np.zeros((n_cells, PTHSK_NS), dtype=np.float64)
    s[:, 0] = swe
    s[:, 1] = sca
    s[:, -1] = q
    return s


def default_pthpsk_parameters() -> np.ndarray:
    """PTHPSKParameter() defaults in the reference get/set order (core/pt_hps_k.h:64-90)."""
    return np.array([
        -2.439, 0.966, -0.10,            # kirchner c1 c2 c3
        1.5,                             # ae.ae_scale_factor
        0.1, 0.0, 0.5,                   # hps lw tx cfr (hbv_physical_snow.h:45-47)
        2.0, 1.0, 30.0,                  # hps wind_scale wind_const surface_magnitude
        0.9, 0.6, 5.0, 5.0, 5.0,         # hps max/min albedo, fast/slow albedo decay rate, snowfall_reset_depth
        0.0,                             # hps.calculate_iso_pot_energy
        6.0,                             # gm.dtf
        1.0,                             # p_corr.scale_factor
        0.2, 1.26,                       # pt.albedo pt.alpha
        1.0, 7.0, 0.0,                   # routing velocity alpha beta
        1.0,                             # msp.reservoir_direct_response_fraction
    ], dtype=np.float64)


PTHPSK_NS = 4 + 4 * HBV_MAX_BINS + 1  # swe sca surface_heat n_bins sp[8] sw[8] albedo[8] iso_pot_energy[8] kirchner.q


def default_pthpsk_state(n_cells: int, q: float = 1.0, swe: float = 0.0, sca: float = 0.0) -> np.ndarray:
    """PTHPSKState(): hbv_physical_snow::state() (surface_heat 30000, undistributed) with kirchner.q = q."""
    s = np.zeros((n_cells, PTHPSK_NS), dtype=np.float64)
    s[:, 0] = swe
    s[:, 1] = sca
    s[:, 2] = 30000.0
    s[:, -1] = q
    return s
