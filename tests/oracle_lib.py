"""ctypes loader for the CPU oracle (oracle/_build/liboracle.so).

Test infrastructure only: used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker / baseline, never by shyft_amd.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "_build", "liboracle.so")
_L = None
_d = C.c_double
_dp = C.POINTER(C.c_double)


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


_CACHE = {}


def load(variant: str = "detmath"):
    """variant 'detmath' (bit-exact checker of the HIP kernels), 'libm' (host libm, as the reference),
    'fullgamma' / 'libm_fullgamma' (gamma_snow's incomplete gamma at full precision: tolerance statement)."""
    if variant in _CACHE:
        return _CACHE[variant]
    names = {"detmath": None, "libm": "liboracle_libm.so", "fullgamma": "liboracle_fullgamma.so",
             "libm_fullgamma": "liboracle_libm_fullgamma.so", "nodeadcss": "liboracle_nodeadcss.so"}
    path = LIB if variant == "detmath" else os.path.join(ORACLE_DIR, "_build", names[variant])
    if not os.path.exists(path):
        build()
    L = C.CDLL(path)
    for fn in ("oracle_exp", "oracle_log", "oracle_lgamma_fn"):
        getattr(L, fn).restype = _d
        getattr(L, fn).argtypes = [_d]
    L.oracle_pow.restype = _d
    L.oracle_pow.argtypes = [_d, _d]
    L.oracle_gamma_p.restype = _d
    L.oracle_gamma_p.argtypes = [_d, _d]
    L.oracle_gamma_pq.argtypes = [_d, _d, _dp, _dp, _dp]
    L.oracle_gamma_pq_policy.argtypes = [_d, _d, _dp, _dp, _dp]
    L.oracle_lgamma.restype = _d
    L.oracle_lgamma.argtypes = [_d]
    L.oracle_gs_calc_snow_state.argtypes = [_d] * 7 + [_dp, _dp]
    L.oracle_gs_corr_lwc.restype = _d
    L.oracle_gs_corr_lwc.argtypes = [_d] * 6
    L.oracle_gs_step.restype = C.c_int
    L.oracle_gs_step.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p] + [_d] * 7
    L.oracle_kirchner_step.restype = C.c_int
    L.oracle_kirchner_step.argtypes = [_d] * 5 + [C.c_int64, C.c_int64, _dp, _dp, _d, _d]
    L.oracle_pt_pot_evap.restype = _d
    L.oracle_pt_pot_evap.argtypes = [_d] * 5
    L.oracle_day_of_year.restype = C.c_int
    L.oracle_day_of_year.argtypes = [C.c_int64]
    L.oracle_trim_year.restype = C.c_int64
    L.oracle_trim_year.argtypes = [C.c_int64]
    L.oracle_ptgsk_run.restype = C.c_int
    L.oracle_ptgsk_run.argtypes = ([C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_int64,
                                    C.c_int64, C.c_size_t, C.c_int, C.c_int] + [C.c_void_p] * 8 +
                                   [C.c_int, _dp, C.c_char_p, C.c_size_t])
    L.oracle_hbv_integrate.restype = _d
    L.oracle_hbv_integrate.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, _d, _d, C.c_int]
    L.oracle_hbv_snow_step.restype = C.c_int
    L.oracle_hbv_snow_step.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, _d, _d, C.c_int, _dp,
                                       C.c_char_p, C.c_size_t]
    L.oracle_hbv_soil_step.restype = None
    L.oracle_hbv_soil_step.argtypes = [_d, _d, _dp, _d, _d, _dp]
    L.oracle_hbv_tank_step.restype = None
    L.oracle_hbv_tank_step.argtypes = [C.c_void_p, _dp, _dp, _d, _dp]
    L.oracle_hbv_ae.restype = _d
    L.oracle_hbv_ae.argtypes = [_d] * 4
    L.oracle_hbv_run.restype = C.c_int
    L.oracle_hbv_run.argtypes = ([C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                  C.c_int64, C.c_int64, C.c_size_t, C.c_int, C.c_int] + [C.c_void_p] * 8 +
                                 [C.c_int, _dp, C.c_char_p, C.c_size_t])
    L.oracle_skaugen_step.restype = C.c_int
    L.oracle_skaugen_step.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, _d, _d]
    L.oracle_skaugen_sca_rel_red.restype = _d
    L.oracle_skaugen_sca_rel_red.argtypes = [C.c_uint64, C.c_uint64, _d, _d]
    L.oracle_ptssk_run.restype = C.c_int
    L.oracle_ptssk_run.argtypes = L.oracle_ptgsk_run.argtypes
    L.oracle_pthsk_run.restype = C.c_int
    L.oracle_pthsk_run.argtypes = L.oracle_hbv_run.argtypes
    L.oracle_route.restype = C.c_int
    L.oracle_route.argtypes = [C.c_size_t, C.c_size_t, C.c_int64] + [C.c_void_p] * 4 + [C.c_size_t] + \
        [C.c_void_p] * 4 + [C.c_int64] + [C.c_void_p] * 3
    L.oracle_make_uhg.restype = None
    L.oracle_make_uhg.argtypes = [C.c_int, _d, _d, C.c_void_p, C.POINTER(C.c_int)]
    _CACHE[variant] = L
    return L


def idw_run(kind, src_xyz, src_values, dst_xyz, param, dst_slope=None, variant="detmath"):
    """inverse_distance run_interpolation of one variable (oracle kinds: 0 temperature, 1 precipitation, 2 radiation,
    3 wind_speed, 4 rel_hum); src_values [T][S] -> [T][N] (oracle/src/idw.hpp)."""
    L = load(variant)
    L.oracle_idw_run.restype = C.c_int
    L.oracle_idw_run.argtypes = [C.c_int, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                 C.c_size_t, C.c_void_p, C.c_void_p]
    src_xyz = np.ascontiguousarray(src_xyz, dtype=np.float64)
    src_values = np.ascontiguousarray(src_values, dtype=np.float64)
    dst_xyz = np.ascontiguousarray(dst_xyz, dtype=np.float64)
    S, N, T = src_xyz.shape[0], dst_xyz.shape[0], src_values.shape[0]
    slope = None if dst_slope is None else np.ascontiguousarray(dst_slope, dtype=np.float64)
    out = np.empty((T, N))
    prm = np.ascontiguousarray(param, dtype=np.float64)
    L.oracle_idw_run(int(kind), S, _p(src_xyz), _p(src_values), N, _p(dst_xyz), None if slope is None else _p(slope),
                     T, _p(prm), _p(out))
    return out


def route(q, dt_us, cell_rid, cell_dist, cell_vab, rivers, query, variant="detmath"):
    """routing::model (routing.h:347-387) on the oracle. q [T][N] avg_discharge; rivers: list of
    (id, downstream_id, distance, velocity, alpha, beta). Returns local, upstream, output [T]."""
    L = load(variant)
    q = np.ascontiguousarray(q, dtype=np.float64)
    T, N = q.shape
    crid = np.ascontiguousarray(cell_rid, dtype=np.int64)
    cd = np.ascontiguousarray(cell_dist, dtype=np.float64)
    cv = np.ascontiguousarray(cell_vab, dtype=np.float64).reshape(N, 3)
    rv = np.asarray(rivers, dtype=np.float64).reshape(-1, 6)
    rid = np.ascontiguousarray(rv[:, 0], dtype=np.int64)
    ds = np.ascontiguousarray(rv[:, 1], dtype=np.int64)
    rd = np.ascontiguousarray(rv[:, 2])
    rvab = np.ascontiguousarray(rv[:, 3:6])
    out = [np.empty(T) for _ in range(3)]
    if L.oracle_route(N, T, int(dt_us), _p(q), _p(crid), _p(cd), _p(cv), len(rid), _p(rid), _p(ds), _p(rd), _p(rvab),
                      int(query), _p(out[0]), _p(out[1]), _p(out[2])) != 0:
        raise RuntimeError("oracle_route failed")
    return tuple(out)


def make_uhg(n_steps, alpha, beta, variant="detmath"):
    L = load(variant)
    buf = np.empty(max(1, n_steps))
    n = C.c_int(0)
    L.oracle_make_uhg(int(n_steps), float(alpha), float(beta), _p(buf), C.byref(n))
    return buf[:n.value].copy()


SKAUGEN_DEFAULT = (40.77, 113.0, 0.1, 0.1, 0.16, 2.5, 0.14, 0.01)  # skaugen::parameter() (skaugen.h:89-112)
PTSSK_NS = 8        # nu alpha sca swe free_water residual num_units kirchner.q
PTSSK_NSC = 7       # state collector series (pt_ss_k_cell_model.h:185-200)


def skaugen_step(state7, dt_us, T, prec_mm_h, p8=SKAUGEN_DEFAULT, variant="detmath"):
    """One skaugen::calculator::step; state7 (nu alpha sca swe free_water residual num_units) updated in place.
    Returns (outflow, sca, swe) of the response."""
    L = load(variant)
    st = np.ascontiguousarray(state7, dtype=np.float64)
    p = np.ascontiguousarray(p8, dtype=np.float64)
    r = np.zeros(3)
    if L.oracle_skaugen_step(_p(st), _p(r), int(dt_us), _p(p), float(T), float(prec_mm_h)) != 0:
        raise RuntimeError("skaugen step raised")
    state7[:] = st
    return tuple(r)


def ptssk_run(geo11, params, state, t0_us, dt_us, forcing, start_step=0, n_steps=0, set_ix=None, full=False,
              collect_state=False, ncore=0, variant="detmath"):
    """pt_ss_k region on the oracle: 'main' [2][T][N], 'full' [8][T][N], 'state_series' [7][T+1][N], 'state' [N][8]."""
    L = load(variant)
    geo11 = np.ascontiguousarray(geo11, dtype=np.float64)
    N = geo11.shape[0]
    params = np.ascontiguousarray(np.atleast_2d(params), dtype=np.float64)
    st = np.ascontiguousarray(state, dtype=np.float64).reshape(N, PTSSK_NS).copy()
    F = np.ascontiguousarray(forcing, dtype=np.float64)
    T = F.shape[1]
    ix = None if set_ix is None else np.ascontiguousarray(set_ix, dtype=np.int32)
    out_main = np.empty((2, T, N))
    out_full = np.empty((8, T, N)) if full else None
    out_state = np.empty((PTSSK_NSC, T + 1, N)) if collect_state else None
    el = C.c_double(0.0)
    err = C.create_string_buffer(512)
    rc = L.oracle_ptssk_run(N, _p(geo11), _p(params), params.shape[0], _p(ix), _p(st), int(t0_us), int(dt_us), T,
                            int(start_step), int(n_steps), _p(F[0]), _p(F[1]), _p(F[2]), _p(F[3]), _p(F[4]),
                            _p(out_main), _p(out_full), _p(out_state), int(ncore), C.byref(el), err, 512)
    if rc != 0:
        raise RuntimeError(err.value.decode())
    r = {"main": out_main, "state": st, "elapsed_s": el.value}
    if full:
        r["full"] = out_full
    if collect_state:
        r["state_series"] = out_state
    return r


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def ptgsk_run(geo11, params, state, t0_us, dt_us, forcing, start_step=0, n_steps=0, set_ix=None, full=False,
              collect_state=False, ncore=0, variant="detmath"):
    """Run the oracle region model. forcing: [5][T][N]. Returns dict with 'main' [2][T][N],
    'full' [8][T][N] (if full), 'state_series' [9][T+1][N] (if collect_state), 'state' [N][9], 'elapsed_s'."""
    L = load(variant)
    geo11 = np.ascontiguousarray(geo11, dtype=np.float64)
    N = geo11.shape[0]
    params = np.ascontiguousarray(np.atleast_2d(params), dtype=np.float64)
    st = np.ascontiguousarray(state, dtype=np.float64).reshape(N, 9).copy()
    F = np.ascontiguousarray(forcing, dtype=np.float64)
    T = F.shape[1]
    ix = None if set_ix is None else np.ascontiguousarray(set_ix, dtype=np.int32)
    out_main = np.empty((2, T, N))
    out_full = np.empty((8, T, N)) if full else None
    out_state = np.empty((9, T + 1, N)) if collect_state else None
    el = C.c_double(0.0)
    err = C.create_string_buffer(512)
    rc = L.oracle_ptgsk_run(N, _p(geo11), _p(params), params.shape[0], _p(ix), _p(st), int(t0_us), int(dt_us), T,
                            int(start_step), int(n_steps), _p(F[0]), _p(F[1]), _p(F[2]), _p(F[3]), _p(F[4]),
                            _p(out_main), _p(out_full), _p(out_state), int(ncore), C.byref(el), err, 512)
    if rc != 0:
        raise RuntimeError(err.value.decode())
    r = {"main": out_main, "state": st, "elapsed_s": el.value}
    if full:
        r["full"] = out_full
    if collect_state:
        r["state_series"] = out_state
    return r


HBV_MAX_BINS = 8
HBV_FLAT = 6 + 2 * HBV_MAX_BINS   # swe sca sm uz lz n_bins sp[8] sw[8]


def hbv_normalize(s, intervals):
    """hbv_snow::parameter::normalize_snow_distribution (hbv_snow.h:42-47) as set_snow_redistribution_factors
    applies it: s / integrate(s, intervals, n, intervals[0], intervals[-1])."""
    L = load()
    f = np.ascontiguousarray(s, dtype=np.float64)
    x = np.ascontiguousarray(intervals, dtype=np.float64)
    mean = L.oracle_hbv_integrate(f.ctypes.data_as(C.c_void_p), x.ctypes.data_as(C.c_void_p), len(x), float(x[0]),
                                  float(x[-1]), 0)
    return f / mean


def hbv_dist_row(s, intervals):
    """(n_bins, s[8], intervals[8]) row of one parameter set's snow distribution."""
    row = np.zeros(1 + 2 * HBV_MAX_BINS)
    n = len(s)
    row[0] = n
    row[1:1 + n] = s
    row[1 + HBV_MAX_BINS:1 + HBV_MAX_BINS + n] = intervals
    return row


def hbv_run(geo11, params, state, t0_us, dt_us, forcing, start_step=0, n_steps=0, set_ix=None, snow_dist=None,
            full=False, collect_state=False, ncore=0, variant="detmath"):
    """Run the oracle hbv_stack region. params [n_sets][22]; snow_dist [n_sets][17] or None (default 5 bins);
    state [N][22]. Returns dict main [2][T][N], full [9][T][N], state_series [22][T+1][N], state [N][22]."""
    L = load(variant)
    geo11 = np.ascontiguousarray(geo11, dtype=np.float64)
    N = geo11.shape[0]
    params = np.ascontiguousarray(np.atleast_2d(params), dtype=np.float64)
    dist = None if snow_dist is None else np.ascontiguousarray(np.atleast_2d(snow_dist), dtype=np.float64)
    st = np.ascontiguousarray(state, dtype=np.float64).reshape(N, HBV_FLAT).copy()
    F = np.ascontiguousarray(forcing, dtype=np.float64)
    T = F.shape[1]
    ix = None if set_ix is None else np.ascontiguousarray(set_ix, dtype=np.int32)
    out_main = np.empty((2, T, N))
    out_full = np.empty((9, T, N)) if full else None
    out_state = np.empty((HBV_FLAT, T + 1, N)) if collect_state else None
    el = C.c_double(0.0)
    err = C.create_string_buffer(512)
    rc = L.oracle_hbv_run(N, _p(geo11), _p(params), _p(dist), params.shape[0], _p(ix), _p(st), int(t0_us), int(dt_us),
                          T, int(start_step), int(n_steps), _p(F[0]), _p(F[1]), _p(F[2]), _p(F[3]), _p(F[4]),
                          _p(out_main), _p(out_full), _p(out_state), int(ncore), C.byref(el), err, 512)
    if rc != 0:
        raise RuntimeError(err.value.decode())
    r = {"main": out_main, "state": st, "elapsed_s": el.value}
    if full:
        r["full"] = out_full
    if collect_state:
        r["state_series"] = out_state
    return r


def hbv_snow_step(flat_state, prec, temp, t0_us=0, t1_us=3600_000_000, s=None, intervals=None, tx=0.0, cx=1.0,
                  ts=0.0, lw=0.1, cfr=0.5, distribute=0, variant="detmath"):
    """One hbv_snow::calculator::step; returns (new flat state, outflow)."""
    L = load(variant)
    st = np.ascontiguousarray(flat_state, dtype=np.float64).copy()
    dist = None if s is None else hbv_dist_row(s, intervals)
    pv = np.array([tx, cx, ts, lw, cfr], dtype=np.float64)
    out = C.c_double(0.0)
    err = C.create_string_buffer(512)
    rc = L.oracle_hbv_snow_step(_p(pv), _p(dist), _p(st), int(t0_us), int(t1_us), float(prec), float(temp),
                                int(distribute), C.byref(out), err, 512)
    if rc != 0:
        raise RuntimeError(err.value.decode())
    return st, out.value


def hbv_snow_state(swe=0.0, sca=0.0, sm=0.0, uz=20.0, lz=10.0):
    """flat hbv state (HbvState() defaults: soil sm 0, tank uz 20 lz 10, undistributed snow)."""
    v = np.zeros(HBV_FLAT)
    v[:5] = [swe, sca, sm, uz, lz]
    return v


PTHSK_FLAT = 3 + 2 * HBV_MAX_BINS + 1   # swe sca n_bins sp[8] sw[8] kirchner.q
PTHSK_NSC = 3 + 2 * HBV_MAX_BINS        # kirchner_discharge snow_sca snow_swe sp[8] sw[8]


def pthsk_run(geo11, params, state, t0_us, dt_us, forcing, start_step=0, n_steps=0, set_ix=None, snow_dist=None,
              full=False, collect_state=False, ncore=0, variant="detmath"):
    """Run the oracle pt_hs_k region. params [n_sets][18]; snow_dist [n_sets][17] or None (default 5 bins);
    state [N][20]. Returns dict main [2][T][N], full [8][T][N], state_series [19][T+1][N], state [N][20]."""
    L = load(variant)
    geo11 = np.ascontiguousarray(geo11, dtype=np.float64)
    N = geo11.shape[0]
    params = np.ascontiguousarray(np.atleast_2d(params), dtype=np.float64)
    dist = None if snow_dist is None else np.ascontiguousarray(np.atleast_2d(snow_dist), dtype=np.float64)
    st = np.ascontiguousarray(state, dtype=np.float64).reshape(N, PTHSK_FLAT).copy()
    F = np.ascontiguousarray(forcing, dtype=np.float64)
    T = F.shape[1]
    ix = None if set_ix is None else np.ascontiguousarray(set_ix, dtype=np.int32)
    out_main = np.empty((2, T, N))
    out_full = np.empty((8, T, N)) if full else None
    out_state = np.empty((PTHSK_NSC, T + 1, N)) if collect_state else None
    el = C.c_double(0.0)
    err = C.create_string_buffer(512)
    rc = L.oracle_pthsk_run(N, _p(geo11), _p(params), _p(dist), params.shape[0], _p(ix), _p(st), int(t0_us),
                            int(dt_us), T, int(start_step), int(n_steps), _p(F[0]), _p(F[1]), _p(F[2]), _p(F[3]),
                            _p(F[4]), _p(out_main), _p(out_full), _p(out_state), int(ncore), C.byref(el), err, 512)
    if rc != 0:
        raise RuntimeError(err.value.decode())
    r = {"main": out_main, "state": st, "elapsed_s": el.value}
    if full:
        r["full"] = out_full
    if collect_state:
        r["state_series"] = out_state
    return r


PTHPSK_FLAT = 4 + 4 * HBV_MAX_BINS + 1  # swe sca surface_heat n_bins sp[8] sw[8] albedo[8] iso_pot_energy[8] q
PTHPSK_NSC = 4 + 4 * HBV_MAX_BINS       # kirchner_discharge hps_sca hps_swe hps_surface_heat sp sw albedo iso


def hps_step(st36, p12, dist17, distribute, dt_us, T, rad, prec_mm_h, wind_speed, rel_hum, variant="detmath"):
    """One hbv_physical_snow step on a flat state (updated in place). Returns (outflow, sca, storage)."""
    L = load(variant)
    L.oracle_hps_step.restype = C.c_int
    L.oracle_hps_step.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int64] + \
        [C.c_double] * 5 + [C.c_char_p, C.c_size_t]
    st = np.ascontiguousarray(st36, dtype=np.float64)
    p = np.ascontiguousarray(p12, dtype=np.float64)
    d = np.ascontiguousarray(dist17, dtype=np.float64)
    r = np.zeros(3)
    err = C.create_string_buffer(512)
    if L.oracle_hps_step(_p(st), _p(r), _p(p), _p(d), int(distribute), int(dt_us), float(T), float(rad),
                         float(prec_mm_h), float(wind_speed), float(rel_hum), err, 512) != 0:
        raise RuntimeError(err.value.decode())
    st36[:] = st
    return tuple(r)


def pthpsk_run(geo11, params, state, t0_us, dt_us, forcing, start_step=0, n_steps=0, set_ix=None, gm_direct=None,
               snow_dist=None, full=False, collect_state=False, ncore=0, variant="detmath"):
    """Run the oracle pt_hps_k region. params [n_sets][24]; gm_direct [n_sets] or None; snow_dist [n_sets][17] or
    None; state [N][37]. Returns dict main [2][T][N], full [8][T][N], state_series [36][T+1][N], state [N][37]."""
    L = load(variant)
    L.oracle_pthpsk_run.restype = C.c_int
    L.oracle_pthpsk_run.argtypes = ([C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                     C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_size_t, C.c_int, C.c_int] +
                                    [C.c_void_p] * 8 + [C.c_int, C.POINTER(C.c_double), C.c_char_p, C.c_size_t])
    geo11 = np.ascontiguousarray(geo11, dtype=np.float64)
    N = geo11.shape[0]
    params = np.ascontiguousarray(np.atleast_2d(params), dtype=np.float64)
    gm = None if gm_direct is None else np.ascontiguousarray(np.atleast_1d(gm_direct), dtype=np.float64)
    dist = None if snow_dist is None else np.ascontiguousarray(np.atleast_2d(snow_dist), dtype=np.float64)
    st = np.ascontiguousarray(state, dtype=np.float64).reshape(N, PTHPSK_FLAT).copy()
    F = np.ascontiguousarray(forcing, dtype=np.float64)
    T = F.shape[1]
    ix = None if set_ix is None else np.ascontiguousarray(set_ix, dtype=np.int32)
    out_main = np.empty((2, T, N))
    out_full = np.empty((8, T, N)) if full else None
    out_state = np.empty((PTHPSK_NSC, T + 1, N)) if collect_state else None
    el = C.c_double(0.0)
    err = C.create_string_buffer(512)
    rc = L.oracle_pthpsk_run(N, _p(geo11), _p(params), _p(gm), _p(dist), params.shape[0], _p(ix), _p(st),
                             int(t0_us), int(dt_us), T, int(start_step), int(n_steps), _p(F[0]), _p(F[1]), _p(F[2]),
                             _p(F[3]), _p(F[4]), _p(out_main), _p(out_full), _p(out_state), int(ncore), C.byref(el),
                             err, 512)
    if rc != 0:
        raise RuntimeError(err.value.decode())
    r = {"main": out_main, "state": st, "elapsed_s": el.value}
    if full:
        r["full"] = out_full
    if collect_state:
        r["state_series"] = out_state
    return r
