"""Thin Python owner of a C-ABI region handle (include/shyft_hip.h).

This is plumbing for tests, the bench and the Python API layer: every call
goes straight to libshyft_hip.so. Arrays are numpy (host) or, where a
function takes `on_device`, a raw device pointer (e.g. torch tensor.data_ptr()).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._native import check, lib

PT_GS_K, HBV_STACK, PT_SS_K, PT_HS_K, PT_HPS_K = 1, 2, 3, 4, 5
TEMPERATURE, PRECIPITATION, WIND_SPEED, REL_HUM, RADIATION = range(5)
FORCING_NAMES = ("temperature", "precipitation", "wind_speed", "rel_hum", "radiation")
COLLECT_DISCHARGE, COLLECT_DISCHARGE_SNOW, COLLECT_ALL = 0, 1, 2
PTGSK_SERIES = ("avg_discharge", "charge_m3s", "snow_sca", "snow_swe", "snow_outflow", "glacier_melt", "ae_output",
                "pe_output")
PTGSK_STATE = ("albedo", "lwc", "surface_heat", "alpha", "sdc_melt_mean", "acc_melt", "iso_pot_energy", "temp_swe",
               "kirchner_q")
HBV_SERIES = ("avg_discharge", "charge_m3s", "snow_sca", "snow_swe", "snow_outflow", "glacier_melt", "ae_output",
              "pe_output", "soil_outflow")
HBV_MAX_BINS = 8
HBV_STATE = (("swe", "sca", "soil_moisture", "tank_uz", "tank_lz", "n_bins") +
             tuple(f"sp{i}" for i in range(HBV_MAX_BINS)) + tuple(f"sw{i}" for i in range(HBV_MAX_BINS)))
SCOPE_CELL_IX, SCOPE_CATCHMENT = 0, 1
SERIES_FORCING, SERIES_STATE = 100, 200
KNOB_PTGSK_INSTANCE, KNOB_BRENT_READ_DELAY, KNOB_SERIAL_SHARDS, KNOB_CLONE_FAIL_AT = 1, 2, 3, 4
# shyft_hip_region_create_sharded_ex options (include/shyft_hip.h)
SHARD_RCCL_ALWAYS, SHARD_NO_RCCL, SHARD_TEST_FAIL_INIT, SHARD_TEST_FAIL_GATHER, SHARD_TEST_CORRUPT_CHECK = 1, 2, 4, 8, 16
SHARD_BALANCE_Z = 32
SHARD_TEST_STALL_CHECK = 64
# pt_ss_k (core/pt_ss_k.h:154-181, pt_ss_k_cell_model.h:38-200); response series ids are the pt_gs_k ones
PTSSK_STATE = ("nu", "alpha", "sca", "swe", "free_water", "residual", "num_units", "kirchner_q")
PTSSK_STATE_SERIES = ("kirchner_discharge", "snow_sca", "snow_swe", "snow_alpha", "snow_nu", "snow_lwc",
                      "snow_residual")
# pt_hs_k (core/pt_hs_k.h:148-172, pt_hs_k_cell_model.h:148-210); response series ids are the pt_gs_k ones
PTHSK_STATE = (("swe", "sca", "n_bins") + tuple(f"sp{i}" for i in range(HBV_MAX_BINS)) +
               tuple(f"sw{i}" for i in range(HBV_MAX_BINS)) + ("kirchner_q",))
PTHSK_STATE_SERIES = (("kirchner_discharge", "snow_sca", "snow_swe") + tuple(f"sp{i}" for i in range(HBV_MAX_BINS)) +
                      tuple(f"sw{i}" for i in range(HBV_MAX_BINS)))
# pt_hps_k (core/pt_hps_k.h:163-185, pt_hps_k_cell_model.h:160-232); response series ids are the pt_gs_k ones
_B = tuple(range(HBV_MAX_BINS))
PTHPSK_STATE = (("swe", "sca", "surface_heat", "n_bins") + tuple(f"sp{i}" for i in _B) + tuple(f"sw{i}" for i in _B) +
                tuple(f"albedo{i}" for i in _B) + tuple(f"iso_pot_energy{i}" for i in _B) + ("kirchner_q",))
PTHPSK_STATE_SERIES = (("kirchner_discharge", "hps_sca", "hps_swe", "hps_surface_heat") +
                       tuple(f"sp{i}" for i in _B) + tuple(f"sw{i}" for i in _B) + tuple(f"albedo{i}" for i in _B) +
                       tuple(f"iso_pot_energy{i}" for i in _B))
STACK_NPARAM = {PT_GS_K: 31, HBV_STACK: 22, PT_SS_K: 21, PT_HS_K: 18, PT_HPS_K: 24}
STACK_NSTATE = {PT_GS_K: 9, HBV_STACK: len(HBV_STATE), PT_SS_K: len(PTSSK_STATE), PT_HS_K: len(PTHSK_STATE),
                PT_HPS_K: len(PTHPSK_STATE)}
STACK_NSERIES = {PT_GS_K: len(PTGSK_SERIES), HBV_STACK: len(HBV_SERIES), PT_SS_K: len(PTGSK_SERIES),
                 PT_HS_K: len(PTGSK_SERIES), PT_HPS_K: len(PTGSK_SERIES)}


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class HipRegion:
    """A region on one device, or -- with `devices` (a list, one entry per shard, repeats allowed) -- one region
    whose cells are split into len(devices) contiguous shards driven from this process
    (shyft_hip_region_create_sharded): every method below then works on the whole region."""

    def __init__(self, stack: int, n_cells: int, device: int = -1, devices=None, shard_flags: int = 0):
        self._L = lib()
        h = C.c_void_p()
        if devices is None:
            check(self._L.shyft_hip_region_create(stack, n_cells, device, C.byref(h)), None)
        else:
            d = np.ascontiguousarray(list(devices), dtype=np.int32)
            check(self._L.shyft_hip_region_create_sharded_ex(stack, n_cells, _ptr(d), d.size, int(shard_flags),
                                                             C.byref(h)), None)
        self.h = h
        self.stack = stack
        self.n = n_cells
        self.n_steps = 0
        self.window = 0

    def shards(self) -> list:
        """[(device, first cell, n_cells)] of every shard ([(device, 0, n)] for an unsharded region)."""
        dev, c0, nc = C.c_int(), C.c_size_t(), C.c_size_t()
        S = int(self._L.shyft_hip_region_shards(self.h, 0, None, None, None))
        out = []
        for k in range(S):
            self._L.shyft_hip_region_shards(self.h, k, C.byref(dev), C.byref(c0), C.byref(nc))
            out.append((dev.value, c0.value, nc.value))
        return out

    def combine_path(self) -> str:
        """How shard partial sums are combined: "none" (unsharded), "copy" (shards share a device), "rccl"."""
        return ("none", "copy", "rccl")[int(self._L.shyft_hip_region_combine_path(self.h))]

    def combine_report(self) -> str:
        """The combine path's decision: why RCCL or copies, the RCCL self-check result, run-time fallbacks."""
        r = self._L.shyft_hip_region_combine_report(self.h)
        return r.decode() if r else ""

    def close(self):
        if getattr(self, "h", None):
            self._L.shyft_hip_region_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, status):
        check(status, self.h)

    def set_geo(self, geo11: np.ndarray, routing_id=None, routing_distance=None):
        g = np.ascontiguousarray(geo11, dtype=np.float64).reshape(self.n, 11)
        rid = None if routing_id is None else np.ascontiguousarray(routing_id, dtype=np.int64)
        rd = None if routing_distance is None else np.ascontiguousarray(routing_distance, dtype=np.float64)
        self._chk(self._L.shyft_hip_set_geo(self.h, _ptr(g), _ptr(rid), _ptr(rd)))

    def set_parameters(self, params: np.ndarray, set_ix: np.ndarray | None = None):
        p = np.ascontiguousarray(params, dtype=np.float64)
        if p.ndim == 1:
            p = p.reshape(1, -1)
        ix = None if set_ix is None else np.ascontiguousarray(set_ix, dtype=np.int32)
        self._chk(self._L.shyft_hip_set_parameters(self.h, _ptr(p), p.shape[0], p.shape[1], _ptr(ix)))

    def set_time_axis(self, t0_us: int, dt_us: int, n_steps: int, window_steps: int = 0):
        self._chk(self._L.shyft_hip_set_time_axis(self.h, int(t0_us), int(dt_us), int(n_steps), int(window_steps)))
        self.n_steps = n_steps
        self.window = n_steps if window_steps in (0, None) or window_steps > n_steps else window_steps

    def set_window(self, w0: int):
        self._chk(self._L.shyft_hip_set_window(self.h, int(w0)))

    def move_window(self, w0: int, fill_mask: int = 0):
        """set_window without (or with a subset of) the NaN fill; for callers that rewrite the whole window."""
        self._chk(self._L.shyft_hip_move_window(self.h, int(w0), int(fill_mask)))

    def set_collection(self, collect: int, collect_state: bool = False):
        self._chk(self._L.shyft_hip_set_collection(self.h, int(collect), int(bool(collect_state))))

    def set_catchment_filter(self, cids):
        c = np.ascontiguousarray(cids, dtype=np.int64)
        self._chk(self._L.shyft_hip_set_catchment_filter(self.h, _ptr(c) if c.size else None, c.size))

    def set_state(self, state: np.ndarray):
        s = np.ascontiguousarray(state, dtype=np.float64).reshape(self.n, -1)
        self._chk(self._L.shyft_hip_set_state(self.h, _ptr(s), s.shape[1]))

    def get_state(self, n_fields: int | None = None) -> np.ndarray:
        nf = n_fields or STACK_NSTATE[self.stack]
        s = np.empty((self.n, nf), dtype=np.float64)
        self._chk(self._L.shyft_hip_get_state(self.h, _ptr(s), nf))
        return s

    def copy_state_from(self, src: "HipRegion"):
        """This region's state := src's state, device to device (same stack and cell count)."""
        self._chk(self._L.shyft_hip_copy_state(self.h, src.h))

    def set_forcing(self, var: int, step0: int, values: np.ndarray):
        v = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, self.n)
        self._chk(self._L.shyft_hip_set_forcing(self.h, var, step0, v.shape[0], _ptr(v), 0))

    def set_forcing_device(self, var: int, step0: int, n: int, dev_ptr: int):
        self._chk(self._L.shyft_hip_set_forcing(self.h, var, step0, n, C.c_void_p(dev_ptr), 1))

    def get_forcing(self, var: int, step0: int, n: int) -> np.ndarray:
        out = np.empty((n, self.n), dtype=np.float64)
        self._chk(self._L.shyft_hip_get_forcing(self.h, var, step0, n, _ptr(out), 0))
        return out

    def get_forcing_device(self, var: int, step0: int, n: int, dev_ptr: int):
        """[n][cells] forcing rows into device memory (e.g. a torch tensor's data_ptr())."""
        self._chk(self._L.shyft_hip_get_forcing(self.h, var, step0, n, C.c_void_p(dev_ptr), 1))

    def interpolate(self, var: int, src_xyz: np.ndarray, src_values: np.ndarray, step0: int, idw_param):
        """IDW of one forcing variable from sources (src_values [n][S] on the model axis)."""
        xyz = np.ascontiguousarray(src_xyz, dtype=np.float64).reshape(-1, 3)
        v = np.ascontiguousarray(src_values, dtype=np.float64).reshape(-1, xyz.shape[0])
        p = np.ascontiguousarray(idw_param, dtype=np.float64)
        assert p.size == 7
        self._chk(self._L.shyft_hip_interpolate(self.h, var, xyz.shape[0], _ptr(xyz), _ptr(v), step0, v.shape[0],
                                                _ptr(p)))

    def interpolation_path(self, var: int) -> str:
        """The gather the last interpolate of `var` ran: "wave", "tile", "copy" or "none"."""
        k = int(self._L.shyft_hip_interpolation_path(self.h, int(var)))
        if k < 0:
            raise ValueError(f"interpolation_path: invalid variable {var}")
        return ("none", "tile", "wave", "copy")[k]

    def interpolate_btk(self, src_xyz: np.ndarray, src_values: np.ndarray, step0: int, btk_param,
                        prior_gradient=None):
        """Bayesian temperature kriging into the temperature forcing (src_values [n][S] on the model axis).
        btk_param: gradient_sd (C/m), sill, nugget, range, zscale; prior_gradient [n] or None (day-of-year prior)."""
        xyz = np.ascontiguousarray(src_xyz, dtype=np.float64).reshape(-1, 3)
        v = np.ascontiguousarray(src_values, dtype=np.float64).reshape(-1, xyz.shape[0])
        p = np.ascontiguousarray(btk_param, dtype=np.float64)
        assert p.size == 5
        g = None if prior_gradient is None else np.ascontiguousarray(prior_gradient, dtype=np.float64)
        assert g is None or g.size == v.shape[0]
        self._chk(self._L.shyft_hip_interpolate_btk(self.h, xyz.shape[0], _ptr(xyz), _ptr(v), step0, v.shape[0],
                                                    _ptr(g), _ptr(p)))

    def synthetic_forcing(self, seed: int, step0: int, n: int, cell_offset: int = 0):
        self._chk(self._L.shyft_hip_synthetic_forcing(self.h, seed, cell_offset, step0, n))

    def prefetch_synthetic_forcing(self, seed: int, w0_next: int, cell_offset: int = 0, n_cus: int = 8):
        """Generate the next forcing window (rows w0_next .. w0_next + window) on a side stream of n_cus CUs."""
        self._chk(self._L.shyft_hip_prefetch_synthetic_forcing(self.h, seed, cell_offset, w0_next, n_cus))

    def swap_forcing_window(self, w0_next: int):
        self._chk(self._L.shyft_hip_swap_forcing_window(self.h, w0_next))

    def run_cells(self, use_ncore: int = 0, start_step: int = 0, n_steps: int = 0):
        self._chk(self._L.shyft_hip_run_cells(self.h, int(use_ncore), int(start_step), int(n_steps)))

    def run_cells_async(self, start_step: int, n_steps: int):
        self._chk(self._L.shyft_hip_run_cells_async(self.h, int(start_step), int(n_steps)))

    def synchronize(self):
        self._chk(self._L.shyft_hip_synchronize(self.h))

    def last_run_ms(self) -> float:
        return float(self._L.shyft_hip_last_run_ms(self.h))

    def last_interpolate_ms(self) -> float:
        """The last interpolate()'s gather kernel, ms (HIP events on the region's stream)."""
        return float(self._L.shyft_hip_last_interpolate_ms(self.h))

    def last_run_kernel_ms(self) -> list:
        """The last run's kernels separately (pt_gs_k: [snow kernel, flux kernel]; other stacks: [kernel])."""
        buf = (C.c_double * 4)()
        n = self._L.shyft_hip_last_run_kernel_ms(self.h, buf, 4)
        return [float(buf[k]) for k in range(n)]

    def shard_run_ms(self) -> list:
        """Kernel ms of every shard's last run_cells (one entry when unsharded)."""
        buf = (C.c_double * 256)()
        n = int(self._L.shyft_hip_shard_run_ms(self.h, buf, 256))
        return [float(buf[k]) for k in range(min(n, 256))]

    def get_series(self, series: int, step0: int, n: int) -> np.ndarray:
        out = np.empty((n, self.n), dtype=np.float64)
        self._chk(self._L.shyft_hip_get_series(self.h, series, step0, n, _ptr(out), 0))
        return out

    def get_series_device(self, series: int, step0: int, n: int, dev_ptr: int):
        """[n][cells] rows of a collected series into device memory (e.g. a torch tensor's data_ptr())."""
        self._chk(self._L.shyft_hip_get_series(self.h, series, step0, n, C.c_void_p(dev_ptr), 1))

    def get_state_series(self, field: int, step0: int, n: int) -> np.ndarray:
        out = np.empty((n, self.n), dtype=np.float64)
        self._chk(self._L.shyft_hip_get_state_series(self.h, field, step0, n, _ptr(out), 0))
        return out

    def sample_cells(self, series: int, cells, step0: int, n: int) -> np.ndarray:
        """[n][len(cells)] columns of a series (response id, SERIES_FORCING + v, SERIES_STATE + f) for the given
        cells over steps [step0, step0 + n) of the resident window (one device gather; per shard if sharded)."""
        c = np.ascontiguousarray(cells, dtype=np.int64)
        out = np.empty((n, c.size), dtype=np.float64)
        self._chk(self._L.shyft_hip_sample_cells(self.h, int(series), _ptr(c), c.size, int(step0), int(n), _ptr(out)))
        return out

    def set_test_knob(self, knob: int, value: int):
        """KNOB_PTGSK_INSTANCE (0 auto, 2, 4) / KNOB_BRENT_READ_DELAY (s_sleep(127) rounds); tests only."""
        self._chk(self._L.shyft_hip_set_test_knob(self.h, int(knob), int(value)))

    def statistics(self, series: int, ids=(), scope: int = SCOPE_CATCHMENT, weighted: bool = False, step0: int = 0,
                   n: int | None = None) -> np.ndarray:
        n = self.n_steps - step0 if n is None else n
        i = np.ascontiguousarray(list(ids), dtype=np.int64)
        out = np.empty(n, dtype=np.float64)
        self._chk(self._L.shyft_hip_statistics(self.h, series, _ptr(i) if i.size else None, i.size, scope,
                                               int(weighted), step0, n, _ptr(out)))
        return out

    def number_of_catchments(self) -> int:
        return int(self._L.shyft_hip_number_of_catchments(self.h))

    def catchment_ids(self) -> np.ndarray:
        c = np.empty(self.number_of_catchments(), dtype=np.int64)
        self._chk(self._L.shyft_hip_catchment_ids(self.h, _ptr(c)))
        return c

    def catchment_sums(self, series: int, step0: int, n: int) -> np.ndarray:
        out = np.empty((self.number_of_catchments(), n), dtype=np.float64)
        self._chk(self._L.shyft_hip_catchment_sums(self.h, series, step0, n, _ptr(out), 0))
        return out

    def catchment_sums_device(self, series: int, step0: int, n: int, dev_ptr: int):
        self._chk(self._L.shyft_hip_catchment_sums(self.h, series, step0, n, C.c_void_p(dev_ptr), 1))

    # routing (routing.h:239-421): cells sharing (river, UHG) are one group
    def set_routing_groups(self, group_of_cell, n_groups: int):
        g = np.ascontiguousarray(group_of_cell, dtype=np.int32)
        assert g.size == self.n
        self._chk(self._L.shyft_hip_set_routing_groups(self.h, _ptr(g), int(n_groups)))
        self.n_route_groups = int(n_groups)

    def routing_group_sums(self, step0: int, n: int) -> np.ndarray:
        out = np.empty((self.n_route_groups, n), dtype=np.float64)
        self._chk(self._L.shyft_hip_routing_group_sums(self.h, step0, n, _ptr(out), 0))
        return out

    def routing_group_sums_device(self, step0: int, n: int, dev_ptr: int):
        self._chk(self._L.shyft_hip_routing_group_sums(self.h, step0, n, C.c_void_p(dev_ptr), 1))

    # parameter ensembles (model_calibration.h:830-899): n_members parameter vectors in one launch
    def ensemble_run(self, params: np.ndarray, start_step: int = 0, n_steps: int = 0,
                     collect: int = COLLECT_DISCHARGE):
        p = np.ascontiguousarray(params, dtype=np.float64)
        assert p.ndim == 2
        self._chk(self._L.shyft_hip_ensemble_run(self.h, _ptr(p), p.shape[0], p.shape[1], start_step, n_steps,
                                                 collect))
        self.ens_members = p.shape[0]

    def ensemble_sums(self, series: int, step0: int, n: int, area_weighted: bool = False) -> np.ndarray:
        """[n_members][n_catchments][n] sums of `series` over each member's calculated cells per catchment."""
        out = np.empty((self.ens_members, self.number_of_catchments(), n), dtype=np.float64)
        self._chk(self._L.shyft_hip_ensemble_sums(self.h, series, int(area_weighted), step0, n, _ptr(out), 0))
        return out

    def ensemble_last_ms(self) -> float:
        return float(self._L.shyft_hip_ensemble_last_ms(self.h))


def route(group_sums, group_uhgs, group_river, river_uhgs, river_downstream, device: int = -1, sums_dev_ptr=None,
          T: int | None = None):
    """River network evaluation on the device (shyft_hip_route). group_sums [G][T] (numpy) or sums_dev_ptr (+T);
    group_uhgs / river_uhgs: lists of UHG weight vectors; group_river[G] and river_downstream[R] are river
    indices (ascending river id), -1 = no downstream. Returns (local, upstream, output), each [R][T]."""
    L = lib()
    G, R = len(group_uhgs), len(river_uhgs)
    max_len = max([1] + [len(w) for w in group_uhgs] + [len(w) for w in river_uhgs])
    gw = np.zeros((G, max_len))
    for k, w in enumerate(group_uhgs):
        gw[k, :len(w)] = w
    rw = np.zeros((R, max_len))
    for k, w in enumerate(river_uhgs):
        rw[k, :len(w)] = w
    glen = np.array([len(w) for w in group_uhgs], dtype=np.int32)
    rlen = np.array([len(w) for w in river_uhgs], dtype=np.int32)
    gr = np.ascontiguousarray(group_river, dtype=np.int32)
    rd = np.ascontiguousarray(river_downstream, dtype=np.int32)
    if sums_dev_ptr is None:
        s = np.ascontiguousarray(group_sums, dtype=np.float64)
        T = s.shape[1]
        src, on_dev = _ptr(s), 0
    else:
        src, on_dev = C.c_void_p(sums_dev_ptr), 1
    out = [np.empty((R, T)) for _ in range(3)]
    check(L.shyft_hip_route(device, G, T, src, on_dev, _ptr(gw), _ptr(glen), _ptr(gr), R, _ptr(rw), _ptr(rlen),
                            _ptr(rd), max_len, _ptr(out[0]), _ptr(out[1]), _ptr(out[2]), 0), None)
    return tuple(out)


def btk(src_xyz, src_values, prior_gradient, btk_param, dst_xyz, device: int = -1) -> np.ndarray:
    """Stateless Bayesian temperature kriging on the device (shyft_hip_btk): src_values [n][S] on the model axis,
    prior_gradient [n], btk_param (gradient_sd C/m, sill, nugget, range, zscale), dst_xyz [D][3] -> [n][D]."""
    L = lib()
    xyz = np.ascontiguousarray(src_xyz, dtype=np.float64).reshape(-1, 3)
    v = np.ascontiguousarray(src_values, dtype=np.float64).reshape(-1, xyz.shape[0])
    g = np.ascontiguousarray(prior_gradient, dtype=np.float64).reshape(v.shape[0])
    p = np.ascontiguousarray(btk_param, dtype=np.float64).reshape(5)
    d = np.ascontiguousarray(dst_xyz, dtype=np.float64).reshape(-1, 3)
    out = np.empty((v.shape[0], d.shape[0]))
    check(L.shyft_hip_btk(device, xyz.shape[0], _ptr(xyz), _ptr(v), v.shape[0], _ptr(g), _ptr(p), d.shape[0],
                          _ptr(d), _ptr(out)), None)
    return out
