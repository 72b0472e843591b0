"""shyft_amd.api.pt_hps_k -- the reference's `shyft.api.pt_hps_k` (api/boostpython/pt_hps_k.cpp,
shyft/api/pt_hps_k/__init__.py) over the MI355X engine."""
from __future__ import annotations

from .. import (_api, _FlatParameter, _FlatState, _ModelMixin, _Statistics, _Vector, SERIES_STATE,
                make_state_with_id_types)

# get/set order and names (core/pt_hps_k.h:64-159); defaults (kirchner.h:120-125, hbv_physical_snow.h:41-57,
# glacier_melt.h:28-32, routing.h:76, mstack_param.h). gm.direct_response is a member but not a calibration value
# (size() == 24): it rides behind the 24 in the flat vector.
_NAMES = ("kirchner.c1", "kirchner.c2", "kirchner.c3", "ae.ae_scale_factor", "hps.lw", "hps.tx", "hps.cfr",
          "hps.wind_scale", "hps.wind_const", "hps.surface_magnitude", "hps.max_albedo", "hps.min_albedo",
          "hps.fast_albedo_decay_rate", "hps.slow_albedo_decay_rate", "hps.snowfall_reset_depth",
          "hps.calculate_iso_pot_energy", "gm.dtf", "p_corr.scale_factor", "pt.albedo", "pt.alpha",
          "routing.velocity", "routing.alpha", "routing.beta", "msp.reservoir_direct_response_fraction",
          "gm.direct_response")
_DEFAULTS = (-2.439, 0.966, -0.10, 1.5, 0.1, 0.0, 0.5, 2.0, 1.0, 30.0, 0.9, 0.6, 5.0, 5.0, 5.0, 0.0, 6.0, 1.0, 0.2,
             1.26, 1.0, 7.0, 0.0, 1.0, 0.0)
MAX_BINS = 8


class PTHPSKParameter(_FlatParameter):
    NAMES = _NAMES
    DEFAULTS = _DEFAULTS
    ERROR = "pt_ss_k parameter accessor: .set size missmatch"  # the reference's text (pt_hps_k.h:70)

    def __init__(self, *a):
        super().__init__(*a)
        src = a[0] if a and isinstance(a[0], PTHPSKParameter) else None
        self.snow_s = list(src.snow_s) if src else [1.0] * 5
        self.snow_intervals = list(src.snow_intervals) if src else [0.0, 0.25, 0.5, 0.75, 1.0]

    def size(self):
        return 24

    def get_name(self, i):
        if not 0 <= i < self.size():
            raise RuntimeError("pt_hps_k parameter accessor:.get_name(i) Out of range.")
        return self.NAMES[i]

    def to_vector(self):
        nb = len(self.snow_s)
        if not 2 <= nb <= MAX_BINS or len(self.snow_intervals) != nb:
            raise RuntimeError(f"hbv_physical_snow: number of snow bins must be in [2, {MAX_BINS}]")
        x, f = self.snow_intervals, self.snow_s  # normalize_snow_distribution (hbv_physical_snow.h:71-74)
        area = 0.0
        for k in range(nb - 1):
            area += 0.5 * (f[k] + f[k + 1]) * (x[k + 1] - x[k])
        s = [v / area for v in f] + [0.0] * (MAX_BINS - nb)
        i = list(self.snow_intervals) + [0.0] * (MAX_BINS - nb)
        return list(self._v) + [float(nb)] + s + i


_B = range(MAX_BINS)


class PTHPSKState(_FlatState):
    """pt_hps_k::state (pt_hps_k.h:163-185): hps = hbv_physical_snow::state (swe, sca, surface_heat and the
    per-bin sp, sw, albedo, iso_pot_energy), kirchner.q."""
    NAMES = (("hps.swe", "hps.sca", "hps.surface_heat", "hps.n_bins") + tuple(f"hps.sp{i}" for i in _B) +
             tuple(f"hps.sw{i}" for i in _B) + tuple(f"hps.albedo{i}" for i in _B) +
             tuple(f"hps.iso_pot_energy{i}" for i in _B) + ("kirchner.q",))
    DEFAULTS = (0.0, 0.0, 30000.0, 0.0) + (0.0,) * (4 * MAX_BINS) + (0.1,)


class PTHPSKStateVector(_Vector):
    pass


PTHPSKParameterMap = dict
_SERIES = ("avg_discharge", "charge_m3s", "hps_sca", "hps_swe", "hps_outflow", "glacier_melt", "ae_output",
           "pe_output")
_STATE_SERIES = (("kirchner_discharge", "hps_sca", "hps_swe", "hps_surface_heat") + tuple(f"sp{i}" for i in _B) +
                 tuple(f"sw{i}" for i in _B) + tuple(f"albedo{i}" for i in _B) +
                 tuple(f"iso_pot_energy{i}" for i in _B))

PTHPSKStateWithId, PTHPSKStateWithIdVector, deserialize_from_bytes = make_state_with_id_types(
    "PTHPSK", PTHPSKState, PTHPSKStateVector, 5)


class _PTHPSKBase(_ModelMixin):
    _state_with_id_vector_t = PTHPSKStateWithIdVector
    _parameter_t = PTHPSKParameter
    _state_t = PTHPSKState
    _state_vector_t = PTHPSKStateVector
    _SERIES = _SERIES
    _STATE_SERIES = _STATE_SERIES

    def _push_parameters(self):
        self._set_region_parameter(self._region_parameter.to_vector())
        for cid, p in self._catchment_parameters.items():
            self._update_catchment_parameter(cid, p.to_vector())

    @property
    def hbv_physical_snow_state(self):  # hbv_physical_snow_cell_state_statistics (expose_statistics.h:335-360)
        return _Statistics(self, {"swe": (SERIES_STATE + 2, True), "sca": (SERIES_STATE + 1, True),
                                  "surface_heat": (SERIES_STATE + 3, True)})

    @property
    def hbv_physical_snow_response(self):
        return _Statistics(self, {"outflow": (4, False), "sca": (2, True), "swe": (3, True),
                                  "glacier_melt": (5, False)})

    @property
    def kirchner_state(self):
        return _Statistics(self, {"discharge": (SERIES_STATE + 0, False)})

    @property
    def priestley_taylor_response(self):
        return _Statistics(self, {"output": (7, True)})

    @property
    def actual_evaptranspiration_response(self):
        return _Statistics(self, {"output": (6, True), "pot_ratio": ("pot_ratio", True)})


def _ctor(self, full, args, devices=None, shard_flags=0):
    base = _api._PTHPSKRegionModel
    if len(args) == 1 and isinstance(args[0], base):
        other = args[0]
        base.__init__(self, other, full)
        self._region_parameter = PTHPSKParameter(other._region_parameter)
        self._catchment_parameters = {k: PTHPSKParameter(v) for k, v in other._catchment_parameters.items()}
        self._ip, self._env = other._ip, other._env
        return
    geo, region_param = args[0], args[1]
    cps = args[2] if len(args) > 2 else {}
    base.__init__(self, list(geo), region_param.to_vector(), {int(k): v.to_vector() for k, v in cps.items()}, full,
                  [int(d) for d in (devices or [])], int(shard_flags))
    self._init_python(region_param, cps)


class PTHPSKModel(_PTHPSKBase, _api._PTHPSKRegionModel):
    """region_model<pt_hps_k cell_complete_response_t> (pt_hps_k.cpp models())."""

    def __init__(self, *args, devices=None, shard_flags=0):
        _ctor(self, True, args, devices, shard_flags)


class PTHPSKOptModel(_PTHPSKBase, _api._PTHPSKRegionModel):
    """region_model<pt_hps_k cell_discharge_response_t> (pt_hps_k.cpp models())."""

    def __init__(self, *args, devices=None, shard_flags=0):
        _ctor(self, False, args, devices, shard_flags)


def create_opt_model_clone(src_model):
    return PTHPSKOptModel(src_model)


def create_full_model_clone(src_model):
    return PTHPSKModel(src_model)


from .._calibration import make_optimizer_type  # noqa: E402

PTHPSKOptimizer = make_optimizer_type("PTHPSKOptimizer", _api._PTHPSKOptimizer)
for _m in (PTHPSKModel, PTHPSKOptModel):
    _m.optimizer_t = PTHPSKOptimizer
    _m.parameter_t = _PTHPSKBase._parameter_t
    _m.state_t = _PTHPSKBase._state_t
del _m
