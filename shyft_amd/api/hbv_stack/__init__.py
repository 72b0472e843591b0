"""shyft_amd.api.hbv_stack -- the reference's `shyft.api.hbv_stack` (api/boostpython/hbv_stack.cpp,
shyft/api/hbv_stack/__init__.py) over the MI355X engine."""
from __future__ import annotations

from .. import (_api, _FlatParameter, _FlatState, _ModelMixin, _Statistics, _Vector, SERIES_STATE,
                make_state_with_id_types)

# get/set order and names (core/hbv_stack.h:82-170), defaults (hbv_soil.h:19-24, hbv_actual_evapotranspiration.h,
# hbv_tank.h:19-31, hbv_snow.h:49-53, routing.h:76)
_NAMES = ("soil.fc", "soil.beta", "ae.lp", "tank.uz1", "tank.kuz2", "tank.kuz1", "tank.perc", "tank.klz", "hs.lw",
          "hs.tx", "hs.cx", "hs.ts", "hs.cfr", "p_corr.scale_factor", "pt.albedo", "pt.alpha", "gm.dtf",
          "routing.velocity", "routing.alpha", "routing.beta", "gm.direct_response",
          "msp.reservoir_direct_response_fraction")
_DEFAULTS = (300.0, 2.0, 150.0, 25.0, 0.5, 0.3, 0.8, 0.02, 0.1, 0.0, 1.0, 0.0, 0.5, 1.0, 0.2, 1.26, 6.0, 1.0, 7.0,
             0.0, 0.0, 1.0)
MAX_BINS = 8


class HbvParameter(_FlatParameter):
    NAMES = _NAMES
    DEFAULTS = _DEFAULTS
    ERROR = "HBV_Stack Parameter Accessor: .set size missmatch"

    def __init__(self, *a):
        super().__init__(*a)
        # hbv_snow::parameter distribution (hbv_snow.h:21-72): s (normalised bin weights) and intervals
        src = a[0] if a and isinstance(a[0], HbvParameter) else None
        self.snow_s = list(src.snow_s) if src else [1.0] * 5
        self.snow_intervals = list(src.snow_intervals) if src else [0.0, 0.25, 0.5, 0.75, 1.0]

    def to_vector(self):
        nb = len(self.snow_s)
        if not 2 <= nb <= MAX_BINS or len(self.snow_intervals) != nb:
            raise RuntimeError(f"hbv_snow: number of snow bins must be in [2, {MAX_BINS}]")
        # normalize_snow_distribution (hbv_snow.h:63-66): s /= integrate(s, intervals) over the whole range,
        # the trapezoid sum of hbv_snow_common.h:14-40 with a = intervals[0], b = intervals[-1]
        x, f = self.snow_intervals, self.snow_s
        area = 0.0
        for k in range(nb - 1):
            area += 0.5 * (f[k] + f[k + 1]) * (x[k + 1] - x[k])
        s = [v / area for v in f] + [0.0] * (MAX_BINS - nb)
        i = list(self.snow_intervals) + [0.0] * (MAX_BINS - nb)
        return list(self._v) + [float(nb)] + s + i


class _HbvState(_FlatState):
    NAMES = ("snow.swe", "snow.sca", "soil.sm", "tank.uz", "tank.lz", "snow.n_bins") + \
        tuple(f"snow.sp{i}" for i in range(MAX_BINS)) + tuple(f"snow.sw{i}" for i in range(MAX_BINS))
    DEFAULTS = (0.0, 0.0, 0.0, 20.0, 10.0, 0.0) + (0.0,) * (2 * MAX_BINS)


class HbvState(_HbvState):
    """hbv_stack::state (hbv_stack.h:181-201): snow (swe, sca, sp/sw bins), soil.sm, tank.uz/lz."""


class HbvStateVector(_Vector):
    pass


HbvParameterMap = dict
_SERIES = ("avg_discharge", "charge_m3s", "snow_sca", "snow_swe", "snow_outflow", "glacier_melt", "ae_output",
           "pe_output", "soil_outflow")
_STATE_SERIES = ("snow_swe", "snow_sca", "soil_moisture", "tank_uz", "tank_lz", "snow_n_bins") + \
    tuple(f"sp{i}" for i in range(MAX_BINS)) + tuple(f"sw{i}" for i in range(MAX_BINS))


# cell-identified state (api_state.h:62-75) and its serialisation (api/boostpython/api_state.cpp)
HbvStateWithId, HbvStateWithIdVector, deserialize_from_bytes = make_state_with_id_types(
    "Hbv", HbvState, HbvStateVector, 2)


class _HbvBase(_ModelMixin):
    _state_with_id_vector_t = HbvStateWithIdVector
    _parameter_t = HbvParameter
    _state_t = HbvState
    _state_vector_t = HbvStateVector
    _SERIES = _SERIES
    _STATE_SERIES = _STATE_SERIES

    def _push_parameters(self):
        self._set_region_parameter(self._region_parameter.to_vector())
        for cid, p in self._catchment_parameters.items():
            self._update_catchment_parameter(cid, p.to_vector())

    @property
    def hbv_snow_state(self):  # hbv_snow_cell_state_statistics (api.h:1050-1162): averages of sc.snow_swe/sca
        return _Statistics(self, {"swe": (SERIES_STATE + 0, True), "sca": (SERIES_STATE + 1, True)})

    @property
    def hbv_snow_response(self):  # hbv_snow_cell_response_statistics (api.h:1163-1206)
        return _Statistics(self, {"outflow": (4, False), "sca": (2, True), "swe": (3, True),
                                  "glacier_melt": (5, False)})

    @property
    def soil_state(self):  # hbv_soil_cell_state_statistics (api.h:424-444): sums of sc.soil_moisture
        return _Statistics(self, {"discharge": (SERIES_STATE + 2, False)})

    @property
    def tank_state(self):  # hbv_tank_cell_state_statistics (api.h:446-468): sums of sc.tank_uz
        return _Statistics(self, {"discharge": (SERIES_STATE + 3, False), "uz": (SERIES_STATE + 3, False),
                                  "lz": (SERIES_STATE + 4, False)})

    hbv_tank_state = tank_state

    @property
    def priestley_taylor_response(self):
        return _Statistics(self, {"output": (7, True)})

    @property
    def hbv_actual_evaptranspiration_response(self):
        return _Statistics(self, {"output": (6, True)})

    @property
    def soil_response(self):  # hbv_soil_cell_response_statistics (api.h:1472-1497)
        return _Statistics(self, {"output": (8, True)})


def _ctor(self, full, args, devices=None, shard_flags=0):
    base = _api._HbvRegionModel
    if len(args) == 1 and isinstance(args[0], base):
        other = args[0]
        base.__init__(self, other, full)
        self._region_parameter = HbvParameter(other._region_parameter)
        self._catchment_parameters = {k: HbvParameter(v) for k, v in other._catchment_parameters.items()}
        self._ip, self._env = other._ip, other._env  # the reference shares region_env (region_model.h:446-448)
        return
    geo, region_param = args[0], args[1]
    cps = args[2] if len(args) > 2 else {}
    base.__init__(self, list(geo), region_param.to_vector(), {int(k): v.to_vector() for k, v in cps.items()}, full,
                  [int(d) for d in (devices or [])], int(shard_flags))
    self._init_python(region_param, cps)


class HbvModel(_HbvBase, _api._HbvRegionModel):
    """region_model<hbv_stack cell_complete_response_t> (hbv_stack.cpp:140)."""

    def __init__(self, *args, devices=None, shard_flags=0):
        _ctor(self, True, args, devices, shard_flags)


class HbvOptModel(_HbvBase, _api._HbvRegionModel):
    """region_model<hbv_stack cell_discharge_response_t> (hbv_stack.cpp:141)."""

    def __init__(self, *args, devices=None, shard_flags=0):
        _ctor(self, False, args, devices, shard_flags)


def create_opt_model_clone(src_model):
    return HbvOptModel(src_model)


def create_full_model_clone(src_model):
    return HbvModel(src_model)


# the model types know their optimizer, parameter and state types (expose.h:147-170, model_calibrator)
from .._calibration import make_optimizer_type  # noqa: E402

HbvOptimizer = make_optimizer_type("HbvOptimizer", _api._HbvOptimizer)
for _m in (HbvModel, HbvOptModel):
    _m.optimizer_t = HbvOptimizer
    _m.parameter_t = _HbvBase._parameter_t
    _m.state_t = _HbvBase._state_t
del _m
