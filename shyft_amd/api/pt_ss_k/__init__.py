"""shyft_amd.api.pt_ss_k -- the reference's `shyft.api.pt_ss_k` (api/boostpython/pt_ss_k.cpp,
shyft/api/pt_ss_k/__init__.py) over the MI355X engine."""
from __future__ import annotations

from .. import (_api, _FlatParameter, _FlatState, _ModelMixin, _Statistics, _Vector, SERIES_STATE,
                make_state_with_id_types)

# get/set order and names (core/pt_ss_k.h:78-150); defaults of the member structs (skaugen.h:89-112,
# kirchner.h:120-125, priestley_taylor.h, routing.h:76, mstack_param.h)
_NAMES = ("kirchner.c1", "kirchner.c2", "kirchner.c3", "ae.ae_scale_factor", "ss.alpha_0", "ss.d_range",
          "ss.unit_size", "ss.max_water_fraction", "ss.tx", "ss.cx", "ss.ts", "ss.cfr", "p_corr.scale_factor",
          "pt.albedo", "pt.alpha", "gm.dtf", "routing.velocity", "routing.alpha", "routing.beta", "gm.direct_response",
          "msp.reservoir_direct_response_fraction")
_DEFAULTS = (-2.439, 0.966, -0.10, 1.5, 40.77, 113.0, 0.1, 0.1, 0.16, 2.5, 0.14, 0.01, 1.0, 0.2, 1.26, 6.0, 1.0,
             7.0, 0.0, 0.0, 1.0)


class PTSSKParameter(_FlatParameter):
    NAMES = _NAMES
    DEFAULTS = _DEFAULTS
    ERROR = "pt_ss_k parameter accessor: .set size mismatch"


class PTSSKState(_FlatState):
    """pt_ss_k::state (pt_ss_k.h:154-181): snow = skaugen::state, kirchner.q."""
    NAMES = ("snow.nu", "snow.alpha", "snow.sca", "snow.swe", "snow.free_water", "snow.residual", "snow.num_units",
             "kirchner.q")
    DEFAULTS = (4.077, 40.77, 0.0, 0.0, 0.0, 0.0, 0.0, 0.1)


class PTSSKStateVector(_Vector):
    pass


PTSSKParameterMap = dict
_SERIES = ("avg_discharge", "charge_m3s", "snow_sca", "snow_total_stored_water", "snow_outflow", "glacier_melt",
           "ae_output", "pe_output")
_STATE_SERIES = ("kirchner_discharge", "snow_sca", "snow_swe", "snow_alpha", "snow_nu", "snow_lwc", "snow_residual")


# cell-identified state (api_state.h:62-75) and its serialisation (api/boostpython/api_state.cpp)
PTSSKStateWithId, PTSSKStateWithIdVector, deserialize_from_bytes = make_state_with_id_types(
    "PTSSK", PTSSKState, PTSSKStateVector, 3)


class _PTSSKBase(_ModelMixin):
    _state_with_id_vector_t = PTSSKStateWithIdVector
    _parameter_t = PTSSKParameter
    _state_t = PTSSKState
    _state_vector_t = PTSSKStateVector
    _SERIES = _SERIES
    _STATE_SERIES = _STATE_SERIES

    @property
    def skaugen_snow_state(self):  # skaugen_cell_state_statistics (api.h:888-990): averages of sc.snow_*
        return _Statistics(self, {"alpha": (SERIES_STATE + 3, True), "nu": (SERIES_STATE + 4, True),
                                  "lwc": (SERIES_STATE + 5, True), "residual": (SERIES_STATE + 6, True),
                                  "swe": (SERIES_STATE + 2, True), "sca": (SERIES_STATE + 1, True)})

    @property
    def skaugen_snow_response(self):  # skaugen_cell_response_statistics (api.h:991-1048): sums
        return _Statistics(self, {"outflow": (4, False), "total_stored_water": (3, False)})

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
    base = _api._PTSSKRegionModel
    if len(args) == 1 and isinstance(args[0], base):
        other = args[0]
        base.__init__(self, other, full)
        self._region_parameter = PTSSKParameter(other._region_parameter)
        self._catchment_parameters = {k: PTSSKParameter(v) for k, v in other._catchment_parameters.items()}
        self._ip, self._env = other._ip, other._env  # the reference shares region_env (region_model.h:446-448)
        return
    geo, region_param = args[0], args[1]
    cps = args[2] if len(args) > 2 else {}
    base.__init__(self, list(geo), region_param.to_vector(), {int(k): v.to_vector() for k, v in cps.items()}, full,
                  [int(d) for d in (devices or [])], int(shard_flags))
    self._init_python(region_param, cps)


class PTSSKModel(_PTSSKBase, _api._PTSSKRegionModel):
    """region_model<pt_ss_k cell_complete_response_t> (pt_ss_k.cpp:139)."""

    def __init__(self, *args, devices=None, shard_flags=0):
        _ctor(self, True, args, devices, shard_flags)


class PTSSKOptModel(_PTSSKBase, _api._PTSSKRegionModel):
    """region_model<pt_ss_k cell_discharge_response_t> (pt_ss_k.cpp:140)."""

    def __init__(self, *args, devices=None, shard_flags=0):
        _ctor(self, False, args, devices, shard_flags)


def create_opt_model_clone(src_model):
    return PTSSKOptModel(src_model)


def create_full_model_clone(src_model):
    return PTSSKModel(src_model)


# the model types know their optimizer, parameter and state types (expose.h:147-170, model_calibrator)
from .._calibration import make_optimizer_type  # noqa: E402

PTSSKOptimizer = make_optimizer_type("PTSSKOptimizer", _api._PTSSKOptimizer)
for _m in (PTSSKModel, PTSSKOptModel):
    _m.optimizer_t = PTSSKOptimizer
    _m.parameter_t = _PTSSKBase._parameter_t
    _m.state_t = _PTSSKBase._state_t
del _m
