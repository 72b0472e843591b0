"""shyft_amd.api.pt_gs_k -- the reference's `shyft.api.pt_gs_k` (api/boostpython/pt_gs_k.cpp:34-174,
shyft/api/pt_gs_k/__init__.py:5-63) over the MI355X engine."""
from __future__ import annotations

from .. import (_api, _FlatParameter, _FlatState, _ModelMixin, _Statistics, _Vector, SERIES_STATE,
                make_state_with_id_types)

# get/set order and names of pt_gs_k::parameter (core/pt_gs_k.h:77-112, get_name :155-190), defaults of the
# member structs (kirchner.h:120-125, gamma_snow.h:46-97, priestley_taylor.h, routing.h:76, mstack_param.h)
_NAMES = ("kirchner.c1", "kirchner.c2", "kirchner.c3", "ae.ae_scale_factor", "gs.tx", "gs.wind_scale", "gs.max_water",
          "gs.wind_const", "gs.fast_albedo_decay_rate", "gs.slow_albedo_decay_rate", "gs.surface_magnitude",
          "gs.max_albedo", "gs.min_albedo", "gs.snowfall_reset_depth", "gs.snow_cv", "gs.glacier_albedo",
          "p_corr.scale_factor", "gs.snow_cv_forest_factor", "gs.snow_cv_altitude_factor", "pt.albedo", "pt.alpha",
          "gs.initial_bare_ground_fraction", "gs.winter_end_day_of_year", "gs.calculate_iso_pot_energy", "gm.dtf",
          "routing.velocity", "routing.alpha", "routing.beta", "gs.n_winter_days", "gm.direct_response",
          "msp.reservoir_direct_response_fraction")
_DEFAULTS = (-2.439, 0.966, -0.10, 1.5, -0.5, 2.0, 0.1, 1.0, 5.0, 5.0, 30.0, 0.9, 0.6, 5.0, 0.4, 0.4, 1.0, 0.0, 0.0,
             0.2, 1.26, 0.04, 100.0, 0.0, 6.0, 1.0, 7.0, 0.0, 221.0, 0.0, 1.0)


class PTGSKParameter(_FlatParameter):
    NAMES = _NAMES
    DEFAULTS = _DEFAULTS
    ERROR = "PTGSK Parameter Accessor: .set size missmatch"

    def __getattr__(self, name):
        g = super().__getattr__(name)
        if name == "gs":
            # gamma_snow::parameter::effective_snow_cv (gamma_snow.h:87-89)
            object.__setattr__(g, "effective_snow_cv", lambda forest_fraction, altitude:
                               g.snow_cv + forest_fraction * g.snow_cv_forest_factor + altitude * g.snow_cv_altitude_factor)
        return g


# state: gamma_snow::state (gamma_snow.h:101-116) + kirchner::state (kirchner.h:128-131)
class PTGSKState(_FlatState):
    NAMES = ("gs.albedo", "gs.lwc", "gs.surface_heat", "gs.alpha", "gs.sdc_melt_mean", "gs.acc_melt",
             "gs.iso_pot_energy", "gs.temp_swe", "kirchner.q")
    DEFAULTS = (0.4, 0.1, 30000.0, 1.26, 0.0, 0.0, 0.0, 0.0, 0.1)


class PTGSKStateVector(_Vector):
    pass


PTGSKParameterMap = dict

_SERIES = ("avg_discharge", "charge_m3s", "snow_sca", "snow_swe", "snow_outflow", "glacier_melt", "ae_output",
           "pe_output")
_STATE_SERIES = ("kirchner_discharge", "gs_albedo", "gs_lwc", "gs_surface_heat", "gs_alpha", "gs_sdc_melt_mean",
                 "gs_acc_melt", "gs_iso_pot_energy", "gs_temp_swe")


# cell-identified state (api_state.h:62-75) and its serialisation (api/boostpython/api_state.cpp)
PTGSKStateWithId, PTGSKStateWithIdVector, deserialize_from_bytes = make_state_with_id_types(
    "PTGSK", PTGSKState, PTGSKStateVector, 1)


class _PTGSKBase(_ModelMixin):
    _state_with_id_vector_t = PTGSKStateWithIdVector
    _parameter_t = PTGSKParameter
    _state_t = PTGSKState
    _state_vector_t = PTGSKStateVector
    _SERIES = _SERIES
    _STATE_SERIES = _STATE_SERIES

    # decorators of shyft/api/pt_gs_k/__init__.py:5-63 (expose_statistics.h)
    @property
    def gamma_snow_state(self):  # gamma_snow_cell_state_statistics (api.h:470-604): averages of sc.gs_*
        return _Statistics(self, {n: (SERIES_STATE + k, True) for k, n in enumerate(
            ("albedo", "lwc", "surface_heat", "alpha", "sdc_melt_mean", "acc_melt", "iso_pot_energy", "temp_swe"), 1)})

    @property
    def gamma_snow_response(self):  # gamma_snow_cell_response_statistics (api.h:605-676)
        return _Statistics(self, {"sca": (2, True), "swe": (3, True), "outflow": (4, False), "glacier_melt": (5, False)})

    @property
    def kirchner_state(self):  # kirchner_cell_state_statistics (api.h:402-422)
        return _Statistics(self, {"discharge": (SERIES_STATE + 0, False)})

    @property
    def priestley_taylor_response(self):  # priestley_taylor_cell_response_statistics (api.h:1449-1470)
        return _Statistics(self, {"output": (7, True)})

    @property
    def actual_evaptranspiration_response(self):  # actual_evapotranspiration_cell_response_statistics (api.h:1499-1567)
        return _Statistics(self, {"output": (6, True), "pot_ratio": ("pot_ratio", True)})


def _ctor(self, base, full, args, devices=None, shard_flags=0):
    if len(args) == 1 and isinstance(args[0], (_api._PTGSKRegionModel,)):
        other = args[0]
        base.__init__(self, other, full)
        self._region_parameter = PTGSKParameter(other._region_parameter)
        self._catchment_parameters = {k: PTGSKParameter(v) for k, v in other._catchment_parameters.items()}
        self._ip, self._env = other._ip, other._env  # the reference shares region_env (region_model.h:446-448)
        return
    geo, region_param = args[0], args[1]
    cps = args[2] if len(args) > 2 else {}
    base.__init__(self, list(geo), region_param.to_vector(), {int(k): v.to_vector() for k, v in cps.items()}, full,
                  [int(d) for d in (devices or [])], int(shard_flags))
    self._init_python(region_param, cps)


class PTGSKModel(_PTGSKBase, _api._PTGSKRegionModel):
    """region_model<pt_gs_k cell_complete_response_t> (pt_gs_k.cpp:146, all_response_collector)."""

    def __init__(self, *args, devices=None, shard_flags=0):
        _ctor(self, _api._PTGSKRegionModel, True, args, devices, shard_flags)


class PTGSKOptModel(_PTGSKBase, _api._PTGSKRegionModel):
    """region_model<pt_gs_k cell_discharge_response_t> (pt_gs_k.cpp:147, discharge_collector)."""

    def __init__(self, *args, devices=None, shard_flags=0):
        _ctor(self, _api._PTGSKRegionModel, False, args, devices, shard_flags)


def create_opt_model_clone(src_model, with_catchment_params=False):
    """expose.h:447-458: an opt (discharge-collector) model with a deep copy of src's cells, state and env."""
    m = PTGSKOptModel(src_model)
    if not with_catchment_params:
        for cid in list(m._catchment_parameters):
            m.remove_catchment_parameter(cid)
    return m


def create_full_model_clone(src_model, with_catchment_params=False):
    m = PTGSKModel(src_model)
    if not with_catchment_params:
        for cid in list(m._catchment_parameters):
            m.remove_catchment_parameter(cid)
    return m


# the model types know their optimizer, parameter and state types (expose.h:147-170, model_calibrator)
from .._calibration import make_optimizer_type  # noqa: E402

PTGSKOptimizer = make_optimizer_type("PTGSKOptimizer", _api._PTGSKOptimizer)
for _m in (PTGSKModel, PTGSKOptModel):
    _m.optimizer_t = PTGSKOptimizer
    _m.parameter_t = _PTGSKBase._parameter_t
    _m.state_t = _PTGSKBase._state_t
del _m
