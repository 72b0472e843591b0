"""shyft_amd.api.pt_hs_k -- the reference's `shyft.api.pt_hs_k` (api/boostpython/pt_hs_k.cpp,
shyft/api/pt_hs_k/__init__.py) over the MI355X engine."""
from __future__ import annotations

from .. import (_api, _FlatParameter, _FlatState, _ModelMixin, _Statistics, _Vector, SERIES_STATE,
                make_state_with_id_types)

# get/set order and names (core/pt_hs_k.h:66-143); defaults of the member structs (kirchner.h:120-125,
# hbv_snow.h:49-53, priestley_taylor.h, glacier_melt.h, routing.h:76, mstack_param.h)
_NAMES = ("kirchner.c1", "kirchner.c2", "kirchner.c3", "ae.ae_scale_factor", "hs.lw", "hs.tx", "hs.cx", "hs.ts",
          "hs.cfr", "gm.dtf", "p_corr.scale_factor", "pt.albedo", "pt.alpha", "routing.velocity", "routing.alpha",
          "routing.beta", "gm.direct_response", "msp.reservoir_direct_response_fraction")
_DEFAULTS = (-2.439, 0.966, -0.10, 1.5, 0.1, 0.0, 1.0, 0.0, 0.5, 6.0, 1.0, 0.2, 1.26, 1.0, 7.0, 0.0, 0.0, 1.0)
MAX_BINS = 8


class PTHSKParameter(_FlatParameter):
    NAMES = _NAMES
    DEFAULTS = _DEFAULTS
    ERROR = "pt_ss_k parameter accessor: .set size missmatch"  # the reference's text (pt_hs_k.h:68)

    def __init__(self, *a):
        super().__init__(*a)
        # hbv_snow::parameter distribution (hbv_snow.h:21-72): s (normalised bin weights) and intervals
        src = a[0] if a and isinstance(a[0], PTHSKParameter) else None
        self.snow_s = list(src.snow_s) if src else [1.0] * 5
        self.snow_intervals = list(src.snow_intervals) if src else [0.0, 0.25, 0.5, 0.75, 1.0]

    def to_vector(self):
        nb = len(self.snow_s)
        if not 2 <= nb <= MAX_BINS or len(self.snow_intervals) != nb:
            raise RuntimeError(f"hbv_snow: number of snow bins must be in [2, {MAX_BINS}]")
        # normalize_snow_distribution (hbv_snow.h:63-66): s /= integrate(s, intervals) over the whole range
        x, f = self.snow_intervals, self.snow_s
        area = 0.0
        for k in range(nb - 1):
            area += 0.5 * (f[k] + f[k + 1]) * (x[k + 1] - x[k])
        s = [v / area for v in f] + [0.0] * (MAX_BINS - nb)
        i = list(self.snow_intervals) + [0.0] * (MAX_BINS - nb)
        return list(self._v) + [float(nb)] + s + i


class PTHSKState(_FlatState):
    """pt_hs_k::state (pt_hs_k.h:148-172): snow = hbv_snow::state (swe, sca, sp/sw bins), kirchner.q."""
    NAMES = (("snow.swe", "snow.sca", "snow.n_bins") + tuple(f"snow.sp{i}" for i in range(MAX_BINS)) +
             tuple(f"snow.sw{i}" for i in range(MAX_BINS)) + ("kirchner.q",))
    DEFAULTS = (0.0, 0.0, 0.0) + (0.0,) * (2 * MAX_BINS) + (0.1,)


class PTHSKStateVector(_Vector):
    pass


PTHSKParameterMap = dict
_SERIES = ("avg_discharge", "charge_m3s", "snow_sca", "snow_swe", "snow_outflow", "glacier_melt", "ae_output",
           "pe_output")
_STATE_SERIES = (("kirchner_discharge", "snow_sca", "snow_swe") + tuple(f"snow_sp{i}" for i in range(MAX_BINS)) +
                 tuple(f"snow_sw{i}" for i in range(MAX_BINS)))


# cell-identified state (api_state.h:62-75) and its serialisation (api/boostpython/api_state.cpp)
PTHSKStateWithId, PTHSKStateWithIdVector, deserialize_from_bytes = make_state_with_id_types(
    "PTHSK", PTHSKState, PTHSKStateVector, 4)


class _PTHSKBase(_ModelMixin):
    _state_with_id_vector_t = PTHSKStateWithIdVector
    _parameter_t = PTHSKParameter
    _state_t = PTHSKState
    _state_vector_t = PTHSKStateVector
    _SERIES = _SERIES
    _STATE_SERIES = _STATE_SERIES

    def _push_parameters(self):
        self._set_region_parameter(self._region_parameter.to_vector())
        for cid, p in self._catchment_parameters.items():
            self._update_catchment_parameter(cid, p.to_vector())

    @property
    def hbv_snow_state(self):  # hbv_snow_cell_state_statistics (api.h:1050-1162): averages of sc.snow_swe/sca
        return _Statistics(self, {"swe": (SERIES_STATE + 2, True), "sca": (SERIES_STATE + 1, True)})

    @property
    def hbv_snow_response(self):  # hbv_snow_cell_response_statistics (api.h:1163-1206)
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
    base = _api._PTHSKRegionModel
    if len(args) == 1 and isinstance(args[0], base):
        other = args[0]
        base.__init__(self, other, full)
        self._region_parameter = PTHSKParameter(other._region_parameter)
        self._catchment_parameters = {k: PTHSKParameter(v) for k, v in other._catchment_parameters.items()}
        self._ip, self._env = other._ip, other._env  # the reference shares region_env (region_model.h:446-448)
        return
    geo, region_param = args[0], args[1]
    cps = args[2] if len(args) > 2 else {}
    base.__init__(self, list(geo), region_param.to_vector(), {int(k): v.to_vector() for k, v in cps.items()}, full,
                  [int(d) for d in (devices or [])], int(shard_flags))
    self._init_python(region_param, cps)


class PTHSKModel(_PTHSKBase, _api._PTHSKRegionModel):
    """region_model<pt_hs_k cell_complete_response_t> (pt_hs_k.cpp models())."""

    def __init__(self, *args, devices=None, shard_flags=0):
        _ctor(self, True, args, devices, shard_flags)


class PTHSKOptModel(_PTHSKBase, _api._PTHSKRegionModel):
    """region_model<pt_hs_k cell_discharge_response_t> (pt_hs_k.cpp models())."""

    def __init__(self, *args, devices=None, shard_flags=0):
        _ctor(self, False, args, devices, shard_flags)


def create_opt_model_clone(src_model):
    return PTHSKOptModel(src_model)


def create_full_model_clone(src_model):
    return PTHSKModel(src_model)


from .._calibration import make_optimizer_type  # noqa: E402

PTHSKOptimizer = make_optimizer_type("PTHSKOptimizer", _api._PTHSKOptimizer)
for _m in (PTHSKModel, PTHSKOptModel):
    _m.optimizer_t = PTHSKOptimizer
    _m.parameter_t = _PTHSKBase._parameter_t
    _m.state_t = _PTHSKBase._state_t
del _m
