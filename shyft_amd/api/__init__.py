"""shyft_amd.api -- the reference's `shyft.api` names over the MI355X engine.

Mirrors the parts of `shyft.api` (shyft/api/__init__.py, api/boostpython/api_*.cpp,
expose.h, expose_statistics.h) that the region-model hot path uses: geo cells,
time axes and point series, region environment and interpolation parameters,
statistics, river network. The heavy objects (region models, their
interpolation, run_cells, statistics, routing) are the C++ host classes of
shyft_amd/csrc/host bound by pybind11 in `_api`; those drive the HIP engine
through the C ABI of include/shyft_hip.h. There is no CPU fallback: importing
this package requires the built extension and libshyft_hip.so.
"""
from __future__ import annotations

import numpy as np

from .._native import lib as _lib

_lib()  # one HIP runtime per process: map it (and libshyft_hip.so) before the extension module

from ._api import (  # noqa: F401  (re-exported names)
    GeoPoint, LandTypeFractions, RoutingInfo, GeoCellData, TimeAxisFixedDeltaT, point_interpretation_policy,
    POINT_INSTANT_VALUE, POINT_AVERAGE_VALUE, IDWParameter, IDWTemperatureParameter, IDWPrecipitationParameter,
    InterpolationParameter, UHGParameter, River, RiverNetwork, make_uhg_from_gamma, average_values, FlowAdjustResult,
    find_min_single_variable, BTKParameter,
)
from . import _api

TimeAxis = TimeAxisFixedDeltaT
ts_point_fx = point_interpretation_policy


# ---- time (core/utctime_utilities.h; shyft's `time` is seconds) -----------------------------------------------------
def deltahours(n):
    return 3600 * n


def deltaminutes(n):
    return 60 * n


class Calendar:
    """UTC calendar (utctime_utilities.cpp:230-277); only the UTC zone is on the hot path."""

    YEAR, MONTH, DAY, HOUR = 365 * 86400, 30 * 86400, 86400, 3600

    def __init__(self, tz: str | int = 0):
        if tz not in (0, "UTC", "Etc/UTC"):
            raise RuntimeError("Calendar: only UTC is supported by the MI355X engine")

    def time(self, Y, M=1, D=1, h=0, m=0, s=0):
        return int(_api.utc_time(Y, M, D, h, m, s))

    def day_of_year(self, t):
        import datetime
        return datetime.datetime.fromtimestamp(t, datetime.timezone.utc).timetuple().tm_yday


class UtcPeriod:
    def __init__(self, start, end):
        self.start, self.end = start, end

    def timespan(self):
        return self.end - self.start

    def contains(self, t):
        return self.start <= t < self.end

    def __repr__(self):
        return f"UtcPeriod({self.start}, {self.end})"


# ---- vectors (boost.python vector_indexing_suite stand-ins) -----------------------------------------------------------
class _Vector(list):
    def push_back(self, x):
        self.append(x)

    def size(self):
        return len(self)

    def to_numpy(self):
        return np.asarray(self)


class IntVector(_Vector):
    @staticmethod
    def from_numpy(a):
        return IntVector(int(x) for x in np.asarray(a))


class DoubleVector(_Vector):
    @staticmethod
    def from_numpy(a):
        return DoubleVector(float(x) for x in np.asarray(a))


class UtcTimeVector(_Vector):
    pass


class GeoCellDataVector(_Vector):
    pass


class _Scope(int):
    """an enum value (distinct from a time-step index when passed positionally)"""


class stat_scope:  # core/cell_model.h:183-186
    cell = cell_ix = _Scope(0)
    catchment = catchment_ix = _Scope(1)


# ---- point time series (core/time_series.h:323-414) -----------------------------------------------------------------
class TimeSeries:
    """A point series on a fixed_dt or point time axis (the apoint_ts results of the statistics)."""

    def __init__(self, ta=None, values=None, point_fx=POINT_AVERAGE_VALUE, _impl=None, fill_value=None):
        if _impl is not None:
            self._ts = _impl
            return
        if isinstance(ta, TimeSeries):  # copy constructor
            import copy
            self._ts = copy.deepcopy(ta._ts)
            return
        if values is None and fill_value is not None:
            values = float(fill_value)
        if isinstance(values, (int, float)):
            values = [float(values)] * ta.size()
        self._ts = _api._PointTs(ta, [float(v) for v in np.asarray(values, dtype=np.float64)], point_fx)
        self._ta = ta

    def value(self, i):
        return self._ts.value(i)

    def set(self, i, v):
        self._ts.set(i, v)

    def size(self):
        return self._ts.size()

    def __len__(self):
        return self._ts.size()

    def __call__(self, t):
        return self._ts(t)

    def time(self, i):
        return self._ts.time(i)

    def point_interpretation(self):
        return self._ts.point_interpretation()

    def total_period(self):
        return UtcPeriod(*self._ts.total_period())

    @property
    def values(self):
        return DoubleVector(self._ts._values.tolist())

    @property
    def v(self):
        return self.values

    def __deepcopy__(self, memo):
        import copy
        return TimeSeries(_impl=copy.deepcopy(self._ts, memo))

    def average(self, ta):
        """true average onto a fixed_dt axis (average_accessor, time_series.h:2033-2072)."""
        return TimeSeries(ta, self._ts.average(ta), POINT_AVERAGE_VALUE)


class TsFactory:
    """api.TsFactory (api/api.h:1630-1700)."""

    def create_time_point_ts(self, period, times, values, interpretation=POINT_INSTANT_VALUE):
        return TimeSeries(_impl=_api._PointTs([float(t) for t in times], float(period.end),
                                              [float(v) for v in values], interpretation))

    def create_point_ts(self, n, tstart, dt, values, interpretation=POINT_INSTANT_VALUE):
        return TimeSeries(TimeAxisFixedDeltaT(tstart, dt, n), values, interpretation)


# ---- geo-located sources and the region environment (api/api.h:78-168) -----------------------------------------------
class _GeoPointSource:
    def __init__(self, mid_point=None, ts=None):
        self._mid_point = mid_point if mid_point is not None else GeoPoint()
        self.ts = ts
        self.uid = ""

    def mid_point(self):
        return self._mid_point

    def _impl(self):
        g = _api._GeoPointTs(self._mid_point, self.ts._ts)
        g.uid = self.uid or ""
        return g


class TemperatureSource(_GeoPointSource):
    pass


class PrecipitationSource(_GeoPointSource):
    pass


class RadiationSource(_GeoPointSource):
    pass


class WindSpeedSource(_GeoPointSource):
    pass


class RelHumSource(_GeoPointSource):
    pass


class _SourceVector(_Vector):
    def values_at_time(self, t):
        return DoubleVector(s.ts(t) for s in self)


class TemperatureSourceVector(_SourceVector):
    pass


class PrecipitationSourceVector(_SourceVector):
    pass


class RadiationSourceVector(_SourceVector):
    pass


class WindSpeedSourceVector(_SourceVector):
    pass


class RelHumSourceVector(_SourceVector):
    pass


class GeoPointVector(_Vector):
    pass


def bayesian_kriging_temperature(src, dst, time_axis, btk_parameter):
    """Bayesian temperature kriging of the sources onto the destination points over time_axis
    (api/boostpython/api_interpolation.cpp:54-71), computed on the MI355X (shyft_hip_btk).
    Returns a TemperatureSourceVector, one source per destination point."""
    values = _api._bayesian_kriging_temperature([s._impl() for s in (src or [])], list(dst or []), time_axis,
                                                btk_parameter)
    out = TemperatureSourceVector()
    for d, gp in enumerate(dst):
        out.append(TemperatureSource(gp, TimeSeries(time_axis, values[:, d], POINT_AVERAGE_VALUE)))
    return out


class ARegionEnvironment:
    def __init__(self):
        self.temperature = TemperatureSourceVector()
        self.precipitation = PrecipitationSourceVector()
        self.radiation = RadiationSourceVector()
        self.wind_speed = WindSpeedSourceVector()
        self.rel_hum = RelHumSourceVector()

    def _impl(self):
        e = _api._RegionEnvironment()
        for name in ("temperature", "precipitation", "radiation", "wind_speed", "rel_hum"):
            setattr(e, name, [s._impl() for s in (getattr(self, name) or [])])
        return e

    def copy(self):
        import copy
        return copy.deepcopy(self)


# ---- the method-stack parameter / state objects -----------------------------------------------------------------------
class _Group:
    """Attribute view of a slice of a flat parameter/state vector (pt_gs_k.h:77-112 get/set order)."""

    def __init__(self, owner, fields):
        object.__setattr__(self, "_owner", owner)
        object.__setattr__(self, "_fields", fields)

    def __getattr__(self, name):
        f = object.__getattribute__(self, "_fields")
        if name in f:
            return object.__getattribute__(self, "_owner")._v[f[name]]
        raise AttributeError(name)

    def __setattr__(self, name, value):
        f = object.__getattribute__(self, "_fields")
        if name not in f:
            raise AttributeError(name)
        object.__getattribute__(self, "_owner")._v[f[name]] = float(value)


class _FlatParameter:
    """Base of the stack parameter classes: a flat vector with the reference's named groups."""
    NAMES: tuple = ()
    DEFAULTS: tuple = ()
    ERROR = "Parameter Accessor: .set size missmatch"

    def __init__(self, *groups):
        self._v = [float(x) for x in self.DEFAULTS]
        if len(groups) == 1 and isinstance(groups[0], _FlatParameter):
            self._v = list(groups[0]._v)

    def size(self):
        return len(self.NAMES)

    def get(self, i):
        return self._v[i]

    def set(self, p):
        p = list(p)
        if len(p) != self.size():
            raise RuntimeError(self.ERROR)
        self._v[:self.size()] = [float(x) for x in p]

    def get_name(self, i):
        if not 0 <= i < self.size():
            raise RuntimeError(self.ERROR.replace(".set size missmatch", ".get_name(i) Out of range."))
        return self.NAMES[i]

    def to_vector(self):
        return list(self._v)

    def __getattr__(self, name):
        fields = {n.split(".", 1)[1]: k for k, n in enumerate(type(self).NAMES) if n.split(".", 1)[0] == name}
        if not fields:
            raise AttributeError(name)
        return _Group(self, fields)

    def __eq__(self, other):
        return isinstance(other, type(self)) and self._v == other._v

    def __deepcopy__(self, memo):
        c = type(self)()
        c._v = list(self._v)
        return c


class _FlatState:
    NAMES: tuple = ()
    DEFAULTS: tuple = ()

    def __init__(self, v=None):
        self._v = [float(x) for x in (self.DEFAULTS if v is None else v)]

    def to_vector(self):
        return list(self._v)

    def __getattr__(self, name):
        fields = {n.split(".", 1)[1]: k for k, n in enumerate(type(self).NAMES) if n.split(".", 1)[0] == name}
        if not fields:
            raise AttributeError(name)
        return _Group(self, fields)

    def __eq__(self, other):
        return isinstance(other, type(self)) and np.allclose(self._v, other._v, atol=1e-6)


# ---- cell-identified state (api/api_state.h:22-146; api/boostpython/api_state.cpp) -----------------------------------
CellStateId = _api.CellStateId


def byte_vector_to_file(path, byte_vector):
    """api.byte_vector_to_file: write a serialised state blob to a file."""
    with open(path, "wb") as f:
        f.write(bytes(byte_vector))


def byte_vector_from_file(path):
    """api.byte_vector_from_file: read a blob written by byte_vector_to_file."""
    with open(path, "rb") as f:
        return f.read()


class _StateWithId:
    """cell_state_with_id<state_t> (api_state.h:62-75): id + state."""
    _state_t = None

    def __init__(self, id=None, state=None):
        self.id = id if id is not None else CellStateId()
        self.state = state if state is not None else self._state_t()

    def __eq__(self, other):  # only id equality (api_state.h:68-70)
        return isinstance(other, _StateWithId) and self.id == other.id


class _StateWithIdVector(_Vector):
    """vector<cell_state_with_id<state_t>> with the reference's serialisation helpers. The byte layout is this
    engine's own (host/state_io.hpp), tagged with the method stack; it is not a boost archive."""
    _item_t = None
    _state_vector_t = None
    _stack = 0

    def _pairs(self):
        return [(x.id, x.state.to_vector()) for x in self]

    @classmethod
    def _from_pairs(cls, pairs):
        return cls(cls._item_t(i, cls._item_t._state_t(v)) for i, v in pairs)

    def serialize_to_bytes(self):
        return _api._serialize_states(self._stack, len(self._item_t._state_t.NAMES), self._pairs())

    @classmethod
    def deserialize_from_bytes(cls, b):
        return cls._from_pairs(_api._deserialize_states(bytes(b), cls._stack, len(cls._item_t._state_t.NAMES)))

    def serialize_to_str(self):
        import base64
        return base64.b64encode(self.serialize_to_bytes()).decode("ascii")

    @classmethod
    def deserialize_from_str(cls, s):
        import base64
        return cls.deserialize_from_bytes(base64.b64decode(s))

    @property
    def state_vector(self):
        return self._state_vector_t(x.state for x in self)


def make_state_with_id_types(prefix, state_t, state_vector_t, stack_id):
    """<prefix>StateWithId, <prefix>StateWithIdVector and the module-level deserialize_from_bytes of a stack."""
    item = type(prefix + "StateWithId", (_StateWithId,), {"_state_t": state_t})
    vec = type(prefix + "StateWithIdVector", (_StateWithIdVector,),
               {"_item_t": item, "_state_vector_t": state_vector_t, "_stack": stack_id})
    return item, vec, vec.deserialize_from_bytes


class _StateIoHandler:
    """model.state: state_io_handler<cell_t> (api_state.h:99-146)."""

    def __init__(self, model):
        self._m = model

    def extract_state(self, cids):
        """the states of the cells (all, or those of the catchment ids `cids`) with their CellStateId"""
        return self._m._state_with_id_vector_t._from_pairs(self._m._extract_state(list(cids)))

    def apply_state(self, cell_id_state_vector, cids):
        """apply states by CellStateId (filtered by cids); returns the indexes of states that matched no cell"""
        return IntVector(self._m._apply_state(list(cell_id_state_vector._pairs()), list(cids)))


# ---- cell views (core/cell_model.h:47-160) ---------------------------------------------------------------------------
FORCING = ("temperature", "precipitation", "wind_speed", "rel_hum", "radiation")
SERIES_FORCING, SERIES_STATE = 100, 200


class _CellSeries:
    def __init__(self, model, series, cell):
        self._m, self._s, self._c = model, series, cell

    def value(self, i):
        return self._m._cell_value(self._s, self._c, i)

    def set(self, i, v):
        if self._s < SERIES_FORCING or self._s >= SERIES_STATE:
            raise RuntimeError("only cell env_ts series are writable")
        self._m._set_cell_value(self._s - SERIES_FORCING, self._c, i, float(v))

    def size(self):
        n = self._m._time_axis.size()
        return n + 1 if self._s >= SERIES_STATE else n

    def __len__(self):
        return self.size()

    @property
    def values(self):
        return DoubleVector(self._m._cell_series(self._s, self._c).tolist())

    def to_numpy(self):
        return self._m._cell_series(self._s, self._c)


class _Named:
    def __init__(self, model, cell, mapping):
        self._m, self._c, self._map = model, cell, mapping

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        if name not in self._map:
            raise AttributeError(name)
        return _CellSeries(self._m, self._map[name], self._c)


class CellView:
    """model.cells[i]: geo, env_ts, state, rc, sc and parameter of one cell (a view into the device data)."""

    def __init__(self, model, i):
        self._m, self._i = model, i

    @property
    def geo(self):
        return self._m._cell_geo(self._i)

    def mid_point(self):
        return self.geo.mid_point()

    @property
    def env_ts(self):
        return _Named(self._m, self._i, {n: SERIES_FORCING + k for k, n in enumerate(FORCING)})

    @property
    def rc(self):
        return _Named(self._m, self._i, {n: k for k, n in enumerate(self._m._SERIES)})

    @property
    def sc(self):
        return _Named(self._m, self._i, {n: SERIES_STATE + k for k, n in enumerate(self._m._STATE_SERIES)})

    @property
    def state(self):
        return self._m._state_t(self._m._get_states()[self._i])

    @property
    def parameter(self):
        p = self._m._parameter_t()
        p._v = list(self._m._cell_parameter(self._i))
        return p


class CellVector(_Vector):
    pass


# ---- statistics (api/api.h:179-1597, expose_statistics.h) --------------------------------------------------------------
class _Statistics:
    """name -> (series id, weighted): sums (weighted False) or area-weighted averages (True)."""

    def __init__(self, model, spec):
        self._m, self._spec = model, spec

    def _ts(self, sid, weighted, indexes, ix_type):
        v = self._m._stat_series(sid, list(indexes), int(ix_type), weighted)
        ta = self._m._time_axis
        if sid >= SERIES_STATE:
            ta = TimeAxisFixedDeltaT(ta.start, ta.delta_t, ta.size() + 1)
        return TimeSeries(ta, v, POINT_AVERAGE_VALUE)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        spec = self._spec
        if name.endswith("_value") and name[:-6] in spec:
            sid, w = spec[name[:-6]]
            if sid == "pot_ratio":
                return lambda indexes, i, ix_type=stat_scope.catchment: self._m._pot_ratio_value(list(indexes), int(ix_type), i)
            return lambda indexes, i, ix_type=stat_scope.catchment: self._m._stat_value(sid, list(indexes), int(ix_type), w, i)
        if name not in spec:
            raise AttributeError(name)
        sid, w = spec[name]

        def f(indexes, i=None, ix_type=stat_scope.catchment):
            if isinstance(i, _Scope):  # overload (indexes, ix_type) of the reference
                ix_type, i = i, None
            if sid == "pot_ratio":
                if i is None:
                    ta = self._m._time_axis
                    ta1 = TimeAxisFixedDeltaT(ta.start, ta.delta_t, ta.size() + 1)
                    return TimeSeries(ta1, self._m._pot_ratio_series(list(indexes), int(ix_type)), POINT_AVERAGE_VALUE)
                return DoubleVector(self._m._pot_ratio_raster(list(indexes), int(ix_type), int(i)))
            if i is None:
                return self._ts(sid, w, indexes, ix_type)
            return DoubleVector(self._m._stat_raster(sid, list(indexes), int(ix_type), int(i)))
        return f


class BasicStatistics(_Statistics):
    """basic_cell_statistics (api/api.h:179-398): discharge/charge sums, forcing averages, areas."""
    AREAS = ("total_area", "forest_area", "glacier_area", "lake_area", "reservoir_area", "unspecified_area",
             "snow_storage_area", "elevation")

    def __init__(self, model):
        super().__init__(model, {"discharge": (0, False), "charge": (1, False),
                                 "temperature": (SERIES_FORCING + 0, True), "precipitation": (SERIES_FORCING + 1, True),
                                 "wind_speed": (SERIES_FORCING + 2, True), "rel_hum": (SERIES_FORCING + 3, True),
                                 "radiation": (SERIES_FORCING + 4, True)})

    def __getattr__(self, name):
        if name in self.AREAS:
            k = self.AREAS.index(name)
            return lambda indexes, ix_type=stat_scope.catchment: self._m._area_stat(k, list(indexes), int(ix_type))
        return super().__getattr__(name)


# ---- the model base (expose.h:143-430, shyft/api/pt_gs_k/__init__.py) ------------------------------------------------
class _ModelMixin:
    """Python half of a region model: keeps the reference's parameter/state objects live and pushes them into the
    C++ host class before every run (the reference's cells hold shared_ptr parameters, region_model.h:640-700)."""

    def _init_python(self, region_param, catchment_parameters=None):
        self._region_parameter = self._parameter_t(region_param)
        self._catchment_parameters = {int(k): self._parameter_t(v) for k, v in (catchment_parameters or {}).items()}
        self._ip = None
        self._env = None

    def _push_parameters(self):
        self._set_region_parameter(self._region_parameter.to_vector())
        for cid, p in self._catchment_parameters.items():
            self._update_catchment_parameter(cid, p.to_vector())

    # parameters
    def get_region_parameter(self):
        return self._region_parameter

    def set_region_parameter(self, p):
        self._region_parameter._v = list(p._v)
        self._set_region_parameter(p.to_vector())

    def set_catchment_parameter(self, catchment_id, p):
        if int(catchment_id) not in self._catchment_parameters:
            self._catchment_parameters[int(catchment_id)] = self._parameter_t(p)
            self._set_catchment_parameter(int(catchment_id), p.to_vector())

    def get_catchment_parameter(self, catchment_id):
        return self._catchment_parameters.get(int(catchment_id), self._region_parameter)

    def remove_catchment_parameter(self, catchment_id):
        self._catchment_parameters.pop(int(catchment_id), None)
        super().remove_catchment_parameter(int(catchment_id))

    # interpolation
    def interpolate(self, interpolation_parameter, env, best_effort=True):
        self._ip, self._env = interpolation_parameter, env
        return self._interpolate(interpolation_parameter, env._impl(), best_effort)

    def run_interpolation(self, interpolation_parameter, time_axis, env, best_effort=True):
        self._ip, self._env = interpolation_parameter, env
        return self._run_interpolation(interpolation_parameter, time_axis, env._impl(), best_effort)

    @property
    def interpolation_parameter(self):
        return self._ip if self._ip is not None else self._ip_parameter

    @property
    def region_env(self):
        return self._env

    @property
    def time_axis(self):
        return self._time_axis

    def run_cells(self, use_ncore=0, start_step=0, n_steps=0):
        self._push_parameters()
        super().run_cells(use_ncore, start_step, n_steps)

    def adjust_state_to_target_flow(self, wanted_flow_m3s, cids, start_step=0, scale_range=3.0, scale_eps=1e-3,
                                    max_iter=300, n_steps=1):
        """Tune the discharge state of `cids` so the average flow over [start_step, start_step+n_steps) is
        wanted_flow_m3s (region_model.h:626-637); returns FlowAdjustResult(q_0, q_r, diagnostics)."""
        self._push_parameters()
        return super().adjust_state_to_target_flow(float(wanted_flow_m3s), list(cids), int(start_step),
                                                   float(scale_range), float(scale_eps), int(max_iter), int(n_steps))

    # states
    def set_states(self, states):
        self._set_states([s.to_vector() for s in states])

    def get_states(self, end_states=None):
        sv = self._state_vector_t(self._state_t(v) for v in self._get_states())
        if end_states is not None:
            end_states.clear()
            end_states.extend(sv)
            return end_states
        return sv

    @property
    def current_state(self):
        return self.get_states()

    @property
    def state(self):
        return _StateIoHandler(self)

    @property
    def initial_state(self):
        return self._state_vector_t(self._state_t(v) for v in self._initial_state)

    @initial_state.setter
    def initial_state(self, sv):
        self._initial_state = [s.to_vector() for s in sv]

    # cells
    def get_cells(self):
        return CellVector(CellView(self, i) for i in range(self.size()))

    @property
    def cells(self):
        return self.get_cells()

    # statistics
    @property
    def statistics(self):
        return BasicStatistics(self)

    # routing
    @property
    def river_network(self):
        return _RiverNetworkProxy(self)

    @river_network.setter
    def river_network(self, rn):
        self._river_network = rn

    def river_output_flow_m3s(self, rid):
        return TimeSeries(self._time_axis, self._river_output_flow_m3s(rid), POINT_AVERAGE_VALUE)

    def river_upstream_inflow_m3s(self, rid):
        return TimeSeries(self._time_axis, self._river_upstream_inflow_m3s(rid), POINT_AVERAGE_VALUE)

    def river_local_inflow_m3s(self, rid):
        return TimeSeries(self._time_axis, self._river_local_inflow_m3s(rid), POINT_AVERAGE_VALUE)

    # catchment aggregates (region_model.h:873-905)
    def catchment_discharges(self):
        return [TimeSeries(self._time_axis, v, POINT_AVERAGE_VALUE) for v in self._catchment_sums(0)]

    def catchment_charges(self):
        return [TimeSeries(self._time_axis, v, POINT_AVERAGE_VALUE) for v in self._catchment_sums(1)]


class _RiverNetworkProxy:
    """model.river_network: edits go to the model's C++ river network (a by-value member there)."""

    def __init__(self, model):
        self._m = model

    def __getattr__(self, name):
        rn = self._m._river_network
        attr = getattr(rn, name)
        if not callable(attr):
            return attr

        def call(*a, **k):
            rn2 = self._m._river_network
            r = getattr(rn2, name)(*a, **k)
            self._m._river_network = rn2
            return self if r is rn2 else r
        return call


# ---- calibration (model_calibration.h; expose.h:472-730) -------------------------------------------------------------
from ._calibration import (  # noqa: E402,F401
    NASH_SUTCLIFFE, KLING_GUPTA, ABS_DIFF, RMSE, DISCHARGE, SNOW_COVERED_AREA, SNOW_WATER_EQUIVALENT,
    ROUTED_DISCHARGE, CELL_CHARGE, TsTransform, TargetSpecificationPts, TargetSpecificationVector,
)
from ._api import (  # noqa: E402,F401
    nash_sutcliffe_goal_function, kling_gupta_goal_function, rmse_goal_function, abs_diff_sum_goal_function,
    abs_diff_sum_goal_function_scaled,
)
