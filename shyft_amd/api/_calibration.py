"""Calibration surface of `shyft.api` over the MI355X engine: TargetSpecificationPts / TargetSpecificationVector,
TsTransform, the goal-function enums and the per-stack optimizer classes (PTGSKOptimizer, HbvOptimizer,
PTSSKOptimizer) of api/boostpython/expose.h:472-730 (model_calibrator) and api_target_specification.cpp.

The search itself runs in C++ (shyft_amd/csrc/host/calibration.hpp): every goal-function evaluation is a device
run_cells, and independent parameter vectors are evaluated as one device parameter-ensemble launch."""
from __future__ import annotations

import copy

from . import _api

NASH_SUTCLIFFE = _api.NASH_SUTCLIFFE
KLING_GUPTA = _api.KLING_GUPTA
ABS_DIFF = _api.ABS_DIFF
RMSE = _api.RMSE
DISCHARGE = _api.DISCHARGE
SNOW_COVERED_AREA = _api.SNOW_COVERED_AREA
SNOW_WATER_EQUIVALENT = _api.SNOW_WATER_EQUIVALENT
ROUTED_DISCHARGE = _api.ROUTED_DISCHARGE
CELL_CHARGE = _api.CELL_CHARGE


class TsTransform:
    """model_calibration::ts_transform (model_calibration.h:193-214)."""

    def to_average(self, start, dt, n, src):
        """True average of `src` (per its point interpretation) over n intervals of dt from start, as a new
        POINT_AVERAGE_VALUE series (average_accessor, time_series.h:2033-2072)."""
        from . import TimeAxisFixedDeltaT, TimeSeries, POINT_AVERAGE_VALUE
        ta = TimeAxisFixedDeltaT(start, dt, n)
        return TimeSeries(ta, src._ts.average(ta), POINT_AVERAGE_VALUE)


class TargetSpecificationPts:
    """target_specification<apoint_ts> (model_calibration.h:242-330; api_target_specification.cpp).

    TargetSpecificationPts()
    TargetSpecificationPts(ts, cids, scale_factor, calc_mode=KLING_GUPTA, s_r=1, s_a=1, s_b=1,
                           catchment_property=DISCHARGE, uid='')
    TargetSpecificationPts(ts, river_id, scale_factor, calc_mode=KLING_GUPTA, s_r=1, s_a=1, s_b=1, uid='')
    The target keeps its own copy of ts."""

    def __init__(self, ts=None, cids_or_rid=None, scale_factor=1.0, calc_mode=KLING_GUPTA, s_r=1.0, s_a=1.0, s_b=1.0,
                 catchment_property=DISCHARGE, uid=""):
        self.ts = copy.deepcopy(ts) if ts is not None else None
        self.catchment_indexes = []
        self.river_id = 0
        self.scale_factor = float(scale_factor)
        self.calc_mode = NASH_SUTCLIFFE if ts is None else calc_mode
        self.catchment_property = DISCHARGE
        self.s_r, self.s_a, self.s_b = float(s_r), float(s_a), float(s_b)
        self.uid = uid
        if ts is None:
            return
        if isinstance(cids_or_rid, (int,)) and not isinstance(cids_or_rid, bool):
            self.river_id = int(cids_or_rid)  # the river constructor: (ts, rid, scale, mode, s_r, s_a, s_b, uid)
            self.catchment_property = ROUTED_DISCHARGE
            if isinstance(catchment_property, str):
                self.uid = catchment_property
        else:
            self.catchment_indexes = [int(c) for c in (cids_or_rid or [])]
            self.catchment_property = catchment_property

    def __deepcopy__(self, memo):
        c = TargetSpecificationPts()
        c.__dict__.update({k: copy.deepcopy(v, memo) for k, v in self.__dict__.items()})
        return c

    def _impl(self):
        if self.ts is None:
            raise RuntimeError("TargetSpecificationPts: no target time-series")
        t = _api._TargetSpecification()
        t.ts = self.ts._ts
        t.catchment_indexes = list(self.catchment_indexes)
        t.river_id = int(self.river_id)
        t.scale_factor = float(self.scale_factor)
        t.calc_mode = _api.target_spec_calc_type(int(self.calc_mode))
        t.catchment_property = _api.target_property_type(int(self.catchment_property))
        t.s_r, t.s_a, t.s_b = self.s_r, self.s_a, self.s_b
        t.uid = self.uid
        return t


class TargetSpecificationVector(list):
    """vector<target_specification>; TargetSpecificationVector(other) is a deep copy."""

    def __init__(self, other=()):
        super().__init__(copy.deepcopy(t) for t in other)

    def size(self):
        return len(self)

    def push_back(self, t):
        self.append(t)


class _Optimizer:
    """optimizer<region_model, parameter, apoint_ts> (model_calibration.h:404-899) for one stack.

    Methods and arguments as expose.h:472-730: set_target_specification, optimize (local, bounded trust
    region), optimize_global, optimize_sceua, optimize_dream, calculate_goal_function, reset_states,
    set_parameter_ranges, set_verbose_level, establish_initial_state_from_model, get_initial_state,
    parameter_active, trace_size / trace_goal_function_value(s) / trace_parameter,
    target_specification, parameter_lower_bound / parameter_upper_bound.
    MI355X addition: calculate_goal_functions(list of parameters) evaluates them as device ensembles."""

    _impl_t = None  # the C++ optimizer class of the stack

    def __init__(self, model, targets=None, p_min=None, p_max=None):
        self._model = model
        if targets is None:
            model._push_parameters()
            self._o = self._impl_t(model)
        else:
            self._o = self._impl_t(model, [t._impl() for t in targets], self._vec(p_min), self._vec(p_max))
            self._targets = TargetSpecificationVector(targets)
        if targets is None:
            self._targets = TargetSpecificationVector()

    # ---- helpers
    def _vec(self, p):
        return p.to_vector() if hasattr(p, "to_vector") else [float(x) for x in p]

    def _sync_model(self):
        # the C++ optimizer set the region parameter (parameter_accessor.set); mirror it on the Python side
        self._model._region_parameter._v = list(self._model._get_region_parameter())

    def _wrap(self, p, v):
        v = list(v)
        if hasattr(p, "to_vector"):
            r = self._model._parameter_t()
            r._v = v
            return r
        return v

    # ---- configuration
    def set_target_specification(self, target_specification, parameter_lower_bound, parameter_upper_bound):
        self._model._push_parameters()
        self._targets = TargetSpecificationVector(target_specification)
        self._o._set_target_specification([t._impl() for t in self._targets], self._vec(parameter_lower_bound),
                                          self._vec(parameter_upper_bound))

    def set_parameter_ranges(self, p_min, p_max):
        self._o._set_parameter_ranges(self._vec(p_min), self._vec(p_max))

    @property
    def target_specification(self):
        return self._targets

    @target_specification.setter
    def target_specification(self, tv):
        self._targets = TargetSpecificationVector(tv)
        self._o._targets = [t._impl() for t in self._targets]

    @property
    def parameter_lower_bound(self):
        return self._wrap(self._model._parameter_t(), self._o._lower)

    @parameter_lower_bound.setter
    def parameter_lower_bound(self, p):
        self._o._lower = self._vec(p)

    @property
    def parameter_upper_bound(self):
        return self._wrap(self._model._parameter_t(), self._o._upper)

    @parameter_upper_bound.setter
    def parameter_upper_bound(self, p):
        self._o._upper = self._vec(p)

    def parameter_active(self, i):
        return self._o.parameter_active(i)

    def set_verbose_level(self, level):
        self._o.set_verbose_level(level)

    def establish_initial_state_from_model(self):
        self._o.establish_initial_state_from_model()

    def get_initial_state(self, i):
        return self._model._state_t(self._o._get_initial_state(i))

    def reset_states(self):
        self._o.reset_states()

    @property
    def batch_evaluation(self):
        return self._o.batch_evaluation

    @batch_evaluation.setter
    def batch_evaluation(self, on):
        self._o.batch_evaluation = bool(on)

    # ---- evaluation and search
    def calculate_goal_function(self, parameters):
        self._model._push_parameters()
        try:
            return self._o._calculate_goal_function(self._vec(parameters))
        finally:
            self._sync_model()

    def calculate_goal_functions(self, parameter_list):
        self._model._push_parameters()
        try:
            return list(self._o._calculate_goal_functions([self._vec(p) for p in parameter_list]))
        finally:
            self._sync_model()

    def optimize(self, p, max_n_evaluations=1500, tr_start=0.1, tr_stop=1.0e-5):
        self._model._push_parameters()
        try:
            return self._wrap(p, self._o._optimize(self._vec(p), int(max_n_evaluations), float(tr_start), float(tr_stop)))
        finally:
            self._sync_model()

    def optimize_global(self, p, max_n_evaluations, max_seconds, solver_eps):
        self._model._push_parameters()
        try:
            return self._wrap(p, self._o._optimize_global(self._vec(p), int(max_n_evaluations), float(max_seconds),
                                                          float(solver_eps)))
        finally:
            self._sync_model()

    def optimize_sceua(self, p, max_n_evaluations=1500, x_eps=0.0001, y_eps=1.0e-5):
        self._model._push_parameters()
        try:
            return self._wrap(p, self._o._optimize_sceua(self._vec(p), int(max_n_evaluations), float(x_eps),
                                                         float(y_eps)))
        finally:
            self._sync_model()

    def optimize_dream(self, p, max_n_evaluations=1500):
        self._model._push_parameters()
        try:
            return self._wrap(p, self._o._optimize_dream(self._vec(p), int(max_n_evaluations)))
        finally:
            self._sync_model()

    # ---- trace
    @property
    def trace_size(self):
        return self._o.trace_size

    @property
    def trace_goal_function_values(self):
        return list(self._o.trace_goal_function_values)

    def trace_goal_function_value(self, i):
        return self._o.trace_goal_function_value(i)

    def trace_parameter(self, i):
        r = self._model._parameter_t()
        r._v = list(self._o._trace_parameter(i))
        return r


def _from_vector(model, v):
    p = model._parameter_t()
    p._v = list(v)
    return p


def make_optimizer_type(name, impl_t):
    return type(name, (_Optimizer,), {"_impl_t": impl_t, "__doc__": _Optimizer.__doc__})
