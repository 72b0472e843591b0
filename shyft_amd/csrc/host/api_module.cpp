// pybind11 module shyft_amd.api._api: the Python surface of the host layer.
//
// The reference exposes region_model<cell_t> and its data types with
// boost.python (api/boostpython/expose.h:98-430, api_*.cpp, pt_gs_k.cpp:34-174,
// hbv_stack.cpp). boost.python is not available here, so this module binds the
// same C++ host classes (host/region_model.hpp) with pybind11; the Python
// package shyft_amd.api adds the reference's names and decorators on top
// (shyft/api/__init__.py, shyft/api/pt_gs_k/__init__.py).
//
// Time crosses the boundary as seconds (int or float, like shyft's `time`);
// internally it is int64 microseconds.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/functional.h>
#include <pybind11/stl.h>

#include <cmath>

#include "calibration.hpp"
#include "region_model.hpp"

namespace py = pybind11;
using namespace shyft_hip::host;

namespace {

utctime to_us(double seconds) { return utctime(std::llround(seconds * 1e6)); }
double to_s(utctime us) { return double(us) / 1e6; }

template <class Stack>
void bind_model(py::module_& m, const char* name) {
    using M = region_model<Stack>;
    py::class_<M>(m, name, py::dynamic_attr())
        .def(py::init<const std::vector<geo_cell_data>&, const std::vector<double>&, bool, int, const std::vector<int>&,
                      unsigned>(),
             py::arg("geo_data_vector"), py::arg("region_param"), py::arg("full_collection") = true,
             py::arg("device") = -1, py::arg("devices") = std::vector<int>(), py::arg("shard_flags") = 0u)
        .def(py::init<const std::vector<geo_cell_data>&, const std::vector<double>&,
                      const std::map<int64_t, std::vector<double>>&, bool, const std::vector<int>&, unsigned>(),
             py::arg("geo_data_vector"), py::arg("region_param"), py::arg("catchment_parameters"),
             py::arg("full_collection") = true, py::arg("devices") = std::vector<int>(), py::arg("shard_flags") = 0u)
        .def_property_readonly("shard_devices", &M::shard_devices)
        .def(py::init<const M&, bool>(), py::arg("other_model"), py::arg("full_collection"))
        .def_readwrite("ncore", &M::ncore)
        .def_readwrite("_ip_parameter", &M::ip_parameter)
        .def_readwrite("_region_env", &M::region_env)
        .def_readwrite("_initial_state", &M::initial_state)
        .def_readwrite("_river_network", &M::rivers)
        .def_property_readonly("_time_axis", [](const M& x) { return x.time_axis; })
        .def_property_readonly("full_collection", &M::full_collection)
        .def("size", &M::size)
        .def("number_of_catchments", &M::number_of_catchments)
        .def_property_readonly("catchment_ids", &M::catchment_ids)
        .def("extract_geo_cell_data", &M::extract_geo_cell_data)
        .def("_set_region_parameter", &M::set_region_parameter)
        .def("_get_region_parameter", &M::get_region_parameter)
        .def("_set_catchment_parameter", &M::set_catchment_parameter)
        .def("_update_catchment_parameter", &M::update_catchment_parameter)
        .def("remove_catchment_parameter", &M::remove_catchment_parameter, py::arg("catchment_id"))
        .def("has_catchment_parameter", &M::has_catchment_parameter, py::arg("catchment_id"))
        .def("_get_catchment_parameter", &M::get_catchment_parameter)
        .def("set_catchment_calculation_filter", &M::set_catchment_calculation_filter, py::arg("catchment_id_list"))
        .def("set_calculation_filter", &M::set_calculation_filter, py::arg("catchment_id_list"), py::arg("river_id_list"))
        .def("is_calculated", &M::is_calculated, py::arg("catchment_id"))
        .def("initialize_cell_environment", &M::initialize_cell_environment, py::arg("time_axis"))
        .def("_interpolate", &M::interpolate)
        .def("_run_interpolation", &M::run_interpolation)
        .def("is_cell_env_ts_ok", &M::is_cell_env_ts_ok)
        .def("run_cells", &M::run_cells, py::arg("use_ncore") = 0, py::arg("start_step") = 0, py::arg("n_steps") = 0,
             py::call_guard<py::gil_scoped_release>())
        .def("_get_states", [](const M& x) { return x.current_state(); })
        .def("_set_states", &M::set_states)
        .def("revert_to_initial_state", &M::revert_to_initial_state)
        .def("_extract_state", &M::extract_state)
        .def("_apply_state", &M::apply_state)
        .def("adjust_q", &M::adjust_q, py::arg("q_scale"), py::arg("cids"))
        .def("adjust_state_to_target_flow", &M::adjust_state_to_target_flow, py::arg("wanted_flow_m3s"),
             py::arg("cids"), py::arg("start_step") = 0, py::arg("scale_range") = 3.0, py::arg("scale_eps") = 1e-3,
             py::arg("max_iter") = 300, py::arg("n_steps") = 1)
        .def("set_state_collection", &M::set_state_collection, py::arg("catchment_id"), py::arg("on_or_off"))
        .def("set_snow_sca_swe_collection", &M::set_snow_sca_swe_collection, py::arg("catchment_id"), py::arg("on_or_off"))
        .def("_cell_collects_state", &M::cell_collects_state)
        .def("_cell_collects_snow", &M::cell_collects_snow)
        .def("_cell_series", [](const M& x, int s, size_t c) { auto v = x.cell_series(s, c); return py::array_t<double>(v.size(), v.data()); })
        .def("_cell_value", &M::cell_value)
        .def("_set_cell_value", &M::set_cell_value)
        .def("_set_cell_forcing", &M::set_cell_forcing)
        .def("_cell_geo", [](const M& x, size_t i) { return x.cells_geo().at(i); })
        .def("_cell_parameter", &M::cell_parameter)
        .def("_stat_series", [](const M& x, int s, const std::vector<int64_t>& ids, int scope, bool w) {
            auto v = x.stat_series(s, ids, scope, w);
            return py::array_t<double>(v.size(), v.data());
        })
        .def("_stat_value", &M::stat_value)
        .def("_stat_raster", &M::stat_raster)
        .def("_pot_ratio_series", [](const M& x, const std::vector<int64_t>& ids, int scope) {
            auto v = x.pot_ratio_series(ids, scope);
            return py::array_t<double>(v.size(), v.data());
        })
        .def("_pot_ratio_raster", &M::pot_ratio_raster)
        .def("_pot_ratio_value", &M::pot_ratio_value)
        .def("_area_stat", &M::area_stat)
        .def("_catchment_sums", &M::catchment_sums)
        .def("connect_catchment_to_river", &M::connect_catchment_to_river, py::arg("cid"), py::arg("rid"))
        .def("_set_cell_routing", &M::set_cell_routing)
        .def("has_routing", &M::has_routing)
        .def("_river_output_flow_m3s", &M::river_output_flow_m3s)
        .def("_river_upstream_inflow_m3s", &M::river_upstream_inflow_m3s)
        .def("_river_local_inflow_m3s", &M::river_local_inflow_m3s);
}

// model_calibration::optimizer<region_model> (expose.h:472-730 model_calibrator)
template <class Stack>
void bind_optimizer(py::module_& m, const char* name) {
    using M = region_model<Stack>;
    using O = optimizer<M>;
    py::class_<O>(m, name)
        .def(py::init<M&, const std::vector<target_specification>&, const std::vector<double>&, const std::vector<double>&>(),
             py::arg("model"), py::arg("targets"), py::arg("p_min"), py::arg("p_max"), py::keep_alive<1, 2>())
        .def(py::init<M&>(), py::arg("model"), py::keep_alive<1, 2>())
        .def("_set_target_specification", &O::set_target_specification)
        .def("_set_parameter_ranges", &O::set_parameter_ranges)
        .def_readwrite("_targets", &O::targets)
        .def_readwrite("_lower", &O::parameter_lower_bound)
        .def_readwrite("_upper", &O::parameter_upper_bound)
        .def_readwrite("batch_evaluation", &O::batch_evaluation)
        .def_readwrite("max_batch_members", &O::max_batch_members)
        .def("establish_initial_state_from_model", &O::establish_initial_state_from_model)
        .def("_get_initial_state", &O::get_initial_state)
        .def("set_verbose_level", &O::set_verbose_level, py::arg("level"))
        .def("reset_states", &O::reset_states)
        .def("parameter_active", &O::active_parameter, py::arg("i"))
        .def_property_readonly("trace_size", &O::trace_size)
        .def_readonly("trace_goal_function_values", &O::goal_fn_trace)
        .def("trace_goal_function_value", &O::trace_goal_fn, py::arg("i"))
        .def("_trace_parameter", &O::trace_parameter)
        .def("_calculate_goal_function", &O::calculate_goal_function, py::call_guard<py::gil_scoped_release>())
        .def("_calculate_goal_functions", &O::calculate_goal_functions, py::call_guard<py::gil_scoped_release>())
        .def("_optimize", &O::optimize, py::call_guard<py::gil_scoped_release>())
        .def("_optimize_global", &O::optimize_global, py::call_guard<py::gil_scoped_release>())
        .def("_optimize_sceua", &O::optimize_sceua, py::call_guard<py::gil_scoped_release>())
        .def("_optimize_dream", &O::optimize_dream, py::call_guard<py::gil_scoped_release>())
        .def("_to_scaled", &O::to_scaled)
        .def("_from_scaled", &O::from_scaled);
}

}  // namespace

PYBIND11_MODULE(_api, m) {
    m.doc() = "MI355X region engine host layer (C++ over the shyft_hip C ABI)";

    py::class_<geo_point>(m, "GeoPoint")
        .def(py::init<>())
        .def(py::init<double, double, double>(), py::arg("x"), py::arg("y"), py::arg("z"))
        .def_readwrite("x", &geo_point::x)
        .def_readwrite("y", &geo_point::y)
        .def_readwrite("z", &geo_point::z)
        .def("__deepcopy__", [](const geo_point& p, py::dict) { return p; })
        .def_static("distance2", [](const geo_point& a, const geo_point& b) {
            return (a.x - b.x) * (a.x - b.x) + (a.y - b.y) * (a.y - b.y) + (a.z - b.z) * (a.z - b.z);
        })
        .def("__repr__", [](const geo_point& p) {
            return "GeoPoint(" + std::to_string(p.x) + ", " + std::to_string(p.y) + ", " + std::to_string(p.z) + ")";
        });

    py::class_<land_type_fractions>(m, "LandTypeFractions")
        .def(py::init<>())
        .def(py::init<double, double, double, double, double>(), py::arg("glacier"), py::arg("lake"),
             py::arg("reservoir"), py::arg("forest"), py::arg("unspecified"))
        .def("glacier", &land_type_fractions::glacier)
        .def("lake", &land_type_fractions::lake)
        .def("reservoir", &land_type_fractions::reservoir)
        .def("forest", &land_type_fractions::forest)
        .def("unspecified", &land_type_fractions::unspecified)
        .def("snow_storage", &land_type_fractions::snow_storage)
        .def("set_fractions", &land_type_fractions::set_fractions, py::arg("glacier"), py::arg("lake"),
             py::arg("reservoir"), py::arg("forest"));

    py::class_<routing_info>(m, "RoutingInfo")
        .def(py::init<>())
        .def(py::init<int64_t, double>(), py::arg("id"), py::arg("distance") = 0.0)
        .def_readwrite("id", &routing_info::id)
        .def_readwrite("distance", &routing_info::distance);

    py::class_<geo_cell_data>(m, "GeoCellData")
        .def(py::init<>())
        .def(py::init<const geo_point&, double, int64_t, double, const land_type_fractions&>(), py::arg("mid_point"),
             py::arg("area"), py::arg("catchment_id"), py::arg("radiation_slope_factor") = 0.9,
             py::arg("land_type_fractions") = land_type_fractions())
        .def("mid_point", &geo_cell_data::mid_point)
        .def("area", &geo_cell_data::area)
        .def("catchment_id", &geo_cell_data::catchment_id)
        .def("set_catchment_id", [](geo_cell_data& g, int64_t c) { g.catchment_id_ = c; })
        .def("radiation_slope_factor", &geo_cell_data::radiation_slope_factor)
        .def("land_type_fractions_info", [](geo_cell_data& g) -> land_type_fractions& { return g.fractions; },
             py::return_value_policy::reference_internal)
        .def("set_land_type_fractions", [](geo_cell_data& g, const land_type_fractions& f) { g.fractions = f; })
        .def_readwrite("routing_info", &geo_cell_data::routing)
        .def_readwrite("routing", &geo_cell_data::routing);

    py::class_<fixed_dt>(m, "TimeAxisFixedDeltaT")
        .def(py::init([](double t0, double dt, size_t n) { return fixed_dt(to_us(t0), to_us(dt), n); }), py::arg("start"),
             py::arg("delta_t"), py::arg("n"))
        .def("size", &fixed_dt::size)
        .def("__len__", &fixed_dt::size)
        .def_property_readonly("start", [](const fixed_dt& a) { return to_s(a.t); })
        .def_property_readonly("delta_t", [](const fixed_dt& a) { return to_s(a.dt); })
        .def_property_readonly("n", [](const fixed_dt& a) { return a.n; })
        .def("time", [](const fixed_dt& a, size_t i) { return to_s(a.time(i)); })
        .def("period", [](const fixed_dt& a, size_t i) { auto p = a.period(i); return std::make_pair(to_s(p.start), to_s(p.end)); })
        .def("total_period", [](const fixed_dt& a) { auto p = a.total_period(); return std::make_pair(to_s(p.start), to_s(p.end)); })
        .def("index_of", [](const fixed_dt& a, double t) { auto i = a.index_of(to_us(t)); return i == npos ? int64_t(-1) : int64_t(i); })
        .def("__eq__", &fixed_dt::operator==);

    py::enum_<ts_point_fx>(m, "point_interpretation_policy")
        .value("POINT_INSTANT_VALUE", POINT_INSTANT_VALUE)
        .value("POINT_AVERAGE_VALUE", POINT_AVERAGE_VALUE)
        .export_values();

    py::class_<point_ts>(m, "_PointTs")
        .def(py::init([](const fixed_dt& ta, std::vector<double> v, ts_point_fx fx) { return point_ts(ta, std::move(v), fx); }))
        .def(py::init([](const std::vector<double>& t, double t_end, std::vector<double> v, ts_point_fx fx) {
            std::vector<utctime> tu(t.size());
            for (size_t i = 0; i < t.size(); ++i) tu[i] = to_us(t[i]);
            return point_ts(std::move(tu), to_us(t_end), std::move(v), fx);
        }))
        .def("__deepcopy__", [](const point_ts& s, py::dict) { return point_ts(s); })
        .def("size", &point_ts::size)
        .def("value", &point_ts::value)
        .def("set", &point_ts::set)
        .def("time", [](const point_ts& s, size_t i) { return to_s(s.time(i)); })
        .def("point_interpretation", [](const point_ts& s) { return s.fx; })
        .def("total_period", [](const point_ts& s) { auto p = s.total_period(); return std::make_pair(to_s(p.start), to_s(p.end)); })
        .def("__call__", [](const point_ts& s, double t) { return s(to_us(t)); })
        .def_property_readonly("_values", [](const point_ts& s) { return py::array_t<double>(s.v.size(), s.v.data()); })
        .def_property_readonly("_times", [](const point_ts& s) {
            std::vector<double> t(s.t.size());
            for (size_t i = 0; i < t.size(); ++i) t[i] = to_s(s.t[i]);
            return t;
        })
        .def_property_readonly("_t_end", [](const point_ts& s) { return to_s(s.t_end); })
        .def("average", [](const point_ts& s, const fixed_dt& ta) {
            auto v = average_values(s, ta);
            return py::array_t<double>(v.size(), v.data());
        });

    py::class_<geo_point_ts>(m, "_GeoPointTs")
        .def(py::init([](const geo_point& p, const point_ts& ts) { return geo_point_ts{p, ts, ""}; }))
        .def_readwrite("_mid_point", &geo_point_ts::mid_point)
        .def_readwrite("_ts", &geo_point_ts::ts)
        .def_readwrite("uid", &geo_point_ts::uid);

    py::class_<region_environment>(m, "_RegionEnvironment")
        .def(py::init<>())
        .def_readwrite("temperature", &region_environment::temperature)
        .def_readwrite("precipitation", &region_environment::precipitation)
        .def_readwrite("wind_speed", &region_environment::wind_speed)
        .def_readwrite("rel_hum", &region_environment::rel_hum)
        .def_readwrite("radiation", &region_environment::radiation);

    py::class_<idw_parameter>(m, "IDWParameter")
        .def(py::init<>())
        .def(py::init([](size_t mm, double md, double f, double zs) {
                 idw_parameter p; p.max_members = mm; p.max_distance = md; p.distance_measure_factor = f; p.zscale = zs;
                 return p;
             }),
             py::arg("max_members") = 10, py::arg("max_distance") = 200000.0, py::arg("distance_measure_factor") = 2.0,
             py::arg("zscale") = 1.0)
        .def_readwrite("max_members", &idw_parameter::max_members)
        .def_readwrite("max_distance", &idw_parameter::max_distance)
        .def_readwrite("distance_measure_factor", &idw_parameter::distance_measure_factor)
        .def_readwrite("zscale", &idw_parameter::zscale);
    py::class_<idw_temperature_parameter, idw_parameter>(m, "IDWTemperatureParameter")
        .def(py::init<>())
        .def(py::init([](double g, size_t mm, double md, bool eq) {
                 idw_temperature_parameter p; p.default_temp_gradient = g; p.max_members = mm; p.max_distance = md;
                 p.gradient_by_equation = eq; return p;
             }),
             py::arg("default_gradient") = -0.006, py::arg("max_members") = 20, py::arg("max_distance") = 200000.0,
             py::arg("gradient_by_equation") = false)
        .def_readwrite("default_temp_gradient", &idw_temperature_parameter::default_temp_gradient)
        .def_readwrite("gradient_by_equation", &idw_temperature_parameter::gradient_by_equation);
    py::class_<idw_precipitation_parameter, idw_parameter>(m, "IDWPrecipitationParameter")
        .def(py::init<>())
        .def(py::init([](double s, size_t mm, double md) {
                 idw_precipitation_parameter p; p.scale_factor = s; p.max_members = mm; p.max_distance = md; return p;
             }),
             py::arg("scale_factor") = 1.02, py::arg("max_members") = 20, py::arg("max_distance") = 200000.0)
        .def_readwrite("scale_factor", &idw_precipitation_parameter::scale_factor);
    // CellStateId (api/api_state.h:34-59; api/boostpython/api_state.cpp)
    py::class_<cell_state_id>(m, "CellStateId")
        .def(py::init<>())
        .def(py::init<int64_t, int64_t, int64_t, int64_t>(), py::arg("cid"), py::arg("x"), py::arg("y"), py::arg("area"))
        .def_readwrite("cid", &cell_state_id::cid)
        .def_readwrite("x", &cell_state_id::x)
        .def_readwrite("y", &cell_state_id::y)
        .def_readwrite("area", &cell_state_id::area)
        .def("__eq__", &cell_state_id::operator==)
        .def("__ne__", &cell_state_id::operator!=)
        .def("__lt__", &cell_state_id::operator<)
        .def("__hash__", [](const cell_state_id& c) { return py::hash(py::make_tuple(c.cid, c.x, c.y, c.area)); })
        .def("__repr__", [](const cell_state_id& c) {
            return "CellStateId(" + std::to_string(c.cid) + ", " + std::to_string(c.x) + ", " + std::to_string(c.y) +
                   ", " + std::to_string(c.area) + ")";
        });
    m.def("_serialize_states", [](int stack, size_t n_fields, const std::vector<state_with_id>& v) {
        auto b = serialize_states(stack, n_fields, v);
        return py::bytes(b.data(), b.size());
    });
    m.def("_deserialize_states", [](const py::bytes& b, int stack, size_t n_fields) {
        std::string s = b;
        return deserialize_states(std::vector<char>(s.begin(), s.end()), stack, n_fields);
    });
    // BTKParameter (api/boostpython/api_interpolation.cpp:188-200)
    py::class_<btk_parameter>(m, "BTKParameter")
        .def(py::init<>())
        .def(py::init<double, double>(), py::arg("temperature_gradient"), py::arg("temperature_gradient_sd"))
        .def(py::init<double, double, double, double, double, double>(), py::arg("temperature_gradient"),
             py::arg("temperature_gradient_sd"), py::arg("sill"), py::arg("nugget"), py::arg("range"), py::arg("zscale"))
        .def("temperature_gradient", [](const btk_parameter& p, std::pair<double, double> period) {
                 return p.temperature_gradient(utcperiod(to_us(period.first), to_us(period.second)));
             }, py::arg("p"))
        .def("temperature_gradient_sd", &btk_parameter::temperature_gradient_sd)
        .def("sill", &btk_parameter::sill)
        .def("nug", &btk_parameter::nug)
        .def("range", &btk_parameter::range)
        .def("zscale", &btk_parameter::zscale);
    // bayesian_kriging_temperature (api_interpolation.cpp:54-71): validation, sources averaged onto the axis,
    // one source copied, else the device BTK
    m.def("_bayesian_kriging_temperature", [](const std::vector<geo_point_ts>& src, const std::vector<geo_point>& dst,
                                              const fixed_dt& ta, const btk_parameter& p) {
        if (src.empty() || dst.empty())
            throw std::runtime_error("the supplied src and dst_points should be non-null and have at least one time-series");
        if (ta.size() == 0 || ta.dt == 0)
            throw std::runtime_error("the supplied destination time-axis should have more than 0 element, and a delta-t larger than 0");
        const size_t S = src.size(), T = ta.size(), D = dst.size();
        std::vector<double> xyz(3 * S), vals(T * S), prior(T), prm(5), dxyz(3 * D), out(T * D);
        for (size_t s = 0; s < S; ++s) {
            xyz[3 * s] = src[s].mid_point.x;
            xyz[3 * s + 1] = src[s].mid_point.y;
            xyz[3 * s + 2] = src[s].mid_point.z;
            auto v = average_values(src[s].ts, ta);
            for (size_t t = 0; t < T; ++t) vals[t * S + s] = v[t];
        }
        for (size_t d = 0; d < D; ++d) {
            dxyz[3 * d] = dst[d].x;
            dxyz[3 * d + 1] = dst[d].y;
            dxyz[3 * d + 2] = dst[d].z;
        }
        for (size_t t = 0; t < T; ++t) prior[t] = p.temperature_gradient(ta.period(t));
        p.as_abi(prm.data());
        {
            py::gil_scoped_release nogil;
            throw_if(shyft_hip_btk(-1, S, xyz.data(), vals.data(), T, prior.data(), prm.data(), D, dxyz.data(),
                                   out.data()),
                     nullptr);
        }
        return py::array_t<double>({T, D}, out.data());
    });
    py::class_<interpolation_parameter>(m, "InterpolationParameter")
        .def(py::init<>())
        .def(py::init([](const btk_parameter& t, const idw_precipitation_parameter& p, const idw_parameter& ws,
                         const idw_parameter& rad, const idw_parameter& rh) {
                 interpolation_parameter ip;
                 ip.temperature = t; ip.precipitation = p; ip.wind_speed = ws; ip.radiation = rad; ip.rel_hum = rh;
                 return ip;
             }),
             py::arg("temperature"), py::arg("precipitation"), py::arg("wind_speed"), py::arg("radiation"),
             py::arg("rel_hum"))
        .def(py::init([](const idw_temperature_parameter& t, const idw_precipitation_parameter& p, const idw_parameter& ws,
                         const idw_parameter& rad, const idw_parameter& rh) {
                 interpolation_parameter ip;
                 ip.temperature_idw = t; ip.use_idw_for_temperature = true;  // api_interpolation.cpp:447
                 ip.precipitation = p; ip.wind_speed = ws; ip.radiation = rad; ip.rel_hum = rh;
                 return ip;
             }),
             py::arg("temperature"), py::arg("precipitation"), py::arg("wind_speed"), py::arg("radiation"),
             py::arg("rel_hum"))
        .def_readwrite("temperature", &interpolation_parameter::temperature)
        .def_readwrite("use_idw_for_temperature", &interpolation_parameter::use_idw_for_temperature)
        .def_readwrite("temperature_idw", &interpolation_parameter::temperature_idw)
        .def_readwrite("precipitation", &interpolation_parameter::precipitation)
        .def_readwrite("wind_speed", &interpolation_parameter::wind_speed)
        .def_readwrite("radiation", &interpolation_parameter::radiation)
        .def_readwrite("rel_hum", &interpolation_parameter::rel_hum);

    py::class_<uhg_parameter>(m, "UHGParameter")
        .def(py::init<>())
        .def(py::init<double, double, double>(), py::arg("velocity"), py::arg("alpha") = 7.0, py::arg("beta") = 0.0)
        .def_readwrite("velocity", &uhg_parameter::velocity)
        .def_readwrite("alpha", &uhg_parameter::alpha)
        .def_readwrite("beta", &uhg_parameter::beta);
    py::class_<river>(m, "River")
        .def(py::init([](int64_t id, const routing_info& ds, const uhg_parameter& p) { return river(id, ds.id, ds.distance, p); }),
             py::arg("id"), py::arg("downstream") = routing_info(), py::arg("parameter") = uhg_parameter())
        .def_readwrite("id", &river::id)
        .def_property("downstream", [](const river& r) { return routing_info(r.downstream_id, r.downstream_distance); },
                      [](river& r, const routing_info& ri) { r.downstream_id = ri.id; r.downstream_distance = ri.distance; })
        .def_readwrite("parameter", &river::parameter)
        .def("uhg", [](const river& r, double dt) { return r.uhg(to_us(dt)); });
    py::class_<q_adjust_result>(m, "FlowAdjustResult")
        .def(py::init<>())
        .def_readwrite("q_0", &q_adjust_result::q_0)
        .def_readwrite("q_r", &q_adjust_result::q_r)
        .def_readwrite("diagnostics", &q_adjust_result::diagnostics);
    // the state tuner's 1-D minimiser, exposed for host-side tests (no device work)
    m.def(
        "find_min_single_variable",
        [](const std::function<double(double)>& f, double x, double begin, double end, double eps, long max_iter,
           double radius) {
            const double fx = find_min_single_variable(f, x, begin, end, eps, max_iter, radius);
            return std::make_pair(x, fx);
        },
        py::arg("f"), py::arg("starting_point"), py::arg("begin"), py::arg("end"), py::arg("eps") = 1e-3,
        py::arg("max_iter") = 100, py::arg("initial_search_radius") = 1.0);
    py::class_<river_network>(m, "RiverNetwork")
        .def(py::init<>())
        .def("add", [](river_network& n, const river& r) -> river_network& { return n.add(r); }, py::return_value_policy::reference_internal)
        .def("remove_by_id", &river_network::remove_by_id)
        .def("river_by_id", [](river_network& n, int64_t rid) -> river& { return n.river_by_id(rid); }, py::return_value_policy::reference_internal)
        .def("upstreams_by_id", &river_network::upstreams_by_id)
        .def("downstream_by_id", &river_network::downstream_by_id)
        .def("set_downstream_by_id", &river_network::set_downstream_by_id)
        .def("network_contains_directed_cycle", &river_network::network_contains_directed_cycle);
    m.def("make_uhg_from_gamma", &make_uhg_from_gamma, py::arg("n_steps"), py::arg("alpha"), py::arg("beta"));

    m.def("utc_time", [](int y, int mo, int d, int h, int mi, int s) { return to_s(utc_time(y, mo, d, h, mi, s)); });
    m.def("average_values", [](const point_ts& s, const fixed_dt& ta) {
        auto v = average_values(s, ta);
        return py::array_t<double>(v.size(), v.data());
    });

    bind_model<pt_gs_k_stack>(m, "_PTGSKRegionModel");
    bind_model<hbv_stack_stack>(m, "_HbvRegionModel");
    bind_model<pt_ss_k_stack>(m, "_PTSSKRegionModel");
    bind_model<pt_hs_k_stack>(m, "_PTHSKRegionModel");
    bind_model<pt_hps_k_stack>(m, "_PTHPSKRegionModel");

    py::enum_<target_spec_calc_type>(m, "target_spec_calc_type")
        .value("NASH_SUTCLIFFE", NASH_SUTCLIFFE)
        .value("KLING_GUPTA", KLING_GUPTA)
        .value("ABS_DIFF", ABS_DIFF)
        .value("RMSE", RMSE)
        .export_values();
    py::enum_<target_property_type>(m, "target_property_type")
        .value("DISCHARGE", DISCHARGE)
        .value("SNOW_COVERED_AREA", SNOW_COVERED_AREA)
        .value("SNOW_WATER_EQUIVALENT", SNOW_WATER_EQUIVALENT)
        .value("ROUTED_DISCHARGE", ROUTED_DISCHARGE)
        .value("CELL_CHARGE", CELL_CHARGE)
        .export_values();
    py::class_<target_specification>(m, "_TargetSpecification")
        .def(py::init<>())
        .def_readwrite("ts", &target_specification::ts)
        .def_readwrite("catchment_indexes", &target_specification::catchment_indexes)
        .def_readwrite("river_id", &target_specification::river_id)
        .def_readwrite("scale_factor", &target_specification::scale_factor)
        .def_readwrite("calc_mode", &target_specification::calc_mode)
        .def_readwrite("catchment_property", &target_specification::catchment_property)
        .def_readwrite("s_r", &target_specification::s_r)
        .def_readwrite("s_a", &target_specification::s_a)
        .def_readwrite("s_b", &target_specification::s_b)
        .def_readwrite("uid", &target_specification::uid);
    // goal functions on value vectors (time_series.h:2301-2450), for tests and direct use
    m.def("nash_sutcliffe_goal_function", &goal::nash_sutcliffe, py::arg("observed"), py::arg("model"));
    m.def("kling_gupta_goal_function", &goal::kling_gupta, py::arg("observed"), py::arg("model"), py::arg("s_r"),
          py::arg("s_a"), py::arg("s_b"));
    m.def("rmse_goal_function", &goal::rmse, py::arg("observed"), py::arg("model"));
    m.def("abs_diff_sum_goal_function", &goal::abs_diff_sum, py::arg("observed"), py::arg("model"));
    m.def("abs_diff_sum_goal_function_scaled", &goal::abs_diff_sum_scaled, py::arg("observed"), py::arg("model"),
          py::arg("scale"));
    m.def("_average_onto", &average_onto);
    // search algorithms over a Python callable (scaled space [0,1]^n), for tests of the restatements
    m.def("_sceua_find_min", [](const std::function<double(const std::vector<double>&)>& f, std::vector<double> x,
                                size_t max_n, double x_eps, double y_eps) {
        const size_t n = x.size();
        std::vector<double> lo(n, 0.0), hi(n, 1.0), xe(n, x_eps);
        scaled_fx fx{f, [&f](const std::vector<std::vector<double>>& xs) {
                         std::vector<double> r;
                         for (const auto& v : xs) r.push_back(f(v));
                         return r;
                     }};
        double y = 0;
        auto st = sceua_search().find_min(lo, hi, x, y, fx, y_eps, -1.0, -2.0, xe, max_n, false);
        return std::make_tuple(x, y, int(st));
    });
    m.def("_dream_find_max", [](const std::function<double(const std::vector<double>&)>& f, std::vector<double> x,
                                size_t max_n) {
        scaled_fx fx{f, [&f](const std::vector<std::vector<double>>& xs) {
                         std::vector<double> r;
                         for (const auto& v : xs) r.push_back(f(v));
                         return r;
                     }};
        double y = dream_search().find_max(fx, x, max_n, false);
        return std::make_pair(x, y);
    });
    m.def("_box_trust_region_min", [](const std::function<double(const std::vector<double>&)>& f, std::vector<double> x,
                                      double rho_begin, double rho_end, size_t max_n) {
        scaled_fx fx{f, [&f](const std::vector<std::vector<double>>& xs) {
                         std::vector<double> r;
                         for (const auto& v : xs) r.push_back(f(v));
                         return r;
                     }};
        auto r = box_trust_region::minimize(fx, x, rho_begin, rho_end, max_n);
        return std::make_tuple(r.x, r.f, r.evaluations);
    });
    bind_optimizer<pt_gs_k_stack>(m, "_PTGSKOptimizer");
    bind_optimizer<hbv_stack_stack>(m, "_HbvOptimizer");
    bind_optimizer<pt_ss_k_stack>(m, "_PTSSKOptimizer");
    bind_optimizer<pt_hs_k_stack>(m, "_PTHSKOptimizer");
    bind_optimizer<pt_hps_k_stack>(m, "_PTHPSKOptimizer");

    py::register_exception_translator([](std::exception_ptr p) {
        try {
            if (p) std::rethrow_exception(p);
        } catch (const std::invalid_argument& e) {
            PyErr_SetString(PyExc_RuntimeError, e.what());
        }
    });
}
