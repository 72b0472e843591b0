// region_model<Stack>: the C++ host class that keeps the reference's
// region_model<cell_t, region_env> API (core/region_model.h:211-1049) and
// drives the MI355X engine exclusively through the C ABI of include/shyft_hip.h.
//
// What lives here (host, O(cells) bookkeeping) and what does not:
//  - cells' geo_cell_data, region/catchment parameters, catchment ids and the
//    calculation filter, initial-state snapshot, river network: host mirrors,
//    pushed to the device handle when they change;
//  - source resampling (average_accessor, region_model.h:135-145) of the region
//    environment onto the model time axis: host, once per source;
//  - run_interpolation's inverse-distance work, run_cells, catchment sums and
//    the routing aggregation: device (shyft_hip_interpolate / run_cells /
//    statistics / catchment_sums).
// Errors are std::runtime_error with the reference's messages (the C ABI returns
// them as last_error text).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <utility>
#include <vector>

#include "../../../include/shyft_hip.h"
#include "optimize.hpp"
#include "routing.hpp"
#include "state_io.hpp"
#include "time_series.hpp"

namespace shyft_hip::host {

// ---- geo (core/geo_point.h, core/geo_cell_data.h:36-230) -------------------------------------------------------
struct geo_point {
    double x = 0, y = 0, z = 0;
    geo_point() = default;
    geo_point(double x_, double y_, double z_) : x(x_), y(y_), z(z_) {}
};

struct land_type_fractions {
    double glacier_ = 0, lake_ = 0, reservoir_ = 0, forest_ = 0;
    land_type_fractions() = default;
    // ctor normalises by the sum of the 5 non-negative fractions (geo_cell_data.h:36-51)
    land_type_fractions(double glacier, double lake, double reservoir, double forest, double unspecified) {
        glacier = std::max(0.0, glacier); lake = std::max(0.0, lake); reservoir = std::max(0.0, reservoir);
        forest = std::max(0.0, forest); unspecified = std::max(0.0, unspecified);
        const double sum = glacier + lake + reservoir + forest + unspecified;
        if (sum > 0) {
            glacier_ = glacier / sum; lake_ = lake / sum; reservoir_ = reservoir / sum; forest_ = forest / sum;
        }
    }
    double glacier() const { return glacier_; }
    double lake() const { return lake_; }
    double reservoir() const { return reservoir_; }
    double forest() const { return forest_; }
    double unspecified() const { return 1.0 - glacier_ - lake_ - reservoir_ - forest_; }
    double snow_storage() const { return 1.0 - lake_ - reservoir_; }
    // set_fractions (geo_cell_data.h:67-79)
    void set_fractions(double glacier, double lake, double reservoir, double forest) {
        const double tol = 1.0e-3;
        const double sum = glacier + lake + reservoir + forest;
        if (sum > 1.0 && sum < 1.0 + tol) {
            glacier /= sum; lake /= sum; reservoir /= sum; forest /= sum;
        } else if (sum > 1.0 || glacier < 0.0 || lake < 0.0 || reservoir < 0.0 || forest < 0.0) {
            throw std::invalid_argument("LandTypeFractions:: must be >=0.0 and sum <= 1.0");
        }
        glacier_ = glacier; lake_ = lake; reservoir_ = reservoir; forest_ = forest;
    }
};

struct routing_info {
    int64_t id = 0;
    double distance = 0.0;
    routing_info() = default;
    routing_info(int64_t i, double d) : id(i), distance(d) {}
};

struct geo_cell_data {
    geo_point mid_point_;
    double area_m2 = 1.0e6;
    int64_t catchment_id_ = -1;
    double radiation_slope_factor_ = 0.9;
    land_type_fractions fractions;
    routing_info routing;
    geo_cell_data() = default;
    geo_cell_data(const geo_point& mp, double area, int64_t cid, double slope = 0.9,
                  const land_type_fractions& ltf = land_type_fractions())
        : mid_point_(mp), area_m2(area), catchment_id_(cid), radiation_slope_factor_(slope), fractions(ltf) {}
    const geo_point& mid_point() const { return mid_point_; }
    double area() const { return area_m2; }
    int64_t catchment_id() const { return catchment_id_; }
    double radiation_slope_factor() const { return radiation_slope_factor_; }
    // geo_cell_data_io layout (api/api.h:1598-1621)
    void to_io11(double* g) const {
        g[0] = mid_point_.x; g[1] = mid_point_.y; g[2] = mid_point_.z; g[3] = area_m2; g[4] = double(catchment_id_);
        g[5] = radiation_slope_factor_; g[6] = fractions.glacier(); g[7] = fractions.lake();
        g[8] = fractions.reservoir(); g[9] = fractions.forest(); g[10] = fractions.unspecified();
    }
};

// ---- interpolation parameters (core/inverse_distance.h:38-74, core/region_model.h:60-95) -----------------------
struct idw_parameter {
    size_t max_members = 10;
    double max_distance = 200000.0, distance_measure_factor = 2.0, zscale = 1.0;
};
struct idw_temperature_parameter : idw_parameter {
    double default_temp_gradient = -0.006;
    bool gradient_by_equation = false;
    idw_temperature_parameter() { max_members = 20; }
};
struct idw_precipitation_parameter : idw_parameter {
    double scale_factor = 1.02;
    idw_precipitation_parameter() { max_members = 20; }
};
// bayesian_kriging::parameter (core/bayesian_kriging.h:204-230): the prior gradient follows the day of year
struct btk_parameter {
    double gradient_sd = 0.0025, sill_value = 25.0, nug_value = 0.5, range_value = 200000.0, zscale_value = 20.0;
    btk_parameter() = default;
    btk_parameter(double /*temperature_gradient, not used*/, double temperature_gradient_sd)
        : gradient_sd(temperature_gradient_sd / 100) {}
    btk_parameter(double /*temperature_gradient*/, double temperature_gradient_sd, double sill, double nugget,
                  double range, double zscale)
        : gradient_sd(temperature_gradient_sd / 100), sill_value(sill), nug_value(nugget), range_value(range),
          zscale_value(zscale) {}
    double temperature_gradient(const utcperiod& p) const {
        const double doy = double(day_of_year(p.start + (p.end - p.start) / 2));
        return 1.18e-3 * std::sin(6.2831 / 365 * (doy + 79.0)) - 5.48e-3;
    }
    double temperature_gradient_sd() const { return gradient_sd; }
    double sill() const { return sill_value; }
    double nug() const { return nug_value; }
    double range() const { return range_value; }
    double zscale() const { return zscale_value; }
    void as_abi(double* p) const { p[0] = gradient_sd; p[1] = sill_value; p[2] = nug_value; p[3] = range_value; p[4] = zscale_value; }
};

struct interpolation_parameter {
    bool use_idw_for_temperature = false;
    btk_parameter temperature;
    idw_temperature_parameter temperature_idw;
    idw_precipitation_parameter precipitation;
    idw_parameter wind_speed, radiation, rel_hum;
};

// ---- region environment (core/region_model.h:146-187, api/api.h:78-168) ----------------------------------------
struct geo_point_ts {
    geo_point mid_point;
    point_ts ts;
    std::string uid;
};
struct region_environment {
    // nullptr-equivalent: the vector is empty and the flag unset (the reference keeps shared_ptr<vector<..>>)
    std::vector<geo_point_ts> temperature, precipitation, wind_speed, rel_hum, radiation;
};

inline void throw_if(int status, shyft_hip_region* h) {
    if (status) throw std::runtime_error(shyft_hip_last_error(h));
}

// ---- the method-stack traits -------------------------------------------------------------------------------------
struct pt_gs_k_stack {
    static constexpr int id = SHYFT_HIP_PT_GS_K;
    static constexpr size_t n_param = 31;   // core/pt_gs_k.h:74
    static constexpr size_t n_state = 9;    // gs(8) + kirchner.q
    static constexpr size_t n_full_series = 8;
    static constexpr int k_ae_scale = 3;    // ae.ae_scale_factor in the parameter vector
    static constexpr int k_routing = 25;    // routing.velocity, alpha, beta
    static constexpr int state_q = 8;       // kirchner.q in the state vector
    static constexpr double q_min = 0.0;
    static constexpr const char* param_error = "PTGSK Parameter Accessor: .set size missmatch";
};
struct hbv_stack_stack {
    static constexpr int id = SHYFT_HIP_HBV_STACK;
    static constexpr size_t n_param = 22;   // core/hbv_stack.h:81 (+17 snow distribution values, optional)
    static constexpr size_t n_state = 22;   // swe sca sm uz lz n_bins sp[8] sw[8]
    static constexpr size_t n_full_series = 9;
    static constexpr int k_ae_scale = -1;
    static constexpr int k_routing = 17;
    static constexpr int state_q = -1;
    static constexpr double q_min = 0.0;
    static constexpr const char* param_error = "HBV_Stack Parameter Accessor: .set size missmatch";
};

struct pt_ss_k_stack {
    static constexpr int id = SHYFT_HIP_PT_SS_K;
    static constexpr size_t n_param = 21;   // core/pt_ss_k.h:74
    static constexpr size_t n_state = 8;    // skaugen nu alpha sca swe free_water residual num_units + kirchner.q
    static constexpr size_t n_full_series = 8;
    static constexpr int k_ae_scale = 3;
    static constexpr int k_routing = 16;
    static constexpr int state_q = 7;
    static constexpr double q_min = 0.0;
    static constexpr const char* param_error = "pt_ss_k parameter accessor: .set size mismatch";
};

struct pt_hs_k_stack {
    static constexpr int id = SHYFT_HIP_PT_HS_K;
    static constexpr size_t n_param = 18;   // core/pt_hs_k.h:64 (+17 snow distribution values, optional)
    static constexpr size_t n_state = 20;   // swe sca n_bins sp[8] sw[8] kirchner q
    static constexpr size_t n_full_series = 8;
    static constexpr int k_ae_scale = 3;
    static constexpr int k_routing = 13;
    static constexpr int state_q = 19;
    static constexpr double q_min = 0.0;
    static constexpr const char* param_error = "pt_ss_k parameter accessor: .set size missmatch";  // pt_hs_k.h:68
};

struct pt_hps_k_stack {
    static constexpr int id = SHYFT_HIP_PT_HPS_K;
    static constexpr size_t n_param = 24;   // core/pt_hps_k.h:62 (+ gm.direct_response + 17 distribution values)
    static constexpr size_t n_state = 37;   // swe sca surface_heat n_bins sp[8] sw[8] albedo[8] iso_pot_energy[8] q
    static constexpr size_t n_full_series = 8;
    static constexpr int k_ae_scale = 3;
    static constexpr int k_routing = 20;
    static constexpr int state_q = 36;
    static constexpr double q_min = 0.0;
    static constexpr const char* param_error = "pt_ss_k parameter accessor: .set size missmatch";  // pt_hps_k.h:70
};

// ---- region_model ------------------------------------------------------------------------------------------------
// result of adjust_state_to_target_flow (core/model_state_tuning.h:12-17)
struct q_adjust_result {
    double q_0{0.0};          // m3/s with the state before adjustment
    double q_r{0.0};          // m3/s with the adjusted state
    std::string diagnostics;  // empty if ok
};

template <class Stack>
class region_model {
  public:
    using parameter_t = std::vector<double>;
    using state_t = std::vector<double>;

    // region_model(const vector<geo_cell_data>&, const parameter_t&)  (region_model.h:285-293)
    // devices: the region's cells in shards, one per entry (repeats allowed), all driven from this process
    // (shyft_hip_region_create_sharded_ex; shard_flags e.g. SHYFT_HIP_SHARD_BALANCE_Z); empty: one region on `device`
    region_model(const std::vector<geo_cell_data>& geov, const parameter_t& region_param, bool full_collection = true,
                 int device = -1, const std::vector<int>& devices = {}, unsigned shard_flags = 0)
        : geo_(geov), full_(full_collection) {
        if (geo_.empty()) throw std::runtime_error("region_model: no cells");
        shyft_hip_region* h = nullptr;
        if (devices.empty())
            throw_if(shyft_hip_region_create(Stack::id, geo_.size(), device, &h), nullptr);
        else
            throw_if(shyft_hip_region_create_sharded_ex(Stack::id, geo_.size(), devices.data(), devices.size(),
                                                        shard_flags, &h),
                     nullptr);
        h_.reset(h, shyft_hip_region_destroy);
        ncore = std::max(1u, std::thread::hardware_concurrency());
        state_collection_.assign(geo_.size(), false);
        snow_collection_.assign(geo_.size(), false);
        push_geo();
        set_region_parameter(region_param);
        state_t s0 = default_state();
        std::vector<state_t> sv(geo_.size(), s0);
        put_states(sv);
        push_collection();
    }
    // region_model(cells, region_param, catchment_parameters)  (region_model.h:294-301)
    region_model(const std::vector<geo_cell_data>& geov, const parameter_t& region_param,
                 const std::map<int64_t, parameter_t>& catchment_parameters, bool full_collection = true,
                 const std::vector<int>& devices = {}, unsigned shard_flags = 0)
        : region_model(geov, region_param, full_collection, -1, devices, shard_flags) {
        for (const auto& kv : catchment_parameters) set_catchment_parameter(kv.first, kv.second);
    }
    // copy ctor / clone (region_model.h:297, clone :256-276): a true deep copy, device data included;
    // full_collection selects the collector type of the copy (create_opt/full_model_clone, expose.h:447-470)
    region_model(const region_model& o, bool full_collection) { clone_from(o, full_collection); }
    region_model(const region_model& o) { clone_from(o, o.full_); }
    region_model& operator=(const region_model& o) {
        if (&o != this) clone_from(o, o.full_);
        return *this;
    }

    // ---- properties
    fixed_dt time_axis;
    size_t ncore = 0;
    interpolation_parameter ip_parameter;
    region_environment region_env;
    std::vector<state_t> initial_state;
    river_network rivers;

    shyft_hip_region* handle() const { return h_.get(); }
    // the device of each shard (one entry for an unsharded region)
    std::vector<int> shard_devices() const {
        std::vector<int> d(shyft_hip_region_shards(h_.get(), 0, nullptr, nullptr, nullptr));
        for (size_t k = 0; k < d.size(); ++k) shyft_hip_region_shards(h_.get(), k, &d[k], nullptr, nullptr);
        return d;
    }
    bool full_collection() const { return full_; }
    size_t size() const { return geo_.size(); }
    const std::vector<geo_cell_data>& cells_geo() const { return geo_; }
    std::vector<geo_cell_data> extract_geo_cell_data() const { return geo_; }
    size_t number_of_catchments() const { return cix_to_cid_.size(); }
    std::vector<int64_t> catchment_ids() const { return cix_to_cid_; }

    static state_t default_state() {
        if (Stack::id == SHYFT_HIP_PT_GS_K)  // gamma_snow::state() + kirchner::state() (gamma_snow.h:101-116, kirchner.h:131)
            return {0.4, 0.1, 30000.0, 1.26, 0.0, 0.0, 0.0, 0.0, 0.1};
        if (Stack::id == SHYFT_HIP_PT_SS_K)  // skaugen::state() (skaugen.h:122-124) + kirchner::state()
            return {4.077, 40.77, 0.0, 0.0, 0.0, 0.0, 0.0, 0.1};
        if (Stack::id == SHYFT_HIP_PT_HPS_K) {  // hbv_physical_snow::state() (hbv_physical_snow.h:135-146) + kirchner
            state_t s(Stack::n_state, 0.0);
            s[2] = 30000.0;
            s[Stack::state_q] = 0.1;
            return s;
        }
        if (Stack::id == SHYFT_HIP_PT_HS_K) {  // hbv_snow::state() undistributed (hbv_snow.h:74-99) + kirchner::state()
            state_t s(Stack::n_state, 0.0);
            s[Stack::state_q] = 0.1;
            return s;
        }
        state_t s(Stack::n_state, 0.0);  // hbv_stack::state(): snow undistributed, soil sm 0, tank uz 20 lz 10
        s[3] = 20.0;                    // (hbv_soil.h:28, hbv_tank.h:32)
        s[4] = 10.0;
        return s;
    }

    // ---- parameters (region_model.h:640-700)
    void set_region_parameter(const parameter_t& p) {
        check_param(p);
        region_parameter_ = p;
        params_dirty_ = true;
    }
    const parameter_t& get_region_parameter() const { return region_parameter_; }
    void set_catchment_parameter(int64_t cid, const parameter_t& p) {
        check_param(p);
        if (catchment_parameters_.find(cid) == catchment_parameters_.end()) {
            catchment_parameters_[cid] = p;
            params_dirty_ = true;
        }
        // else: the reference keeps the existing shared parameter untouched (region_model.h:664-667)
    }
    void update_catchment_parameter(int64_t cid, const parameter_t& p) {  // in-place edit of an existing override
        check_param(p);
        catchment_parameters_[cid] = p;
        params_dirty_ = true;
    }
    void remove_catchment_parameter(int64_t cid) {
        if (catchment_parameters_.erase(cid)) params_dirty_ = true;
    }
    bool has_catchment_parameter(int64_t cid) const { return catchment_parameters_.count(cid) != 0; }
    const parameter_t& get_catchment_parameter(int64_t cid) const {
        auto f = catchment_parameters_.find(cid);
        return f != catchment_parameters_.end() ? f->second : region_parameter_;
    }
    const parameter_t& cell_parameter(size_t i) const { return get_catchment_parameter(geo_.at(i).catchment_id()); }

    // ---- catchment filter (region_model.h:715-779)
    void set_catchment_calculation_filter(const std::vector<int64_t>& cids) {
        throw_if(shyft_hip_set_catchment_filter(h_.get(), cids.empty() ? nullptr : cids.data(), cids.size()), h_.get());
        catchment_filter_.clear();
        if (!cids.empty()) {
            catchment_filter_.assign(cix_to_cid_.size(), false);
            for (auto c : cids) catchment_filter_[cid_to_cix_.at(c)] = true;
        }
    }
    void set_calculation_filter(const std::vector<int64_t>& cids, const std::vector<int64_t>& rids) {
        std::set<int64_t> all(cids.begin(), cids.end());
        for (auto rid : rids)
            for (auto c : get_catchment_feeding_to_river(rid)) all.insert(c);
        set_catchment_calculation_filter(std::vector<int64_t>(all.begin(), all.end()));
    }
    std::set<int64_t> get_catchment_feeding_to_river(int64_t rid) const {
        std::set<int64_t> r;
        auto ups = rivers.all_upstreams_by_id(rid);
        ups.push_back(rid);
        for (const auto& g : geo_)
            if (valid_routing_id(g.routing.id) && std::find(ups.begin(), ups.end(), g.routing.id) != ups.end())
                r.insert(g.catchment_id());
        return r;
    }
    bool is_calculated(int64_t cid) const {
        auto f = cid_to_cix_.find(cid);
        if (f == cid_to_cix_.end()) throw std::runtime_error("region_model: no match for cid in map lookup");
        return catchment_filter_.empty() || catchment_filter_[f->second];
    }

    // ---- environment and interpolation (region_model.h:359-555)
    void initialize_cell_environment(const fixed_dt& ta) {
        if (ta.size() == 0 || ta.dt <= 0) throw std::runtime_error("region_model::run with invalid time_axis invoked");
        throw_if(shyft_hip_set_time_axis(h_.get(), ta.t, ta.dt, ta.size(), 0), h_.get());
        time_axis = ta;
        push_collection();
    }

    bool interpolate(const interpolation_parameter& ip, const region_environment& env, bool best_effort = true) {
        if (time_axis.size() == 0) throw std::runtime_error("region_model::interpolate: initialize_cell_environment first");
        ip_parameter = ip;
        region_env = env;
        bool ok = true;
        std::string first_error;
        auto guard = [&](auto&& f) {
            try {
                f();
            } catch (const std::exception& e) {
                ok = false;
                if (first_error.empty()) first_error = e.what();
            }
        };
        guard([&] {
            if (env.temperature.empty()) return;
            if (env.temperature.size() > 1 && !ip.use_idw_for_temperature) {  // region_model.h:463-467
                run_btk(env.temperature, ip.temperature);
                return;
            }
            const idw_temperature_parameter& t = ip.temperature_idw;
            run_idw(SHYFT_HIP_TEMPERATURE, env.temperature, t, t.default_temp_gradient, t.gradient_by_equation, 1.02);
        });
        guard([&] { run_idw(SHYFT_HIP_PRECIPITATION, env.precipitation, ip.precipitation, -0.006, false,
                            ip.precipitation.scale_factor); });
        guard([&] { run_idw(SHYFT_HIP_RADIATION, env.radiation, ip.radiation, -0.006, false, 1.02); });
        guard([&] { run_idw(SHYFT_HIP_WIND_SPEED, env.wind_speed, ip.wind_speed, -0.006, false, 1.02); });
        guard([&] { run_idw(SHYFT_HIP_REL_HUM, env.rel_hum, ip.rel_hum, -0.006, false, 1.02); });
        if (!best_effort && !ok) throw std::runtime_error(first_error);
        return ok;
    }
    bool run_interpolation(const interpolation_parameter& ip, const fixed_dt& ta, const region_environment& env,
                           bool best_effort = true) {
        initialize_cell_environment(ta);
        return interpolate(ip, env, best_effort);
    }
    bool is_cell_env_ts_ok() const {
        int ok = 0;
        throw_if(shyft_hip_forcing_ok(h_.get(), &ok), h_.get());
        return ok != 0;
    }

    // ---- run (region_model.h:578-597)
    void run_cells(size_t use_ncore = 0, int start_step = 0, int n_steps = 0) {
        if (use_ncore == 0) {
            if (ncore == 0) ncore = 4;
            use_ncore = ncore;
        } else if (use_ncore > 100 * ncore) {
            throw std::runtime_error(std::string("illegal parameter value: use_ncore(") + std::to_string(use_ncore) +
                                     std::string(" is more than 100 time available physical cores: ") +
                                     std::to_string(ncore));
        }
        if (!(time_axis.size() > 0)) throw std::runtime_error("region_model::run with invalid time_axis invoked");
        if (start_step < 0 || size_t(start_step + 1) > time_axis.size())
            throw std::runtime_error("region_model::run start_step must in range[0..n_steps-1>");
        if (n_steps < 0) throw std::runtime_error("region_model::run n_steps must be range[0..time-axis-steps]");
        if (size_t(start_step + n_steps) > time_axis.size())
            throw std::runtime_error("region_model::run start_step+n_steps must be within time-axis range");
        if (initial_state.size() != size()) get_states(initial_state);
        push_parameters();
        throw_if(shyft_hip_run_cells(h_.get(), use_ncore, start_step, n_steps), h_.get());
    }

    // ---- states (region_model.h:784-818)
    void get_states(std::vector<state_t>& end_states) const {
        std::vector<double> flat(size() * Stack::n_state);
        throw_if(shyft_hip_get_state(h_.get(), flat.data(), Stack::n_state), h_.get());
        end_states.assign(size(), state_t(Stack::n_state));
        for (size_t i = 0; i < size(); ++i)
            std::copy(flat.begin() + i * Stack::n_state, flat.begin() + (i + 1) * Stack::n_state, end_states[i].begin());
    }
    std::vector<state_t> current_state() const {
        std::vector<state_t> r;
        get_states(r);
        return r;
    }
    void set_states(const std::vector<state_t>& states) {
        if (states.size() != size()) throw std::runtime_error("Length of the state vector must equal number of cells");
        put_states(states);
        if (initial_state.size() != states.size()) initial_state = states;
    }
    // state_io_handler (api/api_state.h:99-146): model.state.extract_state / apply_state
    std::vector<state_with_id> extract_state(const std::vector<int64_t>& cids) const {
        return shyft_hip::host::extract_state(geo_, current_state(), cids);
    }
    std::vector<int64_t> apply_state(const std::vector<state_with_id>& s, const std::vector<int64_t>& cids) {
        auto st = current_state();
        auto missing = shyft_hip::host::apply_state(geo_, st, s, cids);
        put_states(st);  // cell.state = ... (initial_state is not touched, api_state.h:139)
        return missing;
    }
    void revert_to_initial_state() {
        if (initial_state.empty()) throw std::runtime_error("Initial state not yet established or set");
        set_states(initial_state);
    }
    // adjust_q (region_model.h:806-813, kirchner state adjust_q = q *= scale)
    void adjust_q(double q_scale, const std::vector<int64_t>& cids) {
        if (Stack::state_q < 0) {  // hbv: state::adjust_q scales soil sm, tank uz and lz (hbv_stack.h:191-194)
            auto s = current_state();
            for (size_t i = 0; i < size(); ++i)
                if (cids.empty() || std::find(cids.begin(), cids.end(), geo_[i].catchment_id()) != cids.end()) {
                    s[i][2] *= q_scale;
                    s[i][3] *= q_scale;
                    s[i][4] *= q_scale;
                }
            put_states(s);
            return;
        }
        auto s = current_state();
        for (size_t i = 0; i < size(); ++i)
            if (cids.empty() || std::find(cids.begin(), cids.end(), geo_[i].catchment_id()) != cids.end())
                s[i][Stack::state_q] *= q_scale;
        put_states(s);
    }

    // ---- state tuning to a wanted flow (region_model.h:626-637, core/model_state_tuning.h:35-120)
    // Scales the discharge state of the cells in `cids` (adjust_q) so that the average summed discharge over
    // steps [start_step, start_step+n_steps) equals wanted_flow_m3s; the scale is searched in
    // [s/scale_range, s*scale_range] around s = wanted/q_0 with find_min_single_variable. Each evaluation
    // restores the snapshot state, scales it, runs the filtered cells for n_steps on the device and sums
    // discharge there. On return the current state is the tuned one; the calculation filter is restored.
    q_adjust_result adjust_state_to_target_flow(double wanted_flow_m3s, const std::vector<int64_t>& cids,
                                                size_t start_step = 0, double scale_range = 3.0, double scale_eps = 1e-3,
                                                size_t max_iter = 300, size_t n_steps = 1) {
        std::vector<int64_t> old_filter;
        for (size_t c = 0; c < catchment_filter_.size(); ++c)
            if (catchment_filter_[c]) old_filter.push_back(cix_to_cid_[c]);
        q_adjust_result r;
        try {
            set_catchment_calculation_filter(cids);
            const std::vector<state_t> s0 = current_state();
            auto discharge = [&](double q_scale) {
                put_states(s0);
                adjust_q(q_scale, cids);
                run_cells(0, int(start_step), int(n_steps));
                double q_sum = 0.0;
                for (size_t i = start_step; i < start_step + n_steps; ++i)
                    q_sum += stat_value(0, cids, SHYFT_HIP_SCOPE_CATCHMENT, false, i);
                return q_sum / double(n_steps);
            };
            r.q_0 = discharge(1.0);
            double scale = wanted_flow_m3s / r.q_0;
            try {
                if (!std::isfinite(r.q_0)) throw std::runtime_error("the initial simulated discharge is nan");
                find_min_single_variable(
                    [&](double x) {
                        const double d = discharge(x) - wanted_flow_m3s;
                        return d * d;
                    },
                    scale, scale / scale_range, scale * scale_range, scale * scale_eps, long(max_iter));
            } catch (const std::exception& e) {
                r.diagnostics = std::string("failed to find solution within ") + std::to_string(max_iter) +
                                std::string(", exception was:") + e.what();
            }
            r.q_r = discharge(scale);
            put_states(s0);
            adjust_q(scale, cids);
        } catch (const std::exception& e) {
            r.diagnostics = std::string("Failed to tune_flow") + e.what();
        }
        set_catchment_calculation_filter(old_filter);
        return r;
    }

    // ---- collection (region_model.h:806-818)
    void set_state_collection(int64_t cid, bool on) {
        for (size_t i = 0; i < size(); ++i)
            if (cid == -1 || geo_[i].catchment_id() == cid) state_collection_[i] = on;
        push_collection();
    }
    void set_snow_sca_swe_collection(int64_t cid, bool on) {
        for (size_t i = 0; i < size(); ++i)
            if (cid == -1 || geo_[i].catchment_id() == cid) snow_collection_[i] = on;
        push_collection();
    }
    bool cell_collects_state(size_t i) const { return state_collection_.at(i); }
    bool cell_collects_snow(size_t i) const { return full_ || snow_collection_.at(i); }

    // ---- per-cell series views (cell.env_ts / cell.rc / cell.sc, core/cell_model.h:47-160)
    std::vector<double> cell_series(int series, size_t cell) const {
        size_t n = time_axis.size() + (series >= SHYFT_HIP_SERIES_STATE ? 1 : 0);
        std::vector<double> v(n);
        if (n) throw_if(shyft_hip_cell_series(h_.get(), series, cell, 0, n, v.data(), 0), h_.get());
        return v;
    }
    double cell_value(int series, size_t cell, size_t i) const {
        double v = 0;
        throw_if(shyft_hip_cell_series(h_.get(), series, cell, i, 1, &v, 0), h_.get());
        return v;
    }
    void set_cell_value(int var, size_t cell, size_t i, double v) {
        throw_if(shyft_hip_cell_series(h_.get(), SHYFT_HIP_SERIES_FORCING + var, cell, i, 1, &v, 1), h_.get());
    }
    void set_cell_forcing(int var, size_t cell, const std::vector<double>& v) {
        if (v.size() != time_axis.size()) throw std::runtime_error("cell env_ts: size differs from the time axis");
        throw_if(shyft_hip_cell_series(h_.get(), SHYFT_HIP_SERIES_FORCING + var, cell, 0, v.size(),
                                       const_cast<double*>(v.data()), 1),
                 h_.get());
    }

    // ---- statistics (core/cell_model.h:228-368, api/api.h:179-1597)
    // verify_cids_exist + is_match selection in cell order (cell_model.h:198-216)
    std::vector<size_t> select(const std::vector<int64_t>& ids, int scope) const {
        std::vector<size_t> sel;
        if (ids.empty()) {
            for (size_t i = 0; i < size(); ++i) sel.push_back(i);
            return sel;
        }
        if (scope == SHYFT_HIP_SCOPE_CELL_IX) {
            for (auto c : ids)
                if (c < 0 || c > int64_t(size()))
                    throw std::runtime_error(std::string("Supplied cell index reference ") + std::to_string(c) +
                                             " is ouside valid range 0 .." + std::to_string(size()));
        } else {
            for (auto c : ids)
                if (cid_to_cix_.count(c) == 0)
                    throw std::runtime_error(std::string("one or more supplied catchment_indexes does not exist:") +
                                             std::to_string(c));
        }
        for (size_t i = 0; i < size(); ++i)
            for (auto c : ids)
                if ((scope == SHYFT_HIP_SCOPE_CELL_IX && c == int64_t(i)) ||
                    (scope == SHYFT_HIP_SCOPE_CATCHMENT && geo_[i].catchment_id() == c)) {
                    sel.push_back(i);
                    break;
                }
        return sel;
    }
    size_t series_length(int series) const { return time_axis.size() + (series >= SHYFT_HIP_SERIES_STATE ? 1 : 0); }
    // sum_catchment_feature (weighted=false) / average_catchment_feature (weighted=true) as a series
    std::vector<double> stat_series(int series, const std::vector<int64_t>& ids, int scope, bool weighted) const {
        const size_t n = series_length(series);
        std::vector<double> r(n);
        throw_if(shyft_hip_statistics(h_.get(), series, ids.empty() ? nullptr : ids.data(), ids.size(), scope,
                                      weighted ? 1 : 0, 0, n, r.data()),
                 h_.get());
        return r;
    }
    double stat_value(int series, const std::vector<int64_t>& ids, int scope, bool weighted, size_t i) const {
        double r = 0;
        if (i >= series_length(series)) throw std::runtime_error("statistics: time step index out of range");
        throw_if(shyft_hip_statistics(h_.get(), series, ids.empty() ? nullptr : ids.data(), ids.size(), scope,
                                      weighted ? 1 : 0, i, 1, &r),
                 h_.get());
        return r;
    }
    // catchment_feature: the i'th value of every selected cell (cell_model.h:340-366)
    std::vector<double> stat_raster(int series, const std::vector<int64_t>& ids, int scope, size_t i) const {
        auto sel = select(ids, scope);
        std::vector<double> r;
        r.reserve(sel.size());
        for (auto c : sel) r.push_back(cell_value(series, c, i));
        return r;
    }
    // ae pot_ratio (api/api.h:1519-1566): 1 - exp(-3 q_mmh / ae_scale_factor) from the collected kirchner discharge
    std::vector<double> pot_ratio_series(const std::vector<int64_t>& ids, int scope) const {
        auto sel = select(ids, scope);
        const size_t n = time_axis.size() + 1;
        std::vector<double> r(n, 0.0);
        double sum_area = 0;
        for (auto c : sel) {
            auto q = cell_series(SHYFT_HIP_SERIES_STATE + 0, c);
            const double area = geo_[c].area(), sf = cell_parameter(c)[Stack::k_ae_scale];
            for (size_t t = 0; t < n; ++t) r[t] += pot_ratio(q[t], area, sf) * area;
            sum_area += area;
        }
        for (auto& x : r) x *= 1 / sum_area;
        return r;
    }
    std::vector<double> pot_ratio_raster(const std::vector<int64_t>& ids, int scope, size_t i) const {
        auto sel = select(ids, scope);
        std::vector<double> r;
        for (auto c : sel)
            r.push_back(pot_ratio(cell_value(SHYFT_HIP_SERIES_STATE + 0, c, i), geo_[c].area(),
                                  cell_parameter(c)[Stack::k_ae_scale]));
        return r;
    }
    double pot_ratio_value(const std::vector<int64_t>& ids, int scope, size_t i) const {
        auto sel = select(ids, scope);
        double r = 0, sum_area = 0;
        for (auto c : sel) {
            const double area = geo_[c].area();
            r += pot_ratio(cell_value(SHYFT_HIP_SERIES_STATE + 0, c, i), area, cell_parameter(c)[Stack::k_ae_scale]) * area;
            sum_area += area;
        }
        return r / sum_area;
    }
    // area statistics (api/api.h:183-288): kind 0 total, 1 forest, 2 glacier, 3 lake, 4 reservoir, 5 unspecified,
    // 6 snow_storage, 7 elevation (area-weighted mean z)
    double area_stat(int kind, const std::vector<int64_t>& ids, int scope) const {
        auto frac = [&](const geo_cell_data& g) {
            switch (kind) {
                case 1: return g.fractions.forest();
                case 2: return g.fractions.glacier();
                case 3: return g.fractions.lake();
                case 4: return g.fractions.reservoir();
                case 5: return g.fractions.unspecified();
                case 6: return g.fractions.snow_storage();
                default: return 1.0;
            }
        };
        double sum = 0, area_sum = 0;
        if (!ids.empty()) select(ids, scope);  // verify_cids_exist
        auto add = [&](const geo_cell_data& g) {
            if (kind == 7) {
                sum += g.mid_point().z * g.area();
                area_sum += g.area();
            } else {
                sum += g.area() * frac(g);
            }
        };
        if (ids.empty()) {
            for (const auto& g : geo_) add(g);
        } else if (kind == 0) {  // total_area honours the scope (api.h:183-197)
            for (auto c : ids)
                for (size_t j = 0; j < size(); ++j)
                    if ((scope == SHYFT_HIP_SCOPE_CELL_IX && c == int64_t(j)) ||
                        (scope == SHYFT_HIP_SCOPE_CATCHMENT && geo_[j].catchment_id() == c))
                        add(geo_[j]);
        } else {  // the other area statistics match on catchment id (api.h:198-288)
            for (auto c : ids)
                for (const auto& g : geo_)
                    if (int(g.catchment_id()) == c) add(g);
        }
        return kind == 7 ? sum / area_sum : sum;
    }
    // catchment_discharges / catchment_charges (region_model.h:873-905): [catchment][t], calculated catchments only
    std::vector<std::vector<double>> catchment_sums(int series) const {
        const size_t C = number_of_catchments(), T = time_axis.size();
        std::vector<double> flat(C * T);
        throw_if(shyft_hip_catchment_sums(h_.get(), series, 0, T, flat.data(), 0), h_.get());
        std::vector<std::vector<double>> r(C);
        for (size_t c = 0; c < C; ++c) {
            if (catchment_filter_.empty() || catchment_filter_[c]) r[c].assign(flat.begin() + c * T, flat.begin() + (c + 1) * T);
            else r[c].assign(T, 0.0);
        }
        return r;
    }
    // per-catchment sums of value x cell area: [catchment][t], calculated catchments only (others 0)
    std::vector<std::vector<double>> catchment_area_sums(int series) const {
        const size_t C = number_of_catchments(), T = time_axis.size();
        std::vector<double> flat(C * T);
        throw_if(shyft_hip_catchment_area_sums(h_.get(), series, 0, T, flat.data(), 0), h_.get());
        std::vector<std::vector<double>> r(C);
        for (size_t c = 0; c < C; ++c) {
            if (catchment_filter_.empty() || catchment_filter_[c]) r[c].assign(flat.begin() + c * T, flat.begin() + (c + 1) * T);
            else r[c].assign(T, 0.0);
        }
        return r;
    }
    bool is_calculated_by_catchment_ix(size_t cix) const { return catchment_filter_.empty() || catchment_filter_.at(cix); }
    size_t cix_from_cid(int64_t cid) const {
        auto f = cid_to_cix_.find(cid);
        if (f == cid_to_cix_.end()) throw std::runtime_error("region_model: no match for cid in map lookup");
        return f->second;
    }
    size_t catchment_ix_of_cell(size_t i) const { return cid_to_cix_.at(geo_.at(i).catchment_id()); }

    // ---- parameter ensembles (shyft_hip_ensemble_run): every member runs the calculated cells over the whole
    // time axis from the CURRENT state with its own region parameter vector; the model's own state/responses
    // are untouched. collect_snow adds the snow sca/swe series (2, 3).
    void ensemble_run(const std::vector<parameter_t>& members, bool collect_snow) {
        if (members.empty()) throw std::runtime_error("ensemble_run: no members");
        const size_t w = members[0].size();
        std::vector<double> flat;
        flat.reserve(members.size() * w);
        for (const auto& p : members) {
            check_param(p);
            if (p.size() != w) throw std::runtime_error(Stack::param_error);
            flat.insert(flat.end(), p.begin(), p.end());
        }
        throw_if(shyft_hip_ensemble_run(h_.get(), flat.data(), members.size(), w, 0, int(time_axis.size()),
                                        collect_snow ? SHYFT_HIP_COLLECT_DISCHARGE_SNOW : SHYFT_HIP_COLLECT_DISCHARGE),
                 h_.get());
        ens_members_ = members.size();
    }
    // [member][catchment][t] sums (area_weighted: of value x cell area) of the last ensemble run
    std::vector<double> ensemble_sums(int series, bool area_weighted) const {
        const size_t C = number_of_catchments(), T = time_axis.size();
        std::vector<double> flat(ens_members_ * C * T);
        throw_if(shyft_hip_ensemble_sums(h_.get(), series, area_weighted ? 1 : 0, 0, T, flat.data(), 0), h_.get());
        return flat;
    }

    // ---- routing (region_model.h:424-440, 906-949; core/routing.h)
    void connect_catchment_to_river(int64_t cid, int64_t rid) {
        if (cid_to_cix_.find(cid) == cid_to_cix_.end())
            throw std::runtime_error(std::string("specified catchment id=") + std::to_string(cid) + std::string(" not found"));
        if (valid_routing_id(rid)) rivers.check_rid(rid);
        for (auto& g : geo_)
            if (g.catchment_id() == cid) g.routing.id = rid;
        routing_dirty_ = true;
    }
    void set_cell_routing(size_t i, int64_t rid, double distance) {
        geo_.at(i).routing = routing_info(rid, distance);
        routing_dirty_ = true;
    }
    bool has_routing() const {
        for (const auto& g : geo_)
            if (valid_routing_id(g.routing.id)) return true;
        return false;
    }
    // the three river flows; on a model without routing they are 0-series on the time axis
    std::vector<double> river_output_flow_m3s(int64_t rid) const { return routed(rid, 2); }
    std::vector<double> river_upstream_inflow_m3s(int64_t rid) const { return routed(rid, 1); }
    std::vector<double> river_local_inflow_m3s(int64_t rid) const { return routed(rid, 0); }

  private:
    std::shared_ptr<shyft_hip_region> h_;
    std::vector<geo_cell_data> geo_;
    bool full_ = true;
    parameter_t region_parameter_;
    std::map<int64_t, parameter_t> catchment_parameters_;
    std::vector<double> uploaded_params_;
    std::vector<int32_t> uploaded_set_ix_;
    bool params_dirty_ = true;
    std::vector<int64_t> cix_to_cid_;
    std::map<int64_t, size_t> cid_to_cix_;
    std::vector<bool> catchment_filter_;
    std::vector<bool> state_collection_, snow_collection_;
    mutable bool routing_dirty_ = true;
    size_t ens_members_ = 0;

    static double pot_ratio(double q_m3s, double area_m2, double scale_factor) {
        const double water_level = q_m3s * (3600.0 * 1000.0) / area_m2;  // m3s_to_mmh (unit_conversion.h:12-15)
        return 1.0 - std::exp(-water_level * 3.0 / scale_factor);       // calc_pot_ratio (actual_evapotranspiration.h:33-35)
    }

    void check_param(const parameter_t& p) const {
        const bool has_snow_dist = Stack::id == SHYFT_HIP_HBV_STACK || Stack::id == SHYFT_HIP_PT_HS_K;
        const bool hps = Stack::id == SHYFT_HIP_PT_HPS_K;  // + gm.direct_response + distribution
        if (p.size() != Stack::n_param && !(has_snow_dist && p.size() == Stack::n_param + 17) &&
            !(hps && p.size() == Stack::n_param + 18))
            throw std::runtime_error(Stack::param_error);
    }

    void push_geo() {
        const size_t N = geo_.size();
        std::vector<double> g(11 * N), rd(N);
        std::vector<int64_t> rid(N);
        cix_to_cid_.clear();
        cid_to_cix_.clear();
        for (size_t i = 0; i < N; ++i) {
            geo_[i].to_io11(&g[11 * i]);
            rid[i] = geo_[i].routing.id;
            rd[i] = geo_[i].routing.distance;
            const int64_t cid = geo_[i].catchment_id();
            if (cid_to_cix_.find(cid) == cid_to_cix_.end()) {  // update_ix_to_id_mapping (region_model.h:236-252)
                cid_to_cix_[cid] = cix_to_cid_.size();
                cix_to_cid_.push_back(cid);
            }
        }
        throw_if(shyft_hip_set_geo(h_.get(), g.data(), rid.data(), rd.data()), h_.get());
    }

    // region parameter = set 0, catchment overrides = sets 1..; one set index per cell
    void push_parameters() {
        const size_t w = region_parameter_.size();
        std::vector<double> flat(region_parameter_);
        std::map<int64_t, int32_t> set_of;
        int32_t k = 1;
        for (const auto& kv : catchment_parameters_) {
            if (kv.second.size() != w) throw std::runtime_error(Stack::param_error);
            flat.insert(flat.end(), kv.second.begin(), kv.second.end());
            set_of[kv.first] = k++;
        }
        std::vector<int32_t> ix(size(), 0);
        for (size_t i = 0; i < size(); ++i) {
            auto f = set_of.find(geo_[i].catchment_id());
            if (f != set_of.end()) ix[i] = f->second;
        }
        if (!params_dirty_ && flat == uploaded_params_ && ix == uploaded_set_ix_) return;
        throw_if(shyft_hip_set_parameters(h_.get(), flat.data(), flat.size() / w, w, ix.data()), h_.get());
        uploaded_params_.swap(flat);
        uploaded_set_ix_.swap(ix);
        params_dirty_ = false;
    }

    void put_states(const std::vector<state_t>& states) {
        std::vector<double> flat;
        flat.reserve(size() * Stack::n_state);
        for (const auto& s : states) {
            if (s.size() != Stack::n_state) throw std::runtime_error("state: wrong number of state values");
            flat.insert(flat.end(), s.begin(), s.end());
        }
        throw_if(shyft_hip_set_state(h_.get(), flat.data(), Stack::n_state), h_.get());
    }

    void push_collection() {
        bool any_state = std::find(state_collection_.begin(), state_collection_.end(), true) != state_collection_.end();
        bool any_snow = std::find(snow_collection_.begin(), snow_collection_.end(), true) != snow_collection_.end();
        int mode = full_ ? SHYFT_HIP_COLLECT_ALL : (any_snow ? SHYFT_HIP_COLLECT_DISCHARGE_SNOW : SHYFT_HIP_COLLECT_DISCHARGE);
        throw_if(shyft_hip_set_collection(h_.get(), mode, any_state ? 1 : 0), h_.get());
    }

    void run_idw(int var, const std::vector<geo_point_ts>& src, const idw_parameter& p, double gradient, bool by_eq,
                 double scale) {
        if (src.empty()) return;
        const size_t S = src.size(), T = time_axis.size();
        std::vector<double> xyz(3 * S), vals(T * S);
        for (size_t s = 0; s < S; ++s) {
            xyz[3 * s] = src[s].mid_point.x;
            xyz[3 * s + 1] = src[s].mid_point.y;
            xyz[3 * s + 2] = src[s].mid_point.z;
            auto v = average_values(src[s].ts, time_axis);
            for (size_t t = 0; t < T; ++t) vals[t * S + s] = v[t];
        }
        const double prm[7] = {double(p.max_members), p.max_distance, p.distance_measure_factor, p.zscale,
                               gradient, by_eq ? 1.0 : 0.0, scale};
        throw_if(shyft_hip_interpolate(h_.get(), var, S, xyz.data(), vals.data(), 0, T, prm), h_.get());
    }

    // btk::btk_interpolation over the device (bayesian_kriging.h:280-402), sources averaged onto the axis
    void run_btk(const std::vector<geo_point_ts>& src, const btk_parameter& p) {
        const size_t S = src.size(), T = time_axis.size();
        std::vector<double> xyz(3 * S), vals(T * S), prior(T), prm(5);
        for (size_t s = 0; s < S; ++s) {
            xyz[3 * s] = src[s].mid_point.x;
            xyz[3 * s + 1] = src[s].mid_point.y;
            xyz[3 * s + 2] = src[s].mid_point.z;
            auto v = average_values(src[s].ts, time_axis);
            for (size_t t = 0; t < T; ++t) vals[t * S + s] = v[t];
        }
        for (size_t t = 0; t < T; ++t) prior[t] = p.temperature_gradient(time_axis.period(t));
        p.as_abi(prm.data());
        throw_if(shyft_hip_interpolate_btk(h_.get(), S, xyz.data(), vals.data(), 0, T, prior.data(), prm.data()),
                 h_.get());
    }

    // routing::model over the device (routing.h:239-387): which = 0 local_inflow, 1 upstream_inflow, 2 output_m3s
    std::vector<double> routed(int64_t rid, int which) const {
        const size_t T = time_axis.size();
        if (!has_routing()) return std::vector<double>(T, 0.0);
        rivers.check_rid(rid);
        // routing groups: cells sharing (river, UHG length, alpha, beta) (routing.h:326-330)
        std::vector<uhg_group> groups;
        std::vector<int32_t> group_of(size(), -1);
        std::map<std::tuple<int64_t, int, double, double>, size_t> key_to_group;
        for (size_t i = 0; i < size(); ++i) {
            const auto& g = geo_[i];
            if (!valid_routing_id(g.routing.id)) continue;
            // every cell routed to the river counts, whatever the catchment calculation filter says:
            // routing::model::local_inflow (routing.h:345-350) iterates all cells; a filtered-out cell
            // contributes the response series it holds (the last run that included it), as in the reference
            rivers.check_rid(g.routing.id);  // routing::model::verify_cell_river_connections (routing.h:313-320)
            const auto& p = cell_parameter(i);
            const double velocity = p[Stack::k_routing], alpha = p[Stack::k_routing + 1], beta = p[Stack::k_routing + 2];
            const int n_steps = uhg_steps(g.routing.distance, velocity, time_axis.dt);
            auto key = std::make_tuple(g.routing.id, n_steps, alpha, beta);
            auto f = key_to_group.find(key);
            if (f == key_to_group.end()) {
                f = key_to_group.emplace(key, groups.size()).first;
                groups.push_back(uhg_group{g.routing.id, make_uhg_from_gamma(n_steps, alpha, beta), {}});
            }
            group_of[i] = int32_t(f->second);
        }
        const size_t G = groups.size();
        std::vector<double> sums(G * T);
        throw_if(shyft_hip_set_routing_groups(h_.get(), group_of.data(), G), h_.get());
        if (G) throw_if(shyft_hip_routing_group_sums(h_.get(), 0, T, sums.data(), 0), h_.get());
        // rivers indexed in ascending id (the rid_map order)
        std::vector<int64_t> ids;
        std::map<int64_t, int32_t> index_of;
        for (const auto& kv : rivers.rid_map) {
            index_of[kv.first] = int32_t(ids.size());
            ids.push_back(kv.first);
        }
        const size_t R = ids.size();
        std::vector<std::vector<double>> rw(R);
        size_t max_len = 1;
        for (size_t r = 0; r < R; ++r) {
            rw[r] = rivers.rid_map.at(ids[r]).uhg(time_axis.dt);
            max_len = std::max(max_len, rw[r].size());
        }
        for (const auto& g : groups) max_len = std::max(max_len, g.w.size());
        std::vector<double> gw(G * max_len, 0.0), rwf(R * max_len, 0.0);
        std::vector<int32_t> glen(G), griver(G), rlen(R), rdown(R);
        for (size_t k = 0; k < G; ++k) {
            std::copy(groups[k].w.begin(), groups[k].w.end(), gw.begin() + k * max_len);
            glen[k] = int32_t(groups[k].w.size());
            griver[k] = index_of.at(groups[k].rid);
        }
        for (size_t r = 0; r < R; ++r) {
            std::copy(rw[r].begin(), rw[r].end(), rwf.begin() + r * max_len);
            rlen[r] = int32_t(rw[r].size());
            const int64_t ds = rivers.rid_map.at(ids[r]).downstream_id;
            rdown[r] = valid_routing_id(ds) ? index_of.at(ds) : -1;
        }
        std::vector<double> local(R * T), up(R * T), out(R * T);
        throw_if(shyft_hip_route(-1, G, T, sums.data(), 0, gw.data(), glen.data(), griver.data(), R, rwf.data(),
                                 rlen.data(), rdown.data(), max_len, local.data(), up.data(), out.data(), 0),
                 nullptr);
        const auto& sel = which == 0 ? local : (which == 1 ? up : out);
        const size_t r = size_t(index_of.at(rid));
        return std::vector<double>(sel.begin() + r * T, sel.begin() + (r + 1) * T);
    }

    void clone_from(const region_model& o, bool full_collection) {
        shyft_hip_region* h = nullptr;
        throw_if(shyft_hip_region_clone(o.h_.get(), &h), nullptr);
        h_.reset(h, shyft_hip_region_destroy);
        geo_ = o.geo_;
        full_ = full_collection;
        region_parameter_ = o.region_parameter_;
        catchment_parameters_ = o.catchment_parameters_;
        params_dirty_ = true;
        cix_to_cid_ = o.cix_to_cid_;
        cid_to_cix_ = o.cid_to_cix_;
        catchment_filter_ = o.catchment_filter_;
        state_collection_ = o.state_collection_;
        snow_collection_ = o.snow_collection_;
        time_axis = o.time_axis;
        ncore = o.ncore;
        ip_parameter = o.ip_parameter;
        region_env = o.region_env;
        initial_state = o.initial_state;
        rivers = o.rivers;
        if (full_ != o.full_) push_collection();
    }
};

}  // namespace shyft_hip::host
