// ORACLE — test infrastructure only (see common.hpp header).
//
// region.hpp: the region_model::run_cells scheduler (core/region_model.h:578-597,
// 972-1021) over pt_gs_k and hbv_stack cells (core/cell_model.h:112-160), plus cell
// statistics (core/cell_model.h:194-406).
#pragma once
#include <future>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"
#include "hbv.hpp"
#include "ptgsk.hpp"
#include "ptssk.hpp"
#include "pthsk.hpp"
#include "pthpsk.hpp"

namespace oracle {

struct ptgsk_cell {
    geo_cell_data geo;
    const pt_gs_k::parameter* parameter = nullptr;
    pt_gs_k::state state;
    // env_ts (cell_model.h:47-81): five [T] series per cell
    std::vector<double> temp, prec, ws, rh, rad;
    pt_gs_k::collectors col;

    // cell<...>::run specialisation (pt_gs_k_cell_model.h:215-262)
    void run(const fixed_dt& ta, int start_step, int n_steps) {
        if (parameter == nullptr) throw std::runtime_error("pt_gs_k::run with null parameter attempted");
        col.initialize(ta.size(), start_step, n_steps, geo.area);
        pt_gs_k::forcing_view fv{temp.data(), prec.data(), ws.data(), rh.data(), rad.data(), 1};
        pt_gs_k::run_pt_gs_k(geo, *parameter, ta, start_step, n_steps, fv, state, col);
    }
};

// hbv_stack cell (hbv_stack_cell_model.h:247-306)
struct hbv_cell {
    geo_cell_data geo;
    const hbv_stack::parameter* parameter = nullptr;
    hbv_stack::state state;
    std::vector<double> temp, prec, ws, rh, rad;
    hbv_stack::collectors col;
    void run(const fixed_dt& ta, int start_step, int n_steps) {
        if (parameter == nullptr) throw std::runtime_error("pt_hs_k::run with null parameter attempted");
        col.initialize(ta.size(), start_step, n_steps, geo.area);
        pt_gs_k::forcing_view fv{temp.data(), prec.data(), ws.data(), rh.data(), rad.data(), 1};
        hbv_stack::run_hbv_stack(geo, *parameter, ta, start_step, n_steps, fv, state, col);
    }
};

// pt_ss_k cell (pt_ss_k_cell_model.h:205-256)
struct ptssk_cell {
    geo_cell_data geo;
    const pt_ss_k::parameter* parameter = nullptr;
    pt_ss_k::state state;
    std::vector<double> temp, prec, ws, rh, rad;
    pt_ss_k::collectors col;
    void run(const fixed_dt& ta, int start_step, int n_steps) {
        if (parameter == nullptr) throw std::runtime_error("pt_ss_k::run with null parameter attempted");
        col.initialize(ta.size(), start_step, n_steps, geo.area);
        pt_gs_k::forcing_view fv{temp.data(), prec.data(), ws.data(), rh.data(), rad.data(), 1};
        pt_ss_k::run_pt_ss_k(geo, *parameter, ta, start_step, n_steps, fv, state, col);
    }
};

// pt_hs_k cell (pt_hs_k_cell_model.h:218-267)
struct pthsk_cell {
    geo_cell_data geo;
    const pt_hs_k::parameter* parameter = nullptr;
    pt_hs_k::state state;
    std::vector<double> temp, prec, ws, rh, rad;
    pt_hs_k::collectors col;
    void run(const fixed_dt& ta, int start_step, int n_steps) {
        if (parameter == nullptr) throw std::runtime_error("pt_hs_k::run with null parameter attempted");
        col.initialize(ta.size(), start_step, n_steps, geo.area);
        pt_gs_k::forcing_view fv{temp.data(), prec.data(), ws.data(), rh.data(), rad.data(), 1};
        pt_hs_k::run_pt_hs_k(geo, *parameter, ta, start_step, n_steps, fv, state, col);
    }
};

// pt_hps_k cell (pt_hps_k_cell_model.h:236-294)
struct pthpsk_cell {
    geo_cell_data geo;
    const pt_hps_k::parameter* parameter = nullptr;
    pt_hps_k::state state;
    std::vector<double> temp, prec, ws, rh, rad;
    pt_hps_k::collectors col;
    void run(const fixed_dt& ta, int start_step, int n_steps) {
        if (parameter == nullptr) throw std::runtime_error("pt_hps_k::run with null parameter attempted");
        col.initialize(ta.size(), start_step, n_steps, geo.area);
        pt_gs_k::forcing_view fv{temp.data(), prec.data(), ws.data(), rh.data(), rad.data(), 1};
        pt_hps_k::run_pt_hps_k(geo, *parameter, ta, start_step, n_steps, fv, state, col);
    }
};

template <class C, class P>
struct region_of {
    std::vector<C> cells;
    std::vector<P> params;
    std::vector<bool> catchment_filter;  // indexed by catchment_ix
    fixed_dt time_axis;
    size_t ncore = std::thread::hardware_concurrency();

    bool is_calculated_by_catchment_ix(size_t cix) const { return catchment_filter.empty() || catchment_filter[cix]; }

    // region_model::single_run (region_model.h:972-979)
    void single_run(int start_step, int n_steps, size_t ci) {
        auto& c = cells[ci];
        if (is_calculated_by_catchment_ix(c.geo.catchment_ix)) c.run(time_axis, start_step, n_steps);
    }

    // region_model::parallel_run (region_model.h:991-1021): use_ncore async
    // workers, each pulling ONE cell per mutex-protected pos++.
    void parallel_run(int start_step, int n_steps, size_t use_ncore) {
        size_t len = cells.size();
        if (len == 0) return;
        if (use_ncore == 0) throw std::runtime_error("parallel_run: use_ncore is zero ");
        std::vector<std::future<void>> calcs;
        std::mutex pos_mx;
        size_t pos = 0;
        for (size_t i = 0; i < use_ncore; ++i) {
            calcs.emplace_back(std::async(std::launch::async, [this, &pos, &pos_mx, len, start_step, n_steps]() {
                while (true) {
                    size_t ci;
                    {
                        std::lock_guard<std::mutex> lock(pos_mx);
                        if (pos < len) ci = pos++;
                        else break;
                    }
                    this->single_run(start_step, n_steps, ci);
                }
            }));
        }
        for (auto& f : calcs) f.get();
    }

    // region_model::run_cells (region_model.h:578-597)
    void run_cells(size_t use_ncore = 0, int start_step = 0, int n_steps = 0) {
        if (use_ncore == 0) {
            if (ncore == 0) ncore = 4;
            use_ncore = ncore;
        } else if (use_ncore > 100 * ncore) {
            throw std::runtime_error(std::string("illegal parameter value: use_ncore(") + std::to_string(use_ncore) +
                                     std::string(" is more than 100 time available physical cores: ") + std::to_string(ncore));
        }
        if (!(time_axis.size() > 0)) throw std::runtime_error("region_model::run with invalid time_axis invoked");
        if (start_step < 0 || size_t(start_step + 1) > time_axis.size())
            throw std::runtime_error("region_model::run start_step must in range[0..n_steps-1>");
        if (n_steps < 0) throw std::runtime_error("region_model::run n_steps must be range[0..time-axis-steps]");
        if (size_t(start_step + n_steps) > time_axis.size())
            throw std::runtime_error("region_model::run start_step+n_steps must be within time-axis range");
        parallel_run(start_step, n_steps, use_ncore);
    }
};

using ptgsk_region = region_of<ptgsk_cell, pt_gs_k::parameter>;
using hbv_region = region_of<hbv_cell, hbv_stack::parameter>;
using ptssk_region = region_of<ptssk_cell, pt_ss_k::parameter>;
using pthsk_region = region_of<pthsk_cell, pt_hs_k::parameter>;
using pthpsk_region = region_of<pthpsk_cell, pt_hps_k::parameter>;

}  // namespace oracle
