// pt_gs_k cell kernel for gfx950.
//
// region_model::run_cells -> cell::run -> run_pt_gs_k (core/region_model.h:578-597,
// core/pt_gs_k_cell_model.h:243-262, core/pt_gs_k.h:312-398) for every cell of
// the region in ONE launch: lane = cell, the time loop runs inside the kernel
// with the cell state held in registers, forcing read [step][cell] (coalesced,
// 512 B per wave per variable per step) and collector series written
// [series][step][cell].
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device/ptgsk_dev.h"
#include "../include_internal/kernels.h"

using namespace shyft_dev;

namespace {

// error codes written to err[cell]
constexpr int32_t ERR_KIRCHNER_MAX_ITER = 1;

__global__ __launch_bounds__(256) void ptgsk_run_kernel(const ptgsk_kargs a) {
    const int cell = blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= a.n_cells) return;
    if (a.active && !a.active[cell]) return;
    const size_t N = (size_t)a.n_cells;
    const double* __restrict__ P = a.params + (size_t)a.set_ix[cell] * PTGSK_NP;

    // per-cell constants (pt_gs_k.h:347-357)
    const double* __restrict__ cc = a.cellc;
    gs_cell gcell;
    gcell.forest_fraction = cc[PC_FOREST * N + cell];
    gcell.altitude = cc[PC_ALTITUDE * N + cell];
    gcell.cv2 = cc[PC_CV2 * N + cell];
    gcell.inv_cv2 = cc[PC_INV_CV2 * N + cell];
    const double glacier_fraction = cc[PC_GLACIER * N + cell];
    const double snow_storage_fraction = cc[PC_SNOW_STORAGE * N + cell];
    const double kirchner_routed_prec = cc[PC_KIRCHNER_ROUTED_PREC * N + cell];
    const double direct_response_fraction = cc[PC_DIRECT_RESPONSE * N + cell];
    const double kirchner_fraction = cc[PC_KIRCHNER_FRACTION * N + cell];
    const double cell_area_m2 = cc[PC_AREA * N + cell];
    const double glacier_area_m2 = cc[PC_GLACIER_AREA * N + cell];

    const double gm_direct = P[PK_GM_DIRECT];
    const double gm_routed = 1 - gm_direct;
    const double dtf = P[PK_DTF];
    const double p_corr = P[PK_PCORR];
    const double kc1 = P[PK_C1], kc2 = P[PK_C2], kc3 = P[PK_C3];
    const double mmh_to_m3s_scale_factor = 1 / (3600.0 * 1000.0);

    // state -> registers
    double* __restrict__ st = a.state;
    gs_state s;
    s.albedo = st[PS_ALBEDO * N + cell];
    s.lwc = st[PS_LWC * N + cell];
    s.surface_heat = st[PS_SURFACE_HEAT * N + cell];
    s.alpha = st[PS_ALPHA * N + cell];
    s.sdc_melt_mean = st[PS_SDC_MELT_MEAN * N + cell];
    s.acc_melt = st[PS_ACC_MELT * N + cell];
    s.iso_pot_energy = st[PS_ISO_POT_ENERGY * N + cell];
    s.temp_swe = st[PS_TEMP_SWE * N + cell];
    double q = st[PS_KIRCHNER_Q * N + cell];
    lgamma_cache lgc;
    int32_t err = 0;

    const size_t TW = (size_t)a.win_len;
    const double* __restrict__ f_temp = a.forcing + (size_t)FV_TEMPERATURE * TW * N;
    const double* __restrict__ f_prec = a.forcing + (size_t)FV_PRECIPITATION * TW * N;
    const double* __restrict__ f_ws = a.forcing + (size_t)FV_WIND_SPEED * TW * N;
    const double* __restrict__ f_rh = a.forcing + (size_t)FV_REL_HUM * TW * N;
    const double* __restrict__ f_rad = a.forcing + (size_t)FV_RADIATION * TW * N;
    double* __restrict__ R = a.resp;
    const size_t RS = TW * N;  // stride between response series
    double* __restrict__ SS = a.state_series;
    const size_t SSS = (TW + 1) * N;
    const int wed = (int)P[PK_WED];
    const int64_t snow_lo = (int64_t)((int)(P[PK_WED] * 24) - (int)(P[PK_NWD] * 24)) * 3600000000LL;
    const int64_t snow_hi = (int64_t)(int)(P[PK_WED] * 24) * 3600000000LL;

    auto collect_state = [&](size_t wi) {
        // state_collector::collect of state.scale_snow(snow_storage_fraction)
        SS[0 * SSS + wi * N + cell] = cell_area_m2 * q * mmh_to_m3s_scale_factor;
        SS[1 * SSS + wi * N + cell] = s.albedo;
        SS[2 * SSS + wi * N + cell] = s.lwc * snow_storage_fraction;
        SS[3 * SSS + wi * N + cell] = s.surface_heat;
        SS[4 * SSS + wi * N + cell] = s.alpha;
        SS[5 * SSS + wi * N + cell] = s.sdc_melt_mean;
        SS[6 * SSS + wi * N + cell] = s.acc_melt;
        SS[7 * SSS + wi * N + cell] = s.iso_pot_energy;
        SS[8 * SSS + wi * N + cell] = s.temp_swe * snow_storage_fraction;
    };

    const int i_end = a.step0 + a.n_steps;
    for (int i = a.step0; i < i_end; ++i) {
        const size_t wi = (size_t)(i - a.win0);
        const size_t fo = wi * N + cell;
        const double temp = f_temp[fo];
        const double rad = f_rad[fo];
        const double rel_hum = f_rh[fo];
        const double prec = f_prec[fo] * p_corr;
        const double wind_speed = f_ws[fo];
        if (SS) collect_state(wi);

        const bool start_melt = a.doy[i] == wed;
        const int64_t trel = a.t_rel_year_us[i];
        const bool snow_season = trel >= snow_lo && trel < snow_hi;
        double gs_sca, gs_storage, gs_outflow;
        gs_step(s, gs_sca, gs_storage, gs_outflow, start_melt, snow_season, a.dt_s, a.dt_us, P, gcell, temp, rad, prec,
                wind_speed, rel_hum, lgc);
        // glacier_melt::step (glacier_melt.h:47-52)
        const double sca_area = cell_area_m2 * gs_sca;
        double gm_melt_m3s = 0.0;
        if (!(glacier_area_m2 <= sca_area || temp <= 0.0))
            gm_melt_m3s = dtf * temp * (glacier_area_m2 - sca_area) * (0.001 / 86400.0);
        const double pot_evap = pt_pot_evap(P[PK_PT_ALBEDO], P[PK_PT_ALPHA], temp, rad, rel_hum) * 3600.0;
        const double ae = pot_evap * (1.0 - dexp(-q * 3.0 / P[PK_AE_SCALE])) * (1.0 - smax(gs_sca, glacier_fraction));
        const double gm_mmh = gm_melt_m3s / (mmh_to_m3s_scale_factor * cell_area_m2);
        double q_avg;
        if (!kirchner_step(q, q_avg, gs_outflow * snow_storage_fraction + prec * kirchner_routed_prec + gm_routed * gm_mmh,
                           ae, a.t1_hours, kc1, kc2, kc3))
            err = ERR_KIRCHNER_MAX_ITER;
        const double total_discharge = smax(0.0, prec - ae) * direct_response_fraction + gm_direct * gm_mmh +
                                       q_avg * kirchner_fraction;
        const double charge_m3s = +(cell_area_m2 * prec * mmh_to_m3s_scale_factor) -
                                  (cell_area_m2 * ae * mmh_to_m3s_scale_factor) + gm_melt_m3s -
                                  (cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor);
        // collectors (pt_gs_k_cell_model.h:80-89, 116-124) of response.scale_snow(snow_storage_fraction)
        R[0 * RS + fo] = cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor;
        R[1 * RS + fo] = charge_m3s;
        if (a.collect >= 1) {
            R[2 * RS + fo] = gs_sca;
            R[3 * RS + fo] = gs_storage * snow_storage_fraction;
        }
        if (a.collect >= 2) {
            R[4 * RS + fo] = cell_area_m2 * (gs_outflow * snow_storage_fraction) * mmh_to_m3s_scale_factor;
            R[5 * RS + fo] = gm_melt_m3s;
            R[6 * RS + fo] = ae;
            R[7 * RS + fo] = pot_evap;
        }
        if (SS && i + 1 == i_end) collect_state(wi + 1);
    }
    st[PS_ALBEDO * N + cell] = s.albedo;
    st[PS_LWC * N + cell] = s.lwc;
    st[PS_SURFACE_HEAT * N + cell] = s.surface_heat;
    st[PS_ALPHA * N + cell] = s.alpha;
    st[PS_SDC_MELT_MEAN * N + cell] = s.sdc_melt_mean;
    st[PS_ACC_MELT * N + cell] = s.acc_melt;
    st[PS_ISO_POT_ENERGY * N + cell] = s.iso_pot_energy;
    st[PS_TEMP_SWE * N + cell] = s.temp_swe;
    st[PS_KIRCHNER_Q * N + cell] = q;
    if (err) a.err[cell] = err;
}

}  // namespace

hipError_t launch_ptgsk_run(const ptgsk_kargs& a, hipStream_t stream) {
    const int block = 256;
    const int grid = (a.n_cells + block - 1) / block;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(ptgsk_run_kernel, dim3(grid), dim3(block), 0, stream, a);
    return hipGetLastError();
}
