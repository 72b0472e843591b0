// pt_hps_k cell kernel for gfx950.
//
// region_model::run_cells -> cell::run -> pt_hps_k::run (core/region_model.h:578-597,
// core/pt_hps_k_cell_model.h:236-294, core/pt_hps_k.h:203-300) for every cell in ONE launch: lane =
// cell, the time loop inside the kernel, the hbv_physical_snow quantile bins (sp, sw, albedo,
// iso_pot_energy) and kirchner q in registers, forcing read [step][cell] and the collector series
// written [series][step][cell].
//
// Per step: p_corr -> hbv_physical_snow (energy balance per bin) -> glacier melt on the post-step sca ->
// Priestley-Taylor -> actual evapotranspiration -> kirchner (dopri5, shared with pt_gs_k) -> total
// discharge / charge. 40 B of forcing in (wind speed is read: the snow energy balance uses it) and 16 B
// of discharge/charge out per cell-step.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device/stream.h"
#include "../device/hps_dev.h"
#include "../device/pt_dev.h"
#include "../device/ptgsk_dev.h"
#include "../include_internal/kernels.h"

using namespace shyft_dev;

namespace {

// forcing loads / response stores with the nontemporal hint (device/stream.h). r06, 1M cells, the year:
// 63.3 -> 62.2 ms per 730-step chunk (profiles/r06/pthsk_pthpsk_nt_variants.txt), bit-exact
#ifndef SHYFT_PTHPSK_NT
#define SHYFT_PTHPSK_NT 1
#endif
constexpr bool STREAM_NT = SHYFT_PTHPSK_NT != 0;

constexpr int BLOCK = 256;

// occupancy target (waves per SIMD; variant builds override with -DSHYFT_PTHPSK_WAVES=N): per-lane parameter rows
#ifndef SHYFT_PTHPSK_WAVES
#define SHYFT_PTHPSK_WAVES 2  // measured: compiler choice (1) 151 ms, 2: 91, 3: 123
#endif
constexpr int WAVES_UNIFORM = 3;  // the uniform-parameter instance; measured: 2: 93.4, 3: 85.0 ms per chunk (per-lane rows at 2: 91.0)

// UNIFORM: every cell uses parameter set 0 (the parameter row wave-uniform, in SGPRs instead of VGPRs)
template <bool UNIFORM>
__global__ __launch_bounds__(BLOCK)
__attribute__((amdgpu_waves_per_eu(UNIFORM ? WAVES_UNIFORM : SHYFT_PTHPSK_WAVES, UNIFORM ? WAVES_UNIFORM : SHYFT_PTHPSK_WAVES)))
void pthpsk_run_kernel(const pthpsk_kargs a) {
    const int cell = blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= a.n_cells) return;
    if (a.active && !a.active[cell]) return;
    const size_t N = (size_t)a.n_cells;
    const size_t NF = a.fcol ? (size_t)a.f_cols : N;
    const size_t fcl = a.fcol ? (size_t)a.fcol[cell] : (size_t)cell;
    const double* __restrict__ P = UNIFORM ? a.params : a.params + (size_t)a.set_ix[cell] * PTHPSK_NP;

    const double dt_us = a.dt_us;
    const double dts = dt_us / 1e6;  // to_seconds(dt)
    hps_par hp;
    hp.nb = (int)P[PP_NB];
#pragma unroll
    for (int i = 0; i < MB; ++i) {
        hp.s[i] = P[PP_S0 + i];
        hp.I[i] = P[PP_I0 + i];
    }
    hp.tx = P[PP_TX];
    hp.lw = P[PP_LW];
    hp.cfr = P[PP_CFR];
    hp.wind_scale = P[PP_WIND_SCALE];
    hp.wind_const = P[PP_WIND_CONST];
    hp.surface_magnitude = P[PP_SURFACE_MAGNITUDE];
    hp.max_albedo = P[PP_MAX_ALBEDO];
    hp.min_albedo = P[PP_MIN_ALBEDO];
    hp.snowfall_reset_depth = P[PP_SNOWFALL_RESET_DEPTH];
    hp.iso = fabs(P[PP_ISO]) < 0.0001 ? false : true;  // pt_hps_k.h:83
    {
        const double albedo_range = hp.max_albedo - hp.min_albedo;
        const double dt_in_days = dts / 86400.0;
        hp.slow_decay = (0.5 * albedo_range * dt_in_days / P[PP_SLOW_DECAY_RATE]);
        hp.fast_decay = dpow(2.0, -dt_in_days / P[PP_FAST_DECAY_RATE]);
        hp.BB0 = 0.98 * 5.670373e-8 * dpow(273.15, 4.0);
    }
    const double kc1 = P[PP_C1], kc2 = P[PP_C2], kc3 = P[PP_C3];
    const double ae_scale = P[PP_AE_SCALE], p_corr = P[PP_PCORR], dtf = P[PP_DTF];
    const double pt_albedo = P[PP_PT_ALBEDO], pt_alpha = P[PP_PT_ALPHA];
    const double gm_direct = P[PP_GM_DIRECT];
    const double gm_routed = 1 - gm_direct;

    const double* __restrict__ cc = a.cellc;  // pt_hps_k.h:233-242 (same rows as pt_gs_k)
    const double glacier_fraction = cc[PC_GLACIER * N + cell];
    const double snow_storage_fraction = cc[PC_SNOW_STORAGE * N + cell];
    const double kirchner_routed_prec = cc[PC_KIRCHNER_ROUTED_PREC * N + cell];
    const double direct_response_fraction = cc[PC_DIRECT_RESPONSE * N + cell];
    const double kirchner_fraction = cc[PC_KIRCHNER_FRACTION * N + cell];
    const double cell_area_m2 = cc[PC_AREA * N + cell];
    const double glacier_area_m2 = cc[PC_GLACIER_AREA * N + cell];
    const double mmh_to_m3s_scale_factor = 1 / (3600.0 * 1000.0);

    double* __restrict__ st = a.state;
    double swe = st[PPS_SWE * N + cell], sca = st[PPS_SCA * N + cell], surface_heat = st[PPS_SURFACE_HEAT * N + cell];
    double nb_state = st[PPS_NB * N + cell];
    // the state holds nb_state bins (the reference's vectors); the rest read as zero, as the oracle's padding
    const int nbs = (int)nb_state;
    double sp[MB], sw[MB], alb[MB], iso[MB];
#pragma unroll
    for (int i = 0; i < MB; ++i) {
        sp[i] = i < nbs ? st[(PPS_SP0 + i) * N + cell] : 0.0;
        sw[i] = i < nbs ? st[(PPS_SW0 + i) * N + cell] : 0.0;
        alb[i] = i < nbs ? st[(PPS_ALB0 + i) * N + cell] : 0.0;
        iso[i] = i < nbs ? st[(PPS_ISO0 + i) * N + cell] : 0.0;
    }
    double q = st[PPS_KIRCHNER_Q * N + cell];
    // state.hps.distribute(parameter.hps, false) (pt_hps_k.h:236, hbv_physical_snow.h:156-164): only on a
    // bin-count mismatch, and then albedo / iso_pot_energy are re-sized to 0.4 / 0.0
    if ((int)nb_state != hp.nb) {
        hbv_snow_par dp;
        dp.nb = hp.nb;
#pragma unroll
        for (int i = 0; i < MB; ++i) {
            dp.s[i] = hp.s[i];
            dp.I[i] = hp.I[i];
        }
        dp.lw = hp.lw;
        hbv_distribute(dp, sp, sw, swe, sca);
#pragma unroll
        for (int i = 0; i < MB; ++i) {
            alb[i] = i < hp.nb ? 0.4 : 0.0;
            iso[i] = 0.0;
        }
        nb_state = (double)hp.nb;
    }
    int32_t err = 0;

    const size_t TW = (size_t)a.win_len;
    const double* __restrict__ f_temp = a.forcing + (size_t)FV_TEMPERATURE * TW * NF;
    const double* __restrict__ f_prec = a.forcing + (size_t)FV_PRECIPITATION * TW * NF;
    const double* __restrict__ f_ws = a.forcing + (size_t)FV_WIND_SPEED * TW * NF;
    const double* __restrict__ f_rh = a.forcing + (size_t)FV_REL_HUM * TW * NF;
    const double* __restrict__ f_rad = a.forcing + (size_t)FV_RADIATION * TW * NF;
    double* __restrict__ R = a.resp;
    const size_t RS = TW * N;
    double* __restrict__ SS = a.state_series;
    const size_t SSS = (TW + 1) * N;

    // state_collector::collect of state.scale_snow(snow_storage_fraction) (pt_hps_k_cell_model.h:213-228,
    // pt_hps_k.h:178-182: only swe is scaled)
    auto collect_state = [&](size_t wi) {
        const size_t o = wi * N + cell;
        SS[PPC_KIRCHNER * SSS + o] = cell_area_m2 * q * mmh_to_m3s_scale_factor;
        SS[PPC_SCA * SSS + o] = sca;
        SS[PPC_SWE * SSS + o] = swe * snow_storage_fraction;
        SS[PPC_SURFACE_HEAT * SSS + o] = surface_heat;
#pragma unroll
        for (int i = 0; i < MB; ++i) {
            SS[(PPC_SP0 + i) * SSS + o] = sp[i];
            SS[(PPC_SW0 + i) * SSS + o] = sw[i];
            SS[(PPC_ALB0 + i) * SSS + o] = alb[i];
            SS[(PPC_ISO0 + i) * SSS + o] = iso[i];
        }
    };

    const int i_end = a.step0 + a.n_steps;
    for (int i = a.step0; i < i_end; ++i) {
        const size_t wi = (size_t)(i - a.win0);
        const size_t fo = wi * N + cell;
        const size_t ff = wi * NF + fcl;
        const double temp = stream_ld<STREAM_NT>(&f_temp[ff]);
        const double rad = stream_ld<STREAM_NT>(&f_rad[ff]);
        const double rel_hum = stream_ld<STREAM_NT>(&f_rh[ff]);
        const double prec = stream_ld<STREAM_NT>(&f_prec[ff]) * p_corr;
        const double wind_speed = stream_ld<STREAM_NT>(&f_ws[ff]);
        if (SS) collect_state(wi);
        double r_sca, r_storage;
        const double snow_outflow = hps_step(hp, sp, sw, alb, iso, swe, sca, surface_heat, dt_us, dts, temp, rad, prec,
                                             wind_speed, rel_hum, r_sca, r_storage, err);
        const double sca_area = cell_area_m2 * sca;
        double gm_melt_m3s = 0.0;
        if (!(glacier_area_m2 <= sca_area || temp <= 0.0))
            gm_melt_m3s = dtf * temp * (glacier_area_m2 - sca_area) * (0.001 / 86400.0);
        double ae_exp;  // actual_evapotranspiration's exp, evaluated beside Priestley-Taylor's (pt_pot_evap_exp)
        const double pot_evap = pt_pot_evap_exp<true>(pt_albedo, pt_alpha, temp, rad, rel_hum, -q * 3.0 / ae_scale, ae_exp) * 3600.0;
        const double ae = pot_evap * (1.0 - ae_exp) * (1.0 - smax(sca, glacier_fraction));
        const double gm_mmh = gm_melt_m3s / (mmh_to_m3s_scale_factor * cell_area_m2);
        double q_avg;
        if (!kirchner_step<true>(q, q_avg, snow_outflow * snow_storage_fraction + prec * kirchner_routed_prec + gm_routed * gm_mmh,
                           ae, a.t1_hours, kc1, kc2, kc3))
            err = ERR_KIRCHNER_MAX_ITER;
        const double total_discharge = smax(0.0, prec - ae) * direct_response_fraction + gm_direct * gm_mmh +
                                       q_avg * kirchner_fraction;
        const double charge_m3s = +(cell_area_m2 * prec * mmh_to_m3s_scale_factor) -
                                  (cell_area_m2 * ae * mmh_to_m3s_scale_factor) + gm_melt_m3s -
                                  (cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor);
        // all_response_collector of response.scale_snow(snow_storage_fraction) (pt_hps_k_cell_model.h:82-91,
        // pt_hps_k.h:196-202): hps_outflow is collected in mm/h, as the reference does
        stream_st<STREAM_NT>(&R[PR_AVG_DISCHARGE * RS + fo], cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor);
        stream_st<STREAM_NT>(&R[PR_CHARGE_M3S * RS + fo], charge_m3s);
        if (a.collect >= 1) {
            R[PR_SNOW_SCA * RS + fo] = r_sca;
            R[PR_SNOW_SWE * RS + fo] = r_storage * snow_storage_fraction;
        }
        if (a.collect >= 2) {
            R[PR_SNOW_OUTFLOW * RS + fo] = snow_outflow * snow_storage_fraction;
            R[PR_GLACIER_MELT * RS + fo] = gm_melt_m3s;
            R[PR_AE_OUTPUT * RS + fo] = ae;
            R[PR_PE_OUTPUT * RS + fo] = pot_evap;
        }
        if (SS && i + 1 == i_end) collect_state(wi + 1);
    }
    st[PPS_SWE * N + cell] = swe;
    st[PPS_SCA * N + cell] = sca;
    st[PPS_SURFACE_HEAT * N + cell] = surface_heat;
    st[PPS_NB * N + cell] = nb_state;
#pragma unroll
    for (int i = 0; i < MB; ++i) {
        st[(PPS_SP0 + i) * N + cell] = sp[i];
        st[(PPS_SW0 + i) * N + cell] = sw[i];
        st[(PPS_ALB0 + i) * N + cell] = alb[i];
        st[(PPS_ISO0 + i) * N + cell] = iso[i];
    }
    st[PPS_KIRCHNER_Q * N + cell] = q;
    if (err) a.err[cell] = err;
}

}  // namespace

hipError_t launch_pthpsk_run(const pthpsk_kargs& a, hipStream_t stream) {
    const int grid = (a.n_cells + BLOCK - 1) / BLOCK;
    if (grid == 0) return hipSuccess;
    if (a.uniform_params) hipLaunchKernelGGL((pthpsk_run_kernel<true>), dim3(grid), dim3(BLOCK), 0, stream, a);
    else hipLaunchKernelGGL((pthpsk_run_kernel<false>), dim3(grid), dim3(BLOCK), 0, stream, a);
    return hipGetLastError();
}
