// pt_hs_k cell kernel for gfx950.
//
// region_model::run_cells -> cell::run -> pt_hs_k::run (core/region_model.h:578-597,
// core/pt_hs_k_cell_model.h:218-267, core/pt_hs_k.h:199-283) for every cell in ONE launch:
// lane = cell, the time loop inside the kernel, the hbv_snow quantile bins and kirchner q in
// registers, forcing read [step][cell] (coalesced) and the collector series written
// [series][step][cell].
//
// Per step: p_corr -> hbv_snow -> glacier melt on the post-step sca -> Priestley-Taylor ->
// actual evapotranspiration (kirchner-q based, as pt_gs_k) -> kirchner (dopri5, shared with
// pt_gs_k) -> total discharge / charge. 40 B of forcing in (wind is read by the reference's
// accessor set but unused) and 16 B of discharge/charge out per cell-step.
// out-of-line exp / log with their constants from the SGPR table (device/special.h SHYFT_TABLE_CALLS): measured
// r05 (ms per 730-step chunk, year mean) pt_hs_k 34.3 -> 34.0; pt_gs_k keeps the default (80.9 -> 82.7 with the table)
#define SHYFT_TABLE_CALLS 1
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device/stream.h"
#include "../device/hbv_dev.h"
#include "../device/pt_dev.h"
#include "../device/ptgsk_dev.h"
#include "../include_internal/kernels.h"

using namespace shyft_dev;

namespace {

// forcing loads / response stores with the nontemporal hint (device/stream.h). r06, 1M cells, the year:
// 31.7 -> 31.5 ms per 730-step chunk (profiles/r06/pthsk_pthpsk_nt_variants.txt), bit-exact
#ifndef SHYFT_PTHSK_NT
#define SHYFT_PTHSK_NT 1
#endif
constexpr bool STREAM_NT = SHYFT_PTHSK_NT != 0;

constexpr int BLOCK = 256;

// occupancy target (waves per SIMD; variant builds override with -DSHYFT_PTHSK_WAVES=N): per-lane parameter rows
#ifndef SHYFT_PTHSK_WAVES
#define SHYFT_PTHSK_WAVES 3  // measured: compiler choice (1) 123 ms, 2: 70, 3: 64, 4: 70 per 730-step chunk
#endif
constexpr int WAVES_UNIFORM = 4;  // the uniform-parameter instance; measured (5 bins): 2: 69.2, 3: 55.3, 4: 50.6 ms per chunk

// UNIFORM: every cell uses parameter set 0 (the row, incl. the bin distribution, in SGPRs instead of VGPRs).
// NB: register capacity of the snow bins, HBV_MAX_BINS or 5 (as in the hbv_stack kernel: one parameter set of at
// most 5 bins and no state series; bins NB..7 of the state are written as 0, the oracle's padding).
// EXACT: the parameter set has exactly NB bins: the bin count is a compile-time constant (hbv_stack's kernel)
template <bool UNIFORM, int NB, bool EXACT = false>
__global__ __launch_bounds__(BLOCK)
__attribute__((amdgpu_waves_per_eu(UNIFORM ? WAVES_UNIFORM : SHYFT_PTHSK_WAVES, UNIFORM ? WAVES_UNIFORM : SHYFT_PTHSK_WAVES)))
void pthsk_run_kernel(const pthsk_kargs a) {
    const int cell = blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= a.n_cells) return;
    if (a.active && !a.active[cell]) return;
    const size_t N = (size_t)a.n_cells;
    // forcing column: the lane itself, or the shared cell of a parameter-ensemble lane
    const size_t NF = a.fcol ? (size_t)a.f_cols : N;
    const size_t fcl = a.fcol ? (size_t)a.fcol[cell] : (size_t)cell;
    const double* __restrict__ P = UNIFORM ? a.params : a.params + (size_t)a.set_ix[cell] * PTHSK_NP;

    hbv_snow_par_t<NB> sp_par;
    sp_par.nb = EXACT ? NB : (int)P[PH_NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        sp_par.s[i] = P[PH_S0 + i];
        sp_par.I[i] = P[PH_I0 + i];
    }
    sp_par.tx = P[PH_TX];
    sp_par.cx = P[PH_CX];
    sp_par.ts = P[PH_TS];
    sp_par.lw = P[PH_LW];
    sp_par.cfr = P[PH_CFR];
    const double kc1 = P[PH_C1], kc2 = P[PH_C2], kc3 = P[PH_C3];
    const double ae_scale = P[PH_AE_SCALE], p_corr = P[PH_PCORR], dtf = P[PH_DTF];
    const double pt_albedo = P[PH_PT_ALBEDO], pt_alpha = P[PH_PT_ALPHA];
    const double gm_direct = P[PH_GM_DIRECT];
    const double gm_routed = 1 - gm_direct;

    const double* __restrict__ cc = a.cellc;  // pt_hs_k.h:233-242 (same rows as pt_gs_k)
    const double glacier_fraction = cc[PC_GLACIER * N + cell];
    const double snow_storage_fraction = cc[PC_SNOW_STORAGE * N + cell];
    const double kirchner_routed_prec = cc[PC_KIRCHNER_ROUTED_PREC * N + cell];
    const double direct_response_fraction = cc[PC_DIRECT_RESPONSE * N + cell];
    const double kirchner_fraction = cc[PC_KIRCHNER_FRACTION * N + cell];
    const double cell_area_m2 = cc[PC_AREA * N + cell];
    const double glacier_area_m2 = cc[PC_GLACIER_AREA * N + cell];
    const double mmh_to_m3s_scale_factor = 1 / (3600.0 * 1000.0);

    double* __restrict__ st = a.state;
    double swe = st[PHS_SWE * N + cell], sca = st[PHS_SCA * N + cell];
    double nb_state = st[PHS_NB * N + cell];
    // the state holds nb_state bins (the reference's vectors); the rest read as zero, as the oracle's padding
    const int nbs = (int)nb_state;
    double sp[NB], sw[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        sp[i] = i < nbs ? st[(PHS_SP0 + i) * N + cell] : 0.0;
        sw[i] = i < nbs ? st[(PHS_SW0 + i) * N + cell] : 0.0;
    }
    double q = st[PHS_KIRCHNER_Q * N + cell];
    // state.snow.distribute(parameter.hs, false) (pt_hs_k.h:230): only on a bin-count mismatch
    if ((int)nb_state != sp_par.nb) {
        hbv_distribute(sp_par, sp, sw, swe, sca);
        nb_state = (double)sp_par.nb;
    }
    int32_t err = 0;

    const size_t TW = (size_t)a.win_len;
    const double* __restrict__ f_temp = a.forcing + (size_t)FV_TEMPERATURE * TW * NF;
    const double* __restrict__ f_prec = a.forcing + (size_t)FV_PRECIPITATION * TW * NF;
    const double* __restrict__ f_rh = a.forcing + (size_t)FV_REL_HUM * TW * NF;
    const double* __restrict__ f_rad = a.forcing + (size_t)FV_RADIATION * TW * NF;
    double* __restrict__ R = a.resp;
    const size_t RS = TW * N;
    double* __restrict__ SS = a.state_series;
    const size_t SSS = (TW + 1) * N;

    // state_collector::collect of state.scale_snow(snow_storage_fraction) (pt_hs_k_cell_model.h:195-209,
    // pt_hs_k.h:165-169: only swe is scaled)
    auto collect_state = [&](size_t wi) {
        const size_t o = wi * N + cell;
        SS[PHC_KIRCHNER * SSS + o] = cell_area_m2 * q * mmh_to_m3s_scale_factor;
        SS[PHC_SCA * SSS + o] = sca;
        SS[PHC_SWE * SSS + o] = swe * snow_storage_fraction;
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            SS[(PHC_SP0 + i) * SSS + o] = sp[i];
            SS[(PHC_SW0 + i) * SSS + o] = sw[i];
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
        if (SS) collect_state(wi);
        const double snow_outflow = hbv_snow_step(sp_par, sp, sw, swe, sca, a.step_in_days, a.dt_hours, prec, temp, err);
        // glacier_melt::step (glacier_melt.h:47-52) on the post-step snow covered area
        const double sca_area = cell_area_m2 * sca;
        double gm_melt_m3s = 0.0;
        if (!(glacier_area_m2 <= sca_area || temp <= 0.0))
            gm_melt_m3s = dtf * temp * (glacier_area_m2 - sca_area) * (0.001 / 86400.0);
        double ae_exp;  // actual_evapotranspiration's exp, evaluated beside Priestley-Taylor's (pt_pot_evap_exp)
        const double pot_evap = pt_pot_evap_exp<true>(pt_albedo, pt_alpha, temp, rad, rel_hum, -q * 3.0 / ae_scale, ae_exp) * 3600.0;
        // actual_evapotranspiration::calculate_step (actual_evapotranspiration.h:40-62)
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
        // collectors of response.scale_snow(snow_storage_fraction) (pt_hs_k.h:188-194, 274-277): the response
        // carries the post-step snow state, swe and outflow scaled
        stream_st<STREAM_NT>(&R[PR_AVG_DISCHARGE * RS + fo], cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor);
        stream_st<STREAM_NT>(&R[PR_CHARGE_M3S * RS + fo], charge_m3s);
        if (a.collect >= 1) {
            R[PR_SNOW_SCA * RS + fo] = sca;
            R[PR_SNOW_SWE * RS + fo] = swe * snow_storage_fraction;
        }
        if (a.collect >= 2) {
            R[PR_SNOW_OUTFLOW * RS + fo] = cell_area_m2 * (snow_outflow * snow_storage_fraction) * mmh_to_m3s_scale_factor;
            R[PR_GLACIER_MELT * RS + fo] = gm_melt_m3s;
            R[PR_AE_OUTPUT * RS + fo] = ae;
            R[PR_PE_OUTPUT * RS + fo] = pot_evap;
        }
        if (SS && i + 1 == i_end) collect_state(wi + 1);
    }
    st[PHS_SWE * N + cell] = swe;
    st[PHS_SCA * N + cell] = sca;
    st[PHS_NB * N + cell] = nb_state;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        st[(PHS_SP0 + i) * N + cell] = sp[i];
        st[(PHS_SW0 + i) * N + cell] = sw[i];
    }
    if (NB < HBV_MAX_BINS) {
        for (int i = NB; i < HBV_MAX_BINS; ++i) st[(PHS_SP0 + i) * N + cell] = st[(PHS_SW0 + i) * N + cell] = 0.0;
    }
    st[PHS_KIRCHNER_Q * N + cell] = q;
    if (err) a.err[cell] = err;
}

}  // namespace

hipError_t launch_pthsk_run(const pthsk_kargs& a, hipStream_t stream) {
    const int grid = (a.n_cells + BLOCK - 1) / BLOCK;
    if (grid == 0) return hipSuccess;
    if (a.uniform_params && a.nb_max == 5 && !a.state_series)
        hipLaunchKernelGGL((pthsk_run_kernel<true, 5, true>), dim3(grid), dim3(BLOCK), 0, stream, a);
    else if (a.uniform_params && a.nb_max <= 5 && !a.state_series)
        hipLaunchKernelGGL((pthsk_run_kernel<true, 5>), dim3(grid), dim3(BLOCK), 0, stream, a);
    else if (a.uniform_params)
        hipLaunchKernelGGL((pthsk_run_kernel<true, HBV_MAX_BINS>), dim3(grid), dim3(BLOCK), 0, stream, a);
    else
        hipLaunchKernelGGL((pthsk_run_kernel<false, HBV_MAX_BINS>), dim3(grid), dim3(BLOCK), 0, stream, a);
    return hipGetLastError();
}
