// hbv_stack cell kernel for gfx950.
//
// region_model::run_cells -> cell::run -> run_hbv_stack (core/region_model.h:578-597,
// core/hbv_stack_cell_model.h:247-306, core/hbv_stack.h:278-361) for every cell
// in ONE launch: lane = cell, the time loop inside the kernel, the cell state
// (incl. the snow quantile bins) in registers, forcing read [step][cell] and
// the collector series written [series][step][cell]. Wind speed is not read
// (hbv_stack.h:295-301), so a step moves 32 B of forcing in and 16 B of
// discharge/charge out per cell.
// out-of-line exp / log with their constants from the SGPR table (device/special.h SHYFT_TABLE_CALLS): measured
// r05 (ms per 730-step chunk, year mean) hbv_stack 7.75 -> 7.65; pt_gs_k keeps the default (80.9 -> 82.7 with the table)
#define SHYFT_TABLE_CALLS 1
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../device/hbv_dev.h"
#include "../device/pt_dev.h"
#include "../include_internal/kernels.h"

using namespace shyft_dev;

namespace {

constexpr int BLOCK = 256;

// forcing prefetch depth: step i+1's forcing is in flight while step i computes. The kernel moves 48 B per
// cell-step and does little arithmetic per byte, so its HBM rate is set by the bytes in flight (Little's law).
// Depths 2-4, LDS-resident bin arrays and nontemporal loads/stores measured no better.
constexpr int PREFETCH = 1;

// occupancy target (waves per SIMD; variant builds override with -DSHYFT_HBV_WAVES=N). Measured (512K cells, ms
// per 730-step chunk, year mean): per-lane parameter rows: 2 waves 15.0, 3: 16.3, 4: 23.1; uniform rows in SGPRs
// (the default launch): 2: 13.8, 3: 11.5, 4: 11.0, 5: 17.6.
#ifndef SHYFT_HBV_WAVES
#define SHYFT_HBV_WAVES 4
#endif
constexpr int WAVES_PERLANE = 2;  // the per-lane-parameter launch (catchment parameter sets)

// UNIFORM: every cell uses parameter set 0, so the parameter row (incl. the bin distribution s[], I[]) is
// wave-uniform and lives in SGPRs instead of 2 x 8 + 15 per-lane doubles of VGPRs
// NB: register capacity of the bin arrays (HBV_MAX_BINS, or 5 when every parameter set has at most 5 bins and
// no state series is collected: 10.9 -> 9.4 ms per 512K-cell chunk). Bins NB..HBV_MAX_BINS-1 of the state in
// HBM are then written as zeros, as the oracle's state vector (nb entries, padded) reads back.
// LEAN: the instance for the common launch (discharge collector only, no state series, no ensemble forcing columns):
// those paths and their
// pointers are compiled out, which keeps the step loop's scalar registers (the uniform parameter row, the series
// bases) within the SGPR file instead of spilled to VGPR lanes (a v_readlane_b32, VALU issue, per use)
// EXACT: the parameter set has exactly NB bins (the reference's default distribution has 5): the bin count is a
// compile-time constant, so every "i < nb" guard of the bin loops (and the selects it feeds) folds away
template <bool UNIFORM, int NB, bool LEAN = false, bool EXACT = false>
__global__ __launch_bounds__(BLOCK)
__attribute__((amdgpu_waves_per_eu(UNIFORM ? SHYFT_HBV_WAVES : WAVES_PERLANE, UNIFORM ? SHYFT_HBV_WAVES : WAVES_PERLANE)))
void hbv_run_kernel(const hbv_kargs a) {
    const int cell = blockIdx.x * blockDim.x + threadIdx.x;
    if (cell >= a.n_cells) return;
    if (a.active && !a.active[cell]) return;
    const size_t N = (size_t)a.n_cells;
    // forcing column: the lane itself, or the shared cell of a parameter-ensemble lane
    const size_t NF = !LEAN && a.fcol ? (size_t)a.f_cols : N;
    const size_t fcl = !LEAN && a.fcol ? (size_t)a.fcol[cell] : (size_t)cell;
    const double* __restrict__ P = UNIFORM ? a.params : a.params + (size_t)a.set_ix[cell] * HBV_NP;
    hbv_snow_par_t<NB> sp_par;
    sp_par.nb = EXACT ? NB : (int)P[HK_NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        sp_par.s[i] = P[HK_S0 + i];
        sp_par.I[i] = P[HK_I0 + i];
    }
    sp_par.tx = P[HK_TX];
    sp_par.cx = P[HK_CX];
    sp_par.ts = P[HK_TS];
    sp_par.lw = P[HK_LW];
    sp_par.cfr = P[HK_CFR];
    const double fc = P[HK_FC], beta = P[HK_BETA], lp = P[HK_LP];
    const double uz1 = P[HK_UZ1], kuz2 = P[HK_KUZ2], kuz1 = P[HK_KUZ1], perc = P[HK_PERC], klz = P[HK_KLZ];
    const double p_corr = P[HK_PCORR], pt_albedo = P[HK_PT_ALBEDO], pt_alpha = P[HK_PT_ALPHA], dtf = P[HK_DTF];
    const double gm_direct = P[HK_GM_DIRECT];
    const double gm_routed = 1 - gm_direct;

    const double* __restrict__ cc = a.cellc;
    const double glacier_fraction = cc[HC_GLACIER * N + cell];
    const double direct_response_fraction = cc[HC_DIRECT_RESPONSE * N + cell];
    const double land_fraction = cc[HC_LAND_FRACTION * N + cell];
    const double cell_area_m2 = cc[HC_AREA * N + cell];
    const double glacier_area_m2 = cc[HC_GLACIER_AREA * N + cell];
    const double mmh_to_m3s_scale_factor = 1 / (3600.0 * 1000.0);

    // state -> registers
    double* __restrict__ st = a.state;
    double swe = st[HS_SWE * N + cell], sca = st[HS_SCA * N + cell];
    double sm = st[HS_SM * N + cell], uz = st[HS_UZ * N + cell], lz = st[HS_LZ * N + cell];
    double nb_state = st[HS_NB * N + cell];
    // the state holds nb_state bins (the reference's vectors); the rest read as zero, as the oracle's padding
    const int nbs = (int)nb_state;
    double sp[NB], sw[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        sp[i] = i < nbs ? st[(HS_SP0 + i) * N + cell] : 0.0;
        sw[i] = i < nbs ? st[(HS_SW0 + i) * N + cell] : 0.0;
    }
    // state.snow.distribute(parameter.snow, false) (hbv_stack.h:310): only on a bin-count mismatch
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
    double* __restrict__ SS = LEAN ? nullptr : a.state_series;
    const size_t SSS = (TW + 1) * N;

    auto collect_state = [&](size_t wi) {  // state_collector::collect (hbv_stack_cell_model.h:196-212)
        const size_t o = wi * N + cell;
        SS[HS_SWE * SSS + o] = swe;
        SS[HS_SCA * SSS + o] = sca;
        SS[HS_SM * SSS + o] = sm;
        SS[HS_UZ * SSS + o] = uz;
        SS[HS_LZ * SSS + o] = lz;
        SS[HS_NB * SSS + o] = nb_state;
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            SS[(HS_SP0 + i) * SSS + o] = sp[i];
            SS[(HS_SW0 + i) * SSS + o] = sw[i];
        }
    };

    const int i_end = a.step0 + a.n_steps;
    // the next D steps' forcing is loaded before this step's arithmetic, so its HBM latency overlaps D steps
    // instead of stalling the top of every iteration
    constexpr int D = PREFETCH;
    double rt[D], rr[D], rh[D], rp[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        rt[k] = rr[k] = rh[k] = rp[k] = 0.0;
        if (a.step0 + k < i_end) {
            const size_t ff = (size_t)(a.step0 + k - a.win0) * NF + fcl;
            rt[k] = f_temp[ff]; rr[k] = f_rad[ff]; rh[k] = f_rh[ff]; rp[k] = f_prec[ff];
        }
    }
    for (int i = a.step0; i < i_end; ++i) {
        const size_t wi = (size_t)(i - a.win0);
        const size_t fo = wi * N + cell;
        const double temp = rt[0], rad = rr[0], rel_hum = rh[0], prec_raw = rp[0];
#pragma unroll
        for (int k = 0; k + 1 < D; ++k) {
            rt[k] = rt[k + 1]; rr[k] = rr[k + 1]; rh[k] = rh[k + 1]; rp[k] = rp[k + 1];
        }
        if (i + D < i_end) {
            const size_t fn = (wi + D) * NF + fcl;
            rt[D - 1] = f_temp[fn]; rr[D - 1] = f_rad[fn]; rh[D - 1] = f_rh[fn]; rp[D - 1] = f_prec[fn];
        }
        const double prec = prec_raw * p_corr;
        if (SS) collect_state(wi);
#ifdef SHYFT_ABLATE_HSNOW  // instruction-budget ablation only (wrong results): no snow routine
        const double snow_outflow = prec + 0.0 * temp;
#else
        const double snow_outflow =
            hbv_snow_step(sp_par, sp, sw, swe, sca, a.step_in_days, a.dt_hours, prec, temp, err);
#endif
        // glacier_melt::step (glacier_melt.h:47-52) on the snow covered area after the snow step
        const double sca_area = cell_area_m2 * sca;
        double gm_melt_m3s = 0.0;
        if (!(glacier_area_m2 <= sca_area || temp <= 0.0))
            gm_melt_m3s = dtf * temp * (glacier_area_m2 - sca_area) * (0.001 / 86400.0);
#ifdef SHYFT_ABLATE_PT  // instruction-budget ablation only (wrong results): no Priestley-Taylor
        const double pot_evap = (rad * 1e-4 + rel_hum * 1e-5 + temp * 1e-6) * pt_alpha;
#else
        const double pot_evap = pt_pot_evap<true>(pt_albedo, pt_alpha, temp, rad, rel_hum) * 3600.0;
#endif
        // hbv_actual_evapotranspiration::calculate_step (hbv_actual_evapotranspiration.h:32-38)
        const double snow_fraction = smax(sca, glacier_fraction);
        const double ae = (1.0 - snow_fraction) * (sm < lp ? pot_evap * (sm / lp) : pot_evap);
        const double gm_mmh = gm_melt_m3s / (mmh_to_m3s_scale_factor * cell_area_m2);
        // hbv_soil::step (hbv_soil.h:55-64)
        const double soil_temp = sm + snow_outflow;
        // detmath::pow returns x * x for y == 2 (the default beta): beta is wave-uniform with one parameter set, so
        // this takes a scalar branch instead of a call (whose entry would wait for the prefetched forcing)
        const double soil_x = soil_temp / fc;
        const double soil_q = snow_outflow * (beta == 2.0 ? soil_x * soil_x : dpow(soil_x, beta));
        const double soil_outflow = soil_q > soil_temp ? soil_temp : soil_q;
        sm = smax(0.0, sm + snow_outflow - soil_outflow - ae);
        // hbv_tank::step (hbv_tank.h:64-80)
        const double tank_in = soil_outflow + gm_routed * gm_mmh;
        const double tank_temp = uz + tank_in;
        const double q12 = smax(0.0, (tank_temp - uz1) * kuz2);
        const double q11 = smin(tank_temp, uz1) * kuz1;
        uz = uz + tank_in - perc - (q12 + q11);
        const double q2 = (lz + perc) * klz;
        lz = lz + perc - q2;
        const double tank_outflow = q12 + q11 + q2;

        const double total_discharge = smax(0.0, prec - ae) * direct_response_fraction + gm_direct * gm_mmh +
                                       tank_outflow * land_fraction;
        const double charge_m3s = +(cell_area_m2 * prec * mmh_to_m3s_scale_factor) -
                                  (cell_area_m2 * ae * mmh_to_m3s_scale_factor) + gm_melt_m3s -
                                  (cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor);
        R[HR_AVG_DISCHARGE * RS + fo] = cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor;
        R[HR_CHARGE_M3S * RS + fo] = charge_m3s;
        if (!LEAN && a.collect >= 1) {
            // response.snow.snow_state is never written by hbv_snow::step (hbv_snow.h:121-124): the
            // reference collects its default (swe = sca = 0)
            R[HR_SNOW_SCA * RS + fo] = 0.0;
            R[HR_SNOW_SWE * RS + fo] = 0.0;
        }
        if (!LEAN && a.collect >= 2) {
            R[HR_SNOW_OUTFLOW * RS + fo] = cell_area_m2 * snow_outflow * mmh_to_m3s_scale_factor;
            R[HR_GLACIER_MELT * RS + fo] = gm_melt_m3s;
            R[HR_AE_OUTPUT * RS + fo] = ae;
            R[HR_PE_OUTPUT * RS + fo] = pot_evap;
            R[HR_SOIL_OUTFLOW * RS + fo] = soil_outflow;
        }
        if (SS && i + 1 == i_end) collect_state(wi + 1);
    }
    st[HS_SWE * N + cell] = swe;
    st[HS_SCA * N + cell] = sca;
    st[HS_SM * N + cell] = sm;
    st[HS_UZ * N + cell] = uz;
    st[HS_LZ * N + cell] = lz;
    st[HS_NB * N + cell] = nb_state;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        st[(HS_SP0 + i) * N + cell] = sp[i];
        st[(HS_SW0 + i) * N + cell] = sw[i];
    }
    if (NB < HBV_MAX_BINS) {
        for (int i = NB; i < HBV_MAX_BINS; ++i) st[(HS_SP0 + i) * N + cell] = st[(HS_SW0 + i) * N + cell] = 0.0;
    }
    if (err) a.err[cell] = err;
}

}  // namespace

hipError_t launch_hbv_run(const hbv_kargs& a, hipStream_t stream) {
    const int grid = (a.n_cells + BLOCK - 1) / BLOCK;
    if (grid == 0) return hipSuccess;
    if (a.uniform_params && a.nb_max == 5 && !a.state_series && !a.fcol && a.collect == 0)
        hipLaunchKernelGGL((hbv_run_kernel<true, 5, true, true>), dim3(grid), dim3(BLOCK), 0, stream, a);
    else if (a.uniform_params && a.nb_max <= 5 && !a.state_series && !a.fcol && a.collect == 0)
        hipLaunchKernelGGL((hbv_run_kernel<true, 5, true>), dim3(grid), dim3(BLOCK), 0, stream, a);
    else if (a.uniform_params && a.nb_max <= 5 && !a.state_series)
        hipLaunchKernelGGL((hbv_run_kernel<true, 5>), dim3(grid), dim3(BLOCK), 0, stream, a);
    else if (a.uniform_params)
        hipLaunchKernelGGL((hbv_run_kernel<true, HBV_MAX_BINS>), dim3(grid), dim3(BLOCK), 0, stream, a);
    else
        hipLaunchKernelGGL((hbv_run_kernel<false, HBV_MAX_BINS>), dim3(grid), dim3(BLOCK), 0, stream, a);
    return hipGetLastError();
}
