// pt_ss_k cell kernel for gfx950.
//
// region_model::run_cells -> cell::run -> pt_ss_k::run (core/region_model.h:578-597,
// core/pt_ss_k_cell_model.h:205-256, core/pt_ss_k.h:210-291) for every cell of
// the region in ONE launch: lane = cell, the time loop inside the kernel, the
// Skaugen snow state and kirchner q in registers, forcing read [step][cell]
// (coalesced) and the collector series written [series][step][cell].
//
// Per step: p_corr -> skaugen snow -> glacier melt on the post-step sca ->
// Priestley-Taylor -> actual evapotranspiration -> kirchner (dopri5, shared with
// pt_gs_k) -> total discharge / charge.
// out-of-line exp / log with their constants from the SGPR table (device/special.h SHYFT_TABLE_CALLS): measured
// r05 (ms per 730-step chunk, year mean) pt_ss_k 88.0 -> 87.1; pt_gs_k keeps the default (80.9 -> 82.7 with the table)
#define SHYFT_TABLE_CALLS 1
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device/pt_dev.h"
#include "../device/ptgsk_dev.h"
#include "../device/ptssk_dev.h"
#include "../device/wave_place.h"
#include "../include_internal/kernels.h"

using namespace shyft_dev;

namespace {

constexpr int BLOCK = 256;

// occupancy target (waves per SIMD; variant builds override with -DSHYFT_PTSSK_WAVES=N)
#ifndef SHYFT_PTSSK_WAVES
#define SHYFT_PTSSK_WAVES 4  // measured: compiler choice (2) 188 ms, 3: 153, 4: 145, 5: 143, 6: 142
#endif

// sca_rel_red compaction (COMPACT): a partial melt calls statistics::sca_rel_red (skaugen.h:57-82: a 2-bit
// Brent, a bracket walk, a 10-bit bisection and two incomplete-gamma cdfs) for 2-50 % of the cells of a melt-season
// step, scattered over the wavefronts. Each step the workgroup queues its lanes' calls in LDS and the first
// ceil(jobs/64) wavefronts evaluate them, one per lane; every lane then finishes its step with its own result
// (the same function of the same arguments: bit-identical to the per-lane call).
// The solving wavefronts run at issue priority 3 (measured: 135.3 -> 134.5 ms per chunk).
constexpr int JOB_PRIO = 3;

// The 7 per-cell constants live in LDS (14 KB per workgroup next to the 11 KB job queue) instead of VGPRs live
// across the sca_rel_red phase (as in the pt_gs_k kernel).

// UNIFORM: every cell uses parameter set 0, so the parameter row is wave-uniform (SGPRs, not 18 per-lane
// doubles held in VGPRs for the whole launch)
template <bool COMPACT, bool UNIFORM>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(SHYFT_PTSSK_WAVES, SHYFT_PTSSK_WAVES)))
void ptssk_run_kernel(const ptssk_kargs a) {
    const int cell = blockIdx.x * blockDim.x + threadIdx.x;
    bool valid = cell < a.n_cells;
    if (valid && a.active && !a.active[cell]) valid = false;
    if (!COMPACT && !valid) return;
    const int lc = valid ? cell : 0;  // idle lanes of a COMPACT block compute on cell 0 and store nothing
    const size_t N = (size_t)a.n_cells;
    // forcing column: the lane itself, or the shared cell of a parameter-ensemble lane
    const size_t NF = a.fcol ? (size_t)a.f_cols : N;
    const size_t fcl = a.fcol ? (size_t)a.fcol[lc] : (size_t)lc;
    const double* __restrict__ P = UNIFORM ? a.params : a.params + (size_t)a.set_ix[lc] * PTSSK_NP;
    __shared__ uint64_t ju[BLOCK], jn[BLOCK];
    __shared__ double jnu[BLOCK], jal[BLOCK], jres[BLOCK];
    __shared__ int32_t jerr[BLOCK];
    __shared__ int jcount[2];
    if (COMPACT) {
        if (threadIdx.x == 0) jcount[0] = jcount[1] = 0;  // both: the first step may be odd (start_step)
        __syncthreads();
    }

    ss_par sp;
    sp.alpha_0 = P[SK_ALPHA0];
    sp.d_range = P[SK_D_RANGE];
    sp.unit_size = P[SK_UNIT_SIZE];
    sp.max_water_fraction = P[SK_MAX_WATER_FRACTION];
    sp.tx = P[SK_TX];
    sp.cx = P[SK_CX];
    sp.ts = P[SK_TS];
    sp.cfr = P[SK_CFR];
    const double kc1 = P[SK_C1], kc2 = P[SK_C2], kc3 = P[SK_C3];
    const double ae_scale = P[SK_AE_SCALE], p_corr = P[SK_PCORR], dtf = P[SK_DTF];
    const double pt_albedo = P[SK_PT_ALBEDO], pt_alpha = P[SK_PT_ALPHA];
    const double gm_direct = P[SK_GM_DIRECT];
    const double gm_routed = 1 - gm_direct;

    const double* __restrict__ cc = a.cellc;  // pt_ss_k.h:237-245 (same rows as pt_gs_k)
    __shared__ double lcc[7][BLOCK];
    {
        const int t = threadIdx.x;
        lcc[0][t] = cc[PC_GLACIER * N + lc];
        lcc[1][t] = cc[PC_SNOW_STORAGE * N + lc];
        lcc[2][t] = cc[PC_KIRCHNER_ROUTED_PREC * N + lc];
        lcc[3][t] = cc[PC_DIRECT_RESPONSE * N + lc];
        lcc[4][t] = cc[PC_KIRCHNER_FRACTION * N + lc];
        lcc[5][t] = cc[PC_AREA * N + lc];
        lcc[6][t] = cc[PC_GLACIER_AREA * N + lc];
    }
#define glacier_fraction (lcc[0][threadIdx.x])
#define snow_storage_fraction (lcc[1][threadIdx.x])
#define kirchner_routed_prec (lcc[2][threadIdx.x])
#define direct_response_fraction (lcc[3][threadIdx.x])
#define kirchner_fraction (lcc[4][threadIdx.x])
#define cell_area_m2 (lcc[5][threadIdx.x])
#define glacier_area_m2 (lcc[6][threadIdx.x])
    const double mmh_to_m3s_scale_factor = 1 / (3600.0 * 1000.0);

    double* __restrict__ st = a.state;
    ss_state s;
    s.nu = st[SS_NU * N + lc];
    s.alpha = st[SS_ALPHA * N + lc];
    s.sca = st[SS_SCA * N + lc];
    s.swe = st[SS_SWE * N + lc];
    s.free_water = st[SS_FREE_WATER * N + lc];
    s.residual = st[SS_RESIDUAL * N + lc];
    s.num_units = (uint64_t)st[SS_NUM_UNITS * N + lc];
    double q = st[SS_KIRCHNER_Q * N + lc];
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

    // state_collector::collect of state.scale_snow(snow_storage_fraction) (pt_ss_k_cell_model.h:185-200,
    // pt_ss_k.h:171-177)
    auto collect_state = [&](size_t wi) {
        const size_t o = wi * N + cell;
        const double swe_s = s.swe * snow_storage_fraction;
        const double fw_s = s.free_water * snow_storage_fraction;
        SS[SSC_KIRCHNER * SSS + o] = cell_area_m2 * q * mmh_to_m3s_scale_factor;
        SS[SSC_SCA * SSS + o] = s.sca;
        SS[SSC_SWE * SSS + o] = (fw_s + swe_s) * s.sca;
        SS[SSC_ALPHA * SSS + o] = s.alpha;
        SS[SSC_NU * SSS + o] = s.nu;
        SS[SSC_LWC * SSS + o] = fw_s * s.sca;
        SS[SSC_RESIDUAL * SSS + o] = s.residual;
    };

    // the lane that solves job 0: the first lane of the solving wavefront (device/wave_place.h)
    __shared__ int wsimd[BLOCK / 64];
    publish_wave_simd(wsimd);
    __syncthreads();
    const int jrot = solver_lane0<BLOCK>(wsimd);

    const int i_end = a.step0 + a.n_steps;
    for (int i = a.step0; i < i_end; ++i) {
        const size_t wi = (size_t)(i - a.win0);
        const size_t fo = wi * N + cell;
        const size_t ff = wi * NF + fcl;
        const double temp = f_temp[ff];
        const double rad = f_rad[ff];
        const double rel_hum = f_rh[ff];
        const double prec = f_prec[ff] * p_corr;
        if (SS && valid) collect_state(wi);
        double snow_outflow = 0, snow_sca = 0, snow_swe = 0;
        ss_mid m;
        ss_front(sp, a.step_in_days, a.dt_hours, temp, prec, s, m, snow_outflow, snow_sca, snow_swe);
        if (!valid) m.need = false;
        double rel = 0.0;
        if (COMPACT) {
            if (threadIdx.x == 0) jcount[(i + 1) & 1] = 0;  // next step's counter (as in the pt_gs_k kernel)
            int slot = -1;
            if (m.need) {
                slot = atomicAdd(&jcount[i & 1], 1);
                ju[slot] = m.u; jn[slot] = m.nnn; jnu[slot] = m.nu; jal[slot] = m.alpha;
            }
            __syncthreads();
            const int nj = jcount[i & 1];
            if (nj > 0) {
                const int t = (int)((threadIdx.x - jrot) & (BLOCK - 1));
                if (t < nj) __builtin_amdgcn_s_setprio(JOB_PRIO);  // the workgroup's critical path
                for (int j = t; j < nj; j += BLOCK) {
                    int32_t e = 0;
                    jres[j] = ss_sca_rel_red(ju[j], jn[j], jnu[j], jal[j], e);
                    jerr[j] = e;
                }
                __builtin_amdgcn_s_setprio(0);
                __syncthreads();
                if (slot >= 0) {
                    rel = jres[slot];
                    if (jerr[slot]) err = jerr[slot];
                }
            }
        } else if (m.need) {
            rel = ss_sca_rel_red(m.u, m.nnn, m.nu, m.alpha, err);
        }
        if (!valid) continue;
        ss_back(sp, a.dt_hours, s, m, rel, snow_outflow, snow_sca, snow_swe);
        // glacier_melt::step (glacier_melt.h:47-52) on the post-step snow covered area
        const double sca_area = cell_area_m2 * s.sca;
        double gm_melt_m3s = 0.0;
        if (!(glacier_area_m2 <= sca_area || temp <= 0.0))
            gm_melt_m3s = dtf * temp * (glacier_area_m2 - sca_area) * (0.001 / 86400.0);
        double ae_exp;  // actual_evapotranspiration's exp, evaluated beside Priestley-Taylor's (pt_pot_evap_exp)
        const double pot_evap = pt_pot_evap_exp(pt_albedo, pt_alpha, temp, rad, rel_hum, -q * 3.0 / ae_scale, ae_exp) * 3600.0;
        const double ae = pot_evap * (1.0 - ae_exp) * (1.0 - smax(s.sca, glacier_fraction));
        const double gm_mmh = gm_melt_m3s / (mmh_to_m3s_scale_factor * cell_area_m2);
        double q_avg;
        if (!kirchner_step(q, q_avg, snow_outflow * snow_storage_fraction + prec * kirchner_routed_prec + gm_routed * gm_mmh,
                           ae, a.t1_hours, kc1, kc2, kc3))
            err = ERR_KIRCHNER_MAX_ITER;
        const double total_discharge = smax(0.0, prec - ae) * direct_response_fraction + gm_direct * gm_mmh +
                                       q_avg * kirchner_fraction;
        const double charge_m3s = +(cell_area_m2 * prec * mmh_to_m3s_scale_factor) -
                                  (cell_area_m2 * ae * mmh_to_m3s_scale_factor) + gm_melt_m3s -
                                  (cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor);
        // collectors of response.scale_snow(snow_storage_fraction) (pt_ss_k.h:198-203)
        R[PR_AVG_DISCHARGE * RS + fo] = cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor;
        R[PR_CHARGE_M3S * RS + fo] = charge_m3s;
        if (a.collect >= 1) {
            R[PR_SNOW_SCA * RS + fo] = snow_sca;
            R[PR_SNOW_SWE * RS + fo] = snow_swe * snow_storage_fraction;
        }
        if (a.collect >= 2) {
            R[PR_SNOW_OUTFLOW * RS + fo] = cell_area_m2 * (snow_outflow * snow_storage_fraction) * mmh_to_m3s_scale_factor;
            R[PR_GLACIER_MELT * RS + fo] = gm_melt_m3s;
            R[PR_AE_OUTPUT * RS + fo] = ae;
            R[PR_PE_OUTPUT * RS + fo] = pot_evap;
        }
        if (SS && i + 1 == i_end) collect_state(wi + 1);
    }
    if (!valid) return;
    st[SS_NU * N + cell] = s.nu;
    st[SS_ALPHA * N + cell] = s.alpha;
    st[SS_SCA * N + cell] = s.sca;
    st[SS_SWE * N + cell] = s.swe;
    st[SS_FREE_WATER * N + cell] = s.free_water;
    st[SS_RESIDUAL * N + cell] = s.residual;
    st[SS_NUM_UNITS * N + cell] = (double)s.num_units;
    st[SS_KIRCHNER_Q * N + cell] = q;
    if (err) a.err[cell] = err;
}
#undef glacier_fraction
#undef snow_storage_fraction
#undef kirchner_routed_prec
#undef direct_response_fraction
#undef kirchner_fraction
#undef cell_area_m2
#undef glacier_area_m2

}  // namespace

hipError_t launch_ptssk_run(const ptssk_kargs& a, hipStream_t stream) {
    const int grid = (a.n_cells + BLOCK - 1) / BLOCK;
    if (grid == 0) return hipSuccess;
    if (a.uniform_params) hipLaunchKernelGGL((ptssk_run_kernel<true, true>), dim3(grid), dim3(BLOCK), 0, stream, a);
    else hipLaunchKernelGGL((ptssk_run_kernel<true, false>), dim3(grid), dim3(BLOCK), 0, stream, a);
    return hipGetLastError();
}
