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

#ifdef SHYFT_PROF
// phase timing (profiling builds only, tools/ptssk_phases.py): per-wavefront s_memtime deltas summed over the launch;
// [0..5] front / queue + first barrier / job compute / second barrier / ss_back + glacier / PT + AE + kirchner +
// stores, [8] solver-wavefront job cycles, [9] solver wavefront-steps, [10] job lanes of those wavefront-steps,
// [11..15] inside a job (device/ptssk_dev.h SS_JOB_MARK): lgammas / opening evaluations / Brent + walk / bisection /
// final cdfs
__device__ unsigned long long g_ptssk_prof[16];
extern "C" int shyft_ptssk_prof_read(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ptssk_prof), sizeof(g_ptssk_prof)) != hipSuccess) return 1;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_ptssk_prof), z, sizeof z) != hipSuccess;
}
#define SS_JOB_T0() unsigned long long ss_jt_ = __builtin_amdgcn_s_memtime()
#define SS_JOB_MARK(k)                                                                                      \
    do {                                                                                                    \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                         \
        if (__lane_id() == (unsigned)(__ffsll((unsigned long long)__ballot(1)) - 1))                        \
            atomicAdd(&g_ptssk_prof[11 + (k)], t_ - ss_jt_);                                                \
        ss_jt_ = t_;                                                                                        \
    } while (0)
#endif

#include "../device/pt_dev.h"
#include "../device/ptgsk_dev.h"
#include "../device/ptssk_dev.h"
#include "../device/stream.h"
#include "../device/wave_place.h"
#include "../include_internal/kernels.h"

using namespace shyft_dev;

#ifdef SHYFT_PROF
#define PROF_DECL unsigned long long prof_acc[6] = {0, 0, 0, 0, 0, 0}; unsigned long long prof_t = __builtin_amdgcn_s_memtime();
#define PROF_MARK(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); prof_acc[k] += t_ - prof_t; prof_t = t_; } while (0)
#define PROF_FLUSH() do { if ((threadIdx.x & 63) == 0) for (int k_ = 0; k_ < 6; ++k_) atomicAdd(&g_ptssk_prof[k_], prof_acc[k_]); } while (0)
#else
#define PROF_DECL
#define PROF_MARK(k) ((void)0)
#define PROF_FLUSH() ((void)0)
#endif

namespace {

constexpr int BLOCK = 256;

// forcing loads / response stores with the nontemporal hint (device/stream.h). r06, 1M cells, the year in 730-step
// chunks: 73.6 -> 72.6 ms per chunk, April HBM traffic 2.33x -> 1.41x the algorithmic bytes
// (profiles/r06/ptssk_nt_variants.txt)
#ifndef SHYFT_PTSSK_NT
#define SHYFT_PTSSK_NT 1
#endif
constexpr bool STREAM_NT = SHYFT_PTSSK_NT != 0;

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

// Priestley-Taylor / Kirchner with the inline exp / log (kmath<true>, as pt_gs_k) instead of the out-of-line calls
#ifndef SHYFT_PTSSK_INLINE_MATH
#define SHYFT_PTSSK_INLINE_MATH 1  // r06: 80.5 -> 79.4 ms per 730-step chunk, year mean (profiles/r06/ptssk_variants_g.txt)
#endif
constexpr bool PTSSK_INLINE_MATH = SHYFT_PTSSK_INLINE_MATH != 0;

// r06: a step with few jobs gives each job a group of L lanes of the solving wavefronts (ss_sca_rel_red<L>,
// device/ptssk_dev.h: lgammas, opening evaluations and final cdfs side by side, the bisection 2-3 levels per
// round), as long as the step's jobs fit GROUP_LANES lanes; the same bits as one lane per job
#ifndef SHYFT_PTSSK_GROUP_LANES
#define SHYFT_PTSSK_GROUP_LANES 64
#endif
#ifndef SHYFT_PTSSK_GROUP_MAX_L
#define SHYFT_PTSSK_GROUP_MAX_L 4
#endif
static_assert(SHYFT_PTSSK_GROUP_MAX_L <= 4, "groups of 8 lanes faulted the GPU (device/ptssk_dev.h)");
// a step with at least SELF_MIN jobs: every lane solves its own job, no queue and no second barrier (0: never)
#ifndef SHYFT_PTSSK_SELF_MIN
#define SHYFT_PTSSK_SELF_MIN 0
#endif
constexpr int SELF_MIN = SHYFT_PTSSK_SELF_MIN;
constexpr int GROUP_LANES = SHYFT_PTSSK_GROUP_LANES;
constexpr int GROUP_MAX_L = SHYFT_PTSSK_GROUP_MAX_L;

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
    // job counters, one per step in rotation (cb = step % 3): thread 0 zeroes the NEXT step's counter before this
    // step's first barrier, and a counter is zeroed again only two steps after its step, when every wavefront has
    // passed that step's first barrier and read it (a step without a second barrier -- no jobs, or every lane
    // solving its own -- lets thread 0 run ahead by at most one step)
    __shared__ int jcount[3];
    if (COMPACT) {
        if (threadIdx.x == 0) jcount[0] = jcount[1] = jcount[2] = 0;
        __syncthreads();
    }
    int cb = 0;

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
    PROF_DECL
    for (int i = a.step0; i < i_end; ++i) {
        const size_t wi = (size_t)(i - a.win0);
        const size_t fo = wi * N + cell;
        const size_t ff = wi * NF + fcl;
        const double temp = stream_ld<STREAM_NT>(&f_temp[ff]);
        const double rad = stream_ld<STREAM_NT>(&f_rad[ff]);
        const double rel_hum = stream_ld<STREAM_NT>(&f_rh[ff]);
        const double prec = stream_ld<STREAM_NT>(&f_prec[ff]) * p_corr;
        if (SS && valid) collect_state(wi);
        double snow_outflow = 0, snow_sca = 0, snow_swe = 0;
        ss_mid m;
        ss_front(sp, a.step_in_days, a.dt_hours, temp, prec, s, m, snow_outflow, snow_sca, snow_swe);
        if (!valid) m.need = false;
        double rel = 0.0;
        PROF_MARK(0);
        if (COMPACT) {
            const int nb = cb == 2 ? 0 : cb + 1;
            if (threadIdx.x == 0) jcount[nb] = 0;  // next step's counter
            int slot = -1;
            if (m.need) {
                slot = atomicAdd(&jcount[cb], 1);
                ju[slot] = m.u; jn[slot] = m.nnn; jnu[slot] = m.nu; jal[slot] = m.alpha;
            }
            __syncthreads();
            PROF_MARK(1);
            const int nj = jcount[cb];
            cb = nb;
            if (SELF_MIN > 0 && nj >= SELF_MIN) {
                if (m.need) rel = ss_sca_rel_red(m.u, m.nnn, m.nu, m.alpha, err);
            } else if (nj > 0) {
                const int t = (int)((threadIdx.x - jrot) & (BLOCK - 1));
                // lanes per job (wave-uniform: nj is the workgroup's): the largest L <= GROUP_MAX_L with
                // nj * L <= GROUP_LANES
                const int L = (GROUP_MAX_L >= 4 && nj * 4 <= GROUP_LANES) ? 4
                            : (GROUP_MAX_L >= 2 && nj * 2 <= GROUP_LANES) ? 2 : 1;
                if (t < nj * L) __builtin_amdgcn_s_setprio(JOB_PRIO);  // the workgroup's critical path
#ifdef SHYFT_PROF
                const unsigned long long tj0 = __builtin_amdgcn_s_memtime();
                const unsigned long long jlanes = __builtin_popcountll(__ballot(t < nj * L));
#endif
                if (L == 1) {
                    for (int j = t; j < nj; j += BLOCK) {
                        int32_t e = 0;
                        jres[j] = ss_sca_rel_red(ju[j], jn[j], jnu[j], jal[j], e);
                        jerr[j] = e;
                    }
                } else {  // a group of L consecutive lanes of one wavefront per job
                    const int j = t / L, k = t & (L - 1);
                    if (j < nj) {
                        int32_t e = 0;
                        const double r = ss_sca_rel_red_group(ju[j], jn[j], jnu[j], jal[j], L, k, e);
                        if (k == 0) {
                            jres[j] = r;
                            jerr[j] = e;
                        }
                    }
                }
                __builtin_amdgcn_s_setprio(0);
#ifdef SHYFT_PROF
                if (jlanes && (threadIdx.x & 63) == 0) {
                    atomicAdd(&g_ptssk_prof[8], __builtin_amdgcn_s_memtime() - tj0);
                    atomicAdd(&g_ptssk_prof[9], 1ull);
                    atomicAdd(&g_ptssk_prof[10], jlanes);
                }
#endif
                PROF_MARK(2);
                __syncthreads();
                PROF_MARK(3);
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
        PROF_MARK(4);  // ss_back + glacier
        double ae_exp;  // actual_evapotranspiration's exp, evaluated beside Priestley-Taylor's (pt_pot_evap_exp)
        const double pot_evap = pt_pot_evap_exp<PTSSK_INLINE_MATH>(pt_albedo, pt_alpha, temp, rad, rel_hum, -q * 3.0 / ae_scale, ae_exp) * 3600.0;
        const double ae = pot_evap * (1.0 - ae_exp) * (1.0 - smax(s.sca, glacier_fraction));
        const double gm_mmh = gm_melt_m3s / (mmh_to_m3s_scale_factor * cell_area_m2);
        double q_avg;
        if (!kirchner_step<PTSSK_INLINE_MATH>(q, q_avg, snow_outflow * snow_storage_fraction + prec * kirchner_routed_prec + gm_routed * gm_mmh,
                           ae, a.t1_hours, kc1, kc2, kc3))
            err = ERR_KIRCHNER_MAX_ITER;
        const double total_discharge = smax(0.0, prec - ae) * direct_response_fraction + gm_direct * gm_mmh +
                                       q_avg * kirchner_fraction;
        const double charge_m3s = +(cell_area_m2 * prec * mmh_to_m3s_scale_factor) -
                                  (cell_area_m2 * ae * mmh_to_m3s_scale_factor) + gm_melt_m3s -
                                  (cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor);
        // collectors of response.scale_snow(snow_storage_fraction) (pt_ss_k.h:198-203)
        stream_st<STREAM_NT>(&R[PR_AVG_DISCHARGE * RS + fo], cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor);
        stream_st<STREAM_NT>(&R[PR_CHARGE_M3S * RS + fo], charge_m3s);
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
        PROF_MARK(5);
    }
    PROF_FLUSH();
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

// r06, measured (1M cells, 730-step chunks, year mean, tools/ptgsk_variants.py): the two job functions compiled for
// their 4-wave caller alone 85.7 ms, with this budget kernel 80.9 (the kernel saves fewer registers around the calls)
#ifndef SHYFT_PTSSK_CALLEE_BUDGET
#define SHYFT_PTSSK_CALLEE_BUDGET 1
#endif
#if SHYFT_PTSSK_CALLEE_BUDGET
// never launched: an 8-wave caller of the job functions, so that they are register-allocated for 64 VGPRs (the
// pt_gs_k kernel's callee-budget scheme, ptgsk.hip)
__global__ __launch_bounds__(256, 8) void ptssk_callee_budget_kernel(const ptssk_kargs a) {
    if (a.n_cells >= 0) return;
    int32_t e = 0;
    const double x = a.params[0];
    const double r = ss_sca_rel_red((uint64_t)x, 7, x, x, e) + ss_sca_rel_red_group((uint64_t)x, 7, x, x, 2, threadIdx.x & 1, e);
    a.resp[threadIdx.x] = r + e;
}
#endif

}  // namespace

hipError_t launch_ptssk_run(const ptssk_kargs& a, hipStream_t stream) {
    const int grid = (a.n_cells + BLOCK - 1) / BLOCK;
    if (grid == 0) return hipSuccess;
#if SHYFT_PTSSK_CALLEE_BUDGET
    if (a.n_cells < 0) hipLaunchKernelGGL(ptssk_callee_budget_kernel, dim3(1), dim3(BLOCK), 0, stream, a);  // never
#endif
    if (a.uniform_params) hipLaunchKernelGGL((ptssk_run_kernel<true, true>), dim3(grid), dim3(BLOCK), 0, stream, a);
    else hipLaunchKernelGGL((ptssk_run_kernel<true, false>), dim3(grid), dim3(BLOCK), 0, stream, a);
    return hipGetLastError();
}
