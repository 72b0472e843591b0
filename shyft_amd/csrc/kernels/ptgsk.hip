// pt_gs_k cell kernel for gfx950.
//
// region_model::run_cells -> cell::run -> run_pt_gs_k (core/region_model.h:578-597,
// core/pt_gs_k_cell_model.h:243-262, core/pt_gs_k.h:312-398) for every cell of
// the region in ONE launch: lane = cell, the time loop runs inside the kernel
// with the cell state held in registers, forcing read [step][cell] (coalesced,
// 512 B per wave per variable per step) and collector series written
// [series][step][cell].
//
// Brent compaction (COMPACT = true): gamma_snow's corr_lwc Brent minimisation
// (gamma_snow.h:425-435) costs ~30 incomplete-gamma evaluations and fires for a
// random ~10% of cells on a snowfall step, so nearly every wavefront would run
// it for a few lanes. Each step the workgroup queues its lanes' Brent jobs in LDS
// and the first ceil(jobs/64) wavefronts solve them (one job per lane), then
// every lane picks up its own result. Results are bit-identical to the
// per-lane version: the same function on the same arguments.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../device/ptgsk_dev.h"
#include "../device/gs_brent.h"
#include "../device/stream.h"
#include "../device/wave_place.h"
#include "../include_internal/kernels.h"

using namespace shyft_dev;

// the Brent job of the solving wavefront: gs_corr_lwc_lean (device/gs_brent.h), the arithmetic of the
// reference-shaped gs_corr_lwc (device/ptgsk_dev.h) in fewer instructions
#define GS_BRENT_JOB gs_corr_lwc_lean

#ifdef SHYFT_PROF
// phase timing (profiling builds only): per-wavefront s_memtime deltas summed over the launch
__device__ unsigned long long g_ptgsk_prof[12];
extern "C" int shyft_ptgsk_prof_read(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ptgsk_prof), sizeof(g_ptgsk_prof)) != hipSuccess) return 1;
    unsigned long long z[12] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_ptgsk_prof), z, sizeof z) != hipSuccess;
}
#define PROF_DECL unsigned long long prof_acc[6] = {0, 0, 0, 0, 0, 0}; unsigned long long prof_t = __builtin_amdgcn_s_memtime();
#define PROF_MARK(k) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); prof_acc[k] += t_ - prof_t; prof_t = t_; } while (0)
#define PROF_FLUSH() do { if ((threadIdx.x & 63) == 0) for (int k_ = 0; k_ < 6; ++k_) atomicAdd(&g_ptgsk_prof[k_], prof_acc[k_]); } while (0)
#else
#define PROF_DECL
#define PROF_MARK(k) ((void)0)
#define PROF_FLUSH() ((void)0)
#endif

namespace {

// forcing loads / response stores with the nontemporal hint (device/stream.h). r06, 1M cells, the year in 730-step
// chunks: 74.0 -> 73.1 ms per chunk, January HBM traffic 1.84x -> 1.33x the algorithmic bytes
// (profiles/r06/ptgsk_nt_variants.txt, tools/traffic_variants.sh)
#ifndef SHYFT_PTGSK_NT
#define SHYFT_PTGSK_NT 1
#endif
constexpr bool STREAM_NT = SHYFT_PTGSK_NT != 0;

// (128- and 512-lane workgroups measured 7 % and 4 % slower over the year, r05)
constexpr int BLOCK = 256;

#ifndef SHYFT_LB_WAVES
#define SHYFT_LB_WAVES 4
#endif

// issue priority (s_setprio) of the Brent-solving wavefront: 138.2 -> 134.5 ms per chunk (year mean, 1M cells)
constexpr int BRENT_PRIO = 3;

// UNIFORM: every cell of the launch uses parameter set 0 (the region parameter, no catchment overrides):
// the parameter row is then wave-uniform and lives in SGPRs (scalar loads), which frees the VGPRs the
// per-lane copies would take in the register-bound time loop.
// ENS: a parameter-ensemble launch (lanes = cells x members): forcing is read from the shared column fcol[lane].
// The 11 per-cell constants live in LDS (22 KB per workgroup, 38.9 KB with the job queue: 4 workgroups = 16
// waves per CU still fit the 160 KB) instead of VGPRs live across the Brent phase. Scratch 400 -> 320 B/lane;
// 124.8 -> 119.1 ms per 1M-cell chunk over the bench year, bit-exact.
// WAVES: the occupancy target. 4 waves per SIMD (128 VGPRs, spilling) is the measured best when the launch fills
// the GPU; a region too small to give every SIMD 4 waves (<= 2 workgroups per CU, e.g. a strong-scaled shard of
// 131K cells) gets the 2-wave instance instead (256 VGPRs, no spills): it cannot be 4-deep anyway.
// B: cells (lanes) per workgroup. SPEC: the speculative Brent opening (device/gs_brent.h), for small regions.
template <bool COMPACT, bool UNIFORM, bool ENS = false, int WAVES = SHYFT_LB_WAVES, int B = BLOCK, bool SPEC = false>
__global__ __launch_bounds__(B, WAVES) void ptgsk_run_kernel(const ptgsk_kargs a) {
    static_assert(COMPACT, "the Brent jobs always go through the workgroup queue");
    const int cell = blockIdx.x * blockDim.x + threadIdx.x;
    bool valid = cell < a.n_cells;
    if (valid && a.active && !a.active[cell]) valid = false;
    const int lc = valid ? cell : 0;  // out-of-range lanes of a COMPACT block read cell 0 and store nothing
    const size_t N = (size_t)a.n_cells;
    const size_t NF = ENS ? (size_t)a.f_cols : N;
    const size_t fcl = ENS ? (size_t)a.fcol[lc] : (size_t)lc;
    const double* __restrict__ Pg = UNIFORM ? a.params : a.params + (size_t)a.set_ix[lc] * PTGSK_NP;
    // the uniform parameter row in LDS (288 B next to the 38.9 KB of job queue and cell constants): the step loop
    // reads it with ds_read_b64 where it is used instead of holding 36 doubles in SGPRs, which spilled to VGPR lanes
    // (a v_readlane per use) beside the inline exp / log constant table. r05: 80.8 -> 79.0 ms per 730-step chunk,
    // v_readlane_b32 326 -> 270 in the kernel's code. (Read after the first barrier below.)
    __shared__ double lpar[UNIFORM ? PTGSK_NP : 1];
    if (UNIFORM && threadIdx.x < PTGSK_NP) lpar[threadIdx.x] = a.params[threadIdx.x];
    const double* __restrict__ P = UNIFORM ? (const double*)lpar : Pg;

    // per-cell constants (pt_gs_k.h:347-357)
    const double* __restrict__ cc = a.cellc;
    gs_cell gcell;
    gcell.forest_fraction = cc[PC_FOREST * N + lc];
    gcell.altitude = cc[PC_ALTITUDE * N + lc];
    gcell.cv2 = cc[PC_CV2 * N + lc];
    gcell.inv_cv2 = cc[PC_INV_CV2 * N + lc];
    // the cell constants live in LDS, not in VGPRs: each use reloads its lane's slot (the barriers of the
    // step keep the compiler from hoisting the loads), so none of them is live across the Brent phase
    // rows 0-8: the cell constants; rows 9-10: the lane's lgamma cache (shape, value), so that every per-lane LDS
    // slot is one address register plus an immediate offset. Two constants are formed from the others with the
    // host's own expressions (region.hip update_derived): kirchner_fraction = 1 - direct_response_fraction and
    // glacier_area_m2 = area * glacier, the same operations on the same doubles
    __shared__ double lcc[11][B];
    {
        const int t = threadIdx.x;
        lcc[0][t] = gcell.forest_fraction;
        lcc[1][t] = gcell.altitude;
        lcc[2][t] = gcell.cv2;
        lcc[3][t] = gcell.inv_cv2;
        lcc[4][t] = cc[PC_GLACIER * N + lc];
        lcc[5][t] = cc[PC_SNOW_STORAGE * N + lc];
        lcc[6][t] = cc[PC_KIRCHNER_ROUTED_PREC * N + lc];
        lcc[7][t] = cc[PC_DIRECT_RESPONSE * N + lc];
        lcc[8][t] = cc[PC_AREA * N + lc];
    }
#define glacier_fraction (lcc[4][threadIdx.x])
#define snow_storage_fraction (lcc[5][threadIdx.x])
#define kirchner_routed_prec (lcc[6][threadIdx.x])
#define direct_response_fraction (lcc[7][threadIdx.x])
#define kirchner_fraction (1 - lcc[7][threadIdx.x])                   // PC_KIRCHNER_FRACTION = 1 - direct
#define cell_area_m2 (lcc[8][threadIdx.x])
#define glacier_area_m2 (lcc[8][threadIdx.x] * lcc[4][threadIdx.x])  // PC_GLACIER_AREA = area * glacier
#define LOAD_GCELL()                                   \
    do {                                               \
        gcell.forest_fraction = lcc[0][threadIdx.x];   \
        gcell.altitude = lcc[1][threadIdx.x];          \
        gcell.cv2 = lcc[2][threadIdx.x];               \
        gcell.inv_cv2 = lcc[3][threadIdx.x];           \
    } while (0)

    const double mmh_to_m3s_scale_factor = 1 / (3600.0 * 1000.0);

    // state -> registers
    double* __restrict__ st = a.state;
    gs_state s;
    s.albedo = st[PS_ALBEDO * N + lc];
    s.lwc = st[PS_LWC * N + lc];
    s.surface_heat = st[PS_SURFACE_HEAT * N + lc];
    s.alpha = st[PS_ALPHA * N + lc];
    s.sdc_melt_mean = st[PS_SDC_MELT_MEAN * N + lc];
    s.acc_melt = st[PS_ACC_MELT * N + lc];
    s.iso_pot_energy = st[PS_ISO_POT_ENERGY * N + lc];
    s.temp_swe = st[PS_TEMP_SWE * N + lc];
    double q = st[PS_KIRCHNER_Q * N + lc];
    lcc[9][threadIdx.x] = -1.0;  // the lgamma cache (device/ptgsk_dev.h)
    lcc[10][threadIdx.x] = 0.0;
    lgamma_cache_lds lgc{lcc[9], lcc[10]};
    gs_carry carry;
    int32_t err = 0;

    const size_t TW = (size_t)a.win_len;
    const double* __restrict__ f_temp = a.forcing + (size_t)FV_TEMPERATURE * TW * NF;
    const double* __restrict__ f_prec = a.forcing + (size_t)FV_PRECIPITATION * TW * NF;
    const double* __restrict__ f_ws = a.forcing + (size_t)FV_WIND_SPEED * TW * NF;
    const double* __restrict__ f_rh = a.forcing + (size_t)FV_REL_HUM * TW * NF;
    const double* __restrict__ f_rad = a.forcing + (size_t)FV_RADIATION * TW * NF;
    double* __restrict__ R = a.resp;
    const size_t RS = TW * N;  // stride between response series
    double* __restrict__ SS = a.state_series;
    const size_t SSS = (TW + 1) * N;
    const int wed = (int)Pg[PK_WED];
    const int64_t snow_lo = (int64_t)((int)(Pg[PK_WED] * 24) - (int)(Pg[PK_NWD] * 24)) * 3600000000LL;
    const int64_t snow_hi = (int64_t)(int)(Pg[PK_WED] * 24) * 3600000000LL;

    // Brent job queue of the workgroup (COMPACT)
    // (jres is not aliased with a job array: a lane reads its result after the step's second barrier, and another
    // wavefront may already be enqueueing the next step's jobs by then)
    __shared__ double jz1[B], ja1[B], jb1[B], ja2[B], jb2[B], jq1[B], jlg2[B], jres[B];
    __shared__ double jsz[SPEC ? 64 : 1], jsf[SPEC ? 64 : 1];  // speculative opening: point and f of lane t
    __shared__ int jcount[2];
    __shared__ int wsimd[B / 64];
    publish_wave_simd(wsimd);
    if (COMPACT) {
        if (threadIdx.x == 0) jcount[0] = jcount[1] = 0;  // both: the first step may be odd (start_step)
        __syncthreads();
    }
    // the lane that solves job 0: the first lane of the solving wavefront (device/wave_place.h)
    const int jrot = solver_lane0<B>(wsimd);

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
    PROF_DECL
    for (int i = a.step0; i < i_end; ++i) {
        const double gm_direct = P[PK_GM_DIRECT];
        const double gm_routed = 1 - gm_direct;
        const double dtf = P[PK_DTF];
        const double p_corr = P[PK_PCORR];
        const double kc1 = P[PK_C1], kc2 = P[PK_C2], kc3 = P[PK_C3];
        const size_t wi = (size_t)(i - a.win0);
        const size_t fo = wi * N + lc;
        const size_t ff = ENS ? wi * NF + fcl : fo;
        double temp = 0, rad = 0, rel_hum = 0, prec = 0, wind_speed = 0;
        if (valid) {
            temp = stream_ld<STREAM_NT && !ENS>(&f_temp[ff]);
            rad = stream_ld<STREAM_NT && !ENS>(&f_rad[ff]);
            rel_hum = stream_ld<STREAM_NT && !ENS>(&f_rh[ff]);
            prec = stream_ld<STREAM_NT && !ENS>(&f_prec[ff]) * p_corr;
            wind_speed = stream_ld<STREAM_NT && !ENS>(&f_ws[ff]);
            if (SS) collect_state(wi);
        }
        const bool start_melt = a.doy[i] == wed;
        const int64_t trel = a.t_rel_year_us[i];
        const bool snow_season = trel >= snow_lo && trel < snow_hi;

        gs_mid m;
        m.need = false;
        m.done = true;
        LOAD_GCELL();
        if (threadIdx.x == 0) jcount[(i + 1) & 1] = 0;  // next step's counter (race-free: see DESIGN.md)
        int slot = -1;
        // the step's Brent job goes into the queue where gs_front forms it
        auto enqueue = [&](double z1, double a1, double b1, double a2, double b2, double q1, double lga2) {
            slot = atomicAdd(&jcount[i & 1], 1);
            jz1[slot] = z1; ja1[slot] = a1; jb1[slot] = b1; ja2[slot] = a2; jb2[slot] = b2;
            jq1[slot] = q1; jlg2[slot] = lga2;
        };
#ifndef SHYFT_ABLATE_SNOW
        if (valid)
            gs_front(s, m, start_melt, a.dt_s, a.dt_us, P, gcell, temp, rad, prec, wind_speed, rel_hum, lgc, carry, enqueue);
#endif
        PROF_MARK(0);  // forcing + gs_front
        double z = 0.0;
        {
            __syncthreads();
            PROF_MARK(1);  // job queue + barrier
            const int nj = jcount[i & 1];
            if (nj > 0) {
#ifdef SHYFT_PROF
                const unsigned long long tb = __builtin_amdgcn_s_memtime();
                if (threadIdx.x < nj) __builtin_amdgcn_s_setprio(BRENT_PRIO);
                for (int j = threadIdx.x; j < nj; j += B) jres[j] = GS_BRENT_JOB(jz1[j], ja1[j], jb1[j], ja2[j], jb2[j], jq1[j], jlg2[j]);
                __builtin_amdgcn_s_setprio(0);
                if (threadIdx.x < nj && (threadIdx.x & 63) == 0)
                    atomicAdd(&g_ptgsk_prof[8], (unsigned long long)(__builtin_amdgcn_s_memtime() - tb));
#else
                const int t = SPEC ? (int)threadIdx.x : (int)((threadIdx.x - jrot) & (B - 1));
                // the solving wavefront is the workgroup's critical path (its other wavefronts wait at the
                // barrier below): it gets issue priority over the other workgroups' wavefronts on its SIMD
                if (t < nj) __builtin_amdgcn_s_setprio(BRENT_PRIO);
                // the speculative opening when the jobs' point lanes fit the solving wavefront: 4 lanes per job
                // (z1, u1, u2a, u2b: two f rounds saved) or 2 (z1, u1: one round saved)
                const int L = SPEC ? (4 * nj <= 64 ? 4 : 2 * nj <= 64 ? 2 : 0) : 0;
                if (L) {
                    const int jj = L == 4 ? t >> 2 : t >> 1;
                    if (t < 64 && jj < nj) {
                        const gsb_zf r = gs_corr_lwc_spec(jz1[jj], ja1[jj], jb1[jj], ja2[jj], jb2[jj], jq1[jj], jlg2[jj], t & (L - 1));
                        jsz[t] = r.z;
                        jsf[t] = r.f;
                    }
                    __syncthreads();
                    if (t < nj) {
                        gsb_memo mm;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {  // with 2 points, entries 2 and 3 repeat entry 0
                            const int e = L * t + (k < L ? k : 0);
                            mm.z[k] = jsz[e];
                            mm.f[k] = jsf[e];
                        }
                        jres[t] = gs_corr_lwc_memo(jz1[t], ja1[t], jb1[t], ja2[t], jb2[t], jq1[t], jlg2[t], mm);
                    }
                } else {
                    for (int j = t; j < nj; j += B) jres[j] = GS_BRENT_JOB(jz1[j], ja1[j], jb1[j], ja2[j], jb2[j], jq1[j], jlg2[j]);
                }
                __builtin_amdgcn_s_setprio(0);
#endif
                __syncthreads();
                // test knob: the other wavefronts read their results late, so a fast first wavefront is already
                // enqueueing the next step's jobs (jres must not alias the job arrays for this to stay exact)
                if (a.read_delay > 0 && (threadIdx.x >> 6) != 0)
                    for (int k = 0; k < a.read_delay; ++k) __builtin_amdgcn_s_sleep(127);
                if (slot >= 0) z = jres[slot];
            }
        }
        PROF_MARK(2);  // Brent phase
        if (!valid) {
            carry = gs_carry();  // (dead: keeps the carry out of the values live across the Brent phase)
            continue;
        }
        double gs_sca, gs_storage, gs_outflow;
        LOAD_GCELL();
#ifdef SHYFT_ABLATE_SNOW  // instruction-budget ablation only (wrong results): no snow routine at all
        gs_sca = 0.0; gs_storage = 0.0; gs_outflow = prec + 0.0 * z;
#else
        gs_back(s, m, z, gs_sca, gs_storage, gs_outflow, snow_season, a.dt_us, P, gcell, prec, lgc, carry);
#endif
        PROF_MARK(3);  // gs_back

        // glacier_melt::step (glacier_melt.h:47-52)
        const double sca_area = cell_area_m2 * gs_sca;
        double gm_melt_m3s = 0.0;
        if (!(glacier_area_m2 <= sca_area || temp <= 0.0))
            gm_melt_m3s = dtf * temp * (glacier_area_m2 - sca_area) * (0.001 / 86400.0);
        // Priestley-Taylor's saturation-pressure exp and actual_evapotranspiration's exp in one dexp2 call
        double ae_exp;
        const double pot_evap =
            pt_pot_evap_exp<true>(P[PK_PT_ALBEDO], P[PK_PT_ALPHA], temp, rad, rel_hum, -q * 3.0 / P[PK_AE_SCALE], ae_exp) *
            3600.0;
        const double ae = pot_evap * (1.0 - ae_exp) * (1.0 - smax(gs_sca, glacier_fraction));
        const double gm_mmh = gm_melt_m3s / (mmh_to_m3s_scale_factor * cell_area_m2);
        PROF_MARK(4);  // glacier, PT, AE
        double q_avg;
        if (!kirchner_step<true>(q, q_avg, gs_outflow * snow_storage_fraction + prec * kirchner_routed_prec + gm_routed * gm_mmh,
                           ae, a.t1_hours, kc1, kc2, kc3))
            err = ERR_KIRCHNER_MAX_ITER;
        const double total_discharge = smax(0.0, prec - ae) * direct_response_fraction + gm_direct * gm_mmh +
                                       q_avg * kirchner_fraction;
        const double charge_m3s = +(cell_area_m2 * prec * mmh_to_m3s_scale_factor) -
                                  (cell_area_m2 * ae * mmh_to_m3s_scale_factor) + gm_melt_m3s -
                                  (cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor);
        // collectors (pt_gs_k_cell_model.h:80-89, 116-124) of response.scale_snow(snow_storage_fraction)
        stream_st<STREAM_NT>(&R[0 * RS + fo], cell_area_m2 * total_discharge * mmh_to_m3s_scale_factor);
        stream_st<STREAM_NT>(&R[1 * RS + fo], charge_m3s);
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
        PROF_MARK(5);  // kirchner, outputs
    }
    PROF_FLUSH();
    if (!valid) return;
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
#undef LOAD_GCELL
#undef glacier_fraction
#undef snow_storage_fraction
#undef kirchner_routed_prec
#undef direct_response_fraction
#undef kirchner_fraction
#undef cell_area_m2
#undef glacier_area_m2

// The step's out-of-line device functions (dexp / dexp2 / dlog / dlgamma, the Brent job) are shared by every
// kernel of this file, and the AMDGPU attributor compiles a shared callee for the range of its callers' occupancy.
// This never-launched 8-wave caller makes that range tight: the callees are register-allocated for 64 VGPRs, so
// they clobber fewer registers and the 4-wave step loop keeps more values live across its calls (VGPR spills of
// the bench instance 164 -> 127). Measured on the 1M-cell bench year, 730-step chunks: 105.3 -> 100.0 ms per chunk,
// bit-exact (tools/ptgsk_variants.py). Round 6 re-measured the budget against the current step
// (detmath's one-division log and degree-11 exp): 7 waves (72 VGPRs for the callees) 75.5 -> 74.2 ms per chunk,
// 6 waves 74.8, bit-exact (profiles/r06/ptgsk_budget_variants.txt); the caller spills a few more VGPRs (32 -> 39)
// but saves more in the calls.
#ifndef SHYFT_PTGSK_BUDGET_WAVES
#define SHYFT_PTGSK_BUDGET_WAVES 7
#endif
__global__ __launch_bounds__(256, SHYFT_PTGSK_BUDGET_WAVES) void ptgsk_callee_budget_kernel(const ptgsk_kargs a) {
    if (a.n_cells >= 0) return;  // never runs: launch_ptgsk_run only references it
    const int c = threadIdx.x;
    gs_state s{};
    gs_mid m{};
    lgamma_cache lgc;
    gs_carry carry;
    gs_cell gc{};
    double q = a.dt_s, qa = 0.0, sca, sto, outf;
    double j[7] = {};
    gs_front(s, m, c == 0, a.dt_s, a.dt_us, a.params, gc, q, q, q, q, q, lgc, carry,
             [&](double z1, double a1, double b1, double a2, double b2, double q1, double lga2) {
                 j[0] = z1; j[1] = a1; j[2] = b1; j[3] = a2; j[4] = b2; j[5] = q1; j[6] = lga2;
             });
    const double z = gs_corr_lwc_lean(j[0], j[1], j[2], j[3], j[4], j[5], j[6]);
    gs_back(s, m, z, sca, sto, outf, c == 1, a.dt_us, a.params, gc, q, lgc, carry);
    double e;
    const double pe = pt_pot_evap_exp<true>(0.2, 1.26, q, q, q, q, e);
    kirchner_step<true>(q, qa, outf, pe * e, a.t1_hours, -2.4, 0.9, -0.1);
    a.resp[c] = q + qa + sca + sto + s.lwc;
}

}  // namespace


hipError_t launch_ptgsk_run(const ptgsk_kargs& a, hipStream_t stream) {
    const int grid = (a.n_cells + BLOCK - 1) / BLOCK;
    if (grid == 0) return hipSuccess;
    // workgroups resident at 4 waves per SIMD: 4 per CU (16 waves of 256-lane workgroups)
    int n_cu = 256;
    {
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess) {
            int v = 0;
            if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) n_cu = v;
        }
    }
    static const char* force = getenv("SHYFT_PTGSK_WAVES");  // measurement knob: "2" / "4" forces an instance
    const bool small = a.instance ? a.instance == 2 : force ? force[0] == '2' : grid <= 2 * n_cu;
    if (a.n_cells < 0)  // never (n_cells > 0): keeps ptgsk_callee_budget_kernel in the module
        hipLaunchKernelGGL(ptgsk_callee_budget_kernel, dim3(1), dim3(BLOCK), 0, stream, a);
    if (a.fcol) {
        hipLaunchKernelGGL((ptgsk_run_kernel<true, false, true>), dim3(grid), dim3(BLOCK), 0, stream, a);
    } else if (small) {
        // small regions: one-wavefront workgroups (each wavefront solves its own ~7 winter Brent jobs: no workgroup
        // barrier wait) with the speculative Brent opening (4 lanes per job, free in a wavefront that has the lanes)
        const int g64 = (a.n_cells + 63) / 64;
        if (a.uniform_params) hipLaunchKernelGGL((ptgsk_run_kernel<true, true, false, 2, 64, true>), dim3(g64), dim3(64), 0, stream, a);
        else hipLaunchKernelGGL((ptgsk_run_kernel<true, false, false, 2, 64, true>), dim3(g64), dim3(64), 0, stream, a);
    } else {
        // (the speculative Brent opening in this instance measured 100.5 -> 134.7 ms per 1M-cell chunk, year mean:
        // its memo registers spill in every phase of the 128-VGPR step loop, so it stays a small-region feature)
        if (a.uniform_params) hipLaunchKernelGGL((ptgsk_run_kernel<true, true>), dim3(grid), dim3(BLOCK), 0, stream, a);
        else hipLaunchKernelGGL((ptgsk_run_kernel<true, false>), dim3(grid), dim3(BLOCK), 0, stream, a);
    }
    return hipGetLastError();
}
