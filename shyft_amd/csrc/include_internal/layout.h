// Device data layout shared by the HIP kernels and the C-ABI host code.
//
// All per-cell arrays are structure-of-arrays [field][n_cells] in HBM so that
// lane i of a wavefront touches cell i: every per-step load/store of a wave is
// one contiguous 512-byte fp64 segment.
#pragma once
#include <stdint.h>

// pt_gs_k parameter row (per parameter set). Indices 0..30 are the reference's
// calibration order (core/pt_gs_k.h:77-112); the rest are derived on the host
// with the same expressions the reference evaluates per step.
enum ptgsk_param_index {
    PK_C1 = 0, PK_C2, PK_C3, PK_AE_SCALE, PK_TX, PK_WIND_SCALE, PK_MAX_WATER, PK_WIND_CONST,
    PK_FAST_DECAY_RATE, PK_SLOW_DECAY_RATE, PK_SURFACE_MAG, PK_MAX_ALBEDO, PK_MIN_ALBEDO,
    PK_SNOWFALL_RESET, PK_SNOW_CV, PK_GLACIER_ALBEDO, PK_PCORR, PK_CV_FOREST, PK_CV_ALT,
    PK_PT_ALBEDO, PK_PT_ALPHA, PK_IBGF, PK_WED, PK_ISO, PK_DTF, PK_R_VELOCITY, PK_R_ALPHA,
    PK_R_BETA, PK_NWD, PK_GM_DIRECT, PK_RSV_DRF,
    // derived (host, per run's dt): gamma_snow.h:340-343, :188, :271
    PK_ALBEDO_RANGE,    // max_albedo - min_albedo
    PK_SLOW_DECAY,      // 0.5*albedo_range*dt_in_days/slow_albedo_decay_rate
    PK_FAST_DECAY,      // pow(2.0, -dt_in_days/fast_albedo_decay_rate)
    PK_BB0,             // 0.98*sigma*pow(273.15, 4)
    PK_INV_CV2_PARAM,   // 1.0/(snow_cv*snow_cv) with the parameter (not effective) cv
    PTGSK_NP
};
#define PTGSK_NP_REF 31

// pt_gs_k state fields (SoA rows); order = the oracle/C-ABI order
enum ptgsk_state_index {
    PS_ALBEDO = 0, PS_LWC, PS_SURFACE_HEAT, PS_ALPHA, PS_SDC_MELT_MEAN, PS_ACC_MELT,
    PS_ISO_POT_ENERGY, PS_TEMP_SWE, PS_KIRCHNER_Q, PTGSK_NS
};

// per-cell constants of pt_gs_k (pt_gs_k.h:347-357 + effective snow cv)
enum ptgsk_cell_index {
    PC_FOREST = 0, PC_GLACIER, PC_SNOW_STORAGE, PC_KIRCHNER_ROUTED_PREC, PC_DIRECT_RESPONSE,
    PC_KIRCHNER_FRACTION, PC_AREA, PC_GLACIER_AREA, PC_ALTITUDE, PC_CV2, PC_INV_CV2, PTGSK_NC
};

// response series (all_response_collector order, pt_gs_k_cell_model.h:41-98)
enum ptgsk_series_index {
    PR_AVG_DISCHARGE = 0, PR_CHARGE_M3S, PR_SNOW_SCA, PR_SNOW_SWE, PR_SNOW_OUTFLOW,
    PR_GLACIER_MELT, PR_AE_OUTPUT, PR_PE_OUTPUT, PTGSK_NR
};

// forcing variables (env_ts order used everywhere in this repo)
enum forcing_index { FV_TEMPERATURE = 0, FV_PRECIPITATION, FV_WIND_SPEED, FV_REL_HUM, FV_RADIATION, N_FORCING };

// collection modes
enum collect_mode { COLLECT_DISCHARGE = 0, COLLECT_DISCHARGE_SNOW = 1, COLLECT_ALL = 2 };

// ------------------------------------------------------------------ hbv_stack
// parameter row: 22 reference values (core/hbv_stack.h:82-109 order), then the
// hbv_snow distribution (n_bins, s[HBV_MAX_BINS], intervals[HBV_MAX_BINS]),
// which the reference keeps in hbv_snow::parameter (hbv_snow.h:21-72).
#define HBV_MAX_BINS 8
enum hbv_param_index {
    HK_FC = 0, HK_BETA, HK_LP, HK_UZ1, HK_KUZ2, HK_KUZ1, HK_PERC, HK_KLZ, HK_LW, HK_TX, HK_CX, HK_TS, HK_CFR,
    HK_PCORR, HK_PT_ALBEDO, HK_PT_ALPHA, HK_DTF, HK_R_VELOCITY, HK_R_ALPHA, HK_R_BETA, HK_GM_DIRECT, HK_RSV_DRF,
    HK_NB, HK_S0, HK_I0 = HK_S0 + HBV_MAX_BINS, HBV_NP = HK_I0 + HBV_MAX_BINS
};
#define HBV_NP_REF 22

// hbv_stack state (hbv_stack.h:181-201): swe sca sm uz lz, the number of
// distributed snow bins (0 = not yet distributed, hbv_snow.h:95-99) and the bins
enum hbv_state_index {
    HS_SWE = 0, HS_SCA, HS_SM, HS_UZ, HS_LZ, HS_NB, HS_SP0, HS_SW0 = HS_SP0 + HBV_MAX_BINS,
    HBV_NS = HS_SW0 + HBV_MAX_BINS
};

// per-cell constants of hbv_stack (hbv_stack.h:311-318)
enum hbv_cell_index { HC_GLACIER = 0, HC_DIRECT_RESPONSE, HC_LAND_FRACTION, HC_AREA, HC_GLACIER_AREA, HBV_NC };

// response series (hbv all_response_collector, hbv_stack_cell_model.h:40-92, in this
// repo's series-id order so the discharge collector is the prefix [0, 2) / [0, 4))
enum hbv_series_index {
    HR_AVG_DISCHARGE = 0, HR_CHARGE_M3S, HR_SNOW_SCA, HR_SNOW_SWE, HR_SNOW_OUTFLOW, HR_GLACIER_MELT, HR_AE_OUTPUT,
    HR_PE_OUTPUT, HR_SOIL_OUTFLOW, HBV_NR
};

// ------------------------------------------------------------------ pt_ss_k
// parameter row: the 21 reference values in get/set order (core/pt_ss_k.h:78-101)
enum ptssk_param_index {
    SK_C1 = 0, SK_C2, SK_C3, SK_AE_SCALE, SK_ALPHA0, SK_D_RANGE, SK_UNIT_SIZE, SK_MAX_WATER_FRACTION, SK_TX, SK_CX,
    SK_TS, SK_CFR, SK_PCORR, SK_PT_ALBEDO, SK_PT_ALPHA, SK_DTF, SK_R_VELOCITY, SK_R_ALPHA, SK_R_BETA, SK_GM_DIRECT,
    SK_RSV_DRF, PTSSK_NP
};

// pt_ss_k state (pt_ss_k.h:154-181): skaugen nu alpha sca swe free_water residual num_units, kirchner q
enum ptssk_state_index {
    SS_NU = 0, SS_ALPHA, SS_SCA, SS_SWE, SS_FREE_WATER, SS_RESIDUAL, SS_NUM_UNITS, SS_KIRCHNER_Q, PTSSK_NS
};

// pt_ss_k state-collector series (pt_ss_k_cell_model.h:185-200)
enum ptssk_state_series_index {
    SSC_KIRCHNER = 0, SSC_SCA, SSC_SWE, SSC_ALPHA, SSC_NU, SSC_LWC, SSC_RESIDUAL, PTSSK_NSC
};
// per-cell constants: the pt_gs_k PC_* rows (pt_ss_k.h:237-245 are the same expressions)
// response series: the pt_gs_k PR_* ids (snow_swe = snow_total_stored_water of the all-collector)

// ------------------------------------------------------------------ pt_hs_k
// parameter row: the 18 reference values in get/set order (core/pt_hs_k.h:66-88), then the hbv_snow
// distribution (n_bins, s[HBV_MAX_BINS], intervals[HBV_MAX_BINS]) as for hbv_stack (hbv_snow.h:21-72)
enum pthsk_param_index {
    PH_C1 = 0, PH_C2, PH_C3, PH_AE_SCALE, PH_LW, PH_TX, PH_CX, PH_TS, PH_CFR, PH_DTF, PH_PCORR, PH_PT_ALBEDO,
    PH_PT_ALPHA, PH_R_VELOCITY, PH_R_ALPHA, PH_R_BETA, PH_GM_DIRECT, PH_RSV_DRF,
    PH_NB, PH_S0, PH_I0 = PH_S0 + HBV_MAX_BINS, PTHSK_NP = PH_I0 + HBV_MAX_BINS
};
#define PTHSK_NP_REF 18

// pt_hs_k state (pt_hs_k.h:148-172): hbv_snow swe sca, the number of distributed bins (0 = not yet
// distributed), the bins sp / sw, kirchner q
enum pthsk_state_index {
    PHS_SWE = 0, PHS_SCA, PHS_NB, PHS_SP0, PHS_SW0 = PHS_SP0 + HBV_MAX_BINS, PHS_KIRCHNER_Q = PHS_SW0 + HBV_MAX_BINS,
    PTHSK_NS
};
// pt_hs_k state-collector series (pt_hs_k_cell_model.h:148-210): kirchner_discharge, snow_sca, snow_swe, sp[], sw[]
enum pthsk_state_series_index {
    PHC_KIRCHNER = 0, PHC_SCA, PHC_SWE, PHC_SP0, PHC_SW0 = PHC_SP0 + HBV_MAX_BINS, PTHSK_NSC = PHC_SW0 + HBV_MAX_BINS
};
// per-cell constants: the pt_gs_k PC_* rows (pt_hs_k.h:233-242 are the same expressions); response series: PR_*

// ------------------------------------------------------------------ pt_hps_k
// parameter row: the 24 reference values in get/set order (core/pt_hps_k.h:64-90), gm.direct_response (not a
// calibration value there, glacier_melt::parameter default 0), then the hbv_physical_snow distribution
// (n_bins, s[HBV_MAX_BINS], intervals[HBV_MAX_BINS], hbv_physical_snow.h:43-44)
enum pthpsk_param_index {
    PP_C1 = 0, PP_C2, PP_C3, PP_AE_SCALE, PP_LW, PP_TX, PP_CFR, PP_WIND_SCALE, PP_WIND_CONST, PP_SURFACE_MAGNITUDE,
    PP_MAX_ALBEDO, PP_MIN_ALBEDO, PP_FAST_DECAY_RATE, PP_SLOW_DECAY_RATE, PP_SNOWFALL_RESET_DEPTH, PP_ISO, PP_DTF,
    PP_PCORR, PP_PT_ALBEDO, PP_PT_ALPHA, PP_R_VELOCITY, PP_R_ALPHA, PP_R_BETA, PP_RSV_DRF,
    PP_GM_DIRECT, PP_NB, PP_S0, PP_I0 = PP_S0 + HBV_MAX_BINS, PTHPSK_NP = PP_I0 + HBV_MAX_BINS
};
#define PTHPSK_NP_REF 24

// pt_hps_k state (pt_hps_k.h:163-185; hbv_physical_snow.h:135-190): swe sca surface_heat, the number of
// distributed bins, the bins sp / sw / albedo / iso_pot_energy, kirchner q
enum pthpsk_state_index {
    PPS_SWE = 0, PPS_SCA, PPS_SURFACE_HEAT, PPS_NB, PPS_SP0, PPS_SW0 = PPS_SP0 + HBV_MAX_BINS,
    PPS_ALB0 = PPS_SW0 + HBV_MAX_BINS, PPS_ISO0 = PPS_ALB0 + HBV_MAX_BINS, PPS_KIRCHNER_Q = PPS_ISO0 + HBV_MAX_BINS,
    PTHPSK_NS
};
// pt_hps_k state-collector series (pt_hps_k_cell_model.h:160-232)
enum pthpsk_state_series_index {
    PPC_KIRCHNER = 0, PPC_SCA, PPC_SWE, PPC_SURFACE_HEAT, PPC_SP0, PPC_SW0 = PPC_SP0 + HBV_MAX_BINS,
    PPC_ALB0 = PPC_SW0 + HBV_MAX_BINS, PPC_ISO0 = PPC_ALB0 + HBV_MAX_BINS, PTHPSK_NSC = PPC_ISO0 + HBV_MAX_BINS
};

// per-cell error codes written by the stack kernels
enum cell_error { ERR_NONE = 0, ERR_KIRCHNER_MAX_ITER = 1, ERR_NEGATIVE_OUTFLOW = 2, ERR_SKAUGEN_BISECT = 3,
                  ERR_SKAUGEN_PDF = 4 };
