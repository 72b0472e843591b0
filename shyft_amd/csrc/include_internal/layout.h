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
