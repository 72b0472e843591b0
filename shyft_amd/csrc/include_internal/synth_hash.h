// Synthetic workload generator shared by the device kernel and the host
// (elevations). Spec (restated for exact host/device equality):
//   SM(x)       = SplitMix64 finaliser of x + 0x9E3779B97F4A7C15
//   key         = SM(SM(seed ^ cell*0xD1B54A32D192ED03) ^ step)
//   u(var)      = (SM(key ^ var*0xA24BAED4963EE407) >> 11) * 2^-53
//   f = (step % 8760)/8760, g = f(1-f), b = 16 g^2, h = step % 24,
//   d = max(0, 1-((h-12)/6)^2)
//   T   = 8 + 12(2b-1) - 0.006 z + 4(u0-0.5)      [degC]
//   P   = u1 < 0.15 ? 3 u5 : 0                     [mm/h]
//   WS  = 10 u2                                    [m/s]
//   RH  = 0.5 + 0.5 u3                             [-]
//   RAD = 800 d (0.3 + 0.7 b)                      [W/m2]
//   z(cell) = 2000 u(seed, var 7, cell, step 0)    [m]
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SYNTH_HD __host__ __device__
#else
#define SYNTH_HD
#endif

SYNTH_HD inline uint64_t synth_sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

SYNTH_HD inline uint64_t synth_key(uint64_t seed, uint64_t cell, uint64_t step) {
    return synth_sm64(synth_sm64(seed ^ (cell * 0xD1B54A32D192ED03ull)) ^ step);
}

SYNTH_HD inline double synth_u(uint64_t key, uint64_t var) {
    return (double)(synth_sm64(key ^ (var * 0xA24BAED4963EE407ull)) >> 11) * 0x1p-53;
}

SYNTH_HD inline double synth_elevation(uint64_t seed, uint64_t cell) { return 2000.0 * synth_u(synth_key(seed, cell, 0), 7); }

// the cell part of synth_key: synth_key(seed, cell, step) == synth_sm64(synth_cell_key(seed, cell) ^ step)
SYNTH_HD inline uint64_t synth_cell_key(uint64_t seed, uint64_t cell) {
    return synth_sm64(seed ^ (cell * 0xD1B54A32D192ED03ull));
}

// v[5] in forcing order: temperature, precipitation, wind_speed, rel_hum, radiation; ck = synth_cell_key(seed, cell)
// (hoisted out of a caller's step loop)
SYNTH_HD inline void synth_values_ck(uint64_t ck, uint64_t step, double z, double* v) {
#pragma clang fp contract(off)
    const uint64_t key = synth_sm64(ck ^ step);
    // step % 8760 and step % 24 in 32-bit arithmetic when the step fits (the same remainders)
    const bool s32 = (step >> 32) == 0;
    const uint64_t m8760 = s32 ? (uint64_t)((uint32_t)step % 8760u) : step % 8760;
    const uint64_t m24 = s32 ? (uint64_t)((uint32_t)step % 24u) : step % 24;
    const double f = (double)m8760 / 8760.0;
    const double g = f * (1.0 - f);
    const double b = 16.0 * g * g;
    const double h = (double)m24;
    const double dd = (h - 12.0) / 6.0;
    double di = 1.0 - dd * dd;
    if (di < 0.0) di = 0.0;
    const double u0 = synth_u(key, 0), u1 = synth_u(key, 1), u2 = synth_u(key, 2), u3 = synth_u(key, 3),
                 u5 = synth_u(key, 5);
    v[0] = 8.0 + 12.0 * (2.0 * b - 1.0) - 0.006 * z + 4.0 * (u0 - 0.5);
    v[1] = (u1 < 0.15) ? 3.0 * u5 : 0.0;
    v[2] = 10.0 * u2;
    v[3] = 0.5 + 0.5 * u3;
    v[4] = 800.0 * di * (0.3 + 0.7 * b);
}

SYNTH_HD inline void synth_values(uint64_t seed, uint64_t cell, uint64_t step, double z, double* v) {
    synth_values_ck(synth_cell_key(seed, cell), step, z, v);
}
