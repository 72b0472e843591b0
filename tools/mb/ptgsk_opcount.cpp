// Analysis (CPU): the fp64 operation count of the pt_gs_k oracle (oracle/src/ptgsk.hpp, the restatement of
// core/pt_gs_k.h:312-398 with detmath's elementary functions -- the arithmetic the HIP kernel performs bit for bit) on
// the bench region's cells, per cell-step and by chunk of the year, for comparison with the kernel's VALU instruction
// counts (rocprofv3 SQ_INSTS_VALU*, profiles/r06/pmc_*.json). Every double of the oracle is a counting type here:
// additions, subtractions, multiplications, divisions, fused multiply-adds, square roots, comparisons and conversions
// to integers are counted as the oracle executes them (the CPU build, -ffp-contract=off, so no operation is fused behind the count).
// build: g++ -O2 -std=c++17 -mfma -ffp-contract=off -o tools/mb/ptgsk_opcount tools/mb/ptgsk_opcount.cpp
// usage: ptgsk_opcount [cells (1024)] [stride (1024)]  -- cells 0, stride, 2 stride, ... of the 1M-cell bench region
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <limits>
#include <map>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../shyft_amd/csrc/include_internal/synth_hash.h"

namespace opc {
struct counts {
    unsigned long long add = 0, mul = 0, div = 0, fma = 0, sqrt = 0, cmp = 0, cvt = 0;
};
counts C;
}  // namespace opc

struct CD {
    double v;
    CD() = default;
    constexpr CD(double x) : v(x) {}
    template <class I, class = std::enable_if_t<std::is_integral<I>::value>>
    constexpr CD(I x) : v(double(x)) {}
    template <class T, class = std::enable_if_t<std::is_arithmetic<T>::value>>
    explicit operator T() const { if (std::is_integral<T>::value) ++opc::C.cvt; return T(v); }
    constexpr CD operator-() const { return CD(-v); }
    constexpr CD operator+() const { return *this; }
    CD& operator+=(CD o) { ++opc::C.add; v += o.v; return *this; }
    CD& operator-=(CD o) { ++opc::C.add; v -= o.v; return *this; }
    CD& operator*=(CD o) { ++opc::C.mul; v *= o.v; return *this; }
    CD& operator/=(CD o) { ++opc::C.div; v /= o.v; return *this; }
    friend CD operator+(CD a, CD b) { ++opc::C.add; return CD(a.v + b.v); }
    friend CD operator-(CD a, CD b) { ++opc::C.add; return CD(a.v - b.v); }
    friend CD operator*(CD a, CD b) { ++opc::C.mul; return CD(a.v * b.v); }
    friend CD operator/(CD a, CD b) { ++opc::C.div; return CD(a.v / b.v); }
    friend bool operator<(CD a, CD b) { ++opc::C.cmp; return a.v < b.v; }
    friend bool operator>(CD a, CD b) { ++opc::C.cmp; return a.v > b.v; }
    friend bool operator<=(CD a, CD b) { ++opc::C.cmp; return a.v <= b.v; }
    friend bool operator>=(CD a, CD b) { ++opc::C.cmp; return a.v >= b.v; }
    friend bool operator==(CD a, CD b) { ++opc::C.cmp; return a.v == b.v; }
    friend bool operator!=(CD a, CD b) { ++opc::C.cmp; return a.v != b.v; }
};
static_assert(sizeof(CD) == 8 && std::is_trivially_copyable<CD>::value, "CD must be a double in memory");

namespace std {
inline CD fma(CD a, CD b, CD c) { ++opc::C.fma; return CD(std::fma(a.v, b.v, c.v)); }
inline CD fabs(CD a) { return CD(std::fabs(a.v)); }
inline CD sqrt(CD a) { ++opc::C.sqrt; return CD(std::sqrt(a.v)); }
inline CD ldexp(CD a, int e) { return CD(std::ldexp(a.v, e)); }
inline CD rint(CD a) { return CD(std::rint(a.v)); }
inline long lrint(CD a) { ++opc::C.cvt; return std::lrint(a.v); }
inline CD floor(CD a) { return CD(std::floor(a.v)); }
inline bool isfinite(CD a) { return std::isfinite(a.v); }
inline bool isnan(CD a) { return std::isnan(a.v); }
inline bool isinf(CD a) { return std::isinf(a.v); }
inline bool signbit(CD a) { return std::signbit(a.v); }
inline CD nextafter(CD a, CD b) { return CD(std::nextafter(a.v, b.v)); }
inline const CD& max(const CD& a, const CD& b) { ++opc::C.cmp; return (a.v < b.v) ? b : a; }
inline const CD& min(const CD& a, const CD& b) { ++opc::C.cmp; return (b.v < a.v) ? b : a; }
template <>
struct numeric_limits<CD> {
    static constexpr CD quiet_NaN() { return CD(numeric_limits<double>::quiet_NaN()); }
    static constexpr CD infinity() { return CD(numeric_limits<double>::infinity()); }
    static constexpr CD max() { return CD(numeric_limits<double>::max()); }
    static constexpr CD min() { return CD(numeric_limits<double>::min()); }
    static constexpr CD lowest() { return CD(numeric_limits<double>::lowest()); }
    static constexpr CD epsilon() { return CD(numeric_limits<double>::epsilon()); }
    static constexpr bool is_specialized = true;
    static constexpr int digits = 53;
};
}  // namespace std

#define double CD
#include "../../oracle/src/ptgsk.hpp"
#undef double

using namespace oracle;

int main(int argc, char** argv) {
    const int n_cells = argc > 1 ? atoi(argv[1]) : 1024;
    const int stride = argc > 2 ? atoi(argv[2]) : 1024;
    const uint64_t seed = 20251015ull;
    const int T = 8760, CH = 438;
    const int64_t T0 = 1420070400LL * 1000000LL, HOUR = 3600LL * 1000000LL;
    // PTGSKParameter() defaults in the get/set order (shyft_amd/synthetic.py default_ptgsk_parameters)
    const double pv[31] = {-2.439, 0.966, -0.10, 1.5, -0.5, 2.0, 0.1, 1.0, 5.0, 5.0, 30.0, 0.9, 0.6, 5.0, 0.4, 0.4,
                           1.0, 0.0, 0.0, 0.2, 1.26, 0.04, 100.0, 0.0, 6.0, 1.0, 7.0, 0.0, 221.0, 0.0, 1.0};
    const double sv[9] = {0.4, 0.1, 30000.0, 1.26, 0.0, 0.0, 0.0, 0.0, 1.0};
    CD pcd[31], scd[9];
    for (int k = 0; k < 31; ++k) pcd[k] = CD(pv[k]);
    for (int k = 0; k < 9; ++k) scd[k] = CD(sv[k]);
    pt_gs_k::parameter par;
    par.set(pcd);
    const fixed_dt ta(T0, HOUR, T);
    std::vector<opc::counts> by_chunk(T / CH);
    std::vector<CD> fv[5];
    for (auto& v : fv) v.resize(T);
    const int W = 1024;  // ceil(sqrt(2^20)): the geo11 grid of the 1M-cell region
    for (int c = 0; c < n_cells; ++c) {
        const uint64_t cell = (uint64_t)c * stride;
        const double z = synth_elevation(seed, cell);
        const uint64_t ck = synth_cell_key(seed, cell);
        for (int i = 0; i < T; ++i) {
            double v[5];
            synth_values_ck(ck, (uint64_t)i, z, v);
            for (int k = 0; k < 5; ++k) fv[k][i] = CD(v[k]);
        }
        // geo11 row of the cell (shyft_amd/synthetic.py geo11 with n_total = 2^20, 100 catchments)
        const double g[11] = {500.0 + 1000.0 * double(cell % W), 500.0 + 1000.0 * double(cell / W), z, 1.0e6,
                              double(1 + (cell * 100) / (1u << 20)), 0.9, 0.01, 0.05, 0.19, 0.30,
                              1.0 - 0.01 - 0.05 - 0.19 - 0.30};
        CD gcd[11];
        for (int k = 0; k < 11; ++k) gcd[k] = CD(g[k]);
        const geo_cell_data geo = geo_cell_data::from_raw(gcd);
        pt_gs_k::state st;
        st.set(scd);
        pt_gs_k::collectors col;
        col.full = false;
        col.initialize(T, 0, T, geo.area);
        const pt_gs_k::forcing_view view{fv[0].data(), fv[1].data(), fv[2].data(), fv[3].data(), fv[4].data(), 1};
        for (int ch = 0; ch < T / CH; ++ch) {
            const opc::counts before = opc::C;
            pt_gs_k::run_pt_gs_k(geo, par, ta, ch * CH, CH, view, st, col);
            opc::counts& d = by_chunk[ch];
            d.add += opc::C.add - before.add; d.mul += opc::C.mul - before.mul; d.div += opc::C.div - before.div;
            d.fma += opc::C.fma - before.fma; d.sqrt += opc::C.sqrt - before.sqrt; d.cmp += opc::C.cmp - before.cmp;
            d.cvt += opc::C.cvt - before.cvt;
        }
    }
    const double cs = double(n_cells) * CH;
    printf("{\"cells\": %d, \"stride\": %d, \"steps_per_chunk\": %d, \"per_cell_step_by_chunk\": [", n_cells, stride, CH);
    for (size_t ch = 0; ch < by_chunk.size(); ++ch) {
        const opc::counts& d = by_chunk[ch];
        printf("%s{\"add\": %.2f, \"mul\": %.2f, \"div\": %.2f, \"fma\": %.2f, \"sqrt\": %.3f, \"cmp\": %.2f, \"cvt\": %.2f}",
               ch ? ", " : "", d.add / cs, d.mul / cs, d.div / cs, d.fma / cs, d.sqrt / cs, d.cmp / cs, d.cvt / cs);
    }
    printf("]}\n");
    return 0;
}
