// Cell-identified state: api::cell_state_id, cell_state_with_id and state_io_handler
// (api/api_state.h:22-146), plus a byte format for state vectors.
//
// The reference serialises state vectors with boost binary/text archives
// (api/api_serialization.cpp), a third-party format that is not in this image; the
// bytes below are this engine's own little-endian layout (not wire-compatible with
// boost archives). A blob records the method stack it belongs to and is refused by
// another stack.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace shyft_hip::host {

// api::cell_state_id (api_state.h:34-55)
struct cell_state_id {
    int64_t cid = 0, x = 0, y = 0, area = 0;
    cell_state_id() = default;
    cell_state_id(int64_t c, int64_t x_, int64_t y_, int64_t a) : cid(c), x(x_), y(y_), area(a) {}
    bool operator==(const cell_state_id& o) const { return cid == o.cid && x == o.x && y == o.y && area == o.area; }
    bool operator!=(const cell_state_id& o) const { return !operator==(o); }
    bool operator<(const cell_state_id& o) const {
        if (cid != o.cid) return cid < o.cid;
        if (x != o.x) return x < o.x;
        if (y != o.y) return y < o.y;
        return area < o.area;
    }
};

// cell_state_id_of (api_state.h:57-59): the integer portions of cid, mid_point.x/y and area
template <class G>
cell_state_id cell_state_id_of(const G& g) {
    return cell_state_id(g.catchment_id(), int(g.mid_point().x), int(g.mid_point().y), int(g.area()));
}

using state_with_id = std::pair<cell_state_id, std::vector<double>>;

// ---- bytes: "SHYFTHIPSTATE1\0\0" | int32 stack | int32 n_fields | uint64 count | count x (4 x int64 id, n_fields x f64)
constexpr char state_magic[16] = {'S', 'H', 'Y', 'F', 'T', 'H', 'I', 'P', 'S', 'T', 'A', 'T', 'E', '1', 0, 0};

inline std::vector<char> serialize_states(int stack, size_t n_fields, const std::vector<state_with_id>& v) {
    std::vector<char> b(16 + 4 + 4 + 8 + v.size() * (32 + 8 * n_fields));
    char* p = b.data();
    auto put = [&p](const void* src, size_t n) { std::memcpy(p, src, n); p += n; };
    put(state_magic, 16);
    const int32_t st = stack, nf = int32_t(n_fields);
    const uint64_t cnt = v.size();
    put(&st, 4);
    put(&nf, 4);
    put(&cnt, 8);
    for (const auto& e : v) {
        if (e.second.size() != n_fields) throw std::runtime_error("serialize_to_bytes: state size mismatch");
        const int64_t id[4] = {e.first.cid, e.first.x, e.first.y, e.first.area};
        put(id, 32);
        put(e.second.data(), 8 * n_fields);
    }
    return b;
}

inline std::vector<state_with_id> deserialize_states(const std::vector<char>& b, int stack, size_t n_fields) {
    if (b.size() < 32 || std::memcmp(b.data(), state_magic, 16) != 0)
        throw std::runtime_error("deserialize_from_bytes: not a state blob of this engine");
    int32_t st, nf;
    uint64_t cnt;
    std::memcpy(&st, b.data() + 16, 4);
    std::memcpy(&nf, b.data() + 20, 4);
    std::memcpy(&cnt, b.data() + 24, 8);
    if (st != stack || size_t(nf) != n_fields)
        throw std::runtime_error("deserialize_from_bytes: the blob holds states of another method stack");
    const size_t rec = 32 + 8 * size_t(nf);
    if (cnt > (b.size() - 32) / rec || b.size() != 32 + cnt * rec)
        throw std::runtime_error("deserialize_from_bytes: truncated or oversized state blob");
    std::vector<state_with_id> v(cnt);
    const char* p = b.data() + 32;
    for (auto& e : v) {
        int64_t id[4];
        std::memcpy(id, p, 32);
        e.first = cell_state_id(id[0], id[1], id[2], id[3]);
        e.second.resize(nf);
        std::memcpy(e.second.data(), p + 32, 8 * size_t(nf));
        p += rec;
    }
    return v;
}

// state_io_handler::extract_state / apply_state (api_state.h:112-145) over a cell geometry vector and the
// current states (same order)
template <class G>
std::vector<state_with_id> extract_state(const std::vector<G>& geo, const std::vector<std::vector<double>>& states,
                                         const std::vector<int64_t>& cids) {
    std::vector<state_with_id> r;
    r.reserve(geo.size());
    for (size_t i = 0; i < geo.size(); ++i)
        if (cids.empty() || std::find(cids.begin(), cids.end(), geo[i].catchment_id()) != cids.end())
            r.emplace_back(cell_state_id_of(geo[i]), states[i]);
    return r;
}

// applies the matching states into `states`; returns the indexes into `s` that matched no cell
template <class G>
std::vector<int64_t> apply_state(const std::vector<G>& geo, std::vector<std::vector<double>>& states,
                                 const std::vector<state_with_id>& s, const std::vector<int64_t>& cids) {
    std::map<cell_state_id, size_t> cmap;
    for (size_t i = 0; i < geo.size(); ++i)
        if (cids.empty() || std::find(cids.begin(), cids.end(), geo[i].catchment_id()) != cids.end())
            cmap[cell_state_id_of(geo[i])] = i;
    std::vector<int64_t> missing;
    for (size_t i = 0; i < s.size(); ++i) {
        if (cids.empty() || std::find(cids.begin(), cids.end(), s[i].first.cid) != cids.end()) {
            auto f = cmap.find(s[i].first);
            if (f != cmap.end()) {
                if (s[i].second.size() != states[f->second].size())
                    throw std::runtime_error("apply_state: state size mismatch");
                states[f->second] = s[i].second;
            } else {
                missing.push_back(int64_t(i));
            }
        }
    }
    return missing;
}

}  // namespace shyft_hip::host
