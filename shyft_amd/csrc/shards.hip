// Sharded regions: one region_model whose cells are split into contiguous shards, each shard an ordinary region
// (region.hip) on its own device (or several shards on one device), driven from one host process.
//
// The reference runs a whole region in one process and sums every catchment over all of its cells
// (core/region_model.h:972-1021 parallel_run, core/cell_model.h:308-333 cell_statistics, core/routing.h:344-383
// river inflows). Here run_cells is per-cell independent, so each shard runs its cells on its device with no
// data-path exchange; the only cross-shard step is the combination of per-catchment / per-routing-group partial
// sums:
//   - every shard reduces its cells into [rows][steps] partials on its device (the deterministic segment sums of
//     region.hip), scattered to the region's global row order;
//   - the partials are all-gathered: RCCL ncclAllGather over xGMI when every shard has its own device (one
//     communicator per device from ncclCommInitAll), device-to-device copies when shards share a device;
//   - each device adds the gathered partials in shard order (fixed order: deterministic, and bit-equal to the
//     unsharded region wherever a catchment / group lies inside one shard, since the other partials are +0.0).
// Host-side fan-out runs the shards' calls on one host thread per shard, so the devices work concurrently.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <exception>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "include_internal/region_impl.h"
#include "include_internal/shards.h"

namespace shyft_hip_impl {

struct shard_bufs {
    dbuf<double> part, full, gath, out;  // child partial [R_k][n], scattered [R][n], gathered [S][R][n], sum [R][n]
    dbuf<int32_t> rows;                  // child row -> global row
};

struct shard_set {
    int stack = 0;
    size_t n = 0;
    std::vector<shyft_hip_region*> r;  // owned
    std::vector<size_t> b, e;          // cell range of each shard
    std::vector<int> dev;
    std::vector<char> idle;            // no calculated cell under the catchment filter: not run, not interpolated
    std::vector<int64_t> cix_to_cid;   // the region's catchments in first-appearance order (region_model.h:236-252)
    std::map<int64_t, size_t> cid_to_cix;
    std::vector<std::vector<int64_t>> child_cids;
    size_t n_groups = 0;               // routing groups
    std::vector<ncclComm_t> comms;     // one per shard when the devices are distinct
    std::vector<hipStream_t> streams;  // one per shard, on its device
    std::vector<std::unique_ptr<shard_bufs>> bufs;
    int path = SHYFT_HIP_COMBINE_COPY;
    unsigned flags = 0;                // SHYFT_HIP_SHARD_* options of shyft_hip_region_create_sharded_ex
    std::string report;                // how the combine path was chosen, its self-check, run-time fallbacks
    bool gather_fail_armed = false;    // SHYFT_HIP_SHARD_TEST_FAIL_GATHER: the next all-gather fails
    bool stall_armed = false;          // SHYFT_HIP_SHARD_TEST_STALL_CHECK: the self-check's all-gather is not seen to end
    std::string rccl_error;            // the last RCCL failure of exchange()
    size_t ens_members = 0;
    // SHYFT_HIP_SHARD_BALANCE_Z: the cells are dealt to the shards by elevation rank (fixed at the first set_geo), so
    // every shard holds the same mix of elevations; each shard keeps its cells in region order
    bool serial = false;                       // SHYFT_HIP_KNOB_SERIAL_SHARDS: run_cells one shard after another
    mutable int64_t clone_fail_at = -1;        // SHYFT_HIP_KNOB_CLONE_FAIL_AT: the next clone fails at this shard
    bool permuted = false;
    std::vector<std::vector<int64_t>> cells;   // permuted: region cells of shard k, ascending
    std::vector<int32_t> cell_k, cell_j;       // permuted: region cell -> (shard, index in the shard)

    size_t S() const { return r.size(); }
    size_t nk(size_t k) const { return e[k] - b[k]; }
    // shard and index in the shard of a region cell
    void locate(size_t cell, size_t& k, size_t& j) const {
        if (permuted) {
            k = size_t(cell_k[cell]);
            j = size_t(cell_j[cell]);
        } else {
            k = size_t(std::upper_bound(b.begin(), b.end(), cell) - b.begin()) - 1;
            j = cell - b[k];
        }
    }
    // region cell of index j of shard k
    int64_t cell_at(size_t k, size_t j) const { return permuted ? cells[k][j] : int64_t(b[k] + j); }
};

namespace {

void ck(shyft_hip_region* child, int rc) {
    if (rc) throw std::runtime_error(shyft_hip_last_error(child));
}

void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

// f(k) for every shard, shard k on its own host thread with its device current; the first error is rethrown
template <class F>
void for_shards(shard_set* s, F&& f, bool parallel = true) {
    const size_t S = s->S();
    std::vector<std::string> errs(S);
    auto one = [&](size_t k) {
        try {
            hip_check(hipSetDevice(s->dev[k]), "hipSetDevice");
            f(k);
        } catch (const std::exception& e) {
            errs[k] = e.what();
        }
    };
    if (!parallel || S == 1) {
        for (size_t k = 0; k < S; ++k) one(k);
    } else {
        std::vector<std::thread> th;
        for (size_t k = 1; k < S; ++k) th.emplace_back(one, k);
        one(0);
        for (auto& t : th) t.join();
    }
    for (size_t k = 0; k < S; ++k)
        if (!errs[k].empty()) throw std::runtime_error(errs[k]);
}

// columns of a [n][N] host array <-> the [n][n_k] block of shard k
void split_cols(const shard_set* s, const double* src, size_t n, size_t k, std::vector<double>& dst) {
    const size_t N = s->n, nk = s->nk(k);
    dst.resize(n * nk);
    if (!s->permuted) {
        for (size_t t = 0; t < n; ++t) std::copy(src + t * N + s->b[k], src + t * N + s->e[k], dst.begin() + t * nk);
        return;
    }
    const std::vector<int64_t>& c = s->cells[k];
    for (size_t t = 0; t < n; ++t)
        for (size_t j = 0; j < nk; ++j) dst[t * nk + j] = src[t * N + size_t(c[j])];
}
void join_cols(const shard_set* s, const std::vector<double>& src, size_t n, size_t k, double* dst) {
    const size_t N = s->n, nk = s->nk(k);
    if (!s->permuted) {
        for (size_t t = 0; t < n; ++t)
            std::copy(src.begin() + t * nk, src.begin() + (t + 1) * nk, dst + t * N + s->b[k]);
        return;
    }
    const std::vector<int64_t>& c = s->cells[k];
    for (size_t t = 0; t < n; ++t)
        for (size_t j = 0; j < nk; ++j) dst[t * N + size_t(c[j])] = src[t * nk + j];
}
// rows of a [N][width] host array of shard k's cells: a pointer into src (contiguous shards) or a gathered copy
template <class T>
const T* shard_rows(const shard_set* s, size_t k, const T* src, size_t width, std::vector<T>& tmp) {
    if (!src) return nullptr;
    if (!s->permuted) return src + s->b[k] * width;
    const std::vector<int64_t>& c = s->cells[k];
    tmp.resize(c.size() * width);
    for (size_t j = 0; j < c.size(); ++j) std::copy(src + size_t(c[j]) * width, src + (size_t(c[j]) + 1) * width,
                                                     tmp.begin() + j * width);
    return tmp.data();
}

void drop_comms(shard_set* s) {
    for (auto& c : s->comms)
        if (c) (void)ncclCommAbort(c);
    s->comms.clear();
}

// Every RCCL step of a region -- communicator initialisation and each all-gather -- has a deadline
// (SHYFT_HIP_RCCL_DEADLINE_MS, default 120 s): the communicators are non-blocking (ncclConfig_t.blocking = 0), their
// state is polled (ncclCommGetAsyncError) and the streams' completion too (hipStreamQuery), so a step that stalls
// fails like one that errs -- the communicators are aborted and the region continues on device copies.
using clock_t_ = std::chrono::steady_clock;
long long rccl_deadline_ms() {
    const char* e = getenv("SHYFT_HIP_RCCL_DEADLINE_MS");  // read at every step: a test may change it
    const long long ms = e ? atoll(e) : 0;
    return ms > 0 ? ms : 120000;
}

clock_t_::time_point rccl_deadline() { return clock_t_::now() + std::chrono::milliseconds(rccl_deadline_ms()); }

std::string deadline_text() { return std::to_string(rccl_deadline_ms()) + " ms"; }

// a non-blocking RCCL call: ncclInProgress is the normal answer
void nccl_nb(ncclResult_t r, const char* what) {
    if (r != ncclSuccess && r != ncclInProgress) nccl_check(r, what);
}

// wait until no communicator is ncclInProgress; throws on an error state or at the deadline
void wait_comms(shard_set* s, const char* what, clock_t_::time_point until) {
    for (;;) {
        bool pending = false;
        for (ncclComm_t c : s->comms) {
            ncclResult_t st = ncclSuccess;
            nccl_check(ncclCommGetAsyncError(c, &st), "ncclCommGetAsyncError");
            if (st == ncclInProgress) pending = true;
            else nccl_check(st, what);
        }
        if (!pending) return;
        if (clock_t_::now() > until)
            throw std::runtime_error(std::string(what) + " did not complete within " + deadline_text());
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

// wait for the shards' streams; throws on an error or at the deadline. stall: the test of a stalled collective
// (SHYFT_HIP_SHARD_TEST_STALL_CHECK) -- the work has completed, but the wait behaves as if it had not
bool wait_streams(shard_set* s, clock_t_::time_point until, bool stall = false) {
    for (size_t k = 0; k < s->S(); ++k) {
        hip_check(hipSetDevice(s->dev[k]), "hipSetDevice");
        for (;;) {
            const hipError_t q = stall ? hipErrorNotReady : hipStreamQuery(s->streams[k]);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) hip_check(q, "ncclAllGather completion");
            if (clock_t_::now() > until) return false;
            std::this_thread::sleep_for(std::chrono::microseconds(stall ? 2000 : 20));
        }
    }
    return true;
}

// the all-gather step of combine(): bufs[k]->full [M] of every shard -> [S][M] partials on shard 0's device in
// bufs[0]->gath (RCCL: on every shard's device). An RCCL failure at run time (an error status from the group) drops
// the communicators and switches the region to device copies for this and every later combine: the reference's
// one-process region has no exchange that can fail, so a failing interconnect costs speed, never a result.
void exchange(shard_set* s, size_t M) {
    const size_t S = s->S();
    if (s->path == SHYFT_HIP_COMBINE_RCCL) {
        bool group_open = false;
        try {
            if (s->gather_fail_armed) {
                s->gather_fail_armed = false;
                throw std::runtime_error("ncclAllGather: injected failure (SHYFT_HIP_SHARD_TEST_FAIL_GATHER)");
            }
            const clock_t_::time_point until = rccl_deadline();
            nccl_check(ncclGroupStart(), "ncclGroupStart");
            group_open = true;
            for (size_t k = 0; k < S; ++k) {
                hip_check(hipSetDevice(s->dev[k]), "hipSetDevice");
                nccl_nb(ncclAllGather(s->bufs[k]->full.p, s->bufs[k]->gath.p, M, ncclDouble, s->comms[k], s->streams[k]),
                        "ncclAllGather");
            }
            group_open = false;
            nccl_nb(ncclGroupEnd(), "ncclGroupEnd");
            wait_comms(s, "ncclAllGather", until);
            const bool stall = s->stall_armed;
            s->stall_armed = false;
            if (!wait_streams(s, until, stall))
                throw std::runtime_error("ncclAllGather did not complete within " + deadline_text() +
                                         (stall ? " (injected stall, SHYFT_HIP_SHARD_TEST_STALL_CHECK)" : ""));
            hip_check(hipSetDevice(s->dev[0]), "hipSetDevice");
            return;
        } catch (const std::exception& e) {
            // a group left open would defer this thread's next RCCL calls: close it first
            if (group_open) (void)ncclGroupEnd();
            drop_comms(s);  // ncclCommAbort: pending RCCL work of the region ends
            (void)wait_streams(s, rccl_deadline());
            s->path = SHYFT_HIP_COMBINE_COPY;
            s->rccl_error = e.what();
            s->report += std::string("; RCCL failed at run time (") + e.what() + "): device copies from then on";
        }
    }
    hip_check(hipSetDevice(s->dev[0]), "hipSetDevice");
    for (size_t k = 0; k < S; ++k)
        hip_check(hipMemcpyPeerAsync(s->bufs[0]->gath.p + k * M, s->dev[0], s->bufs[k]->full.p, s->dev[k],
                                     M * sizeof(double), s->streams[0]),
                  "gather partials");
}

// The first RCCL use of a region, before any data goes through it: every shard contributes M known doubles
// (signed, spread over 60 binades), the all-gather must deliver all S x M bit for bit on every device, and the
// shard-order sum of the gathered partials must equal the one of the device-copy path bitwise. Any mismatch or
// error is returned as text (empty: passed).
std::string rccl_self_check(shard_set* s) {
    const size_t S = s->S(), M = 4096;
    std::vector<std::vector<double>> in(S, std::vector<double>(M));
    for (size_t k = 0; k < S; ++k)
        for (size_t j = 0; j < M; ++j) {
            const double m = double((k * 2654435761ull + j * 40503ull) % 1000003ull) + 0.5;
            in[k][j] = std::ldexp((j & 1) ? -m : m, int(j % 61) - 30);
        }
    try {
        for (size_t k = 0; k < S; ++k) {
            hip_check(hipSetDevice(s->dev[k]), "hipSetDevice");
            shard_bufs& q = *s->bufs[k];
            q.full.alloc(M);
            q.gath.alloc(S * M);
            q.out.alloc(M);
            hip_check(hipMemcpyAsync(q.full.p, in[k].data(), M * sizeof(double), hipMemcpyHostToDevice, s->streams[k]),
                      "self-check upload");
            hip_check(hipStreamSynchronize(s->streams[k]), "self-check upload");
        }
        exchange(s, M);
        if (s->path != SHYFT_HIP_COMBINE_RCCL) return "the all-gather failed: " + s->rccl_error;
        std::vector<double> got(S * M);
        for (size_t k = 0; k < S; ++k) {
            hip_check(hipSetDevice(s->dev[k]), "hipSetDevice");
            hip_check(hipMemcpy(got.data(), s->bufs[k]->gath.p, S * M * sizeof(double), hipMemcpyDeviceToHost),
                      "self-check download");
            for (size_t r = 0; r < S; ++r)
                if (std::memcmp(got.data() + r * M, in[r].data(), M * sizeof(double)) != 0)
                    return "device " + std::to_string(s->dev[k]) + " received shard " + std::to_string(r) +
                           "'s partials with different bits";
        }
        hip_check(hipSetDevice(s->dev[0]), "hipSetDevice");
        shard_bufs& q0 = *s->bufs[0];
        std::vector<double> sum_rccl(M), sum_copy(M);
        hip_check(launch_ordered_sum(q0.gath.p, S, M, q0.out.p, s->streams[0]), "ordered_sum");
        hip_check(hipMemcpyAsync(sum_rccl.data(), q0.out.p, M * sizeof(double), hipMemcpyDeviceToHost, s->streams[0]),
                  "self-check download");
        hip_check(hipMemsetAsync(q0.gath.p, 0xff, S * M * sizeof(double), s->streams[0]), "memset");
        for (size_t k = 0; k < S; ++k)
            hip_check(hipMemcpyPeerAsync(q0.gath.p + k * M, s->dev[0], s->bufs[k]->full.p, s->dev[k], M * sizeof(double),
                                         s->streams[0]),
                      "self-check copy path");
        hip_check(launch_ordered_sum(q0.gath.p, S, M, q0.out.p, s->streams[0]), "ordered_sum");
        hip_check(hipMemcpyAsync(sum_copy.data(), q0.out.p, M * sizeof(double), hipMemcpyDeviceToHost, s->streams[0]),
                  "self-check download");
        hip_check(hipStreamSynchronize(s->streams[0]), "self-check");
        if (s->flags & SHYFT_HIP_SHARD_TEST_CORRUPT_CHECK) sum_rccl[M / 2] = std::nextafter(sum_rccl[M / 2], 0.0);
        if (std::memcmp(sum_rccl.data(), sum_copy.data(), M * sizeof(double)) != 0)
            return "shard-order sums of the RCCL and the device-copy gathers differ";
        return "";
    } catch (const std::exception& e) {
        return e.what();
    }
}

// the combine path of a new region (shard_set_create, clone): RCCL when every shard has its own device (or when
// asked for), verified by rccl_self_check; otherwise, or on any RCCL failure, device copies
void choose_path(shard_set* s) {
    const size_t S = s->S();
    std::vector<int> sorted(s->dev);
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    std::string devs;
    for (size_t k = 0; k < S; ++k) devs += (k ? "," : "") + std::to_string(s->dev[k]);
    s->path = SHYFT_HIP_COMBINE_COPY;
    if (s->flags & SHYFT_HIP_SHARD_NO_RCCL) {
        s->report = "copy: RCCL not requested (SHYFT_HIP_SHARD_NO_RCCL)";
        return;
    }
    const bool want = (S > 1 && distinct) || (s->flags & SHYFT_HIP_SHARD_RCCL_ALWAYS);
    if (!want) {
        // RCCL does not put two ranks of one communicator on one device
        s->report = S > 1 ? "copy: shards share a device (devices " + devs + ")" : "copy: one shard";
        return;
    }
    try {
        if (s->flags & SHYFT_HIP_SHARD_TEST_FAIL_INIT)
            throw std::runtime_error("ncclCommInitAll: injected failure (SHYFT_HIP_SHARD_TEST_FAIL_INIT)");
        // one non-blocking communicator per device, created in one group (ncclCommInitAll's communicators, with a
        // deadline on their initialisation)
        const clock_t_::time_point until = rccl_deadline();
        ncclUniqueId id;
        nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
        s->comms.assign(S, nullptr);
        nccl_check(ncclGroupStart(), "ncclGroupStart");
        try {
            for (size_t k = 0; k < S; ++k) {
                hip_check(hipSetDevice(s->dev[k]), "hipSetDevice");
                ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
                cfg.blocking = 0;
                nccl_nb(ncclCommInitRankConfig(&s->comms[k], int(S), id, int(k), &cfg), "ncclCommInitRankConfig");
            }
        } catch (...) {
            (void)ncclGroupEnd();
            throw;
        }
        nccl_nb(ncclGroupEnd(), "ncclGroupEnd");
        wait_comms(s, "RCCL communicator initialisation", until);
        hip_check(hipSetDevice(s->dev[0]), "hipSetDevice");
    } catch (const std::exception& e) {
        drop_comms(s);
        (void)hipSetDevice(s->dev[0]);
        s->report = std::string("copy: RCCL initialisation failed (") + e.what() + "), device copies instead";
        return;
    }
    s->path = SHYFT_HIP_COMBINE_RCCL;
    s->stall_armed = (s->flags & SHYFT_HIP_SHARD_TEST_STALL_CHECK) != 0;
    const std::string bad = rccl_self_check(s);
    if (!bad.empty()) {
        drop_comms(s);
        s->path = SHYFT_HIP_COMBINE_COPY;
        s->report = "copy: RCCL self-check failed (" + bad + "), device copies instead";
        return;
    }
    s->report = "rccl: non-blocking communicators over devices " + devs + "; self-check passed (all-gather of " +
                std::to_string(S) + " x 4096 known doubles bit-exact on every device, shard-order sums bit-equal to "
                "the device-copy path)";
    s->gather_fail_armed = (s->flags & SHYFT_HIP_SHARD_TEST_FAIL_GATHER) != 0;
}

// The combination of per-shard partial sums (see the file header). part(k, dev_ptr) writes shard k's partial
// [R_k][n] to a device buffer on its device and returns R_k; rowmap(k) maps its rows to the R global rows (empty:
// identity, R_k == R). The result [R][n] is written to dst (host, or a device pointer on shard 0's device).
// skip_idle: an idle shard (no calculated cell) contributes zeros instead of calling part (ensembles: it ran none);
// otherwise its cells count like any others (catchment sums over uncalculated cells, as the unsharded region)
template <class Part, class RowMap>
void combine(shard_set* s, size_t R, size_t n, Part&& part, RowMap&& rowmap, double* dst, int dst_on_device,
             bool skip_idle = false) {
    const size_t S = s->S(), M = R * n;
    if (M == 0) return;
    for_shards(s, [&](size_t k) {
        shard_bufs& q = *s->bufs[k];
        const std::vector<int32_t> map = rowmap(k);
        const size_t Rk = map.empty() ? R : map.size();
        q.full.alloc(M);
        q.gath.alloc(S * M);
        q.out.alloc(M);
        if ((skip_idle && s->idle[k]) || Rk == 0) {
            hip_check(hipMemsetAsync(q.full.p, 0, M * sizeof(double), s->streams[k]), "memset");
        } else if (map.empty()) {
            part(k, q.full.p);  // synchronous on the shard's stream
        } else {
            q.part.alloc(Rk * n);
            q.rows.alloc(Rk);
            part(k, q.part.p);
            hip_check(hipMemcpyAsync(q.rows.p, map.data(), Rk * sizeof(int32_t), hipMemcpyHostToDevice, s->streams[k]),
                      "upload rows");
            hip_check(hipMemsetAsync(q.full.p, 0, M * sizeof(double), s->streams[k]), "memset");
            hip_check(launch_scatter_rows(q.part.p, q.rows.p, Rk, n, q.full.p, s->streams[k]), "scatter_rows");
        }
        hip_check(hipStreamSynchronize(s->streams[k]), "partials");
    });
    // RCCL: every device holds the same gathered partials; shard 0's device sums them for the caller
    exchange(s, M);
    shard_bufs& q0 = *s->bufs[0];
    double* out = dst_on_device ? dst : q0.out.p;
    hip_check(launch_ordered_sum(q0.gath.p, S, M, out, s->streams[0]), "ordered_sum");
    if (!dst_on_device)
        hip_check(hipMemcpyAsync(dst, q0.out.p, M * sizeof(double), hipMemcpyDeviceToHost, s->streams[0]), "download");
    for (size_t k = 0; k < S; ++k) {  // RCCL: every stream; copies: stream 0
        hip_check(hipSetDevice(s->dev[k]), "hipSetDevice");
        hip_check(hipStreamSynchronize(s->streams[k]), "combine");
    }
}

// the region's catchment map from its geo rows (cid = int(geo[4]), first appearance in cell order)
void map_catchments(shard_set* s, const double* geo11) {
    s->cix_to_cid.clear();
    s->cid_to_cix.clear();
    for (size_t i = 0; i < s->n; ++i) {
        const int64_t c = int64_t(int(geo11[i * 11 + 4]));
        if (s->cid_to_cix.emplace(c, s->cix_to_cid.size()).second) s->cix_to_cid.push_back(c);
    }
    s->child_cids.assign(s->S(), {});
    for (size_t k = 0; k < s->S(); ++k) {
        s->child_cids[k].resize(shyft_hip_number_of_catchments(s->r[k]));
        ck(s->r[k], shyft_hip_catchment_ids(s->r[k], s->child_cids[k].data()));
    }
}

std::vector<int32_t> catchment_rows(const shard_set* s, size_t k) {
    std::vector<int32_t> m;
    for (int64_t c : s->child_cids[k]) m.push_back(int32_t(s->cid_to_cix.at(c)));
    return m;
}

}  // namespace

shard_set* shard_set_create(int stack, size_t n_cells, const int* devices, size_t n_shards, unsigned flags) {
    if (n_shards == 0 || !devices) throw std::runtime_error("shyft_hip_region_create_sharded: no devices");
    if (n_cells < n_shards) throw std::runtime_error("shyft_hip_region_create_sharded: fewer cells than shards");
    int n_dev = 0;
    hip_check(hipGetDeviceCount(&n_dev), "hipGetDeviceCount");
    for (size_t k = 0; k < n_shards; ++k)
        if (devices[k] < 0 || devices[k] >= n_dev)
            throw std::runtime_error("shyft_hip_region_create_sharded: device " + std::to_string(devices[k]) +
                                     " does not exist (" + std::to_string(n_dev) + " visible)");
    std::unique_ptr<shard_set, void (*)(shard_set*)> s(new shard_set(), shard_set_destroy);
    s->stack = stack;
    s->n = n_cells;
    s->flags = flags;
    // every per-shard vector is complete before any shard resource exists, so a failure part-way (a shard that
    // cannot be allocated) unwinds through shard_set_destroy with consistent indexes
    for (size_t k = 0; k < n_shards; ++k) {
        if (flags & SHYFT_HIP_SHARD_BALANCE_Z) {
            // the deal of shyft_hip_set_geo (rank r -> shard r % S) gives the first n % S shards one cell more
            const size_t q = n_cells / n_shards, rem = n_cells % n_shards;
            s->b.push_back(k * q + std::min(k, rem));
            s->e.push_back(s->b.back() + q + (k < rem ? 1 : 0));
        } else {
            s->b.push_back(n_cells * k / n_shards);
            s->e.push_back(n_cells * (k + 1) / n_shards);
        }
        s->dev.push_back(devices[k]);
        s->idle.push_back(0);
    }
    for (size_t k = 0; k < n_shards; ++k) {
        shyft_hip_region* c = nullptr;
        if (shyft_hip_region_create(stack, s->e[k] - s->b[k], devices[k], &c))
            throw std::runtime_error(shyft_hip_last_error(nullptr));
        s->r.push_back(c);
        hipStream_t st = nullptr;
        hip_check(hipSetDevice(devices[k]), "hipSetDevice");
        hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
        s->streams.push_back(st);
        s->bufs.emplace_back(new shard_bufs());
    }
    choose_path(s.get());
    return s.release();
}

void shard_set_destroy(shard_set* s) {
    if (!s) return;
    for (auto& c : s->comms)
        if (c) (void)ncclCommDestroy(c);
    for (size_t k = 0; k < s->streams.size(); ++k) {
        (void)hipSetDevice(s->dev[k]);
        (void)hipStreamSynchronize(s->streams[k]);
        if (k < s->bufs.size()) s->bufs[k].reset();  // device buffers freed on their device
        (void)hipStreamDestroy(s->streams[k]);
    }
    for (auto* c : s->r) shyft_hip_region_destroy(c);
    delete s;
}

namespace shards {

size_t info(const shard_set* s, size_t k, int* device, size_t* cell0, size_t* n_cells) {
    if (k < s->S()) {
        if (device) *device = s->dev[k];
        if (cell0) *cell0 = s->b[k];
        if (n_cells) *n_cells = s->e[k] - s->b[k];
    }
    return s->S();
}

int combine_path(const shard_set* s) { return s->path; }

const char* combine_report(const shard_set* s) { return s->report.c_str(); }

void set_test_knob(shard_set* s, int knob, int64_t value) {
    if (knob == SHYFT_HIP_KNOB_SERIAL_SHARDS) {
        s->serial = value != 0;
        return;
    }
    if (knob == SHYFT_HIP_KNOB_CLONE_FAIL_AT) {
        s->clone_fail_at = value < 0 ? -1 : value;
        return;
    }
    for_shards(s, [&](size_t k) { ck(s->r[k], shyft_hip_set_test_knob(s->r[k], knob, value)); }, false);
}

size_t shard_run_ms(const shard_set* s, double* ms, size_t n) {
    for (size_t k = 0; k < s->S() && k < n; ++k) ms[k] = s->idle[k] ? 0.0 : shyft_hip_last_run_ms(s->r[k]);
    return s->S();
}

// SHYFT_HIP_SHARD_BALANCE_Z: rank the cells by elevation (geo z, ties and NaN by cell index) and deal rank r to
// shard r % S, so that every shard gets every S-th cell of the elevation order. Snow-season cost grows with elevation
// (more snow, more corr_lwc Brent jobs: gamma_snow.h:425-435), and real regions hold their catchments -- and so their
// elevations -- in contiguous cell blocks, which contiguous shards would hand to one device each.
void deal_by_elevation(shard_set* s, const double* geo11) {
    const size_t N = s->n, S = s->S();
    std::vector<int64_t> order(N);
    for (size_t i = 0; i < N; ++i) order[i] = int64_t(i);
    auto z = [&](int64_t i) { return geo11[size_t(i) * 11 + 2]; };
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
        const double za = z(a), zb = z(b);
        if (za != za || zb != zb) return zb != zb && za == za;  // NaN last
        return za < zb;
    });
    s->cells.assign(S, {});
    for (size_t r = 0; r < N; ++r) s->cells[r % S].push_back(order[r]);
    s->cell_k.assign(N, 0);
    s->cell_j.assign(N, 0);
    for (size_t k = 0; k < S; ++k) {
        std::sort(s->cells[k].begin(), s->cells[k].end());
        if (s->cells[k].size() != s->nk(k)) throw std::runtime_error("set_geo: elevation deal does not match the shard sizes");
        for (size_t j = 0; j < s->cells[k].size(); ++j) {
            s->cell_k[size_t(s->cells[k][j])] = int32_t(k);
            s->cell_j[size_t(s->cells[k][j])] = int32_t(j);
        }
    }
    s->permuted = true;
    for_shards(s, [&](size_t k) { region_set_cell_ids(s->r[k], s->cells[k].data()); });
}

// SHYFT_HIP_SHARD_BALANCE_Z deals the cells at the first set_geo; per-cell data given before that would be split
// by contiguous ranges and then belong to the wrong cells, so it is refused
void require_dealt(const shard_set* s, const char* what) {
    if ((s->flags & SHYFT_HIP_SHARD_BALANCE_Z) && !s->permuted)
        throw std::runtime_error(std::string(what) + ": a region whose shards are dealt by elevation "
                                 "(SHYFT_HIP_SHARD_BALANCE_Z) takes per-cell data only after its first set_geo");
}

void set_geo(shard_set* s, const double* geo11, const int64_t* rid, const double* rdist) {
    // the deal is fixed by the first geometry (later set_geo calls keep it: a layout, not a result)
    if ((s->flags & SHYFT_HIP_SHARD_BALANCE_Z) && !s->permuted) deal_by_elevation(s, geo11);
    for_shards(s, [&](size_t k) {
        std::vector<double> g, d;
        std::vector<int64_t> id;
        ck(s->r[k], shyft_hip_set_geo(s->r[k], shard_rows(s, k, geo11, 11, g), shard_rows(s, k, rid, 1, id),
                                      shard_rows(s, k, rdist, 1, d)));
    });
    map_catchments(s, geo11);
    std::fill(s->idle.begin(), s->idle.end(), 0);  // set_geo clears the filter state of each shard
}

void set_parameters(shard_set* s, const double* params, size_t n_sets, size_t n_per_set, const int32_t* set_ix) {
    if (set_ix) require_dealt(s, "set_parameters (per-cell set index)");
    for_shards(s, [&](size_t k) {
        std::vector<int32_t> ix;
        ck(s->r[k], shyft_hip_set_parameters(s->r[k], params, n_sets, n_per_set, shard_rows(s, k, set_ix, 1, ix)));
    });
}

void set_time_axis(shard_set* s, int64_t t0, int64_t dt, size_t n_steps, size_t window) {
    for_shards(s, [&](size_t k) { ck(s->r[k], shyft_hip_set_time_axis(s->r[k], t0, dt, n_steps, window)); });
}

void move_window(shard_set* s, size_t w0, int fill_mask) {
    for_shards(s, [&](size_t k) { ck(s->r[k], shyft_hip_move_window(s->r[k], w0, fill_mask)); });
}

void set_collection(shard_set* s, int collect, int collect_state) {
    for_shards(s, [&](size_t k) { ck(s->r[k], shyft_hip_set_collection(s->r[k], collect, collect_state)); });
}

// region_model::set_catchment_calculation_filter (region_model.h:356-370) over the whole region: checked against
// the region's catchments, then each shard gets the filtered catchments it holds; a shard holding none is idle
void set_catchment_filter(shard_set* s, const int64_t* cids, size_t n) {
    if (n > 0) {
        if (n > s->cix_to_cid.size())
            throw std::runtime_error("set_catchment_calculation_filter: supplied list > available catchments");
        for (size_t j = 0; j < n; ++j)
            if (s->cid_to_cix.find(cids[j]) == s->cid_to_cix.end())
                throw std::runtime_error("set_catchment_calculation_filter: no cells have supplied cid");
    }
    for_shards(s, [&](size_t k) {
        // each catchment once: a list with repeats that passed the region's check must not fail a shard's
        // "supplied list > available catchments" check because that shard holds fewer catchments
        std::vector<int64_t> mine;
        for (size_t j = 0; j < n; ++j)
            if (std::find(s->child_cids[k].begin(), s->child_cids[k].end(), cids[j]) != s->child_cids[k].end() &&
                std::find(mine.begin(), mine.end(), cids[j]) == mine.end())
                mine.push_back(cids[j]);
        s->idle[k] = n > 0 && mine.empty();
        ck(s->r[k], shyft_hip_set_catchment_filter(s->r[k], mine.empty() ? nullptr : mine.data(), mine.size()));
    });
}

void set_state(shard_set* s, const double* state, size_t n_fields) {
    require_dealt(s, "set_state");
    for_shards(s, [&](size_t k) {
        std::vector<double> rows;
        ck(s->r[k], shyft_hip_set_state(s->r[k], shard_rows(s, k, state, n_fields, rows), n_fields));
    });
}

void get_state(shard_set* s, double* state, size_t n_fields) {
    require_dealt(s, "get_state");
    for_shards(s, [&](size_t k) {
        if (!s->permuted) {
            ck(s->r[k], shyft_hip_get_state(s->r[k], state + s->b[k] * n_fields, n_fields));
            return;
        }
        std::vector<double> rows(s->nk(k) * n_fields);
        ck(s->r[k], shyft_hip_get_state(s->r[k], rows.data(), n_fields));
        for (size_t j = 0; j < s->nk(k); ++j)
            std::copy(rows.begin() + j * n_fields, rows.begin() + (j + 1) * n_fields,
                      state + size_t(s->cells[k][j]) * n_fields);
    });
}

void copy_state(shard_set* d, const shard_set* src) {
    if (d->S() != src->S() || d->b != src->b || d->permuted != src->permuted || d->cells != src->cells)
        throw std::runtime_error("copy_state: regions are sharded differently");
    for_shards(d, [&](size_t k) { ck(d->r[k], shyft_hip_copy_state(d->r[k], src->r[k])); });
}

void set_forcing(shard_set* s, int var, size_t step0, size_t n, const double* src, int on_device) {
    if (on_device) throw std::runtime_error("set_forcing: a sharded region takes forcing from host memory");
    require_dealt(s, "set_forcing");
    for_shards(s, [&](size_t k) {
        std::vector<double> blk;
        split_cols(s, src, n, k, blk);
        ck(s->r[k], shyft_hip_set_forcing(s->r[k], var, step0, n, blk.data(), 0));
    });
}

// get_forcing (what 0), get_series (1), get_state_series (2) into host [n][cells]
void get_rows(shard_set* s, int what, int id, size_t step0, size_t n, double* dst, int on_device) {
    if (on_device) throw std::runtime_error("a sharded region returns series to host memory");
    for_shards(s, [&](size_t k) {
        const size_t nk = s->nk(k);
        std::vector<double> blk(n * nk);
        shyft_hip_region* c = s->r[k];
        ck(c, what == 0   ? shyft_hip_get_forcing(c, id, step0, n, blk.data(), 0)
              : what == 1 ? shyft_hip_get_series(c, id, step0, n, blk.data(), 0)
                          : shyft_hip_get_state_series(c, id, step0, n, blk.data(), 0));
        join_cols(s, blk, n, k, dst);
    });
}

void interpolate(shard_set* s, int var, size_t n_sources, const double* xyz, const double* vals, size_t step0, size_t n,
                 const double* prm) {
    for_shards(s, [&](size_t k) {
        if (!s->idle[k]) ck(s->r[k], shyft_hip_interpolate(s->r[k], var, n_sources, xyz, vals, step0, n, prm));
    });
}

int interpolation_path(const shard_set* s, int var) {
    // the gather of the shards that interpolated: none if one has not, tile if one ran tiles, copy if all copied
    bool tile = false, copy = true, seen = false;
    for (size_t k = 0; k < s->S(); ++k) {
        if (s->idle[k]) continue;
        const int q = shyft_hip_interpolation_path(s->r[k], var);
        if (q <= SHYFT_HIP_IDW_NONE) return q;
        seen = true;
        tile = tile || q == SHYFT_HIP_IDW_TILE;
        copy = copy && q == SHYFT_HIP_IDW_COPY;
    }
    if (!seen) return SHYFT_HIP_IDW_NONE;
    return tile ? SHYFT_HIP_IDW_TILE : copy ? SHYFT_HIP_IDW_COPY : SHYFT_HIP_IDW_WAVE;
}

void interpolate_btk(shard_set* s, size_t n_sources, const double* xyz, const double* vals, size_t step0, size_t n,
                     const double* prior, const double* prm) {
    for_shards(s, [&](size_t k) {
        if (!s->idle[k]) ck(s->r[k], shyft_hip_interpolate_btk(s->r[k], n_sources, xyz, vals, step0, n, prior, prm));
    });
}

void synthetic_forcing(shard_set* s, uint64_t seed, uint64_t cell_offset, size_t step0, size_t n) {
    require_dealt(s, "synthetic_forcing");
    for_shards(s, [&](size_t k) {
        // generator cell of shard cell j: cell_offset + its region cell (contiguous: b[k] + j; dealt: the shard's
        // cell ids, region_set_cell_ids)
        ck(s->r[k], shyft_hip_synthetic_forcing(s->r[k], seed, cell_offset + (s->permuted ? 0 : s->b[k]), step0, n));
    });
}

void prefetch_synthetic_forcing(shard_set* s, uint64_t seed, uint64_t cell_offset, size_t w0_next, int n_cus) {
    require_dealt(s, "prefetch_synthetic_forcing");
    for_shards(s, [&](size_t k) {
        ck(s->r[k], shyft_hip_prefetch_synthetic_forcing(s->r[k], seed, cell_offset + (s->permuted ? 0 : s->b[k]),
                                                         w0_next, n_cus));
    });
}

void swap_forcing_window(shard_set* s, size_t w0_next) {
    for_shards(s, [&](size_t k) { ck(s->r[k], shyft_hip_swap_forcing_window(s->r[k], w0_next)); });
}

// run_cells on every shard at once (region_model::parallel_run over the whole region, region_model.h:991-1021)
void run_cells(shard_set* s, size_t use_ncore, int start_step, int n_steps) {
    for_shards(s, [&](size_t k) {
        if (!s->idle[k]) ck(s->r[k], shyft_hip_run_cells(s->r[k], use_ncore, start_step, n_steps));
    }, !s->serial);
}

void run_cells_async(shard_set* s, int start_step, int n_steps) {
    for_shards(s, [&](size_t k) {
        if (!s->idle[k]) ck(s->r[k], shyft_hip_run_cells_async(s->r[k], start_step, n_steps));
    }, false);  // launches only: no threads needed
}

void synchronize(shard_set* s) {
    for_shards(s, [&](size_t k) {
        if (!s->idle[k]) ck(s->r[k], shyft_hip_synchronize(s->r[k]));
    });
}

double last_run_ms(const shard_set* s) {
    double m = 0.0;
    for (size_t k = 0; k < s->S(); ++k)
        if (!s->idle[k]) m = std::max(m, shyft_hip_last_run_ms(s->r[k]));
    return m;
}

double last_interpolate_ms(const shard_set* s) {
    double m = 0.0;
    for (size_t k = 0; k < s->S(); ++k)
        if (!s->idle[k]) m = std::max(m, shyft_hip_last_interpolate_ms(s->r[k]));
    return m;
}

int last_run_kernel_ms(const shard_set* s, double* ms, int n) {
    int parts = 1;
    std::vector<double> mx(4, 0.0);
    for (size_t k = 0; k < s->S(); ++k) {
        if (s->idle[k]) continue;  // not run: its timing is from an earlier run (as last_run_ms)
        double v[4] = {0, 0, 0, 0};
        parts = shyft_hip_last_run_kernel_ms(s->r[k], v, 4);
        for (int j = 0; j < 4; ++j) mx[size_t(j)] = std::max(mx[size_t(j)], v[j]);
    }
    for (int j = 0; j < n && j < parts; ++j) ms[j] = mx[size_t(j)];
    return parts;
}

void cell_series(shard_set* s, int series, size_t cell, size_t step0, size_t n, double* buf, int write) {
    if (cell >= s->n) throw std::runtime_error("cell_series: cell index out of range");
    size_t k, j;
    s->locate(cell, k, j);
    hip_check(hipSetDevice(s->dev[k]), "hipSetDevice");
    ck(s->r[k], shyft_hip_cell_series(s->r[k], series, j, step0, n, buf, write));
}

// columns of selected cells: each shard gathers the ones it holds, into their columns of dst [n][n_cells]
void sample_cells(shard_set* s, int series, const int64_t* cells, size_t m, size_t step0, size_t n, double* dst) {
    std::vector<std::vector<int64_t>> loc(s->S());
    std::vector<std::vector<size_t>> col(s->S());
    for (size_t j = 0; j < m; ++j) {
        if (cells[j] < 0 || size_t(cells[j]) >= s->n) throw std::runtime_error("sample_cells: cell index out of range");
        size_t k, jj;
        s->locate(size_t(cells[j]), k, jj);
        loc[k].push_back(int64_t(jj));
        col[k].push_back(j);
    }
    for_shards(s, [&](size_t k) {
        const size_t mk = loc[k].size();
        if (mk == 0) return;
        std::vector<double> blk(n * mk);
        ck(s->r[k], shyft_hip_sample_cells(s->r[k], series, loc[k].data(), mk, step0, n, blk.data()));
        for (size_t t = 0; t < n; ++t)
            for (size_t q = 0; q < mk; ++q) dst[t * m + col[k][q]] = blk[t * mk + q];
    });
}

void forcing_ok(shard_set* s, int* ok) {
    std::vector<int> oks(s->S(), 1);
    for_shards(s, [&](size_t k) {
        if (!s->idle[k]) ck(s->r[k], shyft_hip_forcing_ok(s->r[k], &oks[k]));
    });
    *ok = 1;
    for (int v : oks) *ok = *ok && v;
}

// cell_statistics over the whole region (cell_model.h:228-333): the selection is resolved against the region
// (cell indexes / catchment ids, verify_cids_exist), each shard sums its selected cells (value, or value x area
// with the area sum for the weighted average), the partial sums are added in shard order
void statistics(shard_set* s, int series, const int64_t* ids, size_t n_ids, int scope, int weighted, size_t step0,
                size_t n, double* dst) {
    std::vector<std::vector<int64_t>> sel(s->S());
    std::vector<char> any(s->S(), n_ids == 0);
    if (n_ids) {
        for (size_t j = 0; j < n_ids; ++j) {
            if (scope == SHYFT_HIP_SCOPE_CELL_IX) {
                if (ids[j] < 0 || ids[j] > int64_t(s->n))
                    throw std::runtime_error("Supplied cell index reference " + std::to_string(ids[j]) +
                                             " is ouside valid range 0 .." + std::to_string(s->n));
                if (ids[j] == int64_t(s->n)) continue;  // valid index, no cell (the reference's range check is <=)
                size_t k, jj;
                s->locate(size_t(ids[j]), k, jj);
                sel[k].push_back(int64_t(jj));
                any[k] = 1;
            } else {
                if (s->cid_to_cix.count(ids[j]) == 0)
                    throw std::runtime_error("one or more supplied catchment_indexes does not exist:" +
                                             std::to_string(ids[j]));
                for (size_t k = 0; k < s->S(); ++k)
                    if (std::find(s->child_cids[k].begin(), s->child_cids[k].end(), ids[j]) != s->child_cids[k].end()) {
                        sel[k].push_back(ids[j]);
                        any[k] = 1;
                    }
            }
        }
    }
    std::vector<std::vector<double>> part(s->S(), std::vector<double>(n, 0.0));
    std::vector<double> area(s->S(), 0.0);
    for_shards(s, [&](size_t k) {
        if (!any[k]) return;
        ck(s->r[k], region_selected_sums(s->r[k], series, sel[k].empty() ? nullptr : sel[k].data(), sel[k].size(),
                                         scope, weighted, step0, n, part[k].data(), &area[k], nullptr));
    });
    bool found = false;
    double sum_area = 0.0;
    for (size_t t = 0; t < n; ++t) dst[t] = 0.0;
    for (size_t k = 0; k < s->S(); ++k) {
        if (!any[k]) continue;
        if (!found) {
            for (size_t t = 0; t < n; ++t) dst[t] = part[k][t];
            sum_area = area[k];
            found = true;
        } else {
            for (size_t t = 0; t < n; ++t) dst[t] += part[k][t];
            sum_area += area[k];
        }
    }
    if (weighted) {
        if (!found) {
            for (size_t t = 0; t < n; ++t) dst[t] = NAN;
            return;
        }
        const double f = 1 / sum_area;  // scale_by(1/sum_area) (cell_model.h:252)
        for (size_t t = 0; t < n; ++t) dst[t] *= f;
    }
}

void catchment_sums(shard_set* s, int series, size_t step0, size_t n, double* dst, int on_device, bool area) {
    combine(
        s, s->cix_to_cid.size(), n,
        [&](size_t k, double* p) {
            ck(s->r[k], area ? shyft_hip_catchment_area_sums(s->r[k], series, step0, n, p, 1)
                             : shyft_hip_catchment_sums(s->r[k], series, step0, n, p, 1));
        },
        [&](size_t k) { return catchment_rows(s, k); }, dst, on_device);
}

size_t number_of_catchments(const shard_set* s) { return s->cix_to_cid.size(); }

void catchment_ids(const shard_set* s, int64_t* cids) {
    std::copy(s->cix_to_cid.begin(), s->cix_to_cid.end(), cids);
}

void set_routing_groups(shard_set* s, const int32_t* group_of_cell, size_t n_groups) {
    require_dealt(s, "set_routing_groups");
    for_shards(s, [&](size_t k) {
        std::vector<int32_t> g;
        ck(s->r[k], shyft_hip_set_routing_groups(s->r[k], shard_rows(s, k, group_of_cell, 1, g), n_groups));
    });
    s->n_groups = n_groups;
}

void routing_group_sums(shard_set* s, size_t step0, size_t n, double* dst, int on_device) {
    combine(
        s, s->n_groups, n,
        [&](size_t k, double* p) { ck(s->r[k], shyft_hip_routing_group_sums(s->r[k], step0, n, p, 1)); },
        [&](size_t) { return std::vector<int32_t>(); }, dst, on_device);
}

// parameter ensembles over a sharded region: each shard runs the members over its calculated cells; the
// per-(member, catchment) sums combine like the catchment sums
void ensemble_run(shard_set* s, const double* params, size_t n_members, size_t n_per_set, int start_step, int n_steps,
                  int collect) {
    bool any = false;
    for (char i : s->idle) any = any || !i;
    if (!any) throw std::runtime_error("ensemble_run: no calculated cells");
    for_shards(s, [&](size_t k) {
        if (!s->idle[k])
            ck(s->r[k], shyft_hip_ensemble_run(s->r[k], params, n_members, n_per_set, start_step, n_steps, collect));
    });
    s->ens_members = n_members;
}

void ensemble_sums(shard_set* s, int series, int area_weighted, size_t step0, size_t n, double* dst, int on_device) {
    if (s->ens_members == 0) throw std::runtime_error("ensemble_sums: no ensemble run");
    const size_t P = s->ens_members, C = s->cix_to_cid.size();
    combine(
        s, P * C, n,
        [&](size_t k, double* p) { ck(s->r[k], shyft_hip_ensemble_sums(s->r[k], series, area_weighted, step0, n, p, 1)); },
        [&](size_t k) {
            const std::vector<int32_t> rows = catchment_rows(s, k);
            std::vector<int32_t> m;
            for (size_t j = 0; j < P; ++j)
                for (int32_t c : rows) m.push_back(int32_t(j * C) + c);
            return m;
        },
        dst, on_device, true);
}

double ensemble_last_ms(const shard_set* s) {
    double m = 0.0;
    for (size_t k = 0; k < s->S(); ++k)
        if (!s->idle[k]) m = std::max(m, shyft_hip_ensemble_last_ms(s->r[k]));
    return m;
}

shard_set* clone(const shard_set* src) {
    std::unique_ptr<shard_set, void (*)(shard_set*)> s(new shard_set(), shard_set_destroy);
    s->stack = src->stack;
    s->n = src->n;
    // host members first (shard_set_destroy reads dev[k] for every stream created below, on any failure)
    s->b = src->b;
    s->e = src->e;
    s->dev = src->dev;
    s->idle = src->idle;
    s->cix_to_cid = src->cix_to_cid;
    s->cid_to_cix = src->cid_to_cix;
    s->child_cids = src->child_cids;
    s->n_groups = src->n_groups;
    s->flags = src->flags & ~unsigned(SHYFT_HIP_SHARD_TEST_FAIL_GATHER);
    s->permuted = src->permuted;   // (the shard regions' cell ids are cloned with them)
    s->cells = src->cells;
    s->cell_k = src->cell_k;
    s->cell_j = src->cell_j;
    const int64_t fail_at = src->clone_fail_at;
    src->clone_fail_at = -1;
    for (size_t k = 0; k < src->S(); ++k) {
        if (int64_t(k) == fail_at) throw std::runtime_error("clone: injected failure at shard " + std::to_string(k));
        hip_check(hipSetDevice(src->dev[k]), "hipSetDevice");
        shyft_hip_region* c = nullptr;
        if (shyft_hip_region_clone(src->r[k], &c)) throw std::runtime_error(shyft_hip_last_error(nullptr));
        s->r.push_back(c);
        hipStream_t st = nullptr;
        hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
        s->streams.push_back(st);
        s->bufs.emplace_back(new shard_bufs());
    }
    // the clone's own communicators (and self-check) if the source combines by RCCL; a source that fell back to
    // copies stays on copies
    if (src->path == SHYFT_HIP_COMBINE_RCCL) {
        choose_path(s.get());
    } else {
        s->path = src->path;
        s->report = src->report;
    }
    return s.release();
}

}  // namespace shards
}  // namespace shyft_hip_impl
