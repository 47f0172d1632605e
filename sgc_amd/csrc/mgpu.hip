// mgpu.hip -- one process drives several devices: X_K = S^K X_0 with the
// feature columns split over them (sgc_mgpu_init / attach /
// propagate / detach / finalize, the C-ABI form of the multi-GPU path that the
// reference's single sgc_precompute call -- reddit.py:43 -> utils.py:92-97 --
// would bind to).
//
// Why the feature partition here.  The caller hands over X_0 on its own
// device and wants X_K back there.  Column f of X_{k+1} depends only on column
// f of X_k, so device d needs just its column block of X_0 (pulled once over
// xGMI: 1/P of X each) and runs all K hops over its own replica of S with no
// exchange between hops; its last hop stores straight into the caller's X_K
// (peer writes).  A row partition would first have to broadcast ALL of X_0 to
// every device (P-1 full copies out of one GPU's links) and exchange X_k after
// every hop.  Every output element is still one sequential FMA chain over its
// row in CSR order, so the result is bit-identical to one device's.
//
// Devices may repeat (virtual devices on one GPU): each entry gets its own
// stream and buffers, replicas of S are shared per physical device.  That is
// how the engine is rehearsed on a one-GPU box.
//
// Ordering: the caller's stream records `ready`; every device's stream waits
// for it, pulls its block, runs its hops and records `done`; the caller's
// stream waits for every `done`.  All asynchronous after attach (which copies
// S and builds plans synchronously, once per adjacency).
#include <algorithm>
#include <cmath>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "common.h"

namespace sgc {

int64_t plan_sorted_workspace(int64_t n_rows);
int plan_sorted(const int32_t *row_ptr, int64_t row_begin, int64_t row_end, int32_t threshold,
                int32_t hub_threshold, int32_t *plan, void *workspace, int64_t workspace_bytes,
                int64_t *counts_host, hipStream_t stream);
int launch_spmm(const int32_t *row_ptr, const int32_t *col_idx, const float *val,
                int64_t row_begin, int64_t row_end, const float *X, int64_t ldx, float *Y,
                int64_t ldy, int64_t F, const int32_t *heavy_rows, int64_t n_heavy,
                int64_t n_hub, int32_t heavy_threshold, uint32_t flags, hipStream_t stream);
int launch_pad_rows(const float *src, int64_t lds, float *dst, int64_t ldd, int64_t n_rows,
                    int64_t F, hipStream_t stream);
int64_t colsplit_workspace(int64_t n_rows, int32_t groups);
int colsplit(const int32_t *row_ptr, const int32_t *col_idx, const float *val, int64_t n_rows,
             int64_t n_cols, int32_t groups, const int32_t *cuts_host, int32_t *row_ptrs,
             int32_t *col_out, float *val_out, void *workspace, int64_t workspace_bytes,
             hipStream_t stream);
int csr_cols_ascending(const int32_t *row_ptr, const int32_t *col_idx, int64_t n_rows,
                       hipStream_t stream, bool *ascending);
int column_groups_rule(int64_t nnz, int64_t width);

namespace {

// Launch-size schedule thresholds: the rule of sgc_amd/propagate.py
// (auto_heavy_threshold / auto_hub_threshold / HUB_SERIAL_MAX_DEGREE).
int32_t heavy_threshold_for(int64_t nnz, int64_t width) {
    const double work = std::max(1.0, (double)nnz * (double)std::max<int64_t>(1, width) /
                                          (double)(1 << 23));
    const int p = (int)std::lround(std::log2(work));
    return (int32_t)std::min<int64_t>(512, std::max<int64_t>(64, int64_t(1) << std::min(p, 30)));
}

int32_t hub_threshold_for(int64_t nnz, int32_t heavy) {
    int64_t hub = nnz / 1024;
    if (nnz < (int64_t(1) << 24)) hub = std::min<int64_t>(hub, 8192);
    return (int32_t)std::max<int64_t>({(int64_t)heavy, hub, 256});
}

constexpr int64_t kHubSerialMaxDegree = 3072;

int64_t aligned_ld(int64_t F) { return (F + 31) / 32 * 32; }

// One device-resident launch plan (heavy rows heaviest first, then every
// light row longest first: SGC_SPMM_LIGHT_ORDER).
struct Plan {
    int32_t *rows = nullptr;
    int64_t n_heavy = 0, n_hub = 0;
    int32_t threshold = 0;
    uint32_t flags = 0;
};

// S on one device split into G column groups (G = 1: S itself; else
// sgc_csr_colsplit's group-major copy, row_ptrs [G][n+1] absolute into it)
// and the plans of every group per (heavy, hub) thresholds.
struct GroupSet {
    int G = 1;
    int32_t *row_ptrs = nullptr, *col = nullptr;
    float *val = nullptr;
    bool owned = false;
    std::map<std::pair<int32_t, int32_t>, std::vector<Plan>> plans;
};

// S on one physical device: the caller's arrays on the home device, a copy
// elsewhere; its column-group sets by G.
struct Replica {
    int dev = -1;
    int32_t *row_ptr = nullptr, *col = nullptr;
    float *val = nullptr;
    bool owned = false;
    std::map<int, GroupSet> sets;
};

struct Graph {
    int64_t n = 0, nnz = 0;
    bool cols_ascending = false;  // column groups allowed (checked at attach)
    std::map<int, Replica> replicas;  // physical device -> replica
};

// One entry of the device list.
struct Slot {
    int dev = -1;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    float *buf[2] = {nullptr, nullptr};  // ping-pong feature buffers [rows, ld]
    size_t buf_floats = 0;
};

struct Engine {
    std::vector<Slot> slots;
    hipEvent_t ready = nullptr;  // on the home device
    std::map<int64_t, Graph> graphs;
};

std::mutex g_mu;
std::unique_ptr<Engine> g_engine;
// Handles are unique for the whole process, not per engine: a caller's
// handle from an engine since re-initialised must never name another
// adjacency attached to the new one (it is simply unknown there).
int64_t g_next_handle = 1;

struct DeviceGuard {  // restores the caller's current device
    int saved = 0;
    DeviceGuard() { (void)hipGetDevice(&saved); }
    ~DeviceGuard() { (void)hipSetDevice(saved); }
};

hipError_t free_sets(Replica &r) {
    hipError_t first = hipSuccess;
    auto keep = [&](hipError_t e) {
        if (first == hipSuccess && e != hipSuccess) first = e;
    };
    for (auto &sv : r.sets) {
        GroupSet &gs = sv.second;
        for (auto &pv : gs.plans)
            for (Plan &p : pv.second) keep(hipFree(p.rows));
        if (gs.owned) {
            keep(hipFree(gs.row_ptrs));
            keep(hipFree(gs.col));
            keep(hipFree(gs.val));
        }
    }
    r.sets.clear();
    return first;
}

int free_engine(Engine &e) {
    hipError_t first = hipSuccess;
    auto keep = [&](hipError_t r) {
        if (first == hipSuccess && r != hipSuccess) first = r;
    };
    for (auto &kv : e.graphs)
        for (auto &rv : kv.second.replicas) {
            Replica &r = rv.second;
            keep(hipSetDevice(r.dev));
            keep(free_sets(r));
            if (r.owned) {
                keep(hipFree(r.row_ptr));
                keep(hipFree(r.col));
                keep(hipFree(r.val));
            }
        }
    e.graphs.clear();
    for (Slot &s : e.slots) {
        keep(hipSetDevice(s.dev));
        if (s.stream) keep(hipStreamSynchronize(s.stream));
        for (float *b : s.buf) keep(hipFree(b));
        if (s.done) keep(hipEventDestroy(s.done));
        if (s.stream) keep(hipStreamDestroy(s.stream));
    }
    if (e.ready && !e.slots.empty()) {
        keep(hipSetDevice(e.slots[0].dev));
        keep(hipEventDestroy(e.ready));
    }
    e.slots.clear();
    SGC_HIP_CHECK(first);
    return SGC_OK;
}

int release_graph(Graph &g) {
    for (auto &rv : g.replicas) {
        Replica &r = rv.second;
        SGC_HIP_CHECK(hipSetDevice(r.dev));
        SGC_HIP_CHECK(hipDeviceSynchronize());
        SGC_HIP_CHECK(free_sets(r));
        if (r.owned) {
            SGC_HIP_CHECK(hipFree(r.row_ptr));
            SGC_HIP_CHECK(hipFree(r.col));
            SGC_HIP_CHECK(hipFree(r.val));
        }
    }
    g.replicas.clear();
    return SGC_OK;
}

// The column-group set of a replica for G groups, split on first use on
// that device (G = 1: the replica itself).  Synchronous when it builds.
int set_for(Graph &g, Replica &r, int G, hipStream_t stream, GroupSet **out) {
    auto it = r.sets.find(G);
    if (it != r.sets.end()) {
        *out = &it->second;
        return SGC_OK;
    }
    GroupSet gs;
    gs.G = G;
    if (G == 1) {
        gs.row_ptrs = r.row_ptr;
        gs.col = r.col;
        gs.val = r.val;
    } else {
        gs.owned = true;
        const size_t nz = (size_t)std::max<int64_t>(1, g.nnz);
        SGC_HIP_CHECK(hipMalloc(&gs.row_ptrs, (size_t)G * (g.n + 1) * sizeof(int32_t)));
        SGC_HIP_CHECK(hipMalloc(&gs.col, nz * sizeof(int32_t)));
        SGC_HIP_CHECK(hipMalloc(&gs.val, nz * sizeof(float)));
        std::vector<int32_t> cuts(G + 1);
        for (int i = 0; i <= G; ++i) cuts[i] = (int32_t)((int64_t)i * g.n / G);
        const int64_t ws_bytes = colsplit_workspace(g.n, G);
        void *ws = nullptr;
        SGC_HIP_CHECK(hipMalloc(&ws, (size_t)ws_bytes));
        int rc = colsplit(r.row_ptr, r.col, r.val, g.n, g.n, G, cuts.data(), gs.row_ptrs, gs.col,
                          gs.val, ws, ws_bytes, stream);
        const hipError_t sync = hipStreamSynchronize(stream);
        (void)hipFree(ws);
        if (rc == SGC_OK && sync != hipSuccess) {
            set_error("mgpu: column split failed: %s", hipGetErrorString(sync));
            rc = SGC_EHIP;
        }
        if (rc != SGC_OK) {
            (void)hipFree(gs.row_ptrs);
            (void)hipFree(gs.col);
            (void)hipFree(gs.val);
            return rc;
        }
    }
    *out = &(r.sets[G] = std::move(gs));
    return SGC_OK;
}

// The plans of a group set at a launch width (one per group: sizes from the
// whole S's nonzeros, as the Python layer's plans), built on first use.
int plans_for(Graph &g, GroupSet &gs, int64_t width, hipStream_t stream,
              const std::vector<Plan> **out) {
    const int32_t th = heavy_threshold_for(g.nnz, width);
    const int32_t hub = std::max(th, hub_threshold_for(g.nnz, th));
    auto it = gs.plans.find({th, hub});
    if (it != gs.plans.end()) {
        *out = &it->second;
        return SGC_OK;
    }
    std::vector<Plan> plans;
    const int64_t ws_bytes = plan_sorted_workspace(g.n);
    void *ws = nullptr;
    SGC_HIP_CHECK(hipMalloc(&ws, (size_t)ws_bytes));
    int rc = SGC_OK;
    for (int k = 0; k < gs.G && rc == SGC_OK; ++k) {
        Plan p;
        p.threshold = th;
        if (hipMalloc(&p.rows, (size_t)std::max<int64_t>(1, g.n) * sizeof(int32_t)) != hipSuccess) {
            set_error("mgpu: plan allocation failed");
            rc = SGC_EHIP;
            break;
        }
        int64_t counts[3] = {0, 0, 0};
        rc = plan_sorted(gs.row_ptrs + (int64_t)k * (g.n + 1), 0, g.n, th, hub, p.rows, ws,
                         ws_bytes, counts, stream);  // synchronous
        p.n_heavy = counts[0];
        p.n_hub = counts[1];
        if (p.n_hub > 0 && counts[2] <= kHubSerialMaxDegree) p.flags |= SGC_SPMM_HUB_SERIAL;
        if (g.n > p.n_heavy) p.flags |= SGC_SPMM_LIGHT_ORDER;
        plans.push_back(p);
    }
    (void)hipFree(ws);
    if (rc != SGC_OK) {
        for (Plan &p : plans) (void)hipFree(p.rows);
        return rc;
    }
    *out = &(gs.plans[{th, hub}] = std::move(plans));
    return SGC_OK;
}

}  // namespace

int mgpu_init(int ndev, const int *devices) {
    SGC_REQUIRE(ndev >= 1 && devices, SGC_EINVAL, "mgpu_init: need at least one device");
    int count = 0;
    SGC_HIP_CHECK(hipGetDeviceCount(&count));
    for (int i = 0; i < ndev; ++i)
        SGC_REQUIRE(devices[i] >= 0 && devices[i] < count, SGC_EDEVICE,
                    "mgpu_init: device %d not present (%d visible)", devices[i], count);
    std::lock_guard<std::mutex> lock(g_mu);
    DeviceGuard guard;
    if (g_engine) {
        int rc = free_engine(*g_engine);
        g_engine.reset();
        if (rc != SGC_OK) return rc;
    }
    auto e = std::make_unique<Engine>();
    // peer access between every pair of distinct physical devices (xGMI)
    for (int i = 0; i < ndev; ++i)
        for (int j = 0; j < ndev; ++j) {
            const int a = devices[i], b = devices[j];
            if (a == b) continue;
            int can = 0;
            SGC_HIP_CHECK(hipDeviceCanAccessPeer(&can, a, b));
            SGC_REQUIRE(can, SGC_EDEVICE, "mgpu_init: device %d cannot access device %d", a, b);
            SGC_HIP_CHECK(hipSetDevice(a));
            hipError_t r = hipDeviceEnablePeerAccess(b, 0);
            if (r == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
            else SGC_HIP_CHECK(r);
        }
    for (int i = 0; i < ndev; ++i) {
        Slot s;
        s.dev = devices[i];
        SGC_HIP_CHECK(hipSetDevice(s.dev));
        SGC_HIP_CHECK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
        SGC_HIP_CHECK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        e->slots.push_back(s);
    }
    SGC_HIP_CHECK(hipSetDevice(devices[0]));
    SGC_HIP_CHECK(hipEventCreateWithFlags(&e->ready, hipEventDisableTiming));
    g_engine = std::move(e);
    return SGC_OK;
}

int mgpu_finalize() {
    std::lock_guard<std::mutex> lock(g_mu);
    if (!g_engine) return SGC_OK;
    DeviceGuard guard;
    int rc = free_engine(*g_engine);
    g_engine.reset();
    return rc;
}

int mgpu_attach(const int32_t *row_ptr, const int32_t *col_idx, const float *val, int64_t n,
                int64_t nnz, hipStream_t stream, int64_t *handle) {
    SGC_REQUIRE(row_ptr && handle && (nnz == 0 || (col_idx && val)), SGC_EINVAL,
                "mgpu_attach: null pointer");
    SGC_REQUIRE(n >= 0 && n < INT32_MAX && nnz >= 0 && nnz < INT32_MAX, SGC_ERANGE,
                "mgpu_attach: CSR exceeds the int32 limits");
    std::lock_guard<std::mutex> lock(g_mu);
    SGC_REQUIRE(g_engine, SGC_EINVAL, "mgpu_attach: sgc_mgpu_init first");
    Engine &e = *g_engine;
    DeviceGuard guard;
    const int home = e.slots[0].dev;
    SGC_HIP_CHECK(hipSetDevice(home));
    SGC_HIP_CHECK(hipStreamSynchronize(stream));  // S may still be in the making
    Graph g;
    g.n = n;
    g.nnz = nnz;
    if (nnz > 0) {
        const int rc = csr_cols_ascending(row_ptr, col_idx, n, stream, &g.cols_ascending);
        if (rc != SGC_OK) return rc;
    }
    for (const Slot &s : e.slots) {
        if (g.replicas.count(s.dev)) continue;
        Replica r;
        r.dev = s.dev;
        if (s.dev == home) {
            r.row_ptr = const_cast<int32_t *>(row_ptr);
            r.col = const_cast<int32_t *>(col_idx);
            r.val = const_cast<float *>(val);
        } else {
            r.owned = true;
            SGC_HIP_CHECK(hipSetDevice(s.dev));
            SGC_HIP_CHECK(hipMalloc(&r.row_ptr, (size_t)(n + 1) * sizeof(int32_t)));
            SGC_HIP_CHECK(hipMalloc(&r.col, (size_t)std::max<int64_t>(1, nnz) * sizeof(int32_t)));
            SGC_HIP_CHECK(hipMalloc(&r.val, (size_t)std::max<int64_t>(1, nnz) * sizeof(float)));
            SGC_HIP_CHECK(hipMemcpyPeer(r.row_ptr, s.dev, row_ptr, home,
                                        (size_t)(n + 1) * sizeof(int32_t)));
            if (nnz) {
                SGC_HIP_CHECK(hipMemcpyPeer(r.col, s.dev, col_idx, home, (size_t)nnz * 4));
                SGC_HIP_CHECK(hipMemcpyPeer(r.val, s.dev, val, home, (size_t)nnz * 4));
            }
        }
        g.replicas[s.dev] = r;
    }
    const int64_t h = g_next_handle++;
    e.graphs[h] = std::move(g);
    *handle = h;
    return SGC_OK;
}

int mgpu_detach(int64_t handle) {
    std::lock_guard<std::mutex> lock(g_mu);
    if (!g_engine) return SGC_OK;  // finalize already freed everything
    auto it = g_engine->graphs.find(handle);
    if (it == g_engine->graphs.end()) return SGC_OK;
    DeviceGuard guard;
    int rc = release_graph(it->second);
    g_engine->graphs.erase(it);
    return rc;
}

int mgpu_propagate(int64_t handle, const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t F,
                   int32_t K, hipStream_t stream) {
    SGC_REQUIRE(X && Y, SGC_EINVAL, "mgpu_propagate: null pointer");
    SGC_REQUIRE(F > 0 && F < (1 << 24) && ldx >= F && ldy >= F && K >= 1, SGC_EINVAL,
                "mgpu_propagate: bad F/ld/K (%lld/%lld/%lld/%d)", (long long)F, (long long)ldx,
                (long long)ldy, (int)K);
    std::lock_guard<std::mutex> lock(g_mu);
    SGC_REQUIRE(g_engine, SGC_EINVAL, "mgpu_propagate: sgc_mgpu_init first");
    Engine &e = *g_engine;
    auto git = e.graphs.find(handle);
    SGC_REQUIRE(git != e.graphs.end(), SGC_EINVAL, "mgpu_propagate: unknown handle %lld",
                (long long)handle);
    Graph &g = git->second;
    if (g.n == 0) return SGC_OK;
    DeviceGuard guard;
    const int P = (int)e.slots.size();
    // column blocks: B = ceil(F / P) rounded up to 4 floats (16-B lanes);
    // the last blocks may be short or empty (sgc_amd.distributed.feature_bounds)
    int64_t B = (F + P - 1) / P;
    B = (B + 3) / 4 * 4;
    // 1. everything that may fail or synchronise -- column groups (the size
    // rule of the Python layer, rows with ascending columns only), plans,
    // buffers -- before any work is enqueued, so an error leaves nothing in
    // flight
    struct Job {
        int64_t c0 = 0, w = 0, ld = 0;
        GroupSet *gs = nullptr;
        const std::vector<Plan> *plans = nullptr;
    };
    std::vector<Job> jobs(P);
    for (int d = 0; d < P; ++d) {
        Slot &s = e.slots[d];
        Job &j = jobs[d];
        j.c0 = std::min<int64_t>(d * B, F);
        j.w = std::min<int64_t>((d + 1) * B, F) - j.c0;
        if (j.w <= 0) continue;
        SGC_HIP_CHECK(hipSetDevice(s.dev));
        Replica &r = g.replicas.at(s.dev);
        const int G = g.cols_ascending ? column_groups_rule(g.nnz, j.w) : 1;
        int rc = set_for(g, r, G, s.stream, &j.gs);
        if (rc == SGC_OK) rc = plans_for(g, *j.gs, j.w, s.stream, &j.plans);
        if (rc != SGC_OK) return rc;
        j.ld = aligned_ld(j.w);
        const size_t need = (size_t)g.n * (size_t)j.ld;
        const int nb = K >= 2 ? 2 : 1;
        if (s.buf_floats < need) {
            SGC_HIP_CHECK(hipStreamSynchronize(s.stream));
            for (float *&b : s.buf) {
                SGC_HIP_CHECK(hipFree(b));
                b = nullptr;
            }
            s.buf_floats = 0;
            for (int i = 0; i < nb; ++i) SGC_HIP_CHECK(hipMalloc(&s.buf[i], need * sizeof(float)));
            s.buf_floats = need;
        } else if (nb == 2 && !s.buf[1]) {
            SGC_HIP_CHECK(hipMalloc(&s.buf[1], s.buf_floats * sizeof(float)));
        }
    }
    // 2. enqueue.  From the first wait on `ready` on, every exit records
    // `done` on the slots that waited and makes the caller's stream wait for
    // them: the caller never frees X / Y under a device still reading or
    // writing them.
    struct Join {
        Engine &e;
        hipStream_t stream;
        int started = 0;  // slots whose stream waits on `ready`
        bool armed = true;
        ~Join() {
            if (!armed) return;
            for (int d = 0; d < started; ++d) {
                (void)hipSetDevice(e.slots[d].dev);
                (void)hipEventRecord(e.slots[d].done, e.slots[d].stream);
            }
            (void)hipSetDevice(e.slots[0].dev);
            for (int d = 0; d < started; ++d) (void)hipStreamWaitEvent(stream, e.slots[d].done, 0);
        }
    } join{e, stream};
    SGC_HIP_CHECK(hipSetDevice(e.slots[0].dev));
    SGC_HIP_CHECK(hipEventRecord(e.ready, stream));
    for (int d = 0; d < P; ++d) {
        Slot &s = e.slots[d];
        const Job &j = jobs[d];
        SGC_HIP_CHECK(hipSetDevice(s.dev));
        SGC_HIP_CHECK(hipStreamWaitEvent(s.stream, e.ready, 0));
        join.started = d + 1;
        if (j.w > 0) {
            // pull this device's column block of X_0 (peer reads over xGMI)
            int rc = launch_pad_rows(X + j.c0, ldx, s.buf[0], j.ld, g.n, j.w, s.stream);
            if (rc != SGC_OK) return rc;
            const float *src = s.buf[0];
            for (int h = 0; h < K; ++h) {
                const bool last = h == K - 1;
                float *dst = last ? Y + j.c0 : s.buf[(h + 1) & 1];
                const int64_t ldd = last ? ldy : j.ld;
                // the engine's buffers may be read / written in their pad
                // columns; the caller's Y never (its next block lives there)
                const uint32_t flags =
                    SGC_SPMM_X_PADDED | (last ? 0u : (uint32_t)SGC_SPMM_Y_PADDED) |
                    (g.n < (int64_t(1) << 24) && g.n * j.ld * 4 < (int64_t(1) << 32)
                         ? (uint32_t)SGC_SPMM_X_UNDER_4G : 0u);
                // column groups: group 0 plain, groups 1.. continue its chains
                for (int k = 0; k < j.gs->G; ++k) {
                    const Plan &pl = (*j.plans)[k];
                    rc = launch_spmm(j.gs->row_ptrs + (int64_t)k * (g.n + 1), j.gs->col,
                                     j.gs->val, 0, g.n, src, j.ld, dst, ldd, j.w, pl.rows,
                                     pl.n_heavy, pl.n_hub, pl.threshold,
                                     flags | pl.flags | (k ? (uint32_t)SGC_SPMM_ACCUMULATE : 0u),
                                     s.stream);
                    if (rc != SGC_OK) return rc;
                }
                src = dst;
            }
        }
        SGC_HIP_CHECK(hipEventRecord(s.done, s.stream));
    }
    join.armed = false;
    SGC_HIP_CHECK(hipSetDevice(e.slots[0].dev));
    for (const Slot &s : e.slots) SGC_HIP_CHECK(hipStreamWaitEvent(stream, s.done, 0));
    return SGC_OK;
}

}  // namespace sgc
