// dcol_capi.cpp — host side of the C-ABI declared in include/dcol.h.
//
//  * dcol_table_create: digests the primitive descriptors into DevShape records and a pool
//    of orthant-row descriptors (DevRow), uploaded once to HBM.  This is the static part of
//    problem_matrices() (primitives/problem_matrices.py:4-209): the per-type constant rows;
//    the pose-dependent part (DCM, rotation, h) runs inside the kernel.
//  * dcol_plan_create: classifies each pair (combine_problem_matrices.py:3-70 cases 1-3 vs
//    the unsupported case 4) and buckets pairs by kernel variant (N, NSOC, OMAX).
//  * dcol_plan_run: one kernel launch per non-empty bucket, asynchronous on the caller's
//    stream, no allocation (graph-capturable) -- or, for a small plan that mixes variants,
//    ONE fused launch covering every bucket (dcol_kernels_fused.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <list>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "../../include/dcol.h"
#include "dcol_device.hpp"
#include "dcol_host.hpp"
#include "dcol_launch.hpp"

using namespace dcol;
using namespace dcol_host;

namespace {

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(DCOL_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    bool switched = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) switched = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (switched && prev >= 0) (void)hipSetDevice(prev);
    }
};

// The side streams of a device, created once per process at the first table of the device
// and shared by all tables.  Early on purpose: HIP maps streams onto a few hardware queues
// (GPU_MAX_HW_QUEUES, 4 by default) in creation order, and side streams created after a
// framework's stream pool (torch creates 32 at its first side stream) can share a queue with
// each other or with the caller's stream, which serialises the fan-out -- measured on the
// 1M mixed plan: 1.25 ms per solve with late side streams, 1.10 ms with early ones.
struct DeviceSide {
    std::mutex mu;
    bool tried = false, ok = false;
    hipStream_t s[kSideStreams] = {};
};
DeviceSide& device_side(int dev) {
    static DeviceSide g[64];
    return g[dev & 63];
}
// side streams per device: 3 (with the caller's stream, 4 = HIP's default hardware queues),
// DCOL_SIDE_STREAMS=<1..7> for A/B runs (then raise GPU_MAX_HW_QUEUES to match)
int side_streams() {
    static const int n = [] {
        const char* e = std::getenv("DCOL_SIDE_STREAMS");
        const int v = e ? std::atoi(e) : 3;
        return v < 1 ? 1 : (v > kSideStreams ? kSideStreams : v);
    }();
    return n;
}
// side streams a plan that fills the GPU fans out over: 2 -- three buckets in flight with the
// caller's stream.  Fewer concurrent buckets finish a large mixed step sooner: the
// one-wave-per-SIMD kernels (400-500 registers) need a whole SIMD's register file and wait
// behind co-running buckets' waves when four run at once (1M mixed plan, synchronised
// steps: 0.87 ms at 2 against 0.94 ms at 3 and 1).  A small plan (its
// buckets cannot fill the GPU, each runs its latency configuration) keeps every side
// stream.  DCOL_SIDE_STREAMS_LARGE=<1..side_streams()> for A/B runs.
int large_side_streams() {
    static const int n = [] {
        const char* e = std::getenv("DCOL_SIDE_STREAMS_LARGE");
        const int v = e ? std::atoi(e) : 2;
        return v < 1 ? 1 : (v > side_streams() ? side_streams() : v);
    }();
    return n;
}

// dcol_prox_pair's one-pair server: how long (us) it stays resident without a request
// (DCOL_PAIR_SERVER_IDLE_US, default 1000); DCOL_PAIR_SERVER=0: no server, one launch per
// call.  Read per call (tests switch it).
int pair_server_idle_us() {
    const char* on = std::getenv("DCOL_PAIR_SERVER");
    if (on && std::atoi(on) == 0) return 0;
    const char* e = std::getenv("DCOL_PAIR_SERVER_IDLE_US");
    const long v = e ? std::atol(e) : 1000;
    return v < 0 ? 0 : (v > 1000000 ? 1000000 : (int)v);
}
// Tables of the process, so that dcol_shutdown can stop every resident pair server before
// the process's HIP context and the servers' mapped mailboxes go away.  dcol_shutdown runs
// from an exit handler registered at the first server start -- after the HIP runtime
// initialised, so before its own exit-time teardown (exit handlers run last-registered
// first) -- and from the Python binding's atexit hook (dcol_amd/_lib.py).  Lock order:
// g_tables_mu, then a table's mu (dcol_prox_pair holds only the latter).
std::mutex g_tables_mu;
std::vector<dcol_table*> g_tables;
std::atomic<bool> g_shutdown{false};   // set by dcol_shutdown: no new server starts
std::atomic<int> g_server_tables{0};   // tables whose pair server was ever started
std::once_flag g_exit_hook;
// how long table destroy / shutdown / a restart wait for a server to leave (it leaves at its
// next poll, i.e. after at most the solve in hand: microseconds)
constexpr int kServerStopMs = 5000;

bool device_side_streams(int dev, hipStream_t out[kSideStreams]) {
    DeviceSide& d = device_side(dev);
    std::lock_guard<std::mutex> lk(d.mu);
    if (!d.tried) {
        d.tried = true;
        d.ok = true;
        for (int i = 0; d.ok && i < side_streams(); ++i) d.ok = hipStreamCreateWithFlags(&d.s[i], hipStreamNonBlocking) == hipSuccess;
        if (!d.ok) (void)hipGetLastError();
    }
    if (d.ok)
        for (int i = 0; i < side_streams(); ++i) out[i] = d.s[i];
    return d.ok;
}

}  // namespace

static_assert(dcol::kRec == DCOL_REC, "record width");

namespace dcol {
// pairs rejected on the host (unsupported combination / too many rows)
__global__ void __launch_bounds__(256) reject_kernel(KArgs A, int32_t code) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.n) return;
    const int64_t pi = A.perm ? (int64_t)A.perm[A.slot0 + t] : (A.slot0 + t);
    const int64_t B = A.B;
    const double nan = __builtin_nan("");
    if (A.alpha) A.alpha[pi] = nan;
    if (A.iters) A.iters[pi] = 0;
    if (A.status) A.status[pi] = code;
    if ((A.flags & F_CONTACT) && A.contact)
        for (int q = 0; q < 3; ++q) A.contact[q * B + pi] = nan;
    if ((A.flags & (F_GRAD_FD | F_GRAD_ENV | F_GRAD_IMP)) && A.grad)
        for (int q = 0; q < 12; ++q) A.grad[q * B + pi] = nan;
    if (A.rec) {
        double* r = A.rec + (int64_t)kRec * pi;
        for (int q = 0; q < 13; ++q) r[q] = nan;
        r[13] = rec_ints(code, 0);
    }
}

}  // namespace dcol

struct dcol_table {
    int device = 0;
    std::vector<DevShape> shapes;
    std::vector<DevRow> rows;
    DevShape* d_shapes = nullptr;
    DevRow* d_rows = nullptr;
    // staging for dcol_prox_batch_host: device buffer + pinned host buffer (grow-only)
    std::mutex mu;
    void* stage = nullptr;
    size_t stage_bytes = 0;
    void* hstage = nullptr;
    size_t hstage_bytes = 0;
    int simds = 1024;   // SIMDs of the device (CUs x 4): below one wave per SIMD a launch is latency-bound
    // side streams for the concurrent variant launches of mixed plans: the process-wide set
    // of the device (device_side_streams), shared by every table
    hipStream_t side[kSideStreams] = {};
    bool side_ready = false;
    // dcol_prox_pair: one-pair plans per (shape1, shape2), at most DCOL_PAIR_PLANS_MAX, least
    // recently used first out (pair_lru: most recent at the front), a stream for their
    // launches, and the device-mapped pinned mailbox (PairBox: poses, outputs, the request of
    // the one-pair server and its stream)
    std::list<std::pair<int64_t, dcol_plan*>> pair_lru;
    std::unordered_map<int64_t, std::list<std::pair<int64_t, dcol_plan*>>::iterator> pair_plans;
    hipStream_t pair_stream = nullptr;
    hipStream_t server_stream = nullptr;
    PairBox* pair_host = nullptr;
    PairBox* pair_dev = nullptr;
    int64_t wall_ticks_us = 0;     // device wall-clock ticks per microsecond (0: unknown, no server)
    bool server_launched = false;  // a server was launched at least once (destroy stops it)
    int64_t n_served = 0, n_launched = 0, n_starts = 0;   // dcol_table_pair_stats
    int32_t srv_mismatch = 0;      // consecutive calls whose flags / tol / max_iter differ from the server's
    std::atomic<bool> stop_req{false};   // a batch launch asked the server to leave (yield_pair_servers)
    double srv_us = 0.0, srv_cycles = 0.0;
};

struct Launch {
    int kind;       // 0 = solve, 1 = reject
    int N, nsoc, omax, lpp;
    int oe = 0;          // row-partitioned bucket (extra-row slots; 0: dense-row kernels)
    // suspend / resume pair (DCOL_PLAN_SUSPEND): continuation entries, their buffers
    bool susp = false;
    int susp_fields = 0;
    int64_t susp_cap = 0;
    int32_t* d_susp_count = nullptr;
    int32_t* d_susp_pi = nullptr;
    double* d_susp_state = nullptr;
    bool full = false;   // every pair has o == omax: the padding-free kernel (DCOL_FULL_VARIANTS) if built
    bool ball = false;   // every SOC block is a ball block: the structured kernel (DCOL_BALL_VARIANTS) if built
    bool cone = false;   // every SOC block is a cone block (N = 4): DCOL_CONE_VARIANTS if built
    bool box = false;    // every pair is box x box (DevShape::boxp; with full): DCOL_BOX_VARIANTS if built
    int flags() const { return (full ? LF_FULL : 0) | (ball ? LF_BALL : 0) | (cone ? LF_CONE : 0) | (box ? LF_BOX : 0); }
    int32_t code;   // reject status
    int64_t slot0, n;
    int lane = 0;   // 0 = caller's stream, 1..kSideStreams = table side stream
};

struct dcol_plan {
    const dcol_table* table = nullptr;
    int64_t B = 0;
    int32_t* d_s1 = nullptr;
    int32_t* d_s2 = nullptr;
    int32_t* d_perm = nullptr;   // nullptr when the whole batch is one variant
    bool owns = false;           // device arrays owned (false: views into table staging)
    std::vector<Launch> launches;
    int lanes = 1;               // streams the launches are spread over (1 = serial)
    bool small = false;          // the plan cannot fill the GPU (bucket_pairs: small_plan)
    std::vector<int> issue;      // launch issue order (assign_lanes: longest first); empty = as built
    hipEvent_t fork = nullptr;   // recorded on the caller's stream, awaited by the side streams
    hipEvent_t join[kSideStreams] = {};
    // fused launch (small mixed plans) or packed launch (mid-size plans, packed = true): one
    // segment per solve bucket, in descending per-pair cost (plan_segments)
    std::vector<FusedSeg> segs;
    FusedSeg* d_segs = nullptr;
    int64_t fused_blocks = 0;
    bool packed = false;
    bool fused() const { return !segs.empty(); }
    void* d_susp = nullptr;      // DCOL_PLAN_SUSPEND scratch (one allocation for every such launch)
    ~dcol_plan() {
        if (fork) (void)hipEventDestroy(fork);
        for (hipEvent_t& e : join)
            if (e) (void)hipEventDestroy(e);
    }
};

namespace {

// Stop a table's pair server, if one may be running: raise `stop` and wait for the server
// stream to drain, at most timeout_ms.  false: it did not drain -- the wave may still read
// the mailbox, which must then stay allocated.  The caller holds t->mu (or owns t).
bool stop_pair_server(dcol_table* t, int timeout_ms) {
    if (!t->server_launched || !t->pair_host) return true;
    __atomic_store_n(&t->pair_host->stop, 1, __ATOMIC_SEQ_CST);
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipStreamQuery(t->server_stream);
        if (q != hipErrorNotReady) {
            if (q != hipSuccess) (void)hipGetLastError();
            break;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) return false;
        std::this_thread::yield();
    }
    __atomic_store_n(&t->pair_host->stop, 0, __ATOMIC_SEQ_CST);
    __atomic_store_n(&t->pair_host->alive, 0, __ATOMIC_SEQ_CST);
    return true;
}

// A batch launch that can fill `device` (a plan that is not small: bucket_pairs) asks every
// resident pair server there to leave (it does after
// the request in hand, at its next poll), without waiting: a kernel resident beside a batch
// plan slowed the plan by 1.3-2x depending on the server stream's kind and the number of
// hardware queues (tools/server_tax.py, profiles/r05_d/, r05_e/), so the latency path gives
// way to the throughput path.  The table's next dcol_prox_pair drains it and starts a new
// server (one launch, ~10 us).  Small plans (ALTRO-sized batches, one-pair launches) leave it
// resident: a caller interleaving them with drop-in calls would otherwise restart the server
// at nearly every pair call, and a latency-bound plan of a few waves is not what the
// server's hardware-queue tax was measured on.
void yield_pair_servers(int device) {
    if (g_server_tables.load(std::memory_order_acquire) == 0) return;
    static const bool off = [] {   // DCOL_PAIR_SERVER_YIELD=0: the server stays (A/B: tools/server_tax.py)
        const char* e = std::getenv("DCOL_PAIR_SERVER_YIELD");
        return e && std::atoi(e) == 0;
    }();
    if (off) return;
    std::lock_guard<std::mutex> lk(g_tables_mu);
    for (dcol_table* t : g_tables) {
        // (pair_host is published by dcol_prox_pair with a release store after its memset)
        PairBox* h = __atomic_load_n(&t->pair_host, __ATOMIC_ACQUIRE);
        if (t->device != device || !h) continue;
        if (!__atomic_load_n(&h->alive, __ATOMIC_ACQUIRE)) continue;
        __atomic_store_n(&h->stop, 1, __ATOMIC_SEQ_CST);
        t->stop_req.store(true, std::memory_order_release);
    }
}

hipError_t launch_variant(int N, int nsoc, int omax, int lpp, int flags, const KArgs& a, hipStream_t st, int oe = 0) {
    if (oe > 0) {
        if (N == 5 && nsoc == 1) return launch_part_n5s1(omax, oe, lpp, flags, a, st);
        if (N == 5 && nsoc == 2) return launch_part_n5s2(omax, oe, lpp, flags, a, st);
        if (N == 6 && nsoc == 1) return launch_part_n6s1(omax, oe, lpp, flags, a, st);
        if (N == 6 && nsoc == 2) {   // the ball-row copies first (a bucket's list order), then the dense ones
            const hipError_t e = launch_part_n6s2(omax, oe, lpp, flags, a, st);
            return e == hipErrorInvalidValue ? launch_part_n6s2_dense(omax, oe, lpp, flags, a, st) : e;
        }
        return hipErrorInvalidValue;
    }
    if (N == 4) return launch_n4(nsoc, omax, lpp, flags, a, st);
    if (N == 5) return launch_n5(nsoc, omax, lpp, flags, a, st);
    if (N == 6) return launch_n6(nsoc, omax, lpp, flags, a, st);
    if (N == 7) return launch_n7(nsoc, omax, lpp, flags, a, st);
    if (N == 8) return launch_n8(nsoc, omax, lpp, flags, a, st);
    return hipErrorInvalidValue;
}

}  // namespace

extern "C" {

int dcol_abi_version(void) { return DCOL_ABI_VERSION; }

const char* dcol_status_string(int32_t s) {
    switch (s) {
        case DCOL_OK: return "ok";
        case DCOL_MAXITER: return "Maximum number of iterations reached, PDIP failed";
        case DCOL_UNSUPPORTED: return "Failed to combine problem matrices.";
        case DCOL_NOT_PD: return "Matrix is not positive definite";
        case DCOL_NONFINITE: return "array must not contain infs or NaNs";
        case DCOL_TOO_LARGE: return "pair exceeds the engine's orthant-row capacity";
        default: return "unknown status";
    }
}

const char* dcol_last_error(void) { return last_error().c_str(); }

int dcol_device_count(int32_t* count) {
    if (!count) return fail(DCOL_ERR_ARG, "count is NULL");
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    *count = n;
    return DCOL_SUCCESS;
}

int dcol_table_create(const dcol_shape_desc* shapes, int32_t n, int32_t device, dcol_table** out) {
    if (!out || n < 0 || (n > 0 && !shapes)) return fail(DCOL_ERR_ARG, "dcol_table_create: bad arguments");
    *out = nullptr;
    auto* t = new (std::nothrow) dcol_table();
    if (!t) return fail(DCOL_ERR_NOMEM, "host allocation failed");
    t->device = device;
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            t->simds = 4 * cus;
        else
            (void)hipGetLastError();
    }
    t->shapes.resize(n);
    init_row_pool(t->rows);
    for (int32_t i = 0; i < n; ++i) {
        int rc = digest_shape(shapes[i], i, t->shapes[i], t->rows);
        if (rc != DCOL_SUCCESS) {
            delete t;
            return rc;
        }
    }
    if (t->shapes.empty()) t->shapes.resize(1);
    DeviceGuard g(device);
    hipError_t e = hipMalloc(&t->d_shapes, sizeof(DevShape) * t->shapes.size());
    if (e == hipSuccess) e = hipMalloc(&t->d_rows, sizeof(DevRow) * t->rows.size());
    if (e == hipSuccess) e = hipMemcpy(t->d_shapes, t->shapes.data(), sizeof(DevShape) * t->shapes.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(t->d_rows, t->rows.data(), sizeof(DevRow) * t->rows.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (t->d_shapes) (void)hipFree(t->d_shapes);
        if (t->d_rows) (void)hipFree(t->d_rows);
        delete t;
        return fail(DCOL_ERR_HIP, std::string("dcol_table_create: ") + hipGetErrorString(e));
    }
    t->shapes.resize(n);
    t->side_ready = device_side_streams(device, t->side);   // early: see DeviceSide
    {
        std::lock_guard<std::mutex> lk(g_tables_mu);
        g_tables.push_back(t);
    }
    *out = t;
    return DCOL_SUCCESS;
}

int dcol_table_destroy(dcol_table* t) {
    if (!t) return DCOL_SUCCESS;
    DeviceGuard g(t->device);
    // the server exits at its next poll; one that does not (a hung device) keeps the whole
    // table -- its wave may still read the shape table and the mailbox -- registered, so that
    // dcol_shutdown still sees it and can stop it before the process's HIP context goes away,
    // and the call fails.  Only a table whose server has left is unregistered and freed.
    {
        std::lock_guard<std::mutex> tl(t->mu);
        if (!stop_pair_server(t, kServerStopMs))
            return fail(DCOL_ERR_HIP, "dcol_table_destroy: the pair server did not stop within 5 s (table kept)");
    }
    {
        std::lock_guard<std::mutex> lk(g_tables_mu);
        g_tables.erase(std::remove(g_tables.begin(), g_tables.end(), t), g_tables.end());
        if (t->server_launched) g_server_tables.fetch_sub(1, std::memory_order_acq_rel);
    }
    for (auto& kv : t->pair_lru) dcol_plan_destroy(kv.second);
    if (t->pair_stream) (void)hipStreamDestroy(t->pair_stream);
    if (t->server_stream) (void)hipStreamDestroy(t->server_stream);
    if (t->pair_host) (void)hipHostFree(t->pair_host);
    if (t->d_shapes) (void)hipFree(t->d_shapes);
    if (t->d_rows) (void)hipFree(t->d_rows);
    if (t->stage) (void)hipFree(t->stage);
    if (t->hstage) (void)hipHostFree(t->hstage);
    delete t;
    return DCOL_SUCCESS;
}

int dcol_table_size(const dcol_table* t, int32_t* n) {
    if (!t || !n) return fail(DCOL_ERR_ARG, "dcol_table_size: NULL argument");
    *n = (int32_t)t->shapes.size();
    return DCOL_SUCCESS;
}

int dcol_pair_dims(const dcol_table* t, int32_t s1, int32_t s2, int32_t* m, int32_t* n, int32_t* n_soc, int32_t* status) {
    if (!t) return fail(DCOL_ERR_ARG, "dcol_pair_dims: NULL table");
    const int32_t ns = (int32_t)t->shapes.size();
    if (s1 < 0 || s1 >= ns || s2 < 0 || s2 >= ns) return fail(DCOL_ERR_ARG, "dcol_pair_dims: shape id out of range");
    const DevShape& a = t->shapes[s1];
    const DevShape& b = t->shapes[s2];
    PairClass c = classify(a, b);
    const int q1 = a.soc_kind == SOC_NONE ? 0 : (a.soc_kind == SOC_CONE ? 3 : 4);
    const int q2 = b.soc_kind == SOC_NONE ? 0 : (b.soc_kind == SOC_CONE ? 3 : 4);
    if (m) *m = c.o + q1 + q2;
    if (n) *n = c.N;
    if (n_soc) *n_soc = c.nsoc;
    if (status) *status = c.status;
    return DCOL_SUCCESS;
}

}  // extern "C"

namespace {
void assign_lanes(dcol_plan* p);

// DCOL_SMALL_FANOUT=1: a small plan the fused kernel cannot take fans its latency-configured
// buckets out (the behaviour before the packed launch; A/B runs)
bool small_fanout() {
    static const bool on = std::getenv("DCOL_SMALL_FANOUT") != nullptr;
    return on;
}

// DCOL_NO_BALL=1: ball-SOC pairs run the dense kernels too (A/B runs, tests)
bool ball_disabled() {
    static const bool off = std::getenv("DCOL_NO_BALL") != nullptr;
    return off;
}
// DCOL_NO_BOX=1: box x box pairs run the padding-free dense-row kernel (A/B runs, tests)
bool box_disabled() {
    static const bool off = std::getenv("DCOL_NO_BOX") != nullptr;
    return off;
}

// DCOL_NO_CONE=1: cone-SOC pairs run the dense (padded) kernels (A/B runs, tests)
bool cone_disabled() {
    static const bool off = std::getenv("DCOL_NO_CONE") != nullptr;
    return off;
}

// Lanes below which a plan counts as small -- it cannot fill the GPU: every bucket takes its
// latency configuration and a mixed plan runs as one fused launch (bucket_pairs, plan_fuse).
// 64 x SIMDs (one wave per SIMD); DCOL_SMALL_PLAN_LANES=<n> for A/B runs.
int64_t small_lanes(const dcol_table* t) {
    static const int64_t v = [] {
        const char* e = std::getenv("DCOL_SMALL_PLAN_LANES");
        return e ? std::atoll(e) : 0LL;
    }();
    return v > 0 ? v : 64LL * t->simds;
}

// A launch too small to fill the GPU runs the configuration with the shortest per-pair
// latency: fewest orthant slots per lane (omax / lpp), over the pair's bucket and the larger
// buckets up to twice its rows (a tight bucket compiled only with LPP 2 -- 6 or 10 rows --
// loses to the next bucket's 8-lane groups), fewer rows on ties.
void latency_config(Launch& L) {
    if (L.oe > 0) {   // row-partitioned bucket: its largest compiled LPP
        L.lpp = part_lpp(L.N, L.nsoc, L.omax, L.oe, true);
        return;
    }
    const int fl = L.ball ? 2 : (L.cone ? 4 : 0);
    int best_o = L.omax, best_l = max_lpp(L.N, L.nsoc, L.omax, fl);
    for (const int om : buckets().at({L.N, L.nsoc})) {
        if (om <= L.omax || om > 2 * L.omax) continue;
        const int l = max_lpp(L.N, L.nsoc, om, fl);
        if (om * best_l < best_o * l) {   // om / l < best_o / best_l
            best_o = om;
            best_l = l;
        }
    }
    if (best_o != L.omax) L.full = false;   // the pairs no longer fill the bucket
    L.omax = best_o;
    L.lpp = best_l;
}

// Classify + bucket (counting sort by variant key).  Fills p->launches and the slot->pair
// permutation; returns DCOL_SUCCESS or an error.
// O(B): each distinct (shape1, shape2) is classified once (a dense S x S cache when S^2 is
// at most 4M cells and small against B, else a hash map), then a stable counting sort by
// group, groups in key order.
// fused_part: a row-partitioned bucket is used only where the fused small-plan kernel has
// its case (the retry of a small plan that would otherwise lose its single fused launch;
// the other pairs take the dense-row kernels, which the fused kernel covers)
// lat_part: a row-partitioned bucket compiled only for one lane per pair is not used (the
// retry of a plan that cannot fill the GPU: one lane working through every row of the pair
// is slower than the dense rows' multi-lane groups -- polygon x box, 1,000 pairs: 84 us in
// the (11, 5) one-lane bucket against 52 us in the dense (6, 1, 12) four-lane kernel)
// small_out: set to whether the plan cannot fill the GPU (its buckets took their latency
// configurations); force_large: bucket as a plan that fills it (throughput configurations:
// the packed launch of a small plan the fused kernel cannot take, bucket_and_fuse)
int bucket_pairs(const dcol_table* t, int64_t B, const int32_t* s1, const int32_t* s2, dcol_plan* p,
                 std::vector<int32_t>& perm, bool case4, bool fused_part = false, bool lat_part = false,
                 bool* small_out = nullptr, bool force_large = false) {
    const int32_t ns = (int32_t)t->shapes.size();
    // kind, N, nsoc, omax, lpp, ball (SOC blocks all balls: no cone), code, oe (row partition)
    using Key = std::tuple<int, int, int, int, int, int, int, int>;
    struct Group {
        Key key;
        bool full = true;   // every pair class of the group has o == omax
        int64_t n = 0, at = 0;
    };
    std::map<Key, int32_t> gid_of_key;
    std::vector<Group> groups;
    auto classify_pair = [&](int32_t i1, int32_t i2) -> int32_t {
        const DevShape& a = t->shapes[i1];
        const DevShape& b = t->shapes[i2];
        PairClass c = classify(a, b, case4);
        // SOC form: 1 every block a ball (BALL kernels), 2 every block a cone and N = 4
        // (CONE kernels), 0 dense
        const bool none_cone = a.soc_kind != SOC_CONE && b.soc_kind != SOC_CONE;
        const bool all_cone = a.soc_kind != SOC_BALL && b.soc_kind != SOC_BALL;
        if (fused_part && c.status == DCOL_OK && c.oe > 0 &&
            fused_vid(c.N, c.nsoc, c.omax, part_lpp(c.N, c.nsoc, c.omax, c.oe, true),
                      (none_cone && !ball_disabled()) ? LF_BALL : 0, c.oe) < 0)
            c = classify(a, b, case4, false);
        if (lat_part && c.status == DCOL_OK && c.oe > 0 && part_lpp(c.N, c.nsoc, c.omax, c.oe, true) < 2)
            c = classify(a, b, case4, false);
        // (3: box x box in the 12-row bucket -- the BOX kernels' axis-pair rows; nsoc == 0)
        const int ball = c.nsoc == 0 ? ((a.boxp && b.boxp && c.N == 4 && c.omax == 12 && c.o == 12 && !box_disabled()) ? 3 : 0)
                         : (none_cone && !ball_disabled()) ? 1
                         : (all_cone && c.N == 4 && !cone_disabled()) ? 2 : 0;
        // a row-partitioned bucket only where its SOC flavour is compiled: the x polytope
        // (NSOC = 1) buckets exist only with ball rows, so with DCOL_NO_BALL those pairs take
        // the dense-row kernels (N and NSOC do not depend on the partition, so `ball` stands)
        if (c.status == DCOL_OK && c.oe > 0 && !part_flavour_built(c.N, c.nsoc, c.omax, c.oe, c.lpp, ball == 1))
            c = classify(a, b, case4, false);
        // flavour's own list (row-partitioned buckets have theirs: PairClass::lpp)
        if (c.status == DCOL_OK && (ball == 1 || ball == 2) && c.oe == 0) c.lpp = choose_lpp(c.N, c.nsoc, c.omax, 2 * ball);
        Key k = c.status == DCOL_OK ? Key{0, c.N, c.nsoc, c.omax, c.lpp, ball, 0, c.oe} : Key{1, 0, 0, 0, 0, 0, c.status, 0};
        auto it = gid_of_key.emplace(k, (int32_t)groups.size()).first;
        if (it->second == (int32_t)groups.size()) groups.push_back(Group{k});
        Group& g = groups[it->second];
        g.full = g.full && c.o == c.omax;
        return it->second;
    };
    // dense cache only when it is small against the batch (its fill is O(S^2): a small
    // batch against a big table takes the hash map)
    const int64_t cells = (int64_t)ns * ns;
    const bool dense = cells <= ((int64_t)1 << 22) && cells <= 16 * B + 4096;
    std::vector<int32_t> cache(dense ? (size_t)ns * ns : 0, -1);
    std::unordered_map<int64_t, int32_t> sparse;
    std::vector<int32_t> gid((size_t)B);
    for (int64_t i = 0; i < B; ++i) {
        const int32_t i1 = s1[i], i2 = s2[i];
        if (i1 < 0 || i1 >= ns || i2 < 0 || i2 >= ns)
            return fail(DCOL_ERR_ARG, "shape id out of range at pair " + std::to_string(i));
        int32_t g;
        if (dense) {
            int32_t& e = cache[(size_t)i1 * ns + i2];
            if (e < 0) e = classify_pair(i1, i2);
            g = e;
        } else {
            auto it = sparse.find((int64_t)i1 * ns + i2);
            if (it == sparse.end()) it = sparse.emplace((int64_t)i1 * ns + i2, classify_pair(i1, i2)).first;
            g = it->second;
        }
        gid[i] = g;
        ++groups[g].n;
    }
    p->table = t;
    p->B = B;
    p->launches.clear();
    perm.assign((size_t)B, 0);
    // Latency configurations only when the whole plan cannot fill the GPU: the buckets of a
    // large mixed plan run side by side on the fan-out streams, so each keeps its throughput
    // configuration even when it alone would leave SIMDs idle (DCOL_LATENCY_PER_LAUNCH=1:
    // the per-launch rule, for A/B runs).
    static const bool per_launch = std::getenv("DCOL_LATENCY_PER_LAUNCH") != nullptr;
    int64_t plan_lanes = 0;
    for (const Group& G : groups)
        if (std::get<0>(G.key) == 0) plan_lanes += G.n * std::get<4>(G.key);
    const bool small_plan = !force_large && plan_lanes < small_lanes(t);
    if (small_out) *small_out = small_plan;
    int64_t at = 0;
    for (auto& kv : gid_of_key) {   // key order
        Group& G = groups[kv.second];
        G.at = at;
        Launch L;
        L.kind = std::get<0>(G.key);
        L.N = std::get<1>(G.key);
        L.nsoc = std::get<2>(G.key);
        L.omax = std::get<3>(G.key);
        L.lpp = std::get<4>(G.key);
        L.code = std::get<6>(G.key);
        L.oe = std::get<7>(G.key);
        L.full = L.kind == 0 && G.full;
        L.ball = L.kind == 0 && std::get<5>(G.key) == 1;
        L.cone = L.kind == 0 && std::get<5>(G.key) == 2;
        L.box = L.kind == 0 && std::get<5>(G.key) == 3 && L.full;
        L.slot0 = at;
        L.n = G.n;
        if (L.kind == 0 && !lpp_forced() && L.n * L.lpp < 64LL * t->simds && (small_plan || per_launch))
            latency_config(L);   // cannot fill the GPU
        at += G.n;
        p->launches.push_back(L);
    }
    for (int64_t i = 0; i < B; ++i) perm[(size_t)groups[gid[i]].at++] = (int32_t)i;   // stable
    p->small = small_plan;
    assign_lanes(p);
    return DCOL_SUCCESS;
}

// Mixed batches (e.g. an ALTRO phase: one victim against spheres, cylinders, capsules,
// cones, polytopes) split into several small variant launches, each far too small to fill
// the chip; run back to back their latencies add up.  Spread them over the caller's stream
// plus up to kSideStreams side streams (fork/join through events) — longest-first greedy on
// a cost estimate (waves x per-pair work), reject launches stay on the caller's stream.
// Per-pair cost of a solve bucket in ns at full occupancy (least-squares fit to the class
// benchmark of profiles/r03_soc/class_bench.log, within ~17 % on the 13 SOC classes): row
// slots, SOC blocks (dense SOC rows cost more than the structured ball / cone rows) and the
// N x N normal-matrix work; polytope x polytope buckets run at two waves per SIMD (x 0.5).
double bucket_cost(const Launch& L) {
    const bool dense_soc = L.nsoc > 0 && !(L.flags() & (LF_BALL | LF_CONE));
    const double per_pair = 0.0806 * L.omax + 0.127 * L.nsoc + 0.0139 * L.N * L.N + (dense_soc ? 0.143 * L.nsoc : 0.0);
    return (double)L.n * per_pair * (L.nsoc == 0 ? 0.5 : 1.0);
}

void assign_lanes(dcol_plan* p) {
    int solves = 0;
    for (const Launch& L : p->launches) solves += L.kind == 0;
    p->lanes = 1;
    p->issue.clear();
    if (solves < 2) return;
    const int lanes = std::min(solves, (p->small ? side_streams() : large_side_streams()) + 1);
    std::vector<int> order;
    std::vector<double> cost(p->launches.size(), 0.0);
    for (size_t i = 0; i < p->launches.size(); ++i) {
        const Launch& L = p->launches[i];
        if (L.kind != 0) {
            p->issue.push_back((int)i);   // rejects first, on the caller's stream
            continue;
        }
        cost[i] = bucket_cost(L);
        order.push_back((int)i);
    }
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost[a] > cost[b]; });
    // issued longest first: every stream starts on its biggest bucket and the short ones fill
    // the tail, where the other streams' last kernels no longer occupy the whole chip
    p->issue.insert(p->issue.end(), order.begin(), order.end());
    std::vector<double> load(lanes, 0.0);
    for (int i : order) {
        const int l = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        p->launches[i].lane = l;
        load[l] += cost[i];
    }
    static const bool serial = std::getenv("DCOL_NO_FANOUT") != nullptr;   // A/B: one stream
    p->lanes = serial ? 1 : lanes;
}

// A plan with several solve buckets that together leave the GPU mostly idle (fewer lanes
// than one wave per SIMD: every bucket already took its latency configuration) runs as ONE
// fused launch; p->segs is left empty when it does not qualify (large or single-variant
// plans, variants outside the fused kernel, DCOL_PLAN_NO_FUSE).
// DCOL_PLAN_SUSPEND: every large solve bucket with a suspend / resume variant gets its
// continuation buffers (entries: DCOL_SUSPEND_T per wave, default 4; DCOL_NO_SUSPEND=1
// disables).  Allocates; returns DCOL_SUCCESS or an error.
int susp_t_env() {
    static const int t = [] {
        const char* e = std::getenv("DCOL_SUSPEND_T");
        return std::getenv("DCOL_NO_SUSPEND") ? 0 : (e ? std::max(0, std::atoi(e)) : 4);
    }();
    return t;
}
int susp_min_env() {
    static const int m = [] {
        const char* e = std::getenv("DCOL_SUSPEND_MIN");
        return e ? std::max(0, std::atoi(e)) : 6;
    }();
    return m;
}
int plan_susp(const dcol_table* t, dcol_plan* p) {
    const int T = susp_t_env();
    if (T <= 0 || p->fused()) return DCOL_SUCCESS;
    size_t bytes = 0;
    for (Launch& L : p->launches) {
        int f = 0;
        if (L.kind != 0 || L.n * L.lpp < 64LL * t->simds || !susp_available(L.N, L.nsoc, L.omax, L.lpp, L.flags(), L.oe, &f))
            continue;
        L.susp = true;
        L.susp_fields = f;
        L.susp_cap = ((L.n * L.lpp + 63) / 64) * (int64_t)T;
        bytes += 256 + (size_t)L.susp_cap * (sizeof(int32_t) + sizeof(double) * f);
    }
    if (bytes == 0) return DCOL_SUCCESS;
    DeviceGuard g(t->device);
    hipError_t e = hipMalloc(&p->d_susp, bytes);
    if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("suspend scratch: ") + hipGetErrorString(e));
    char* c = static_cast<char*>(p->d_susp);
    for (Launch& L : p->launches) {
        if (!L.susp) continue;
        L.d_susp_count = reinterpret_cast<int32_t*>(c);
        c += 256;
        L.d_susp_state = reinterpret_cast<double*>(c);
        c += sizeof(double) * L.susp_fields * (size_t)L.susp_cap;
        L.d_susp_pi = reinterpret_cast<int32_t*>(c);
        c += sizeof(int32_t) * (size_t)L.susp_cap;
    }
    return DCOL_SUCCESS;
}

bool plan_segments(dcol_plan* p, int (*vid_of)(int, int, int, int, int, int));

// Returns 0 when fused (or not allowed), 1 when the plan does not qualify (large or
// single-variant), 2 when it qualifies but a bucket has no case in the fused kernel.
int plan_fuse(const dcol_table* t, dcol_plan* p, bool allow) {
    p->segs.clear();
    p->fused_blocks = 0;
    p->packed = false;
    if (!allow) return 0;
    int solves = 0;
    int64_t lanes = 0;
    for (const Launch& L : p->launches)
        if (L.kind == 0) {
            ++solves;
            lanes += L.n * L.lpp;
        }
    if (solves < 2 || solves > kMaxFusedSegs || lanes >= small_lanes(t)) return 1;
    return plan_segments(p, fused_vid) ? 0 : 2;
}

// One segment per solve bucket with case ids from vid_of (fused_vid / packed_vid), in
// descending per-pair cost (bucket_cost): the workgroup dispatcher hands out blocks in index
// order as SIMDs free up, so the longest-latency waves start first and the short ones fill
// the tail (list scheduling, longest first); DCOL_FUSED_ORDER=0: key order (A/B).  false (p
// unchanged) when a bucket has no case.
bool plan_segments(dcol_plan* p, int (*vid_of)(int, int, int, int, int, int)) {
    static const bool keyorder = [] {
        const char* e = std::getenv("DCOL_FUSED_ORDER");
        return e && std::atoi(e) == 0;
    }();
    std::vector<int> order;
    for (size_t i = 0; i < p->launches.size(); ++i)
        if (p->launches[i].kind == 0) order.push_back((int)i);
    if (!keyorder)
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
            const Launch& A = p->launches[a];
            const Launch& B = p->launches[b];
            return bucket_cost(A) / (double)A.n > bucket_cost(B) / (double)B.n;
        });
    std::vector<FusedSeg> segs;
    int64_t block = 0;
    for (int i : order) {
        const Launch& L = p->launches[i];
        const int vid = vid_of(L.N, L.nsoc, L.omax, L.lpp, L.flags(), L.oe);
        if (vid < 0) return false;
        segs.push_back(FusedSeg{vid, L.lpp, block, L.slot0, L.n});
        block += (L.n * L.lpp + kBlock - 1) / kBlock;
    }
    p->segs = std::move(segs);
    p->fused_blocks = block;
    p->packed = false;
    p->lanes = 1;   // no fan-out
    return true;
}

// Lanes below which a plan that is not small runs as ONE packed launch (every bucket in its
// throughput configuration, dcol_kernels_packed.hip) instead of one launch per bucket over
// the fan-out streams: mid-size mixed plans whose buckets each cover only part of the SIMDs
// (a rank's shard of configs[4] at 2-8 GPUs).  16 x 64 x SIMDs (~1M lanes): measured on the
// configs[4] shards (tools/shard_bench.py, profiles/r06_c/): packed against the fan-out
// 0.506 / 0.549 ms at 500k pairs (775k lanes), 0.267 / 0.396 at 250k, 0.144 / 0.325 at 125k,
// but 0.98 / 0.87 ms for the whole 1M (1.55M lanes: every bucket fills the GPU by itself and
// its two- and three-wave kernels keep their occupancy).  DCOL_PACK_LANES=<n> for A/B runs
// (0: never).
int64_t pack_lanes(const dcol_table* t) {
    static const int64_t v = [] {
        const char* e = std::getenv("DCOL_PACK_LANES");
        return e ? std::atoll(e) : -1LL;
    }();
    return v >= 0 ? v : 16LL * 64LL * t->simds;
}

// A mid-size plan (not small, below pack_lanes) with several solve buckets, every one of
// which the packed kernel has, becomes one packed launch; otherwise p is unchanged.
void plan_pack(const dcol_table* t, dcol_plan* p) {
    if (p->small || p->fused()) return;
    int solves = 0;
    int64_t lanes = 0;
    for (const Launch& L : p->launches)
        if (L.kind == 0) {
            ++solves;
            lanes += L.n * L.lpp;
        }
    if (solves < 2 || solves > kMaxFusedSegs || lanes >= pack_lanes(t)) return;
    if (!plan_segments(p, packed_vid)) return;
    p->packed = true;
}

int bucket_and_fuse(const dcol_table* t, int64_t B, const int32_t* s1, const int32_t* s2, dcol_plan* p,
                    std::vector<int32_t>& perm, bool case4, bool allow_fuse) {
    bool small = false;
    int rc = bucket_pairs(t, B, s1, s2, p, perm, case4, false, false, &small);
    if (rc != DCOL_SUCCESS) return rc;
    // a plan that cannot fill the GPU: no one-lane row-partitioned buckets (bucket_pairs)
    bool lat_part = false;
    if (small && !lpp_forced())
        for (const Launch& L : p->launches) lat_part = lat_part || (L.kind == 0 && L.oe > 0 && L.lpp < 2);
    if (lat_part) {
        rc = bucket_pairs(t, B, s1, s2, p, perm, case4, false, true);
        if (rc != DCOL_SUCCESS) return rc;
    }
    // only when every bucket the fused kernel lacks is a row-partitioned one (a dense bucket
    // without a case -- a many-row bucket -- keeps the plan unfused whatever the PART pairs
    // do, and they would lose their faster kernels for nothing); when the re-bucketed plan
    // still does not fuse, the first bucketing stands
    bool only_part = true;
    for (const Launch& L : p->launches)
        if (L.kind == 0 && L.oe == 0 && fused_vid(L.N, L.nsoc, L.omax, L.lpp, L.flags(), 0) < 0) only_part = false;
    if (plan_fuse(t, p, true) == 2 && only_part) {
        rc = bucket_pairs(t, B, s1, s2, p, perm, case4, true, lat_part);
        if (rc != DCOL_SUCCESS) return rc;
        if (plan_fuse(t, p, true) == 2) {
            rc = bucket_pairs(t, B, s1, s2, p, perm, case4, false, lat_part);
            if (rc != DCOL_SUCCESS) return rc;
        }
    }
    if (!allow_fuse && p->fused()) {   // same buckets, launched one by one (fan-out)
        p->segs.clear();
        p->fused_blocks = 0;
        assign_lanes(p);
    }
    if (allow_fuse) plan_pack(t, p);   // mid-size plans: one packed launch
    // A small plan the fused kernel cannot take (a bucket without a fused case) would fan
    // its latency-configured buckets out over the streams, one under-filled launch after
    // another; the packed launch of its throughput configurations serves it better (one
    // launch, every wave placed as SIMDs free) when every bucket has a
    // packed case.  Tried on a scratch plan: p stands unless it packs.
    if (allow_fuse && p->small && !p->fused() && !lpp_forced() && !small_fanout()) {
        dcol_plan q;
        std::vector<int32_t> qperm;
        if (bucket_pairs(t, B, s1, s2, &q, qperm, case4, false, false, nullptr, true) == DCOL_SUCCESS) {
            q.small = false;
            plan_pack(t, &q);
            if (q.fused()) {
                p->launches = std::move(q.launches);
                p->segs = std::move(q.segs);
                p->fused_blocks = q.fused_blocks;
                p->packed = true;
                p->small = false;
                p->lanes = q.lanes;
                p->issue.clear();
                perm.swap(qperm);
            }
        }
    }
    return DCOL_SUCCESS;
}

int ensure_fanout(const dcol_table* tc, dcol_plan* p) {
    if (p->lanes <= 1) return DCOL_SUCCESS;
    dcol_table* t = const_cast<dcol_table*>(tc);
    DeviceGuard g(t->device);
    if (!t->side_ready) return fail(DCOL_ERR_HIP, "side streams of the device could not be created");
    hipError_t e = hipEventCreateWithFlags(&p->fork, hipEventDisableTiming);
    for (int i = 0; e == hipSuccess && i < p->lanes - 1; ++i) e = hipEventCreateWithFlags(&p->join[i], hipEventDisableTiming);
    if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("fan-out events: ") + hipGetErrorString(e));
    return DCOL_SUCCESS;
}
}  // namespace

extern "C" {

int dcol_plan_create(const dcol_table* t, int64_t B, const int32_t* s1, const int32_t* s2, dcol_plan** out) {
    return dcol_plan_create_ex(t, B, s1, s2, 0, out);
}

int dcol_plan_create_ex(const dcol_table* t, int64_t B, const int32_t* s1, const int32_t* s2, int32_t options,
                        dcol_plan** out) {
    if (!t || !out || B < 0 || (B > 0 && (!s1 || !s2))) return fail(DCOL_ERR_ARG, "dcol_plan_create: bad arguments");
    if (options & ~(DCOL_PLAN_CASE4 | DCOL_PLAN_NO_FUSE | DCOL_PLAN_SUSPEND))
        return fail(DCOL_ERR_ARG, "dcol_plan_create_ex: unknown option bits");
    if (B > INT32_MAX) return fail(DCOL_ERR_ARG, "dcol_plan_create: B exceeds 2^31-1");
    *out = nullptr;
    auto* p = new (std::nothrow) dcol_plan();
    if (!p) return fail(DCOL_ERR_NOMEM, "host allocation failed");
    std::vector<int32_t> perm;
    int rc = bucket_and_fuse(t, B, s1, s2, p, perm, (options & DCOL_PLAN_CASE4) != 0, (options & DCOL_PLAN_NO_FUSE) == 0);
    if (rc != DCOL_SUCCESS) {
        delete p;
        return rc;
    }
    p->owns = true;
    if (B == 0) {
        *out = p;
        return DCOL_SUCCESS;
    }
    DeviceGuard g(t->device);
    hipError_t e = hipMalloc(&p->d_s1, sizeof(int32_t) * B);
    if (e == hipSuccess) e = hipMalloc(&p->d_s2, sizeof(int32_t) * B);
    if (e == hipSuccess) e = hipMemcpy(p->d_s1, s1, sizeof(int32_t) * B, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_s2, s2, sizeof(int32_t) * B, hipMemcpyHostToDevice);
    if (e == hipSuccess && p->launches.size() > 1) {
        e = hipMalloc(&p->d_perm, sizeof(int32_t) * B);
        if (e == hipSuccess) e = hipMemcpy(p->d_perm, perm.data(), sizeof(int32_t) * B, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && p->fused()) {
        const size_t sb = sizeof(FusedSeg) * p->segs.size();
        e = hipMalloc(&p->d_segs, sb);
        if (e == hipSuccess) e = hipMemcpy(p->d_segs, p->segs.data(), sb, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
        dcol_plan_destroy(p);
        return fail(DCOL_ERR_HIP, std::string("dcol_plan_create: ") + hipGetErrorString(e));
    }
    rc = ensure_fanout(t, p);
    if (rc == DCOL_SUCCESS && (options & DCOL_PLAN_SUSPEND)) rc = plan_susp(t, p);
    if (rc != DCOL_SUCCESS) {
        dcol_plan_destroy(p);
        return rc;
    }
    *out = p;
    return DCOL_SUCCESS;
}

int dcol_plan_destroy(dcol_plan* p) {
    if (!p) return DCOL_SUCCESS;
    if (p->table && p->owns) {
        DeviceGuard g(p->table->device);
        if (p->d_s1) (void)hipFree(p->d_s1);
        if (p->d_s2) (void)hipFree(p->d_s2);
        if (p->d_perm) (void)hipFree(p->d_perm);
        if (p->d_segs) (void)hipFree(p->d_segs);
        if (p->d_susp) (void)hipFree(p->d_susp);
    }
    delete p;
    return DCOL_SUCCESS;
}

int dcol_plan_suspended(const dcol_plan* p, int64_t* n) {
    if (!p || !n) return fail(DCOL_ERR_ARG, "dcol_plan_suspended: NULL argument");
    *n = 0;
    if (!p->d_susp) return DCOL_SUCCESS;
    DeviceGuard g(p->table->device);
    for (const Launch& L : p->launches) {
        if (!L.susp) continue;
        int32_t c = 0;
        const hipError_t e = hipMemcpy(&c, L.d_susp_count, sizeof(c), hipMemcpyDeviceToHost);
        if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("dcol_plan_suspended: ") + hipGetErrorString(e));
        *n += c;
    }
    return DCOL_SUCCESS;
}

int dcol_plan_num_launches(const dcol_plan* p, int32_t* n) {
    if (!p || !n) return fail(DCOL_ERR_ARG, "dcol_plan_num_launches: NULL argument");
    int32_t k = 0;
    for (const Launch& L : p->launches) k += (L.kind != 0 || !p->fused());
    *n = k + (p->fused() ? 1 : 0);
    return DCOL_SUCCESS;
}

int dcol_plan_num_streams(const dcol_plan* p, int32_t* n) {
    if (!p || !n) return fail(DCOL_ERR_ARG, "dcol_plan_num_streams: NULL argument");
    *n = p->fused() ? 1 : p->lanes;
    return DCOL_SUCCESS;
}

int dcol_plan_launch_form(const dcol_plan* p, int32_t* form) {
    if (!p || !form) return fail(DCOL_ERR_ARG, "dcol_plan_launch_form: NULL argument");
    *form = !p->fused() ? DCOL_FORM_BUCKETS : (p->packed ? DCOL_FORM_PACKED : DCOL_FORM_FUSED);
    return DCOL_SUCCESS;
}

int dcol_plan_num_buckets(const dcol_plan* p, int32_t* n) {
    if (!p || !n) return fail(DCOL_ERR_ARG, "dcol_plan_num_buckets: NULL argument");
    *n = (int32_t)p->launches.size();
    return DCOL_SUCCESS;
}

int dcol_plan_bucket(const dcol_plan* p, int32_t i, int32_t info[8], int64_t* pairs) {
    if (!p || !info || !pairs) return fail(DCOL_ERR_ARG, "dcol_plan_bucket: NULL argument");
    if (i < 0 || i >= (int32_t)p->launches.size()) return fail(DCOL_ERR_ARG, "dcol_plan_bucket: index out of range");
    const Launch& L = p->launches[(size_t)i];
    const bool solve = L.kind == 0;
    const int32_t v[8] = {L.kind, solve ? L.N : 0, solve ? L.nsoc : 0, solve ? L.omax : 0, solve ? L.lpp : 0,
                          solve ? L.oe : 0, solve ? L.flags() : 0, solve ? 0 : L.code};
    for (int k = 0; k < 8; ++k) info[k] = v[k];
    *pairs = L.n;
    return DCOL_SUCCESS;
}

}  // extern "C"

namespace {
// dcol_plan_run with an optional record output (rec: [B][DCOL_REC], written by the solver
// epilogues; then alpha / grad / iters / status may be NULL)
int plan_run_rec(const dcol_plan* p, const double* pose1, const double* pose2, double tol, int32_t max_iter,
                 int32_t flags, double* alpha, double* contact, double* grad, int32_t* iters, int32_t* status,
                 double* rec, void* stream, bool yield = true) {
    if (!p) return fail(DCOL_ERR_ARG, "dcol_plan_run: NULL plan");
    // (the pair call's own launch path keeps it).  A small plan keeps it too -- unless it is
    // launched on the null stream: the server runs on a blocking stream (CU-masked streams
    // have no non-blocking form), so null-stream work waits for it to leave, i.e. for its idle
    // time (DCOL_PAIR_SERVER_IDLE_US) -- asking it to leave now costs a restart instead.
    if (yield && (!p->small || stream == nullptr)) yield_pair_servers(p->table->device);
    if (p->B == 0) return DCOL_SUCCESS;
    if (!pose1 || !pose2 || (!alpha && !rec))
        return fail(DCOL_ERR_ARG, "dcol_plan_run: pose1, pose2 and alpha are required");
    if ((flags & DCOL_CONTACT) && !contact) return fail(DCOL_ERR_ARG, "dcol_plan_run: DCOL_CONTACT needs contact[]");
    if ((flags & DCOL_GRAD_ANY) && !grad && !rec) return fail(DCOL_ERR_ARG, "dcol_plan_run: gradient flag needs grad[]");
    if (max_iter < 0) return fail(DCOL_ERR_ARG, "dcol_plan_run: max_iter < 0");
    const dcol_table* t = p->table;
    DeviceGuard g(t->device);
    // the launch checks below read the thread's last HIP error: clear one a caller's earlier
    // HIP call left behind (not ours to report)
    (void)hipGetLastError();
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    KArgs a;
    a.shapes = t->d_shapes;
    a.rows = t->d_rows;
    a.s1 = p->d_s1;
    a.s2 = p->d_s2;
    a.pose1 = pose1;
    a.pose2 = pose2;
    a.perm = p->d_perm;
    a.B = p->B;
    a.tol = tol;
    a.max_iter = max_iter;
    a.flags = flags;
    a.alpha = alpha;
    a.contact = contact;
    a.grad = grad;
    a.iters = iters;
    a.status = status;
    a.rec = rec;
    a.susp_t = 0;
    a.susp_min = 0;
    a.susp_count = nullptr;
    a.susp_pi = nullptr;
    a.susp_state = nullptr;
    a.susp_cap = 0;
    // a run without envelope / implicit gradients may take a bucket's FD-only copy (LF_FDONLY)
    const int fdonly = (flags & (DCOL_GRAD_ENVELOPE | DCOL_GRAD_IMPLICIT)) ? 0 : LF_FDONLY;
    const bool fan = p->lanes > 1 && p->fork;
    hipError_t e = hipSuccess;
    if (fan) {
        e = hipEventRecord(p->fork, st);
        for (int l = 1; e == hipSuccess && l < p->lanes; ++l) e = hipStreamWaitEvent(t->side[l - 1], p->fork, 0);
        if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("dcol_plan_run fork: ") + hipGetErrorString(e));
    }
    const size_t nl = p->launches.size();
    for (size_t li = 0; li < nl; ++li) {
        const Launch& L = p->launches[p->issue.size() == nl ? (size_t)p->issue[li] : li];
        if (L.kind == 0 && p->fused()) continue;   // covered by the fused launch below
        a.slot0 = L.slot0;
        a.n = L.n;
        hipStream_t ls = (fan && L.lane > 0) ? t->side[L.lane - 1] : st;
        if (L.kind == 1) {
            const int64_t grid = (L.n + kBlock - 1) / kBlock;
            hipLaunchKernelGGL(reject_kernel, dim3(grid), dim3(kBlock), 0, ls, a, L.code);
            e = hipGetLastError();
        } else if (L.susp) {   // main + resume launch pair (plan_susp)
            KArgs b = a;
            b.susp_t = susp_t_env();
            b.susp_min = susp_min_env();
            b.susp_count = L.d_susp_count;
            b.susp_pi = L.d_susp_pi;
            b.susp_state = L.d_susp_state;
            b.susp_cap = L.susp_cap;
            e = hipMemsetAsync(L.d_susp_count, 0, sizeof(int32_t), ls);
            if (e == hipSuccess) e = launch_susp(L.N, L.nsoc, L.omax, L.lpp, L.flags(), L.oe, b, ls);
        } else {
            const int split = (L.oe > 0 && L.lpp == 2 && split_enabled() && split_built(L.N, L.nsoc, L.omax, L.oe))
                                  ? LF_SPLIT : 0;
            e = launch_variant(L.N, L.nsoc, L.omax, L.lpp, L.flags() | fdonly | split, a, ls, L.oe);
        }
        if (e != hipSuccess) break;
    }
    if (e == hipSuccess && p->fused()) {
        a.slot0 = 0;
        a.n = 0;
        e = p->packed ? launch_packed(a, p->d_segs, (int)p->segs.size(), p->fused_blocks, st)
                      : launch_fused(a, p->d_segs, (int)p->segs.size(), p->fused_blocks, st);
    }
    if (fan) {   // join even after a failed launch, so the side streams never run ahead
        for (int l = 1; l < p->lanes; ++l) {
            hipError_t j = hipEventRecord(p->join[l - 1], t->side[l - 1]);
            if (j == hipSuccess) j = hipStreamWaitEvent(st, p->join[l - 1], 0);
            if (e == hipSuccess) e = j;
        }
    }
    if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("dcol_plan_run launch: ") + hipGetErrorString(e));
    return DCOL_SUCCESS;
}
}  // namespace

extern "C" {

int dcol_plan_run(const dcol_plan* p, const double* pose1, const double* pose2, double tol, int32_t max_iter,
                  int32_t flags, double* alpha, double* contact, double* grad, int32_t* iters, int32_t* status,
                  void* stream) {
    return plan_run_rec(p, pose1, pose2, tol, max_iter, flags, alpha, contact, grad, iters, status, nullptr, stream);
}

int dcol_prox_pair(const dcol_table* tc, int32_t s1, int32_t s2, const double* pose1, const double* pose2, double tol,
                   int32_t max_iter, int32_t flags, double* alpha, double* contact, double* grad, int32_t* iters,
                   int32_t* status) {
    if (!tc || !pose1 || !pose2 || !alpha) return fail(DCOL_ERR_ARG, "dcol_prox_pair: NULL argument");
    if ((flags & DCOL_CONTACT) && !contact) return fail(DCOL_ERR_ARG, "dcol_prox_pair: DCOL_CONTACT needs contact");
    if ((flags & DCOL_GRAD_ANY) && !grad) return fail(DCOL_ERR_ARG, "dcol_prox_pair: gradient flag needs grad");
    if (max_iter < 0) return fail(DCOL_ERR_ARG, "dcol_prox_pair: max_iter < 0");
    const int32_t ns = (int32_t)tc->shapes.size();
    if (s1 < 0 || s1 >= ns || s2 < 0 || s2 >= ns) return fail(DCOL_ERR_ARG, "dcol_prox_pair: shape id out of range");
    dcol_table* t = const_cast<dcol_table*>(tc);
    std::lock_guard<std::mutex> lk(t->mu);
    DeviceGuard g(t->device);
    if (!t->pair_host) {
        // fine-grained coherent on purpose: the server's handshake (system-scope atomics on
        // req / done / alive / stop) needs host and device to see each other's stores while
        // the wave runs, whatever HIP_HOST_COHERENT says
        PairBox* hb = nullptr;
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&hb), sizeof(PairBox),
                                     hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent);
        if (e == hipSuccess) {
            std::memset(hb, 0, sizeof(PairBox));   // flags and sequence numbers start at 0
            hb->xcd = -1;                           // no server yet
        }
        if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&t->pair_dev), hb, 0);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&t->pair_stream, hipStreamNonBlocking);
        // The server stream: a CU-masked stream (mask = every CU), because HIP never pools a
        // CU-masked stream into a shared hardware queue -- the resident server gets a queue of
        // its own instead of sharing one (GPU_MAX_HW_QUEUES, 4 by default) with the caller's
        // or the side streams, whose kernels would otherwise wait behind it until it idles
        // out.  Not a high-priority stream: a resident kernel on a high-priority queue slowed
        // a normal-priority 100k batch plan 1.7-1.8x whatever its poll rate, a normal or
        // CU-masked one by nothing measurable (tools/server_tax.py, profiles/r05_d/).
        // DCOL_PAIR_SERVER_STREAM=normal / high: those alternatives (A/B).
        const char* sk = std::getenv("DCOL_PAIR_SERVER_STREAM");
        if (e == hipSuccess && sk && (std::strcmp(sk, "normal") == 0 || std::strcmp(sk, "high") == 0)) {
            int prio_lo = 0, prio_hi = 0;
            if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) {
                (void)hipGetLastError();
                prio_lo = prio_hi = 0;
            }
            e = hipStreamCreateWithPriority(&t->server_stream, hipStreamNonBlocking,
                                            std::strcmp(sk, "high") == 0 ? prio_hi : prio_lo);
        } else if (e == hipSuccess) {
            int cus = 0;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, t->device) != hipSuccess || cus <= 0) {
                (void)hipGetLastError();
                cus = 256;
            }
            std::vector<uint32_t> mask((cus + 31) / 32, 0u);
            for (int c = 0; c < cus; ++c) mask[c / 32] |= 1u << (c % 32);
            e = hipExtStreamCreateWithCUMask(&t->server_stream, (uint32_t)mask.size(), mask.data());
        }
        int khz = 0;
        if (e == hipSuccess && hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, t->device) != hipSuccess) {
            (void)hipGetLastError();
            khz = 0;
        }
        if (e != hipSuccess) {   // (never published: nothing else has seen hb)
            if (hb) (void)hipHostFree(hb);
            if (t->pair_stream) (void)hipStreamDestroy(t->pair_stream);
            t->pair_dev = nullptr;
            t->pair_stream = nullptr;
            return fail(DCOL_ERR_HIP, std::string("dcol_prox_pair staging: ") + hipGetErrorString(e));
        }
        t->wall_ticks_us = khz > 0 ? (int64_t)khz / 1000 : 0;
        // published after its initialisation: yield_pair_servers reads it without t->mu
        __atomic_store_n(&t->pair_host, hb, __ATOMIC_RELEASE);
    }
    const int64_t key = (int64_t)s1 * ns + s2;
    const bool c4 = (flags & DCOL_CASE4) != 0;
    const int64_t ck = c4 ? -1 - key : key;   // case-4 plans apart
    dcol_plan* plan = nullptr;
    auto it = t->pair_plans.find(ck);
    if (it != t->pair_plans.end()) {
        t->pair_lru.splice(t->pair_lru.begin(), t->pair_lru, it->second);   // now the most recent
        plan = it->second->second;
    } else {
        const int rc = dcol_plan_create_ex(t, 1, &s1, &s2, c4 ? DCOL_PLAN_CASE4 : 0, &plan);
        if (rc != DCOL_SUCCESS) return rc;
        // the least recently used plan makes room (no launch of it is in flight: every call
        // synchronises its stream before returning)
        if ((int)t->pair_lru.size() >= DCOL_PAIR_PLANS_MAX) {
            t->pair_plans.erase(t->pair_lru.back().first);
            dcol_plan_destroy(t->pair_lru.back().second);
            t->pair_lru.pop_back();
        }
        t->pair_lru.emplace_front(ck, plan);
        t->pair_plans.emplace(ck, t->pair_lru.begin());
    }
    PairBox* h = t->pair_host;
    PairBox* d = t->pair_dev;
    // a batch launch asked the server to leave: drain it (it left at its next poll) and clear
    // the stop flag, so the server started below stays
    if (t->stop_req.exchange(false, std::memory_order_acq_rel) && !stop_pair_server(t, kServerStopMs))
        return fail(DCOL_ERR_HIP, "dcol_prox_pair: the pair server did not stop within 5 s");
    std::memcpy(h->pose1, pose1, 6 * sizeof(double));
    std::memcpy(h->pose2, pose2, 6 * sizeof(double));
    // SoA of one pair = the 6 values in order; the kernel reads / writes the mapped memory.
    const bool single = plan->launches.size() == 1 && plan->launches[0].kind == 0 && !plan->fused() &&
                         !plan->launches[0].susp && plan->lanes <= 1;
    // The one-pair server (PairBox, dcol_kernels_server.hip): a resident workgroup polls the
    // mailbox, so a call whose variant the fused kernel has (the server switches over the
    // same solver copies) costs no launch.
    const int idle_us = pair_server_idle_us();
    const Launch& L0 = plan->launches[0];
    int vid = (single && idle_us > 0 && t->wall_ticks_us > 0 && ns <= (1 << kPairBoxIdBits) && L0.lpp < 65536 &&
               !g_shutdown.load(std::memory_order_acquire))
                  ? fused_vid(L0.N, L0.nsoc, L0.omax, L0.lpp, L0.flags(), L0.oe) : -1;
    const int32_t kflags = flags & ~DCOL_CASE4;
    // Flags / tolerance / iteration cap are the server's launch arguments.  A call with others
    // while a server runs takes the launch path below, and only the second such call in a
    // row restarts the server with the new ones: an ALTRO loop switches between
    // proximity_mrp and proximity_gradient per phase (one launched call, then a restart), a
    // caller alternating the two call by call keeps the server for one of them instead of
    // restarting it at every call (47 us per call measured, against 32).
    bool restart = false;
    if (vid >= 0 && t->server_launched && (h->flags != kflags || h->tol != tol || h->max_iter != max_iter)) {
        if (hipStreamQuery(t->server_stream) == hipSuccess) {   // no server left: a fresh start
            __atomic_store_n(&h->alive, 0, __ATOMIC_SEQ_CST);
            t->srv_mismatch = 0;
        } else if (++t->srv_mismatch < 2) {
            vid = -1;
        } else {
            restart = true;
            t->srv_mismatch = 0;
        }
    } else if (vid >= 0) {
        t->srv_mismatch = 0;
    }
    if (vid >= 0) {
        const auto start_server = [&]() -> hipError_t {
            KArgs a;
            a.shapes = t->d_shapes;
            a.rows = t->d_rows;
            a.s1 = nullptr;   // the shape ids come with each request (PairBox::ids)
            a.s2 = nullptr;
            a.pose1 = d->pose1;
            a.pose2 = d->pose2;
            a.perm = nullptr;
            a.B = 1;
            a.slot0 = 0;
            a.n = 1;
            a.tol = tol;
            a.max_iter = max_iter;
            a.flags = kflags;
            a.alpha = &d->alpha;
            a.contact = d->contact;
            a.grad = d->grad;
            a.iters = &d->iters;
            a.status = &d->status;
            a.rec = nullptr;
            a.susp_t = 0;
            a.susp_min = 0;
            a.susp_count = nullptr;
            a.susp_pi = nullptr;
            a.susp_state = nullptr;
            a.susp_cap = 0;
#ifdef DCOL_STAMPS
            a.stamps = d->stamps;   // (diagnostic build) solve_one's phase stamps of each request
#endif
            h->flags = kflags;
            h->tol = tol;
            h->max_iter = max_iter;
            // a resident wave must not outlive the process's HIP context: stop every server
            // at exit (the handler runs before the HIP runtime's own, registered earlier)
            std::call_once(g_exit_hook, [] { std::atexit([] { (void)dcol_shutdown(); }); });
            if (!t->server_launched) g_server_tables.fetch_add(1, std::memory_order_acq_rel);
            t->server_launched = true;
            ++t->n_starts;
            const char* ps = std::getenv("DCOL_PAIR_SERVER_POLL_SLEEP");
            return launch_pair_server(a, d, (int64_t)idle_us * t->wall_ticks_us, ps ? std::atoi(ps) : 0, t->server_stream);
        };
        if (restart && !stop_pair_server(t, kServerStopMs))   // it leaves at its next poll, then start anew
            return fail(DCOL_ERR_HIP, "dcol_prox_pair: the pair server did not stop within 5 s");
        const uint32_t useq = (uint32_t)(h->req >> 32) + 1u;
        const int32_t seq = (int32_t)useq;
        h->ids = ((uint64_t)(useq & 0xffffu) << 48) | ((uint64_t)(uint32_t)s2 << kPairBoxIdBits) | (uint64_t)(uint32_t)s1;
        __atomic_store_n(&h->req, ((uint64_t)useq << 32) | ((uint64_t)(uint32_t)L0.lpp << 16) | (uint64_t)(uint32_t)vid,
                         __ATOMIC_SEQ_CST);
        // a server that cleared `alive` before this request re-checks `req` on its way out
        // (and serves it), or it is gone: then start one (a redundant one queues behind the
        // old one on the server stream, finds nothing to do and leaves after the idle time)
        if (__atomic_load_n(&h->alive, __ATOMIC_SEQ_CST) == 0) {
            const hipError_t e = start_server();
            if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("dcol_prox_pair server: ") + hipGetErrorString(e));
        }
        int restarts = 0;
        const auto t_post = std::chrono::steady_clock::now();
        for (uint64_t spin = 1;; ++spin) {
            if (__atomic_load_n(&h->done, __ATOMIC_ACQUIRE) == seq) break;
            if ((spin & 4095) == 0) {   // a failed server surfaces here; an idle stream with the request
                const hipError_t q = hipStreamQuery(t->server_stream);   // unserved gets a new server
                if (q == hipErrorNotReady && std::chrono::steady_clock::now() - t_post > std::chrono::seconds(30)) {
                    // a server that never answers (not expected: a solve takes microseconds):
                    // make it leave, so the next call starts clean, and report
                    (void)stop_pair_server(t, kServerStopMs);
                    return fail(DCOL_ERR_HIP, "dcol_prox_pair: the pair server did not answer within 30 s");
                }
                if (q == hipSuccess && __atomic_load_n(&h->done, __ATOMIC_ACQUIRE) != seq) {
                    const hipError_t e = ++restarts > 2 ? hipErrorLaunchFailure : start_server();
                    if (e != hipSuccess)
                        return fail(DCOL_ERR_HIP, std::string("dcol_prox_pair server: ") + hipGetErrorString(e));
                } else if (q != hipSuccess && q != hipErrorNotReady) {
                    return fail(DCOL_ERR_HIP, std::string("dcol_prox_pair server: ") + hipGetErrorString(q));
                }
            }
        }
        ++t->n_served;
        t->srv_us += (double)h->solve_ticks / (double)t->wall_ticks_us;
        t->srv_cycles += (double)h->solve_cycles;
        *alpha = h->alpha;
        if (contact && (flags & DCOL_CONTACT)) std::memcpy(contact, h->contact, 3 * sizeof(double));
        if (grad && (flags & DCOL_GRAD_ANY)) std::memcpy(grad, h->grad, 12 * sizeof(double));
        if (iters) *iters = h->iters;
        if (status) *status = h->status;
        return DCOL_SUCCESS;
    }
    // Otherwise one launch on the pair stream, synchronised.  (A completion flag released by
    // the kernel and polled here saved ~2.5 us per call, but its epilogue cost the one-lane
    // row-partitioned x polytope kernels 4-5 % of throughput; the server serves the latency
    // path now.)
    int rc = plan_run_rec(plan, d->pose1, d->pose2, tol, max_iter, flags & ~DCOL_CASE4, &d->alpha, d->contact,
                          d->grad, &d->iters, &d->status, nullptr, t->pair_stream, false);
    if (rc != DCOL_SUCCESS) return rc;
    ++t->n_launched;
    const hipError_t e = hipStreamSynchronize(t->pair_stream);
    if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("dcol_prox_pair: ") + hipGetErrorString(e));
    *alpha = h->alpha;
    if (contact && (flags & DCOL_CONTACT)) std::memcpy(contact, h->contact, 3 * sizeof(double));
    if (grad && (flags & DCOL_GRAD_ANY)) std::memcpy(grad, h->grad, 12 * sizeof(double));
    if (iters) *iters = h->iters;
    if (status) *status = h->status;
    return DCOL_SUCCESS;
}

int dcol_debug_pair_stamps(const dcol_table* tc, uint64_t out[16]) {
    if (!tc || !out) return fail(DCOL_ERR_ARG, "dcol_debug_pair_stamps: NULL argument");
#ifdef DCOL_STAMPS
    dcol_table* t = const_cast<dcol_table*>(tc);
    std::lock_guard<std::mutex> lk(t->mu);
    if (!t->pair_host) return fail(DCOL_ERR_ARG, "dcol_debug_pair_stamps: no pair call yet");
    for (int k = 0; k < 16; ++k) out[k] = __atomic_load_n(&t->pair_host->stamps[k], __ATOMIC_ACQUIRE);
    return DCOL_SUCCESS;
#else
    return fail(DCOL_ERR_ARG, "dcol_debug_pair_stamps: not a stamps build (make stamps)");
#endif
}

int dcol_table_stop_pair_server(const dcol_table* tc) {
    if (!tc) return fail(DCOL_ERR_ARG, "dcol_table_stop_pair_server: NULL table");
    dcol_table* t = const_cast<dcol_table*>(tc);
    std::lock_guard<std::mutex> lk(t->mu);
    DeviceGuard g(t->device);
    if (!stop_pair_server(t, kServerStopMs))
        return fail(DCOL_ERR_HIP, "dcol_table_stop_pair_server: the pair server did not stop within 5 s");
    return DCOL_SUCCESS;
}

int dcol_table_pair_server_running(const dcol_table* tc, int32_t* running) {
    if (!tc || !running) return fail(DCOL_ERR_ARG, "dcol_table_pair_server_running: NULL argument");
    dcol_table* t = const_cast<dcol_table*>(tc);
    std::lock_guard<std::mutex> lk(t->mu);
    DeviceGuard g(t->device);
    *running = 0;
    if (t->server_launched) {
        const hipError_t q = hipStreamQuery(t->server_stream);
        if (q == hipErrorNotReady)
            *running = 1;
        else if (q != hipSuccess)
            return fail(DCOL_ERR_HIP, std::string("dcol_table_pair_server_running: ") + hipGetErrorString(q));
    }
    return DCOL_SUCCESS;
}

int dcol_shutdown(void) {
    g_shutdown.store(true, std::memory_order_release);
    std::lock_guard<std::mutex> lk(g_tables_mu);
    int running = 0, stuck = 0;
    for (dcol_table* t : g_tables) {
        std::lock_guard<std::mutex> tl(t->mu);
        if (!t->server_launched) continue;
        DeviceGuard g(t->device);
        if (hipStreamQuery(t->server_stream) == hipErrorNotReady) ++running;
        (void)hipGetLastError();
        if (!stop_pair_server(t, kServerStopMs)) ++stuck;
    }
    if (const char* dbg = std::getenv("DCOL_DEBUG_SHUTDOWN"); dbg && *dbg && *dbg != '0')
        std::fprintf(stderr, "dcol_shutdown: %zu tables, %d pair servers running, %d stopped, %d did not stop\n",
                     g_tables.size(), running, running - stuck, stuck);
    return stuck ? fail(DCOL_ERR_HIP, "dcol_shutdown: a pair server did not stop within 5 s") : DCOL_SUCCESS;
}

int dcol_table_pair_plans(const dcol_table* tc, int32_t* n) {
    if (!tc || !n) return fail(DCOL_ERR_ARG, "dcol_table_pair_plans: NULL argument");
    dcol_table* t = const_cast<dcol_table*>(tc);
    std::lock_guard<std::mutex> lk(t->mu);
    *n = (int32_t)t->pair_lru.size();
    return DCOL_SUCCESS;
}

int dcol_table_pair_stats(const dcol_table* tc, int64_t* served, int64_t* launched, int64_t* server_starts,
                          double* server_solve_us, double* server_solve_cycles, int32_t* server_xcd) {
    if (!tc) return fail(DCOL_ERR_ARG, "dcol_table_pair_stats: NULL table");
    dcol_table* t = const_cast<dcol_table*>(tc);
    std::lock_guard<std::mutex> lk(t->mu);
    if (served) *served = t->n_served;
    if (launched) *launched = t->n_launched;
    if (server_starts) *server_starts = t->n_starts;
    if (server_solve_us) *server_solve_us = t->srv_us;
    if (server_solve_cycles) *server_solve_cycles = t->srv_cycles;
    if (server_xcd) *server_xcd = t->pair_host ? __atomic_load_n(&t->pair_host->xcd, __ATOMIC_ACQUIRE) : -1;
    return DCOL_SUCCESS;
}

#ifdef DCOL_CHECK_EXEC
// diagnostic build only (make check-exec; not in include/dcol.h): DPP reads from an
// inactive source lane counted over every kernel launched so far (tools/check_exec.py)
int dcol_debug_exec_violations(uint64_t* out, int32_t reset) {
    if (!out) return fail(DCOL_ERR_ARG, "dcol_debug_exec_violations: NULL out");
    (void)hipDeviceSynchronize();
    uint64_t total = 0;
#define DCOL_EXEC_SUM(tag) total += exec_violations_##tag(reset != 0);
    DCOL_EXEC_TAGS(DCOL_EXEC_SUM)
    DCOL_EXEC_SUM(capi)
#undef DCOL_EXEC_SUM
    *out = total;
    return DCOL_SUCCESS;
}
#endif

#ifdef DCOL_CHECK_EXEC
}  // extern "C"
namespace dcol {
// positive control of the DPP-source check: in each wave the odd lanes leave, then the even
// lanes take a 2-lane group sum whose partner lane is inactive -- 32 counted reads per wave
__global__ void __launch_bounds__(64) exec_selftest_kernel(double* out) {
    const int l = (int)threadIdx.x;
    if (l & 1) return;
    out[l] = Grp<2>::sum((double)l);
}
DCOL_EXEC_READER(capi)
}  // namespace dcol
extern "C" {
int dcol_debug_exec_selftest(uint64_t* counted) {
    if (!counted) return fail(DCOL_ERR_ARG, "dcol_debug_exec_selftest: NULL out");
    double* d = nullptr;
    if (hipMalloc(&d, 64 * sizeof(double)) != hipSuccess) return fail(DCOL_ERR_HIP, "selftest alloc");
    (void)exec_violations_capi(true);
    hipLaunchKernelGGL(exec_selftest_kernel, dim3(1), dim3(64), 0, 0, d);
    (void)hipDeviceSynchronize();
    *counted = exec_violations_capi(true);
    (void)hipFree(d);
    return DCOL_SUCCESS;
}
#endif

int dcol_prox_batch_host(const dcol_table* tc, int64_t B, const int32_t* s1, const int32_t* s2, const double* pose1,
                         const double* pose2, double tol, int32_t max_iter, int32_t flags, double* alpha,
                         double* contact, double* grad, int32_t* iters, int32_t* status) {
    if (!tc || B < 0) return fail(DCOL_ERR_ARG, "dcol_prox_batch_host: bad arguments");
    if (B == 0) return DCOL_SUCCESS;
    if (!s1 || !s2 || !pose1 || !pose2 || !alpha) return fail(DCOL_ERR_ARG, "dcol_prox_batch_host: NULL array");
    if (B > INT32_MAX) return fail(DCOL_ERR_ARG, "dcol_prox_batch_host: B exceeds 2^31-1");
    dcol_table* t = const_cast<dcol_table*>(tc);
    std::lock_guard<std::mutex> lk(t->mu);
    dcol_plan p;   // transient, device arrays are views into the table's staging buffer
    std::vector<int32_t> perm;
    int rc = bucket_and_fuse(t, B, s1, s2, &p, perm, (flags & DCOL_CASE4) != 0, true);
    if (rc != DCOL_SUCCESS) return rc;
    rc = ensure_fanout(t, &p);
    if (rc != DCOL_SUCCESS) return rc;
    DeviceGuard g(t->device);
    // staging: doubles pose1[6B] pose2[6B] | alpha[B] contact[3B] grad[12B] ; fused segments ;
    // ints s1 s2 perm iters status
    const size_t nin = (size_t)12 * B, nout = (size_t)16 * B;
    const size_t segb = sizeof(FusedSeg) * p.segs.size();
    const size_t bytes = (nin + nout) * sizeof(double) + segb + 5 * (size_t)B * sizeof(int32_t);
    if (t->stage_bytes < bytes) {
        if (t->stage) (void)hipFree(t->stage);
        t->stage = nullptr;
        t->stage_bytes = 0;
        hipError_t e = hipMalloc(&t->stage, bytes);
        if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("dcol_prox_batch_host staging: ") + hipGetErrorString(e));
        t->stage_bytes = bytes;
    }
    double* dp1 = static_cast<double*>(t->stage);
    double* dp2 = dp1 + 6 * B;
    double* dal = dp1 + nin;
    double* dct = dal + B;
    double* dgr = dct + 3 * B;
    FusedSeg* dsg = reinterpret_cast<FusedSeg*>(dp1 + nin + nout);
    p.d_segs = p.fused() ? dsg : nullptr;
    int32_t* ib = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(dsg) + segb);
    p.d_s1 = ib;
    p.d_s2 = ib + B;
    p.d_perm = p.launches.size() > 1 ? ib + 2 * B : nullptr;
    int32_t* dit = ib + 3 * B;
    int32_t* dst = ib + 4 * B;
    // pinned host staging (DMA at full link rate): [pose soa (12B) | outputs (16B)] doubles,
    // then [s1 | s2 | perm | iters | status] ints
    const size_t hbytes = (nin + nout) * sizeof(double) + 5 * (size_t)B * sizeof(int32_t);
    if (t->hstage_bytes < hbytes) {
        if (t->hstage) (void)hipHostFree(t->hstage);
        t->hstage = nullptr;
        t->hstage_bytes = 0;
        hipError_t e = hipHostMalloc(&t->hstage, hbytes, hipHostMallocDefault);
        if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("dcol_prox_batch_host pinned staging: ") + hipGetErrorString(e));
        t->hstage_bytes = hbytes;
    }
    double* soa = static_cast<double*>(t->hstage);
    double* outd = soa + nin;
    int32_t* ids = reinterpret_cast<int32_t*>(outd + nout);
    for (int64_t i = 0; i < B; ++i)
        for (int q = 0; q < 6; ++q) {
            soa[q * B + i] = pose1[6 * i + q];
            soa[(6 + q) * B + i] = pose2[6 * i + q];
        }
    std::memcpy(ids, s1, sizeof(int32_t) * B);
    std::memcpy(ids + B, s2, sizeof(int32_t) * B);
    std::memcpy(ids + 2 * B, perm.data(), sizeof(int32_t) * B);
    // one H2D copy: [pose1 soa | pose2 soa] then [s1 | s2 | perm]
    hipError_t e = hipMemcpy(dp1, soa, sizeof(double) * nin, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(ib, ids, sizeof(int32_t) * 3 * B, hipMemcpyHostToDevice);
    if (e == hipSuccess && segb) e = hipMemcpy(dsg, p.segs.data(), segb, hipMemcpyHostToDevice);
    if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("dcol_prox_batch_host H2D: ") + hipGetErrorString(e));
    rc = dcol_plan_run(&p, dp1, dp2, tol, max_iter, flags, dal, dct, dgr, dit, dst, nullptr);
    if (rc != DCOL_SUCCESS) return rc;
    e = hipMemcpy(outd, dal, sizeof(double) * nout, hipMemcpyDeviceToHost);   // synchronises
    if (e == hipSuccess) e = hipMemcpy(ids + 3 * B, dit, sizeof(int32_t) * 2 * B, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("dcol_prox_batch_host D2H: ") + hipGetErrorString(e));
    if (iters) std::memcpy(iters, ids + 3 * B, sizeof(int32_t) * B);
    if (status) std::memcpy(status, ids + 4 * B, sizeof(int32_t) * B);
    std::memcpy(alpha, outd, sizeof(double) * B);
    if (contact && (flags & DCOL_CONTACT))
        for (int64_t i = 0; i < B; ++i)
            for (int q = 0; q < 3; ++q) contact[3 * i + q] = outd[(size_t)B + q * B + i];
    if (grad && (flags & DCOL_GRAD_ANY))
        for (int64_t i = 0; i < B; ++i)
            for (int q = 0; q < 12; ++q) grad[12 * i + q] = outd[(size_t)4 * B + q * B + i];
    return DCOL_SUCCESS;
}

}  // extern "C"

// ------------------------------------------------------------------------------------
// multi-GPU: one all-gather of the packed per-pair record (include/dcol.h).
// RCCL is resolved with dlopen on first use, so libdcol.so itself has no link-time
// dependency on it (single-GPU users never load it).
// ------------------------------------------------------------------------------------
#include <dlfcn.h>
#include <rccl/rccl.h>

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    bool ok = false;
};

// The collective library: librccl, or the one DCOL_RCCL_LIB names (a test stand-in with
// the same five entry points, tests/fake_rccl/), resolved per library path on first use
const Rccl& rccl() {
    static std::mutex mu;
    static std::map<std::string, Rccl> libs;
    const char* env = std::getenv("DCOL_RCCL_LIB");
    const std::string path = (env && *env) ? env : "";
    std::lock_guard<std::mutex> lk(mu);
    auto it = libs.find(path);
    if (it != libs.end()) return it->second;
    Rccl x;
    void* h = nullptr;
    if (!path.empty()) {
        h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    } else {
        h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    }
    if (h) {
        x.get_unique_id = reinterpret_cast<decltype(&ncclGetUniqueId)>(dlsym(h, "ncclGetUniqueId"));
        x.init_rank = reinterpret_cast<decltype(&ncclCommInitRank)>(dlsym(h, "ncclCommInitRank"));
        x.destroy = reinterpret_cast<decltype(&ncclCommDestroy)>(dlsym(h, "ncclCommDestroy"));
        x.all_gather = reinterpret_cast<decltype(&ncclAllGather)>(dlsym(h, "ncclAllGather"));
        x.error_string = reinterpret_cast<decltype(&ncclGetErrorString)>(dlsym(h, "ncclGetErrorString"));
        x.ok = x.get_unique_id && x.init_rank && x.destroy && x.all_gather && x.error_string;
    }
    return libs.emplace(path, x).first->second;   // std::map: references stay valid
}

std::string rccl_error(const Rccl& api, ncclResult_t r) {
    return api.error_string ? api.error_string(r) : std::to_string((int)r);
}

}  // namespace

struct dcol_comm {
    const Rccl* api = nullptr;   // the library the communicator was made with
    ncclComm_t comm = nullptr;
    int32_t nranks = 0, rank = 0, device = 0;
};

namespace dcol {
// rec[i] = [alpha, grad(12), (int32 status, int32 iters)] (dcol_amd/dist.py REC layout);
// rows >= n NaN.
// A block packs kPackRows records: each thread gathers one record's fields from the SoA
// outputs (coalesced reads) into LDS, then the block streams the contiguous
// kPackRows * DCOL_REC doubles out with consecutive threads on consecutive addresses
// (coalesced writes; a record-per-thread store pattern strides 120 B per lane).
constexpr int kPackRows = 256;
__global__ void __launch_bounds__(kPackRows) pack_records(int64_t n, int64_t cap, const double* alpha,
                                                          const double* grad, const int32_t* iters,
                                                          const int32_t* status, double* rec) {
    __shared__ double tile[kPackRows * DCOL_REC];
    const int64_t r0 = (int64_t)blockIdx.x * kPackRows;
    const int64_t i = r0 + threadIdx.x;
    const double nan = __builtin_nan("");
    double* o = tile + DCOL_REC * threadIdx.x;
    if (i < n) {
        o[0] = alpha[i];
#pragma unroll
        for (int c = 0; c < 12; ++c) o[1 + c] = grad ? grad[c * n + i] : nan;
        // the int32 pair in one 8-byte slot (status low, iters high: little-endian)
        o[13] = __longlong_as_double((long long)(((unsigned long long)(unsigned)iters[i] << 32) |
                                                 (unsigned long long)(unsigned)status[i]));
    } else {
#pragma unroll
        for (int c = 0; c < DCOL_REC; ++c) o[c] = nan;
    }
    __syncthreads();
    const int64_t rows = (cap - r0) < kPackRows ? (cap - r0) : kPackRows;
    double* dst = rec + DCOL_REC * r0;
    for (int64_t e = threadIdx.x; e < rows * DCOL_REC; e += kPackRows) dst[e] = tile[e];
}
}  // namespace dcol

extern "C" {

int dcol_comm_unique_id(uint8_t id[DCOL_COMM_ID_BYTES]) {
    if (!id) return fail(DCOL_ERR_ARG, "dcol_comm_unique_id: id is NULL");
    const Rccl& api = rccl();
    if (!api.ok) return fail(DCOL_ERR_HIP, "dcol_comm_unique_id: librccl not loadable");
    ncclUniqueId u;
    ncclResult_t r = api.get_unique_id(&u);
    if (r != ncclSuccess) return fail(DCOL_ERR_HIP, "ncclGetUniqueId: " + rccl_error(api, r));
    static_assert(sizeof(u.internal) == DCOL_COMM_ID_BYTES, "unique id size");
    std::memcpy(id, u.internal, DCOL_COMM_ID_BYTES);
    return DCOL_SUCCESS;
}

int dcol_comm_create(const uint8_t id[DCOL_COMM_ID_BYTES], int32_t nranks, int32_t rank, int32_t device,
                     dcol_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks || device < 0)
        return fail(DCOL_ERR_ARG, "dcol_comm_create: bad arguments");
    *out = nullptr;
    const Rccl& api = rccl();
    if (!api.ok) return fail(DCOL_ERR_HIP, "dcol_comm_create: librccl not loadable");
    DeviceGuard g(device);
    ncclUniqueId u;
    std::memcpy(u.internal, id, DCOL_COMM_ID_BYTES);
    auto* c = new (std::nothrow) dcol_comm();
    if (!c) return fail(DCOL_ERR_NOMEM, "dcol_comm_create");
    c->api = &api;
    ncclResult_t r = api.init_rank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return fail(DCOL_ERR_HIP, "ncclCommInitRank: " + rccl_error(api, r));
    }
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    *out = c;
    return DCOL_SUCCESS;
}

int dcol_comm_destroy(dcol_comm* c) {
    if (!c) return DCOL_SUCCESS;
    if (c->comm) (void)c->api->destroy(c->comm);
    delete c;
    return DCOL_SUCCESS;
}

int dcol_prox_batch_multi_gpu(const dcol_plan* p, dcol_comm* c, const double* pose1, const double* pose2, double tol,
                              int32_t max_iter, int32_t flags, int64_t cap, double* alpha, double* grad,
                              int32_t* iters, int32_t* status, double* rec_local, double* rec_all, void* stream) {
    if (!p || !c || !rec_all || (rec_local && (!alpha || !iters || !status)))
        return fail(DCOL_ERR_ARG, "dcol_prox_batch_multi_gpu: NULL argument");
    if (cap < p->B) return fail(DCOL_ERR_ARG, "dcol_prox_batch_multi_gpu: cap < shard size");
    if (p->table->device != c->device)
        return fail(DCOL_ERR_ARG, "dcol_prox_batch_multi_gpu: plan and communicator on different devices");
    const bool gather = (flags & DCOL_NO_GATHER) == 0;
    if (!gather && rec_local) return fail(DCOL_ERR_ARG, "dcol_prox_batch_multi_gpu: DCOL_NO_GATHER is in place only");
    const int32_t rflags = flags & ~(DCOL_CONTACT | DCOL_NO_GATHER);   // the record carries no contact point
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (!rec_local) {
        // in place: the solver epilogues write this rank's records straight into its slice of
        // rec_all (no pack pass, no local copy inside the all-gather); rows past the shard
        // are all-ones bytes (NaN doubles, int pair (-1, -1))
        double* mine = rec_all + (size_t)c->rank * (size_t)cap * DCOL_REC;
        int rc = plan_run_rec(p, pose1, pose2, tol, max_iter, rflags, alpha, nullptr,
                              (rflags & DCOL_GRAD_ANY) ? grad : nullptr, iters, status, mine, stream);
        if (rc != DCOL_SUCCESS) return rc;
        DeviceGuard g(c->device);
        if (cap > p->B) {
            const hipError_t e = hipMemsetAsync(mine + (size_t)p->B * DCOL_REC, 0xFF,
                                                (size_t)(cap - p->B) * DCOL_REC * sizeof(double), st);
            if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("record tail: ") + hipGetErrorString(e));
        }
        if (!gather) return DCOL_SUCCESS;
        ncclResult_t r = c->api->all_gather(mine, rec_all, (size_t)cap * DCOL_REC, ncclDouble, c->comm, st);
        if (r != ncclSuccess) return fail(DCOL_ERR_HIP, "ncclAllGather: " + rccl_error(*c->api, r));
        return DCOL_SUCCESS;
    }
    int rc = dcol_plan_run(p, pose1, pose2, tol, max_iter, rflags, alpha, nullptr,
                           (rflags & DCOL_GRAD_ANY) ? grad : nullptr, iters, status, stream);
    if (rc != DCOL_SUCCESS) return rc;
    DeviceGuard g(c->device);
    const bool want_grad = (rflags & DCOL_GRAD_ANY) && grad;
    if (cap > 0) {
        const int64_t grid = (cap + kPackRows - 1) / kPackRows;
        hipLaunchKernelGGL(pack_records, dim3(grid), dim3(kPackRows), 0, st, p->B, cap, alpha, want_grad ? grad : nullptr,
                           iters, status, rec_local);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return fail(DCOL_ERR_HIP, std::string("pack_records: ") + hipGetErrorString(e));
    }
    ncclResult_t r = c->api->all_gather(rec_local, rec_all, (size_t)cap * DCOL_REC, ncclDouble, c->comm, st);
    if (r != ncclSuccess) return fail(DCOL_ERR_HIP, "ncclAllGather: " + rccl_error(*c->api, r));
    return DCOL_SUCCESS;
}

int dcol_comm_all_gather(dcol_comm* c, int64_t cap, double* rec_all, void* stream) {
    if (!c || !rec_all || cap < 0) return fail(DCOL_ERR_ARG, "dcol_comm_all_gather: bad arguments");
    DeviceGuard g(c->device);
    double* mine = rec_all + (size_t)c->rank * (size_t)cap * DCOL_REC;
    ncclResult_t r = c->api->all_gather(mine, rec_all, (size_t)cap * DCOL_REC, ncclDouble, c->comm,
                                        reinterpret_cast<hipStream_t>(stream));
    if (r != ncclSuccess) return fail(DCOL_ERR_HIP, "ncclAllGather: " + rccl_error(*c->api, r));
    return DCOL_SUCCESS;
}

}  // extern "C"
