// Test infrastructure (never part of the product library): an in-process stand-in for the
// five collective entry points libdcol.so resolves (ncclGetUniqueId, ncclCommInitRank,
// ncclAllGather, ncclCommDestroy, ncclGetErrorString), so that the C-ABI multi-GPU path
// (dcol_prox_batch_multi_gpu / dcol_comm_all_gather) runs as rank 0 AND rank 1 ... on ONE
// GPU: each "rank" is a host thread of the test process with its own communicator, stream
// and buffers; RCCL itself refuses two ranks on one device.  Selected with DCOL_RCCL_LIB
// (include/dcol.h).
//
// Semantics follow ncclAllGather: rank r's `count` elements of sendbuff land at
// recvbuff + r * count on every rank, in place when sendbuff == recvbuff + rank * count, and
// the collective is ordered on each rank's stream after the work issued before it.  Every
// rank records an event after its pending work, the ranks meet on the host, each rank's
// stream waits on every other rank's event and copies their slices in (device-to-device
// copies on the one GPU), then records a second event that every other rank's stream
// waits on before its next work -- so no rank can overwrite its send slice (its next
// solve) before every rank has read it, as in a real collective.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unistd.h>
#include <vector>

namespace {

constexpr auto kTimeout = std::chrono::seconds(60);   // a rank that never arrives fails the call

struct Group {
    int nranks = 0;
    std::mutex mu;
    std::condition_variable cv;
    int joined = 0;
    int alive = 0;
    uint64_t bgen = 0;   // barrier generation
    int bcount = 0;
    struct Slot {
        const char* send = nullptr;
        hipEvent_t ready = nullptr, done = nullptr;
    };
    std::vector<Slot> slots;

    // all ranks meet; false on timeout (lock held by the caller)
    bool barrier(std::unique_lock<std::mutex>& lk) {
        const uint64_t my = bgen;
        if (++bcount == nranks) {
            bcount = 0;
            ++bgen;
            cv.notify_all();
            return true;
        }
        return cv.wait_for(lk, kTimeout, [&] { return bgen != my; });
    }
};

std::mutex g_mu;
std::map<std::string, std::shared_ptr<Group>> g_groups;
std::atomic<uint64_t> g_ids{0};

size_t type_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

}  // namespace

struct ncclComm {
    std::shared_ptr<Group> g;
    std::string key;
    int rank = 0;
    hipEvent_t ready = nullptr, done = nullptr;
};

extern "C" {

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (fake_rccl)";
        case ncclInvalidArgument: return "invalid argument (fake_rccl)";
        case ncclSystemError: return "rank rendezvous timed out (fake_rccl)";
        default: return "internal error (fake_rccl)";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id->internal, 0, sizeof(id->internal));
    std::snprintf(id->internal, sizeof(id->internal), "fake_rccl:%d:%llu", (int)getpid(),
                  (unsigned long long)g_ids.fetch_add(1));
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    const std::string key(id.internal, strnlen(id.internal, sizeof(id.internal)));
    std::shared_ptr<Group> g;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto& slot = g_groups[key];
        if (!slot) {
            slot = std::make_shared<Group>();
            slot->nranks = nranks;
            slot->slots.resize(nranks);
        }
        g = slot;
    }
    if (g->nranks != nranks) return ncclInvalidArgument;
    auto* c = new ncclComm();
    c->g = g;
    c->key = key;
    c->rank = rank;
    if (hipEventCreateWithFlags(&c->ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return ncclUnhandledCudaError;
    }
    std::unique_lock<std::mutex> lk(g->mu);
    ++g->joined;
    ++g->alive;
    if (!g->barrier(lk)) {   // ncclCommInitRank returns once every rank has joined
        --g->alive;
        lk.unlock();
        (void)hipEventDestroy(c->ready);
        (void)hipEventDestroy(c->done);
        delete c;
        return ncclSystemError;
    }
    *out = c;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
    if (!c) return ncclInvalidArgument;
    (void)hipEventDestroy(c->ready);
    (void)hipEventDestroy(c->done);
    bool last = false;
    {
        std::lock_guard<std::mutex> lk(c->g->mu);
        last = --c->g->alive == 0;
    }
    if (last) {
        std::lock_guard<std::mutex> lk(g_mu);
        g_groups.erase(c->key);
    }
    delete c;
    return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t dt, ncclComm_t c,
                           hipStream_t stream) {
    const size_t es = type_size(dt);
    if (!c || es == 0 || (count > 0 && (!sendbuff || !recvbuff))) return ncclInvalidArgument;
    const size_t bytes = count * es;
    Group& g = *c->g;
    char* recv = static_cast<char*>(recvbuff);
    if (hipEventRecord(c->ready, stream) != hipSuccess) return ncclUnhandledCudaError;
    std::unique_lock<std::mutex> lk(g.mu);
    g.slots[c->rank].send = static_cast<const char*>(sendbuff);
    g.slots[c->rank].ready = c->ready;
    g.slots[c->rank].done = c->done;
    if (!g.barrier(lk)) return ncclSystemError;               // every rank's send slice is registered
    const std::vector<Group::Slot> slots = g.slots;
    lk.unlock();
    hipError_t e = hipSuccess;
    for (int r = 0; r < g.nranks && e == hipSuccess; ++r) {
        char* dst = recv + (size_t)r * bytes;
        if (r == c->rank) {
            if (slots[r].send != dst && bytes) e = hipMemcpyAsync(dst, slots[r].send, bytes, hipMemcpyDeviceToDevice, stream);
            continue;
        }
        e = hipStreamWaitEvent(stream, slots[r].ready, 0);
        if (e == hipSuccess && bytes) e = hipMemcpyAsync(dst, slots[r].send, bytes, hipMemcpyDeviceToDevice, stream);
    }
    if (e == hipSuccess) e = hipEventRecord(c->done, stream);
    lk.lock();
    if (!g.barrier(lk)) return ncclSystemError;               // every rank's copies are issued
    lk.unlock();
    for (int r = 0; r < g.nranks && e == hipSuccess; ++r)
        if (r != c->rank) e = hipStreamWaitEvent(stream, slots[r].done, 0);
    lk.lock();
    if (!g.barrier(lk)) return ncclSystemError;               // nobody re-records its events early
    return e == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

}  // extern "C"
