// The one-pair server of dcol_prox_pair: ONE resident workgroup that serves the drop-in's
// per-pair calls (proximity_mrp / proximity_gradient, one pair at a time from an unchanged
// reference ALTRO loop) without a kernel launch per call.
//
// The caller writes a request into the mailbox (PairBox, device-mapped pinned host memory:
// poses, shape ids, the fused variant id of the pair's shape and its lanes) and releases a
// new sequence number in the request word; the server polls that word, solves the pair with
// the same solve_one<...> copy the fused small-plan kernel switches to (csrc/variants.py
// fused(): every shape's latency configuration), and releases the number into box->done
// after its output stores.  Flags, tolerance and iteration cap are
// the launch's (a call with others restarts the server).  It exits after idle_ticks of the
// device wall clock without a request, or when box->stop is set (table destroy), so the
// grid always drains.
#include "dcol_device.hpp"
#include "dcol_launch.hpp"
#include "dcol_variants.inc"

#ifdef DCOL_NO_FUSED_CASES   // development builds: no cases (dcol_prox_pair then launches per call)
#undef DCOL_FUSED_VARIANTS
#define DCOL_FUSED_VARIANTS(X)
#undef DCOL_FUSED_PART_VARIANTS
#define DCOL_FUSED_PART_VARIANTS(X)
#endif

namespace dcol {

namespace {
// mailbox words: system-scope atomic loads (vector memory instructions, never a cached
// copy), made wave-uniform
template <int ORDER = __ATOMIC_RELAXED>
__device__ __forceinline__ int32_t box_ld(const int32_t* p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, ORDER, __HIP_MEMORY_SCOPE_SYSTEM));
}
template <int ORDER = __ATOMIC_RELAXED>
__device__ __forceinline__ uint64_t box_ld64(const uint64_t* p) {
    const uint64_t v = __hip_atomic_load(p, ORDER, __HIP_MEMORY_SCOPE_SYSTEM);
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)v) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ void box_st(int32_t* p, int32_t v) {
    if (threadIdx.x == 0) __hip_atomic_store(p, v, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
}
using KArgsK = const __attribute__((address_space(4))) KArgs;   // in the kernel-argument segment
}  // namespace

// Args (first kernel argument, offset 0 of the kernel-argument segment): the table pointers,
// the mailbox's one-pair arrays and the server's flags / tolerance / iteration cap.
__global__ void __launch_bounds__(kSolveBlock, 1) prox_pair_server(KArgs Args, PairBox* box, int64_t idle_ticks,
                                                                   int32_t poll_sleep) {
    (void)Args;
    constexpr uint64_t kIdMask = (1ull << kPairBoxIdBits) - 1;
    int32_t last = box_ld(&box->done);
    box_st(&box->alive, 1);
    box_st(&box->xcd, __builtin_amdgcn_s_getreg(6164) & 0xf);   // hwreg(HW_REG_XCC_ID, 0, 4)
    long long t0 = wall_clock64();
    for (;;) {
        // one round trip per poll: the id word and the stop flag in flight with the request
        // word.  All three RELAXED: a system-scope acquire load is followed by a cache
        // invalidation (buffer_inv sc0 sc1), and one per poll -- every microsecond or so --
        // kept invalidating the L2 under whatever else ran on the GPU: a 100k batch plan ran
        // 1.6x slower beside a resident server (tests/test_dropin.py ..._does_not_tax_...).
        // The acquire is one fence per request instead (below).
        uint64_t ids = box_ld64(&box->ids);
        const bool stop = box_ld(&box->stop) != 0;
        const uint64_t r = box_ld64(&box->req);
        const int32_t req = (int32_t)(r >> 32);
        if (req == last) {
            if (!stop && wall_clock64() - t0 < idle_ticks) {
                if (poll_sleep >= 0) __builtin_amdgcn_s_sleep(2);   // (A/B knob: < 0 polls without sleeping)
                for (int i = 0; i < poll_sleep; ++i) __builtin_amdgcn_s_sleep(127);
                continue;
            }
            // leaving: clear alive, then look at the request word once more -- a caller that
            // posted before it could see alive == 0 is served here, one that saw it starts a
            // new server
            box_st(&box->alive, 0);
            __threadfence_system();
            if (stop || (int32_t)(box_ld64<__ATOMIC_SEQ_CST>(&box->req) >> 32) == last) return;
            box_st(&box->alive, 1);
            continue;
        }
        // a new request: acquire it (the poses and the id word were written before it)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        const long long w0 = wall_clock64(), c0 = clock64();
        if ((ids >> 48) != ((uint32_t)req & 0xffffu)) ids = box_ld64(&box->ids);   // read before this request's
        const int vid = (int)(r & 0xffffu);
        const int lpp = (int)((r >> 16) & 0xffffu);
        const int k1 = (int)(ids & kIdMask), k2 = (int)((ids >> kPairBoxIdBits) & kIdMask);
        // The launch arguments and the lane index are made opaque per request, so nothing
        // the solver derives from them is loop-invariant: the kernel arguments are scalar
        // loads from the kernel-argument segment where the solver uses them and the lane
        // masks are computed where they are used, as in the one-shot kernels, instead of
        // being hoisted out of this loop and held in registers across it (every solver copy
        // then spills to scratch).
        KArgsK* ap = (KArgsK*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ap));
        const KArgs& A = *(const KArgs*)ap;
        int q = (int)threadIdx.x;
        asm volatile("" : "+v"(q));
        if (lpp > 0 && q < lpp) {
            switch (vid) {   // NOLINT (empty in development builds)
#define DCOL_SCASE(ID, NN, NS, OM, LP, FL)                                                       \
    case ID:                                                                                     \
        solve_one<NN, NS, OM, LP, (FL & 1) != 0, (FL & 2) != 0, (FL & 4) != 0>(A, 0, q, -1, k1, k2); \
        break;
                DCOL_FUSED_VARIANTS(DCOL_SCASE)
#undef DCOL_SCASE
#define DCOL_SPCASE(ID, NN, NS, OM, LP, FL, OEE)                                                 \
    case ID:                                                                                     \
        solve_one<NN, NS, OM, LP, (FL & 1) != 0, (FL & 2) != 0, false, OEE>(A, 0, q, -1, k1, k2); \
        break;
                DCOL_FUSED_PART_VARIANTS(DCOL_SPCASE)
#undef DCOL_SPCASE
                default:
                    break;
            }
        }
        if (threadIdx.x == 0) {   // request-to-answer time on the device (dcol_table_pair_stats)
            box->solve_ticks = wall_clock64() - w0;
            box->solve_cycles = clock64() - c0;
#ifdef DCOL_STAMPS
            box->stamps[6] = (unsigned long long)c0;
            box->stamps[7] = (unsigned long long)clock64();
#endif
        }
        // the pair's lanes reconverged: the fence waits for all of the wave's output stores
        __threadfence_system();
        last = req;
        box_st(&box->done, req);
        t0 = wall_clock64();
    }
}

hipError_t launch_pair_server(const KArgs& args, PairBox* box, int64_t idle_ticks, int32_t poll_sleep,
                              hipStream_t stream) {
    if (!box || idle_ticks <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(prox_pair_server, dim3(1), dim3(kSolveBlock), 0, stream, args, box, idle_ticks, poll_sleep);
    return hipGetLastError();
}

DCOL_EXEC_READER(server)

}  // namespace dcol
