// Host-side launch entry points of the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include "dcol_device.hpp"

namespace dcol {
// launch flags of a bucket (the variant flags FL of variants.py a launch may use)
enum : int { LF_FULL = 1, LF_BALL = 2, LF_CONE = 4, LF_BOX = 8, LF_SPLIT = 32, LF_FDONLY = 64 };
// (LF_FDONLY: a run without envelope / implicit gradients; LF_SPLIT: DCOL_SPLIT=1 opt-in)
constexpr int kBlock = kSolveBlock;   // threads per workgroup of the solve kernel
constexpr int kSideStreams = 7;   // capacity of the extra streams for concurrent variant launches
                                  // (dcol_capi.cpp side_streams(): 3 by default, DCOL_SIDE_STREAMS)
hipError_t launch_n4(int nsoc, int omax, int lpp, int flags, const KArgs& args, hipStream_t stream);
hipError_t launch_n5(int nsoc, int omax, int lpp, int flags, const KArgs& args, hipStream_t stream);
hipError_t launch_n6(int nsoc, int omax, int lpp, int flags, const KArgs& args, hipStream_t stream);
hipError_t launch_n7(int nsoc, int omax, int lpp, int flags, const KArgs& args, hipStream_t stream);   // case-4 extension
hipError_t launch_n8(int nsoc, int omax, int lpp, int flags, const KArgs& args, hipStream_t stream);   // case-4 extension
// row-partitioned copies (dcol_kernels_p<N><NSOC>.hip): bucket (omax, oe)
hipError_t launch_part_n5s1(int omax, int oe, int lpp, int flags, const KArgs& args, hipStream_t stream);
hipError_t launch_part_n5s2(int omax, int oe, int lpp, int flags, const KArgs& args, hipStream_t stream);
hipError_t launch_part_n6s1(int omax, int oe, int lpp, int flags, const KArgs& args, hipStream_t stream);
hipError_t launch_part_n6s2(int omax, int oe, int lpp, int flags, const KArgs& args, hipStream_t stream);
hipError_t launch_part_n6s2_dense(int omax, int oe, int lpp, int flags, const KArgs& args, hipStream_t stream);

// One bucket of a fused launch (dcol_kernels_fused.hip): workgroups [block0, next block0)
// solve plan slots [slot0, slot0 + n) with fused variant `vid` (DCOL_FUSED_VARIANTS),
// `lpp` lanes per pair.
struct FusedSeg {
    int32_t vid, lpp;
    int64_t block0, slot0, n;
};
constexpr int kMaxFusedSegs = 64;
// suspend / resume launch pairs (dcol_kernels_susp.hip)
bool susp_available(int N, int nsoc, int omax, int lpp, int flags, int oe, int* fields);
hipError_t launch_susp(int N, int nsoc, int omax, int lpp, int flags, int oe, const KArgs& args, hipStream_t stream);
// fused variant id of a kernel shape + (lpp, launch flags, PART extra slots oe), or -1 if
// the fused kernel lacks it
int fused_vid(int N, int nsoc, int omax, int lpp, int flags, int oe = 0);
hipError_t launch_fused(const KArgs& args, const FusedSeg* d_segs, int nseg, int64_t blocks, hipStream_t stream);
// packed multi-bucket launch (dcol_kernels_packed.hip): a mid-size plan's buckets in their
// throughput configurations in ONE launch (segments as FusedSeg, vid = packed case id)
int packed_vid(int N, int nsoc, int omax, int lpp, int flags, int oe = 0);
hipError_t launch_packed(const KArgs& args, const FusedSeg* d_segs, int nseg, int64_t blocks, hipStream_t stream);

// Mailbox of the one-pair server (dcol_prox_pair; dcol_kernels_server.hip prox_pair_server):
// device-mapped pinned host memory, one per table.  The caller writes the poses and the
// shape-id word, then releases the request word: a new sequence number in its high half,
// the pair's fused variant id and lanes in its low half, so one poll of the server reads
// all it needs to branch.  The id word carries the sequence number's low 16 bits: the server
// loads it together with the request word (one round trip) and re-reads it only if it saw
// an older one.  The server solves the pair into the output slots and releases the sequence
// number into `done`.  `alive` is 1 while a server polls (it clears it before it exits and
// then re-checks the request word, so a request posted meanwhile is either served or seen by
// the caller as "start a server"); `stop` makes it exit at its next poll.  flags / tol /
// max_iter: those of the running server (a call with others restarts it).
struct PairBox {
    double pose1[6], pose2[6];
    double alpha, contact[3], grad[12];
    int32_t iters, status;
    double tol;
    int32_t flags, max_iter;
    uint64_t req;   // seq << 32 | lpp << 16 | vid
    uint64_t ids;   // (seq & 0xffff) << 48 | s2 << 24 | s1   (shape ids below 2^24)
    int32_t done, alive, stop;
    int32_t xcd;   // the XCD the running server sits on (HW_REG_XCC_ID; dcol_table_pair_stats)
    int64_t solve_ticks, solve_cycles;   // the last served request: wall-clock ticks and shader cycles
#ifdef DCOL_STAMPS
    // diagnostic build (make stamps): s_memtime at solve_one's phases (DCOL_STAMP 0..5: start,
    // frames, assembly, initialise, PDIP loop, gradient; 8..15: the sub-phases of PDIP
    // iteration 2), the request seen (6) and the answer's release (7); dcol_debug_pair_stamps
    unsigned long long stamps[16];
#endif
};
constexpr int kPairBoxIdBits = 24;
// a server on `stream` serving box (device view) with args' table pointers, flags, tolerance
// and iteration cap; it exits after idle_ticks of the device wall clock
// (hipDeviceAttributeWallClockRate) without a request
// (poll_sleep: extra s_sleep(127) rounds between polls, DCOL_PAIR_SERVER_POLL_SLEEP; A/B)
hipError_t launch_pair_server(const KArgs& args, PairBox* box, int64_t idle_ticks, int32_t poll_sleep,
                              hipStream_t stream);
#ifdef DCOL_CHECK_EXEC
// diagnostic build: host reader of a translation unit's DPP-source violation counter
// (dcol_device.hpp dpp_check), summed by dcol_debug_exec_violations (dcol_capi.cpp)
#define DCOL_EXEC_READER(tag)                                                                  \
    unsigned long long exec_violations_##tag(bool reset) {                                     \
        unsigned long long v = 0, z = 0;                                                       \
        if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(dcol_exec_violations), sizeof(v)) != hipSuccess) \
            v = ~0ull;                                                                         \
        if (reset) (void)hipMemcpyToSymbol(HIP_SYMBOL(dcol_exec_violations), &z, sizeof(z));   \
        return v;                                                                              \
    }
#define DCOL_EXEC_TAGS(X) X(n4) X(n5) X(n6) X(n7) X(n8) X(fused) X(packed) X(p51) X(p52) X(p61) X(p62) X(p62d) X(susp) X(server)
#define DCOL_EXEC_DECL(tag) unsigned long long exec_violations_##tag(bool reset);
DCOL_EXEC_TAGS(DCOL_EXEC_DECL)
DCOL_EXEC_DECL(capi)   // the C-ABI unit's own counter (dcol_debug_exec_selftest)
#undef DCOL_EXEC_DECL
#else
#define DCOL_EXEC_READER(tag)
#endif
}  // namespace dcol
