// Host-side launch entry points of the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include "dcol_device.hpp"

namespace dcol {
// launch flags of a bucket (the variant flags FL of variants.py a launch may use)
enum : int { LF_FULL = 1, LF_BALL = 2, LF_CONE = 4 };
constexpr int kBlock = kSolveBlock;   // threads per workgroup of the solve kernel
constexpr int kSideStreams = 3;   // extra streams for concurrent variant launches (4 HW queues)
hipError_t launch_n4(int nsoc, int omax, int lpp, int flags, const KArgs& args, hipStream_t stream);
hipError_t launch_n5(int nsoc, int omax, int lpp, int flags, const KArgs& args, hipStream_t stream);
hipError_t launch_n6(int nsoc, int omax, int lpp, int flags, const KArgs& args, hipStream_t stream);
hipError_t launch_n7(int nsoc, int omax, int lpp, int flags, const KArgs& args, hipStream_t stream);   // case-4 extension
hipError_t launch_n8(int nsoc, int omax, int lpp, int flags, const KArgs& args, hipStream_t stream);   // case-4 extension

// One bucket of a fused launch (dcol_kernels_fused.hip): workgroups [block0, next block0)
// solve plan slots [slot0, slot0 + n) with fused variant `vid` (DCOL_FUSED_VARIANTS),
// `lpp` lanes per pair.
struct FusedSeg {
    int32_t vid, lpp;
    int64_t block0, slot0, n;
};
constexpr int kMaxFusedSegs = 64;
// fused variant id of a kernel shape + (lpp, launch flags), or -1 if the fused kernel lacks it
int fused_vid(int N, int nsoc, int omax, int lpp, int flags);
hipError_t launch_fused(const KArgs& args, const FusedSeg* d_segs, int nseg, int64_t blocks, hipStream_t stream);
}  // namespace dcol
