// Host-side launch entry points of the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include "dcol_device.hpp"

namespace dcol {
// launch flags of a bucket (the variant flags FL of variants.py a launch may use)
enum : int { LF_FULL = 1, LF_BALL = 2, LF_CONE = 4 };
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
#define DCOL_EXEC_TAGS(X) X(n4) X(n5) X(n6) X(n7) X(n8) X(fused) X(p51) X(p52) X(p61) X(p62) X(susp)
#define DCOL_EXEC_DECL(tag) unsigned long long exec_violations_##tag(bool reset);
DCOL_EXEC_TAGS(DCOL_EXEC_DECL)
DCOL_EXEC_DECL(capi)   // the C-ABI unit's own counter (dcol_debug_exec_selftest)
#undef DCOL_EXEC_DECL
#else
#define DCOL_EXEC_READER(tag)
#endif
}  // namespace dcol
