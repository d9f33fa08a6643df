// Fused multi-variant launch: every bucket of a small mixed plan in ONE kernel launch.
//
// An ALTRO phase batch is one victim against a few obstacle types (quadrotor hallway:
// sphere vs polytopes, spheres, capsules, cylinders, a polygon -> 5 kernel variants of
// 100-400 pairs each).  Such a plan is latency-bound (far fewer waves than SIMDs), and five
// launches spread over streams cost more in launch, fork and join latency than the solves
// themselves.  Here each workgroup finds its bucket in a small segment table (scalar loads,
// uniform per workgroup) and switches on the bucket's variant id to the same
// solve_one<N, NSOC, OMAX, LPP, FULL, BALL, CONE> the per-variant kernels run, with that shape's
// latency configuration (largest LPP; csrc/variants.py fused()).  One wave per workgroup, so
// a wave never mixes variants and never diverges on structure.
#include "dcol_device.hpp"
#include "dcol_launch.hpp"
#include "dcol_variants.inc"

// Development builds (make dev): no cases -- plans launch per bucket (fan-out), and this
// unit, whose compile time is the sum of its ~100 solver copies, builds in seconds.
#ifdef DCOL_NO_FUSED_CASES
#undef DCOL_FUSED_VARIANTS
#define DCOL_FUSED_VARIANTS(X)
#undef DCOL_FUSED_PART_VARIANTS
#define DCOL_FUSED_PART_VARIANTS(X)
#endif

namespace dcol {

__global__ void __launch_bounds__(kSolveBlock, 1) prox_fused_kernel(KArgs A, const FusedSeg* __restrict__ segs,
                                                                    int nseg) {
    int s = 0;
    while (s + 1 < nseg && (int64_t)blockIdx.x >= segs[s + 1].block0) ++s;
    const FusedSeg S = segs[s];
    const int64_t t = ((int64_t)blockIdx.x - S.block0) * blockDim.x + threadIdx.x;
    const int64_t slot = t / S.lpp;
    const int q = (int)(t % S.lpp);
    if (slot >= S.n) return;
    const int64_t pi = A.perm ? (int64_t)A.perm[S.slot0 + slot] : (S.slot0 + slot);
    switch (S.vid) {   // NOLINT (empty in development builds)
#define DCOL_FCASE(ID, NN, NS, OM, LP, FL)                  \
    case ID:                                                \
        solve_one<NN, NS, OM, LP, (FL & 1) != 0, (FL & 2) != 0, (FL & 4) != 0>(A, pi, q); \
        break;
        DCOL_FUSED_VARIANTS(DCOL_FCASE)
#undef DCOL_FCASE
#define DCOL_FPCASE(ID, NN, NS, OM, LP, FL, OEE)           \
    case ID:                                                \
        solve_one<NN, NS, OM, LP, (FL & 1) != 0, (FL & 2) != 0, false, OEE>(A, pi, q); \
        break;
        DCOL_FUSED_PART_VARIANTS(DCOL_FPCASE)
#undef DCOL_FPCASE
        default:
            break;
    }
}

// (a bucket whose pairs all fill OMAX takes the padding-free case if there is one, a bucket
// of ball-SOC or cone-SOC pairs the structured case, else the plain one -- as the
// per-variant launchers do)
int fused_vid(int N, int nsoc, int omax, int lpp, int flags, int oe) {
    if (oe > 0) {   // row-partitioned bucket: FULL|BALL, BALL, FULL, dense
        for (const int want : {(int)(LF_FULL | LF_BALL), (int)LF_BALL, (int)LF_FULL, 0}) {
            if ((want & flags) != want) continue;
#define DCOL_FPID(ID, NN, NS, OM, LP, FL, OEE) \
    if (NN == N && NS == nsoc && OM == omax && OEE == oe && LP == lpp && FL == want) return ID;
            DCOL_FUSED_PART_VARIANTS(DCOL_FPID)
#undef DCOL_FPID
        }
        return -1;
    }
    for (const int want : {(int)LF_FULL, (int)LF_BALL, (int)LF_CONE, 0}) {
        if ((want & flags) != want) continue;
#define DCOL_FID(ID, NN, NS, OM, LP, FL) \
    if (NN == N && NS == nsoc && OM == omax && LP == lpp && FL == want) return ID;
        DCOL_FUSED_VARIANTS(DCOL_FID)
#undef DCOL_FID
    }
    return -1;
}

hipError_t launch_fused(const KArgs& args, const FusedSeg* d_segs, int nseg, int64_t blocks, hipStream_t stream) {
    if (nseg <= 0 || nseg > kMaxFusedSegs || blocks <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(prox_fused_kernel, dim3((unsigned)blocks), dim3(kSolveBlock), 0, stream, args, d_segs, nseg);
    return hipGetLastError();
}

DCOL_EXEC_READER(fused)

}  // namespace dcol
