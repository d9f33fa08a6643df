// Packed multi-bucket launch: every bucket of a MID-SIZE plan in one kernel launch, each in
// its throughput configuration (variants.py packed()).
//
// A rank's shard of a mixed batch (configs[4] at 4-8 GPUs: 125k-250k pairs) splits into ~15
// variant buckets of 8k-17k pairs.  Each bucket alone covers 15-30 % of the SIMDs with waves
// that last 20-80 us (single-wave latency: the slowest pair of the wave), so launched one by
// one -- even three streams at a time -- the step is a chain of under-filled launches
// (0.32 ms per 125k pairs, where 1M pairs take 0.85 ms).  Here one launch carries all of
// them: workgroup w finds its segment (bucket) in the segment table, segments in descending
// per-pair cost (dcol_capi.cpp plan_pack), and switches to that bucket's solver copy.  The
// kernel runs one wave per SIMD (its register allocation is the maximum over the cases), so
// the hardware dispatcher places each next workgroup on the next SIMD that frees up: list
// scheduling of every bucket's waves, longest first, instead of stream chains.
//
// Each case is the same solve_one<...> instance the bucket's per-variant kernel runs, with
// the G rows in registers (GLDS off -- the LDS-rows copies exist for the register budget of
// two waves per SIMD; the codegen-invariance twin already runs every copy that way), so the
// results are bitwise those of the per-bucket launches.
#include "dcol_device.hpp"
#include "dcol_launch.hpp"
#include "dcol_variants.inc"

#ifdef DCOL_NO_PACKED_CASES   // development builds (make dev): plans launch per bucket
#undef DCOL_PACKED_VARIANTS
#define DCOL_PACKED_VARIANTS(X)
#endif

namespace dcol {

__global__ void __launch_bounds__(kSolveBlock, 1) prox_packed_kernel(KArgs A, const FusedSeg* __restrict__ segs,
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
#define DCOL_KCASE(ID, NN, NS, OM, LP, FL, OEE)                                                       \
    case ID:                                                                                        \
        solve_one<NN, NS, OM, LP, (FL & 1) != 0, (FL & 2) != 0, (FL & 4) != 0, OEE, 0, false, (FL & 8) != 0>( \
            A, pi, q);                                                                              \
        break;
        DCOL_PACKED_VARIANTS(DCOL_KCASE)
#undef DCOL_KCASE
        default:
            break;
    }
}

// the case of a bucket: the first entry of its shape (and LPP) whose flavour the bucket's
// launch flags allow -- the list is in the per-variant launchers' preference order
int packed_vid(int N, int nsoc, int omax, int lpp, int flags, int oe) {
#define DCOL_KID(ID, NN, NS, OM, LP, FL, OEE) \
    if (NN == N && NS == nsoc && OM == omax && LP == lpp && OEE == oe && (FL & flags) == FL) return ID;
    DCOL_PACKED_VARIANTS(DCOL_KID)
#undef DCOL_KID
    (void)N; (void)nsoc; (void)omax; (void)lpp; (void)flags; (void)oe;
    return -1;
}

hipError_t launch_packed(const KArgs& args, const FusedSeg* d_segs, int nseg, int64_t blocks, hipStream_t stream) {
    if (nseg <= 0 || nseg > kMaxFusedSegs || blocks <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(prox_packed_kernel, dim3((unsigned)blocks), dim3(kSolveBlock), 0, stream, args, d_segs, nseg);
    return hipGetLastError();
}

DCOL_EXEC_READER(packed)

}  // namespace dcol
