// Suspend / resume launch pairs (variants.py SUSP, dcol_device.hpp KArgs susp_*): the main
// launch (prox_kernel, FL bit 4) and the resume launch (prox_resume_kernel) of each listed
// variant, queued back to back on one stream.
#include "dcol_device.hpp"
#include "dcol_launch.hpp"
#include "dcol_variants.inc"

namespace dcol {

// the launch's (N, NSOC, OMAX, LPP, flags, oe) has a suspend / resume copy; *fields: the
// doubles per continuation entry (Solver::SUSP_FIELDS)
bool susp_available(int N, int nsoc, int omax, int lpp, int flags, int oe, int* fields) {
#define DCOL_SAV(NN, NS, OM, LP, WP, FL, OEE)                                                      \
    if (NN == N && NS == nsoc && OM == omax && LP == lpp && OEE == oe && ((FL & 15) & flags) == (FL & 15)) { \
        if (fields) *fields = Solver<NN, NS, OM, LP, (FL & 2) != 0, (FL & 4) != 0, OEE>::SUSP_FIELDS; \
        return true;                                                                               \
    }
    DCOL_SUSP_VARIANTS(DCOL_SAV)
#undef DCOL_SAV
    (void)N; (void)nsoc; (void)omax; (void)lpp; (void)flags; (void)oe; (void)fields;
    return false;
}

hipError_t launch_susp(int N, int nsoc, int omax, int lpp, int flags, int oe, const KArgs& args, hipStream_t stream) {
#define DCOL_SL(NN, NS, OM, LP, WP, FL, OEE)                                                           \
    if (NN == N && NS == nsoc && OM == omax && LP == lpp && OEE == oe && ((FL & 15) & flags) == (FL & 15)) { \
        const int64_t grid = (args.n * LP + kBlock - 1) / kBlock;                                      \
        hipLaunchKernelGGL((prox_kernel<NN, NS, OM, LP, WP, FL, OEE>), dim3(grid), dim3(kBlock), 0, stream, args); \
        hipError_t e = hipGetLastError();                                                              \
        if (e != hipSuccess) return e;                                                                 \
        const int64_t rgrid = (args.susp_cap * LP + kBlock - 1) / kBlock;                              \
        if (rgrid > 0)                                                                                 \
            hipLaunchKernelGGL((prox_resume_kernel<NN, NS, OM, LP, WP, FL, OEE>), dim3(rgrid), dim3(kBlock), 0, stream, args); \
        return hipGetLastError();                                                                      \
    }
    DCOL_SUSP_VARIANTS(DCOL_SL)
#undef DCOL_SL
    (void)N; (void)nsoc; (void)omax; (void)lpp; (void)flags; (void)oe; (void)args; (void)stream;
    return hipErrorInvalidValue;
}

DCOL_EXEC_READER(susp)

}  // namespace dcol
