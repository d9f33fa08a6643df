// Host-side launch entry points of the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include "dcol_device.hpp"

namespace dcol {
constexpr int kBlock = kSolveBlock;   // threads per workgroup of the solve kernel
constexpr int kSideStreams = 3;   // extra streams for concurrent variant launches (4 HW queues)
hipError_t launch_n4(int nsoc, int omax, int lpp, bool full, const KArgs& args, hipStream_t stream);
hipError_t launch_n5(int nsoc, int omax, int lpp, bool full, const KArgs& args, hipStream_t stream);
hipError_t launch_n6(int nsoc, int omax, int lpp, bool full, const KArgs& args, hipStream_t stream);
hipError_t launch_n7(int nsoc, int omax, int lpp, bool full, const KArgs& args, hipStream_t stream);   // case-4 extension
hipError_t launch_n8(int nsoc, int omax, int lpp, bool full, const KArgs& args, hipStream_t stream);   // case-4 extension
}  // namespace dcol
