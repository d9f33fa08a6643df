// altro_device.hip -- forward-difference dynamics Jacobians of a whole trajectory on the GPU
// ("batch over knots on device"; reference ALTRO.py:77-100
// compute_jacobian, called per knot at ALTRO.py:289-290, over the systems' discrete_dynamics,
// piano_mover.py:28-47, cluttered_hallway_quadrotor.py:86-105, cone_through_wall.py:67-86).
//
// One thread per (knot, column): column c < nx perturbs x_c, nx <= c < nx + nu perturbs
// u_(c - nx), c = nx + nu is the unperturbed step f0.  A workgroup holds kKnots knots x 32
// columns; f0 goes through LDS to the knot's other columns, each of which writes its column
// (f1 - f0) / delta of A or B.  The dynamics are altro_model.hpp, the same source the host
// library runs, and this file is compiled without contraction: A and B equal
// dcol_altro_jacobians bitwise.  X, U, A, B may be device memory or device-mapped pinned
// host memory (the ALTRO driver's zero-copy phase buffers).
#include <hip/hip_runtime.h>

#include "../../include/dcol_altro_device.h"
#include "altro_model.hpp"

namespace {

constexpr int kCols = 32;   // >= DCOL_ALTRO_MAX_NX + DCOL_ALTRO_MAX_NU + 1
constexpr int kKnots = 8;   // knots per workgroup
static_assert(kCols >= DCOL_ALTRO_MAX_NX + DCOL_ALTRO_MAX_NU + 1, "one column per perturbation + the base step");

__global__ void __launch_bounds__(kCols * kKnots) jacobian_kernel(dcol_altro_model m, int64_t T,
                                                                   const double* __restrict__ X,
                                                                   const double* __restrict__ U, double delta,
                                                                   double* __restrict__ A, double* __restrict__ B) {
    __shared__ double f0s[kKnots][DCOL_ALTRO_MAX_NX];
    const int nx = m.nx, nu = m.nu;
    const int c = threadIdx.x, ky = threadIdx.y;
    const int64_t t = (int64_t)blockIdx.x * kKnots + ky;
    const bool active = t < T && c <= nx + nu;
    double f[dcol_altro::MX];
    if (active) {
        double xp[dcol_altro::MX], up[dcol_altro::MU];
        for (int i = 0; i < nx; ++i) xp[i] = X[t * nx + i];
        for (int i = 0; i < nu; ++i) up[i] = U[t * nu + i];
        if (c < nx) xp[c] += delta;
        else if (c < nx + nu) up[c - nx] += delta;
        dcol_altro::rk4(m, xp, up, f);
        if (c == nx + nu)
            for (int i = 0; i < nx; ++i) f0s[ky][i] = f[i];
    }
    __syncthreads();
    if (!active || c == nx + nu) return;
    if (c < nx) {
        double* At = A + t * nx * nx;
        for (int i = 0; i < nx; ++i) At[i * nx + c] = (f[i] - f0s[ky][i]) / delta;
    } else {
        double* Bt = B + t * nx * nu;
        for (int i = 0; i < nx; ++i) Bt[i * nu + (c - nx)] = (f[i] - f0s[ky][i]) / delta;
    }
}

}  // namespace

extern "C" int dcol_altro_jacobians_device(const dcol_altro_model* m, int64_t T, const double* X, const double* U,
                                           double delta, double* A, double* B, void* stream) {
    if (!dcol_altro::model_ok(m) || T < 0 || (T > 0 && (!X || !U || !A || !B)) || !(delta != 0))
        return DCOL_ALTRO_ERR_ARG;
    if (T == 0) return DCOL_ALTRO_OK;
    const int64_t blocks = (T + kKnots - 1) / kKnots;
    hipLaunchKernelGGL(jacobian_kernel, dim3((unsigned)blocks), dim3(kCols, kKnots), 0,
                       reinterpret_cast<hipStream_t>(stream), *m, T, X, U, delta, A, B);
    return hipGetLastError() == hipSuccess ? DCOL_ALTRO_OK : DCOL_ALTRO_ERR_DEVICE;
}
