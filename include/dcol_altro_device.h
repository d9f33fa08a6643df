/*
 * dcol_altro_device.h -- the ALTRO driver's device entry point, exported by the HIP library
 * (lib/libdcol.so) next to the proximity C-ABI of dcol.h.
 *
 *   reference                                              replaced by
 *   ----------------------------------------------------   ---------------------------------
 *   ALTRO.py compute_jacobian (forward differences, delta   dcol_altro_jacobians_device()
 *     1e-6; ALTRO.py:77-100) called per knot at              (all knots, one GPU launch;
 *     ALTRO.py:289-290 over discrete_dynamics                 SURVEY.md section 8 f3)
 *     (piano_mover.py:28-47, cluttered_hallway_quadrotor.py:86-105, cone_through_wall.py:67-86)
 */
#ifndef DCOL_ALTRO_DEVICE_H
#define DCOL_ALTRO_DEVICE_H

#include "dcol_altro.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Forward-difference Jacobians of the discrete dynamics at knots t < T, all knots in one
 * launch on `stream` (a hipStream_t; NULL = the default stream): A [T, nx, nx], B [T, nx, nu],
 * bitwise equal to dcol_altro_jacobians (same dynamics source, no contraction, IEEE division
 * and square root).  X [T, nx], U [T, nu], A, B: device pointers or device-mapped pinned
 * host memory.  Asynchronous; DCOL_ALTRO_ERR_DEVICE if the launch fails. */
int dcol_altro_jacobians_device(const dcol_altro_model* m, int64_t T, const double* X, const double* U,
                                double delta, double* A, double* B, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DCOL_ALTRO_DEVICE_H */
