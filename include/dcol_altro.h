/*
 * dcol_altro.h — C-ABI of the native host kernels of the batched ALTRO constraint driver
 * (SURVEY.md §8 f1/f3).  The proximity solves themselves go through dcol.h on the GPU;
 * this library holds the sequential, knot-coupled host work around them, which the
 * reference runs as per-knot NumPy calls:
 *
 *   reference                                                 replaced by
 *   ------------------------------------------------------   ---------------------------------
 *   systems/<sys>.py discrete_dynamics (RK4 of dynamics)      dcol_altro_dynamics()
 *     piano_mover.py:7-47, cluttered_hallway_quadrotor.py:      (batched over states)
 *     19-105, cone_through_wall.py:19-86
 *   ALTRO.py compute_jacobian (forward differences,           dcol_altro_jacobians()
 *     delta 1e-6) called per knot at ALTRO.py:289-290           (all knots in one call),
 *                                                               (GPU: dcol_altro_device.h)
 *   ALTRO.py backward_pass Riccati recursion :304-336          dcol_altro_backward()
 *     (Quu = luu + B'(Vxx+reg I)B, scipy cho_factor/solve)
 *   ALTRO.py forward_pass rollout :214-217                     dcol_altro_rollout(), dcol_altro_rollouts()
 *     (U - K(Xn - X) - a k, then discrete_dynamics)
 *   ALTRO.py compute_total_cost :103-145                       dcol_altro_cost()
 *   ALTRO.py backward_pass stage / terminal terms :254-300     dcol_altro_stage_terms()
 *   systems/<sys>.py pose map and d(1-alpha)/dx chain rule     dcol_altro_victim_poses(),
 *     (piano_mover.py:60-61, :83-95; quad :127-128, :159-168)  dcol_altro_constraint_jacobian()
 *
 * Row-major float64 arrays; plain pointers and sizes; no allocation visible to callers.
 * Every entry point returns DCOL_ALTRO_OK or a negative DCOL_ALTRO_ERR_*.
 */
#ifndef DCOL_ALTRO_H
#define DCOL_ALTRO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCOL_ALTRO_ABI_VERSION 2
#define DCOL_ALTRO_MAX_NX 16
#define DCOL_ALTRO_MAX_NU 8

enum dcol_altro_system {
    DCOL_SYS_PIANO = 0,     /* planar rigid body, x = [r(2) v(2) theta omega], u (3)       */
    DCOL_SYS_QUADROTOR = 1, /* x = [r v p(MRP) w] (12), u = rotor speeds (4)                */
    DCOL_SYS_RIGID = 2      /* force/torque-actuated rigid body (coneThroughWall), u (6)    */
};

enum dcol_altro_error {
    DCOL_ALTRO_OK = 0,
    DCOL_ALTRO_ERR_ARG = -1,    /* bad pointer / size / system id                             */
    DCOL_ALTRO_ERR_NOT_PD = -2, /* Quu not positive definite (scipy cho_factor LinAlgError)    */
    DCOL_ALTRO_ERR_DEVICE = -3  /* kernel launch failed (device entry point)                  */
};

/* Physical constants of a model.  Fields a system does not use are ignored. */
typedef struct dcol_altro_model {
    int32_t system; /* enum dcol_altro_system                                                */
    int32_t nx, nu;
    double dt;          /* RK4 step                                                            */
    double mass;        /* QUADROTOR / RIGID                                                   */
    double inertia[9];  /* QUADROTOR / RIGID, row-major 3x3 (solved with partial pivoting)     */
    double gravity[3];  /* QUADROTOR                                                           */
    double arm, kf, km; /* QUADROTOR: arm length L, thrust and torque coefficients             */
    double u_scale;     /* PIANO: angular acceleration = u[2] / u_scale (reference: 100)       */
} dcol_altro_model;

/* Cost and AL data of one trajectory-optimisation problem (ALTRO.py params).  u bounds
 * give the control constraints h_u = [u - u_max, -u + u_min] (2 nu rows per knot). */
typedef struct dcol_altro_problem {
    int32_t N, nx, nu, ncx; /* knots, state / control dims, collision constraints per knot      */
    const double* Q;        /* [nx, nx] stage state weight                                        */
    const double* R;        /* [nu, nu] stage control weight                                      */
    const double* Qf;       /* [nx, nx] terminal weight                                           */
    const double* Xref;     /* [N, nx]                                                            */
    const double* Uref;     /* [N-1, nu]                                                          */
    const double* u_min;    /* [nu]                                                               */
    const double* u_max;    /* [nu]                                                               */
} dcol_altro_problem;

int32_t dcol_altro_abi_version(void);

/* Xn[i] = RK4(X[i], U[i]) for i < M (independent states).  X [M, nx], U [M, nu]. */
int dcol_altro_dynamics(const dcol_altro_model* m, int64_t M, const double* X, const double* U, double* Xn);

/* Forward-difference Jacobians of the discrete dynamics at knots t < T:
 * A[t] = d x_{t+1} / d x_t  [T, nx, nx],  B[t] = d x_{t+1} / d u_t  [T, nx, nu]. */
int dcol_altro_jacobians(const dcol_altro_model* m, int64_t T, const double* X, const double* U, double delta,
                         double* A, double* B);

/* Riccati recursion of the regularised AL-iLQR backward pass for knots T-1 .. 0, from the
 * terminal cost-to-go (VxT [nx], VxxT [nx, nx]).  Per knot: A [nx,nx], B [nx,nu],
 * lx [nx], lu [nu], lxx [nx,nx], luu [nu,nu].  Outputs gains K [T, nu, nx], k [T, nu],
 * the expected decrease sum_t Qu'k in *dJ.  On DCOL_ALTRO_ERR_NOT_PD, *fail_knot = t. */
int dcol_altro_backward(int64_t T, int32_t nx, int32_t nu, const double* A, const double* B, const double* lx,
                        const double* lu, const double* lxx, const double* luu, const double* VxT,
                        const double* VxxT, double reg, double* K, double* k, double* dJ, int64_t* fail_knot);

/* Closed-loop rollout: Un[t] = U[t] - K[t](Xn[t] - X[t]) - a k[t];  Xn[t+1] = RK4(Xn[t], Un[t]),
 * Xn[0] = X[0], t < T.  X [T+1, nx], U [T, nu]. */
int dcol_altro_rollout(const dcol_altro_model* m, int64_t T, const double* X, const double* U, const double* K,
                       const double* k, double a, double* Xn, double* Un);

/* na rollouts of the same gains at step lengths a[0..na) (a batch of line-search trials),
 * one per host thread: Xn [na, T+1, nx], Un [na, T, nu]; each equals dcol_altro_rollout
 * with a[j] bitwise. */
int dcol_altro_rollouts(const dcol_altro_model* m, int64_t T, const double* X, const double* U, const double* K,
                        const double* k, const double* a, int32_t na, double* Xn, double* Un);

/* Augmented-Lagrangian objective of a trajectory (compute_total_cost): stage costs, AL
 * terms of the control bounds and of the collision constraints hx [N, ncx] with duals
 * mu [N-1, 2 nu], mux [N, ncx] (active set: dual > 0 or h > 0), terminal cost and the goal
 * constraint x_N - xref_N with dual lam [nx].  Sums in the reference's order. */
int dcol_altro_cost(const dcol_altro_problem* p, const double* X, const double* U, const double* hx,
                    const double* mu, const double* mux, const double* lam, double rho, double* J);

/* Derivatives of the same objective for the backward pass: per knot t < N-1 lx [nx], lu [nu],
 * lxx [nx, nx], luu [nu, nu] (Gx [N, ncx, nx] = d hx / d x), and the terminal cost-to-go
 * VxT [nx], VxxT [nx, nx]. */
int dcol_altro_stage_terms(const dcol_altro_problem* p, const double* X, const double* U, const double* hx,
                           const double* Gx, const double* mu, const double* mux, const double* lam, double rho,
                           double* lx, double* lu, double* lxx, double* luu, double* VxT, double* VxxT);

/* Victim pose per knot, [N, 6] = (r, p MRP), from the state (system-specific map). */
int dcol_altro_victim_poses(const dcol_altro_model* m, int64_t N, const double* X, double* poses);

/* Fused driver phases (each equals the calls it replaces, in order):
 * backward pass at (X, U) from the constraint batch (alpha [N, ncx]; dalpha [N, ncx, 12] when
 * dalpha_comp_stride is 0, else the engine's component-major layout: component c of pair i
 * at dalpha[c * dalpha_comp_stride + i], e.g. dcol_plan_run's grad[12][B] as it comes back)
 * and the dynamics Jacobians A [N-1, nx, nx], B [N-1, nx, nu]: hx = 1 - alpha,
 * dcol_altro_constraint_jacobian, dcol_altro_stage_terms, dcol_altro_backward (-> K, k,
 * dJ, fail_knot) and dcol_altro_cost of (X, U) (-> J); */
int dcol_altro_backward_pass(const dcol_altro_model* m, const dcol_altro_problem* p, const double* X,
                             const double* U, const double* alpha, const double* dalpha, int64_t dalpha_comp_stride,
                             const double* A, const double* B, const double* mu, const double* mux, const double* lam,
                             double rho, double reg, double* K, double* k, double* dJ, double* J, int64_t* fail_knot);
/* one line-search trial: dcol_altro_rollout at step a, then dcol_altro_victim_poses of the
 * T+1 rolled-out states -> poses [T+1, 6]. */
int dcol_altro_trial(const dcol_altro_model* m, int64_t T, const double* X, const double* U, const double* K,
                     const double* k, double a, double* Xn, double* Un, double* poses);

/* d(1 - alpha)/dx [N, ncx, nx] from d alpha / d[r1, p1, r2, p2] [N, ncx, 12] (chain rule
 * through the pose map; the victim is primitive 1). */
int dcol_altro_constraint_jacobian(const dcol_altro_model* m, int64_t N, int32_t ncx, const double* X,
                                   const double* dalpha, double* Gx);

#ifdef __cplusplus
}
#endif

#endif /* DCOL_ALTRO_H */
