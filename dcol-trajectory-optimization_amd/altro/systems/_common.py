"""Pieces shared by the three systems.

Each system module offers two faces:
  * the batched interface the driver uses — ``native_model(params)`` (dcol_altro_model),
    ``victim_poses(params, X)`` -> [N, 6] and ``state_jacobian(params, X, J)`` mapping the
    proximity gradient d alpha / d[r1, p1, r2, p2] [N, n_obs, 12] to d h / d x [N, n_obs, nx];
  * the reference's per-knot functions (discrete_dynamics, inequality_constraints_x[_grad],
    inequality_constraints_u[_grad]) with the same signatures, so the reference's own
    ALTRO.py can run on these modules unchanged (they call the GPU through the drop-in
    ``proximity`` package).
"""
from __future__ import annotations

import numpy as np

from proximity.proximity import proximity_mrp
from proximity.proximity_gradient import proximity_gradient

from .. import _native


def control_bounds(params, u):
    """[u - u_max, -u + u_min] (piano_mover.py:99-113 and the 3-D systems)."""
    return np.concatenate([u - params["u_max"], -u + params["u_min"]])


def control_bounds_grad(params, u):
    nu = params["nu"]
    return np.vstack([np.eye(nu), -np.eye(nu)])


def discrete_dynamics(module, params, x, u, k):
    """One RK4 step through the native library (same arithmetic as the batched driver)."""
    return _native.dynamics(module.native_model(params), np.asarray(x, dtype=np.float64)[None],
                            np.asarray(u, dtype=np.float64)[None])[0]


def _set_pose(params, pose):
    params["P_vic"].r = np.array(pose[:3])
    params["P_vic"].p = np.array(pose[3:6])


def collision_constraints(module, params, x):
    """1 - alpha per obstacle at one state (reference per-knot form)."""
    _set_pose(params, module.victim_poses(params, np.asarray(x, dtype=np.float64)[None])[0])
    return np.array([1 - proximity_mrp(params["P_vic"], o, verbose=False)[0] for o in params["P_obs"]])


def collision_constraints_grad(module, params, x):
    x = np.asarray(x, dtype=np.float64)
    _set_pose(params, module.victim_poses(params, x[None])[0])
    J = np.array([proximity_gradient(params["P_vic"], o)[1] for o in params["P_obs"]])
    return module.state_jacobian(params, x[None], J[None])[0]


def per_knot(module):
    """The reference's per-knot system functions, bound to `module`."""
    def discrete_dynamics_(params, x, u, k):
        return discrete_dynamics(module, params, x, u, k)

    def inequality_constraints_x(params, x):
        return collision_constraints(module, params, x)

    def inequality_constraints_x_grad(params, x):
        return collision_constraints_grad(module, params, x)

    return (discrete_dynamics_, inequality_constraints_x, inequality_constraints_x_grad, control_bounds,
            control_bounds_grad)


def linear_interp(dt, x0, xg, N):
    """Reference trajectory of the 3-D systems (cluttered_hallway_quadrotor.py:196-231,
    cone_through_wall.py:169-200): positions and MRPs interpolated linearly; the velocity
    slot holds the ATTITUDE increment / ((N-1) dt) — the reference reuses delta_p after
    reassigning it to the attitude difference, and that is kept here."""
    dpos = xg[0:3] - x0[0:3]
    datt = xg[6:9] - x0[6:9]
    i = np.arange(N, dtype=np.float64)[:, None]
    pos = i * (dpos / (N - 1)) + x0[0:3]
    att = i * (datt / (N - 1)) + x0[6:9]
    vel = datt / ((N - 1) * dt)
    return [np.concatenate([pos[j], vel, att[j], np.zeros(3)]) for j in range(N)]


def rigid_victim_poses(params, X):
    """(r, p) = (x[0:3], x[6:9]) for the 3-D systems."""
    X = np.asarray(X, dtype=np.float64)
    return np.concatenate([X[:, 0:3], X[:, 6:9]], axis=1)


def rigid_state_jacobian(params, X, J):
    """[-dα/dr1, 0, -dα/dp1, 0] per obstacle (cluttered_hallway_quadrotor.py:159-168)."""
    D = np.zeros(J.shape[:2] + (12,))
    D[..., 0:3] = -J[..., 0:3]
    D[..., 6:9] = -J[..., 3:6]
    return D
