"""Piano mover: a thin rectangular plate (2.5 x 0.15 x 0.01) moved through a corner
between three rectangular walls, N = 80 knots (reference systems/piano_mover.py:137-228).

State x = [rx, ry, vx, vy, theta, omega], control u = [ax, ay, tau]; the plate's attitude
is the planar rotation theta about z, as MRP p = [0, 0, tan(theta / 4)]."""
from __future__ import annotations

import sys

import numpy as np

from primitives.misc_primitive_constructor import create_rect_prism

from .. import _native
from . import _common, _data

U_SCALE = 100.0    # angular acceleration = tau / 100 (piano_mover.py:25)


def native_model(params):
    m = params.get("_native_model")
    if m is None:
        m = _native.make_model(_native.SYS_PIANO, params["nx"], params["nu"], params["dt"], u_scale=U_SCALE)
        params["_native_model"] = m
    return m


def victim_poses(params, X):
    """[N, 6] victim (r, p): r = (rx, ry, 0), p = (0, 0, 1) * tan(theta / 4) (piano_mover.py:60-61)."""
    X = np.asarray(X, dtype=np.float64)
    P = np.zeros((X.shape[0], 6))
    P[:, 0:2] = X[:, 0:2]
    P[:, 3:6] = np.array([0, 0, 1]) * np.tan(X[:, 4] / 4)[:, None]
    return P


def state_jacobian(params, X, J):
    """d(1 - alpha)/dx from d alpha/d[r1, p1, ...]: r chains through (rx, ry), p through
    dp/dtheta = (0, 0, 1) / (4 cos^2(theta / 4)) (piano_mover.py:83-95)."""
    X = np.asarray(X, dtype=np.float64)
    dp = np.array([0, 0, 1]) * (1 / (4 * np.cos(X[:, 4] / 4) ** 2))[:, None]        # [N, 3]
    D = np.zeros(J.shape[:2] + (6,))
    D[..., 0:2] = -J[..., 0:2]
    D[..., 4] = -(J[..., 3] * dp[:, None, 0] + J[..., 4] * dp[:, None, 1] + J[..., 5] * dp[:, None, 2])
    return D


def initialize():
    """-> (params, X, U) of the piano mover (piano_mover.py:137-228)."""
    nx, nu, N = 6, 3, 80
    x0 = np.array([1.5, 1.5, 0, 0, 0, 0])
    xg = np.array([3.5, 3.7, 0, 0, np.deg2rad(90), 0])
    P_vic = create_rect_prism(2.5, 0.15, 0.01)
    P_obs = [create_rect_prism(3.0, 3.0, 1.0), create_rect_prism(4.0, 1.0, 1.0), create_rect_prism(1.0, 5.0, 1.1)]
    for o, r in zip(P_obs, ([1.5, 3.5, 0.0], [2, 0.5, 0], [4.5, 2.5, 0])):
        o.r = r
    params = dict(nx=nx, nu=nu, ncx=len(P_obs), ncu=2 * nu, N=N, Q=np.diag(np.ones(nx)), R=np.diag([1, 1, 0.001]),
                  Qf=np.diag(np.ones(nx)), u_min=-200 * np.ones(nu), u_max=200 * np.ones(nu),
                  x_min=-200 * np.ones(nx), x_max=200 * np.ones(nx), Xref=[np.copy(xg) for _ in range(N)],
                  Uref=[np.zeros(nu) for _ in range(N - 1)], dt=0.1, P_obs=P_obs, P_vic=P_vic,
                  max_linesearch_iters=20, atol=4e-2, max_iters=3000, X_hist=[], U_hist=[], hx_hist=[], hu_hist=[],
                  reg_min=1e-6, reg=1e-6, reg_max=1e2, rho=1e0, phi=10.0, convio_tol=1e-4, system="piano_mover")
    X = [np.copy(x0) for _ in range(N)]
    U = _data.load()["piano_mover_U"].copy()
    params["X_hist"].append(X)
    params["U_hist"].append(U)
    return params, X, U


initialize_piano_mover = initialize


# ----------------------------------------------------- reference per-knot interface
(discrete_dynamics, inequality_constraints_x, inequality_constraints_x_grad, inequality_constraints_u,
 inequality_constraints_u_grad) = _common.per_knot(sys.modules[__name__])
