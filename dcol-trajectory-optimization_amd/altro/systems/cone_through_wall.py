"""Cone through wall: a solid cone (H = 2, half-angle 22 deg) flown through a square hole
formed by four slabs, N = 60 knots (reference systems/cone_through_wall.py:202-330).

State x = [r, v, p (MRP), omega] (12), control u = [force (3), torque (3)] on a rigid body
with the cone's own mass properties (primitives/mass_properties.py:3-31, density 1)."""
from __future__ import annotations

import math
import sys

import numpy as np

from primitives.misc_primitive_constructor import ConeMRP, create_rect_prism

from .. import _native
from . import _common


def mass_properties(cone, rho=1):
    """(mass, inertia) of a solid cone about its centre of mass (mass_properties.py:3-31)."""
    r = np.tan(cone.beta) * cone.H
    m = (1 / 3) * (np.pi * (r ** 2) * cone.H) * rho
    iyy = m * ((3 / 20) * r ** 2 + (3 / 80) * cone.H ** 2)
    return m, np.diag([0.3 * m * r ** 2, iyy, iyy])


def mrp_from_q(q):
    return np.array(q[1:4]) / (1 + q[0])


def native_model(params):
    m = params.get("_native_model")
    if m is None:
        m = _native.make_model(_native.SYS_RIGID, params["nx"], params["nu"], params["dt"], mass=params["m"],
                               inertia=params["J"])
        params["_native_model"] = m
    return m


victim_poses = _common.rigid_victim_poses
state_jacobian = _common.rigid_state_jacobian


def initialize():
    """-> (params, X, U) of the cone-through-wall problem."""
    nx, nu, N, dt = 12, 6, 60, 0.1
    x0 = np.array([-4, -7, 9, 0.0, 0.0, 0.0, 0, 0, 0, 0, 0, 0])
    xg = np.array([-4.5, 7, 3, 0, 0, 0.0, 0.0, 0.0, 0.0, 0, 0, 0])
    P_vic = ConeMRP(height=2.0, beta=math.radians(22))
    mass, inertia = mass_properties(P_vic)
    P_obs = [create_rect_prism(10.0, 10.0, 1.0), create_rect_prism(10.0, 10.0, 1.0),
             create_rect_prism(4.1, 4.1, 1.1), create_rect_prism(4.1, 4.1, 1.1)]
    tilt = mrp_from_q([np.cos(np.pi / 4), np.sin(np.pi / 4), 0, 0])
    for o, r in zip(P_obs, ([-6, 0, 5.0], [6, 0, 5.0], [0, 0, 2.05], [0, 0, 7.96])):
        o.r, o.p = np.array(r), tilt
    params = dict(nx=nx, nu=nu, ncx=len(P_obs), ncu=2 * nu, N=N, Q=np.diag(np.ones(nx)),
                  R=np.diag([1., 1., 1., 100., 100., 100.]), Qf=np.diag(np.ones(nx)), u_min=-20 * np.ones(nu),
                  u_max=20 * np.ones(nu), x_min=-20 * np.ones(nx), x_max=20 * np.ones(nx),
                  Xref=_common.linear_interp(dt, x0, xg, N), Uref=[np.zeros(nu) for _ in range(N - 1)], dt=dt,
                  m=mass, J=inertia, P_obs=P_obs, P_vic=P_vic, max_linesearch_iters=20, atol=1e-1, max_iters=3000,
                  reg_min=1e-6, reg=1e-6, reg_max=1e2, rho=1e0, phi=10.0, convio_tol=1e-4, system="coneThroughWall",
                  X_hist=[], U_hist=[], hx_hist=[], hu_hist=[])
    X = [x0.copy() for _ in range(N)]
    rs = np.random.RandomState(2)      # reference: np.random.seed(2); 0.01 * randn(nu) per knot
    U = [0.01 * rs.randn(nu) for _ in range(N - 1)]
    params["X_hist"].append(X)
    params["U_hist"].append(U)
    return params, X, U


initialize_coneThroughWall = initialize

(discrete_dynamics, inequality_constraints_x, inequality_constraints_x_grad, inequality_constraints_u,
 inequality_constraints_u_grad) = _common.per_knot(sys.modules[__name__])
