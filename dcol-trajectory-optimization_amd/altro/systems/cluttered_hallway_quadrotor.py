"""Cluttered-hallway quadrotor: a sphere (R = 0.25) flown through nine mixed obstacles
between a floor and a ceiling slab, N = 100 knots (reference
systems/cluttered_hallway_quadrotor.py:233-387).

State x = [r, v, p (MRP), omega] (12), control u = four rotor speeds."""
from __future__ import annotations

import sys

import numpy as np

from primitives.misc_primitive_constructor import (CapsuleMRP, ConeMRP, CylinderMRP, PolygonMRP, PolytopeMRP,
                                                   SphereMRP, create_n_sided, create_rect_prism)

from .. import _native
from . import _common, _data

MASS = 0.5
INERTIA = np.diag([0.0023, 0.0023, 0.004])
GRAVITY = (0.0, 0.0, -9.81)
ARM, KF, KM = 0.1750, 1.0, 0.0245

# Obstacle poses the reference hard-codes from the original Julia run (seed 2),
# cluttered_hallway_quadrotor.py:318-335: (r, p) per obstacle 0..8.
_POSES = [
    ([-5.0, -0.3597289068234817, 4.087208492428585], [0.9743462834661368, 0.5695654691654629, -0.929297065594203]),
    ([-3.75, 2.0547630560640364, 3.3248927294469155], [0.44432216225861665, -0.8131633664490159, 0.8533462452863487]),
    ([-2.5, 0.01357380155160959, 3.1056516058837307], [-0.7818142467739891, -1.0606493186561021, -0.6997594248738506]),
    ([-1.25, 0.1520302408349855, 2.100626290031169], [0.09970204047057568, -0.6590733218999884, 0.10747184882042882]),
    ([0.0, 0.27038613194550204, 4.579317307027433], [-1.178486073522902, -0.5852806292416908, -0.5104503832374265]),
    ([1.25, -0.20563037602802728, 3.7707031750912097], [1.322242556684692, 1.477962368008582, -0.09186250030835676]),
    ([2.5, 1.724189934074888, 3.1527083547286816], [-1.670756785490579, -1.6504683581003534, 0.9958143390876766]),
    ([3.75, -0.7885513165549604, 2.3533371368422706], [0.40980738483268503, 0.5108420391824778, 0.42272633604120335]),
    ([5.0, 0.32074771862886275, 4.251199978479224], [1.8822143307659809, -0.7779808480817001, 0.8308676764061569]),
]


def native_model(params):
    m = params.get("_native_model")
    if m is None:
        m = _native.make_model(_native.SYS_QUADROTOR, params["nx"], params["nu"], params["dt"], mass=MASS,
                               inertia=INERTIA, gravity=GRAVITY, arm=ARM, kf=KF, km=KM)
        params["_native_model"] = m
    return m


victim_poses = _common.rigid_victim_poses
state_jacobian = _common.rigid_state_jacobian


def obstacles(jld2_path=None):
    """The reference's eleven obstacles; the 8-face polytope comes from polytopes.jld2
    (read with altro.systems.jld2 when a path is given, else the decoded copy shipped in
    altro/data)."""
    if jld2_path is not None:
        from . import jld2
        d = {f"jld2_{k}": v for k, v in jld2.read(jld2_path, ["A2", "b2"]).items()}
    else:
        d = _data.load()
    poly = create_n_sided(5, 0.6)
    floor = create_rect_prism(length=20, width=5, height=0.2)
    floor.r = [0, 0, 0.9]
    ceiling = create_rect_prism(length=20, width=5, height=0.2)
    ceiling.r = [0, 0, 6.0]
    obs = [CylinderMRP(radius=0.6, height=3.0), CapsuleMRP(radius=0.2, height=5.0), SphereMRP(radius=0.8),
           ConeMRP(height=2.0, beta=np.deg2rad(22)), PolytopeMRP(d["jld2_A2"].T, d["jld2_b2"]),
           PolygonMRP(poly["A"], poly["b"], 0.2), CylinderMRP(radius=1.1, height=2.3),
           CapsuleMRP(radius=0.8, height=1.0), SphereMRP(radius=0.5), floor, ceiling]
    for o, (r, p) in zip(obs, _POSES):
        o.r, o.p = r, p
    return obs


def initialize(jld2_path=None):
    """-> (params, X, U) of the quadrotor problem."""
    nx, nu, N, dt = 12, 4, 100, 0.08
    x0 = np.array([-8, 0, 4, 0, 0, 0.0, 0, 0, 0, 0, 0, 0])
    xg = np.array([8, 0, 4, 0, 0, 0.0, 0, 0, 0, 0, 0, 0])
    P_obs = obstacles(jld2_path)
    params = dict(nx=nx, nu=nu, ncx=len(P_obs), ncu=2 * nu, N=N, Q=np.diag(np.ones(nx)), R=np.diag(np.ones(nu)),
                  Qf=np.diag(np.ones(nx)), u_min=-2000 * np.ones(nu), u_max=2000 * np.ones(nu),
                  Xref=_common.linear_interp(dt, x0, xg, N), Uref=[(9.81 * 0.5 / 4) * np.ones(nu) for _ in range(N)],
                  dt=dt, P_obs=P_obs, P_vic=SphereMRP(radius=0.25), max_linesearch_iters=20, atol=1e-2,
                  max_iters=3000, reg_min=1e-6, reg=1e-6, reg_max=1e2, rho=1e0, phi=10.0, convio_tol=1e-4,
                  system="quadrotor", X_hist=[], U_hist=[], hx_hist=[], hu_hist=[])
    X = [x0.copy() for _ in range(N)]
    U = _data.load()["quadrotor_U"].copy()
    params["X_hist"].append(X)
    params["U_hist"].append(U)
    return params, X, U


initialize_quadrotor = initialize

(discrete_dynamics, inequality_constraints_x, inequality_constraints_x_grad, inequality_constraints_u,
 inequality_constraints_u_grad) = _common.per_knot(sys.modules[__name__])
