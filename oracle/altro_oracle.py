"""TEST INFRASTRUCTURE ONLY — NumPy restatement of the reference's ALTRO host math, per knot.

Used by tests/test_altro.py as the checker of the native host library
(lib/libdcol_altro.so, include/dcol_altro.h).  Each function follows the reference
expression by expression:

  dynamics_piano      systems/piano_mover.py:7-25
  dynamics_quadrotor  systems/cluttered_hallway_quadrotor.py:19-84
  dynamics_rigid      systems/cone_through_wall.py:19-64
  rk4                 discrete_dynamics, piano_mover.py:28-47 (same in the 3-D systems)
  fd_jacobian         ALTRO.py:77-100 compute_jacobian (delta 1e-6)
  riccati             ALTRO.py:304-336 (scipy cho_factor / cho_solve)
  rollout             ALTRO.py:214-217

Whole-run parity of the driver is pinned by tests/golden/altro_*.npz, recorded from the
reference itself (tests/golden/gen_altro.py).
"""
import numpy as np
from scipy.linalg import cho_factor, cho_solve


def _skew(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


def _dcm(p):
    p1, p2, p3 = p
    q1, q2, q3 = p1 ** 2, p2 ** 2, p3 ** 2
    den = (q1 + q2 + q3 + 1) ** 2
    a = 4 * q1 + 4 * q2 + 4 * q3 - 4
    d = lambda u, v: -((8 * u + 8 * v) / den - 1) * den  # noqa: E731
    return np.array([[d(q2, q3), 8 * p1 * p2 + p3 * a, 8 * p1 * p3 - p2 * a],
                     [8 * p1 * p2 - p3 * a, d(q1, q3), 8 * p2 * p3 + p1 * a],
                     [8 * p1 * p3 + p2 * a, 8 * p2 * p3 - p1 * a, d(q1, q2)]]) / den


def dynamics_piano(x, u):
    return np.concatenate([x[2:4], u[:2], [x[5]], [u[2] / 100]])


def dynamics_quadrotor(x, u, mass=0.5, J=np.diag([0.0023, 0.0023, 0.004]), g=np.array([0, 0, -9.81]), L=0.175,
                       kf=1.0, km=0.0245):
    p, w = x[6:9], x[9:12]
    Q = _dcm(p)
    F = [max(0, kf * wi) for wi in u]
    M = [km * wi for wi in u]
    Fb = np.array([0., 0., F[0] + F[1] + F[2] + F[3]])
    tau = np.array([L * (F[1] - F[3]), L * (F[2] - F[0]), (M[0] - M[1] + M[2] - M[3])])
    f_world = mass * g + Q @ Fb
    n2 = np.dot(p, p)
    S = _skew(p)
    pk = ((1 + n2) / 4) * (np.eye(3) + 2 * (np.dot(S, S) + S) / (1 + n2))
    wd = np.linalg.solve(J, tau - np.cross(w, J @ w))
    return np.concatenate([x[3:6], f_world / mass, np.dot(pk, w), wd])


def dynamics_rigid(x, u, mass, J):
    p, w = x[6:9], x[9:12]
    n = np.linalg.norm(p)
    S = _skew(p)
    pd = ((1 + n ** 2) / 4) * (np.eye(3) + 2 * (np.dot(S, S) + S) / (1 + n ** 2)).dot(w)
    wd = np.linalg.solve(J, u[3:6] - np.cross(w, J @ w))
    return np.concatenate([x[3:6], u[:3] / mass, pd, wd])


def rk4(f, x, u, dt):
    k1 = dt * f(x, u)
    k2 = dt * f(x + 0.5 * k1, u)
    k3 = dt * f(x + 0.5 * k2, u)
    k4 = dt * f(x + k3, u)
    return x + (1 / 6) * (k1 + 2 * k2 + 2 * k3 + k4)


def fd_jacobian(fn, v, delta=1e-6):
    y0 = fn(v)
    Jm = np.zeros((len(y0), len(v)))
    for i in range(len(v)):
        vp = v.copy()
        vp[i] += delta
        Jm[:, i] = (fn(vp) - y0) / delta
    return Jm


def riccati(A, B, lx, lu, lxx, luu, VxT, VxxT, reg):
    """Backward recursion over knots T-1..0 -> (K [T,nu,nx], k [T,nu], dJ)."""
    T, nx = len(A), len(VxT)
    Vx, Vxx = VxT.copy(), VxxT.copy()
    Ks, ks, dJ = [None] * T, [None] * T, 0.0
    for t in range(T - 1, -1, -1):
        At, Bt = A[t], B[t]
        P = Vxx + reg * np.eye(nx)
        Qu = lu[t] + Bt.T @ Vx
        Quu = luu[t] + Bt.T @ P @ Bt
        Qux = Bt.T @ P @ At
        c = cho_factor(Quu)
        k = cho_solve(c, Qu)
        K = cho_solve(c, Qux)
        Acl = At - Bt @ K
        Vxx_n = lxx[t] + K.T @ luu[t] @ K + Acl.T @ Vxx @ Acl
        Vx_n = lx[t] - K.T @ lu[t] + K.T @ luu[t] @ k + Acl.T @ (Vx - Vxx @ Bt @ k)
        Vx, Vxx = Vx_n, Vxx_n
        dJ += Qu.T @ k
        Ks[t], ks[t] = K, k
    return np.array(Ks), np.array(ks), dJ


def rollout(step, X, U, K, k, a):
    Xn, Un = X.copy(), U.copy()
    for t in range(len(U)):
        Un[t] = U[t] - K[t] @ (Xn[t] - X[t]) - a * k[t]
        Xn[t + 1] = step(Xn[t], Un[t])
    return Xn, Un
