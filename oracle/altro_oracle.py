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


def _mask(dual, h):
    return np.diag([(d > 0 or v > 0) for d, v in zip(dual, h)]).astype(float)   # ALTRO.py:16-31


def al_cost(Q, R, Qf, Xref, Uref, u_min, u_max, X, U, hx, mu, mux, lam, rho):
    """compute_total_cost, ALTRO.py:103-145 (per knot, the reference's accumulation order)."""
    N = len(X)
    cost = 0.0
    for t in range(N - 1):
        dx, du = X[t] - Xref[t], U[t] - Uref[t]
        cost += 0.5 * dx.T @ Q @ dx + 0.5 * du.T @ R @ du
        hu = np.concatenate([U[t] - u_max, -U[t] + u_min])
        cost += np.dot(mu[t], hu) + 0.5 * rho * hu.T @ _mask(mu[t], hu) @ hu
        cost += np.dot(mux[t], hx[t]) + 0.5 * rho * hx[t].T @ _mask(mux[t], hx[t]) @ hx[t]
    dx = X[-1] - Xref[-1]
    cost += 0.5 * dx.T @ Qf @ dx
    cost += np.dot(mux[-1], hx[-1]) + 0.5 * rho * hx[-1].T @ _mask(mux[-1], hx[-1]) @ hx[-1]
    cost += np.dot(lam, dx) + 0.5 * rho * dx.T @ dx
    return cost


def stage_terms(Q, R, Qf, Xref, Uref, u_min, u_max, X, U, hx, Gx, mu, mux, lam, rho):
    """Cost derivatives of backward_pass, ALTRO.py:254-300 -> (lx, lu, lxx, luu, VxT, VxxT)."""
    N, nu = len(X), U.shape[1]
    Gu = np.vstack([np.eye(nu), -np.eye(nu)])
    lx, lu, lxx, luu = [], [], [], []
    for t in range(N - 1):
        hu = np.concatenate([U[t] - u_max, -U[t] + u_min])
        mu_m, mx_m = _mask(mu[t], hu), _mask(mux[t], hx[t])
        lx.append(Q @ (X[t] - Xref[t]) + Gx[t].T @ (mux[t] + rho * (mx_m @ hx[t])))
        lu.append(R @ (U[t] - Uref[t]) + Gu.T @ (mu[t] + rho * (mu_m @ hu)))
        lxx.append(Q + rho * Gx[t].T @ mx_m @ Gx[t])
        luu.append(R + rho * Gu.T @ mu_m @ Gu)
    g = X[-1] - Xref[-1]
    m = _mask(mux[-1], hx[-1])
    VxT = Qf @ g + Gx[-1].T @ (mux[-1] + rho * (m @ hx[-1])) + (lam + rho * g)
    VxxT = Qf + rho * Gx[-1].T @ m @ Gx[-1] + rho * np.eye(len(g))
    return np.array(lx), np.array(lu), np.array(lxx), np.array(luu), VxT, VxxT


def victim_poses_piano(X):
    """piano_mover.py:60-61: r = (x0, x1, 0), p = (0, 0, 1) tan(theta / 4)."""
    return np.array([np.concatenate([[x[0], x[1], 0.0], np.array([0, 0, 1]) * np.tan(x[4] / 4)]) for x in X])


def constraint_jacobian_piano(X, J):
    """piano_mover.py:83-95 chain rule -> d(1 - alpha)/dx [N, ncx, 6]."""
    out = []
    for x, Jt in zip(X, J):
        dp = np.array([0, 0, 1]) * (1 / (4 * np.cos(x[4] / 4) ** 2))
        out.append([np.concatenate([-j[:2], [0, 0], [-np.dot(j[3:6], dp)], [0]]) for j in Jt])
    return np.array(out)


def constraint_jacobian_rigid(J):
    """cluttered_hallway_quadrotor.py:159-168 / cone_through_wall.py:157-166."""
    return np.array([[np.concatenate([-j[:3], np.zeros(3), -j[3:6], np.zeros(3)]) for j in Jt] for Jt in J])
