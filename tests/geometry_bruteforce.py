"""TEST INFRASTRUCTURE: minimum uniform scaling alpha of two primitives by brute-force
geometry, independent of the conic formulation — the checker of the case-4 extension
(DCOL_PLAN_CASE4), for which the reference has no answer (it raises,
combine_problem_matrices.py:58-67).

Each primitive is described by its geometric meaning (the sets the reference's conic
blocks encode, problem_matrices.py:4-120), with y = p - r_eff and body axes Qe:

  capsule   {y : dist(y, segment t * bx, |t| <= a L / 2) <= a R}
  cylinder  {y : |bx . y| <= a L / 2,  |y - (bx . y) bx| <= a R}
  polygon   {y : y = Qe[:, :2] u + w,  A u <= a b,  |w| <= a R}

Its gauge g(y) = min {a : y in a * shape} is computed in closed form (cylinder) or by
bisection of a monotone residual (capsule, polygon), and

  alpha* = min over p of max(g1(p - r1_eff), g2(p - r2_eff))

is minimised directly over the point p (convex, derivative-free, several starts).
"""
import numpy as np
from scipy.optimize import minimize
from scipy.spatial import ConvexHull, HalfspaceIntersection

CAPSULE, CYLINDER, POLYGON = 3, 4, 5


def _dcm(p):
    p1, p2, p3 = p
    q = p1 * p1 + p2 * p2 + p3 * p3
    S = np.array([[0, -p3, p2], [p3, 0, -p1], [-p2, p1, 0]])
    return np.eye(3) + (8 * S @ S + 4 * (1 - q) * S) / (1 + q) ** 2


def _bisect(phi, lo, hi, iters=80):
    """Smallest a in [lo, hi] with phi(a) <= 0 for a non-increasing phi."""
    if phi(lo) <= 0:
        return lo
    for _ in range(iters):
        mid = 0.5 * (lo + hi)
        if phi(mid) <= 0:
            hi = mid
        else:
            lo = mid
        if hi - lo <= 1e-14 * max(1.0, hi):
            break
    return hi


class Body:
    def __init__(self, kind, pose, R=0.0, L=0.0, A=None, b=None, r_offset=np.zeros(3), Q_offset=np.eye(3)):
        r, p = np.asarray(pose[:3], float), np.asarray(pose[3:], float)
        Q = _dcm(p)
        self.kind, self.R, self.L = kind, float(R), float(L)
        self.re = r + Q @ np.asarray(r_offset, float)
        self.Qe = Q @ np.asarray(Q_offset, float)
        self.bx = self.Qe[:, 0]
        if kind == POLYGON:
            A = np.asarray(A, float)
            b = np.asarray(b, float)
            self.A, self.b = A, b
            hs = HalfspaceIntersection(np.hstack([A, -b[:, None]]), np.zeros(2))
            V = hs.intersections
            self.V = V[ConvexHull(V).vertices]          # counter-clockwise polygon

    def _poly_dist(self, u, a):
        """distance from 2-D point u to the polygon a * P."""
        if np.all(self.A @ u <= a * self.b):
            return 0.0
        if a <= 0.0:
            return float(np.hypot(u[0], u[1]))
        P0 = a * self.V
        D = np.roll(P0, -1, axis=0) - P0
        t = np.clip(np.einsum("ij,ij->i", u - P0, D) / np.einsum("ij,ij->i", D, D), 0.0, 1.0)
        E = u - (P0 + t[:, None] * D)
        return float(np.sqrt(np.min(np.einsum("ij,ij->i", E, E))))

    def gauge(self, p):
        y = np.asarray(p, float) - self.re
        if self.kind == CYLINDER:
            ax = np.dot(self.bx, y)
            rho = np.linalg.norm(y - ax * self.bx)
            return max(abs(ax) / (self.L / 2), rho / self.R)
        if self.kind == CAPSULE:
            ax = np.dot(self.bx, y)
            rho = np.linalg.norm(y - ax * self.bx)
            phi = lambda a: np.hypot(rho, max(0.0, abs(ax) - a * self.L / 2)) - a * self.R  # noqa: E731
            return _bisect(phi, 0.0, max(2 * abs(ax) / self.L, rho / self.R) + 1e-300)
        if self.kind == POLYGON:
            u = self.Qe[:, :2].T @ y
            n = np.dot(self.Qe[:, 2], y)
            hi = max(float(np.max(self.A @ u / self.b)), abs(n) / self.R, 0.0) + 1e-300
            phi = lambda a: np.hypot(n, self._poly_dist(u, a)) - a * self.R  # noqa: E731
            return _bisect(phi, 0.0, hi)
        raise ValueError(self.kind)


def min_scaling(b1, b2, starts=()):
    """alpha* = min_p max(g1, g2) by derivative-free search from several starts."""
    F = lambda p: max(b1.gauge(p), b2.gauge(p))  # noqa: E731
    x0s = [0.5 * (b1.re + b2.re)] + [np.asarray(s, float) for s in starts]
    best = (np.inf, None)
    for x0 in x0s:
        r = minimize(F, x0, method="Powell", options=dict(xtol=1e-10, ftol=1e-14, maxiter=4000))
        r = minimize(F, r.x, method="Nelder-Mead", options=dict(xatol=1e-11, fatol=1e-14, maxiter=4000))
        if r.fun < best[0]:
            best = (float(r.fun), r.x)
    return best
