"""TEST INFRASTRUCTURE: a CPU constraint evaluator for the batched ALTRO driver, backed by
the C oracle (oracle/dcol_oracle.c, OpenMP).  Same interface as altro.constraints.
ObstacleField, so the driver's host logic runs on the CPU-only container; the GPU tests use
the real ObstacleField."""
import os

import numpy as np

from dcol_amd import _lib
from dcol_amd.engine import raise_for_status
from dcol_amd.shapes import pose_of, spec_from_object
from oracle import c_oracle


def specs_to_tab(specs):
    """ShapeSpec list -> shape table in the tests/golden array layout."""
    S = len(specs)
    tab = dict(type=np.zeros(S, np.int32), nh=np.zeros(S, np.int32), A_off=np.zeros(S, np.int32),
               params=np.zeros((S, 4)), r_offset=np.zeros((S, 3)), Q_offset=np.zeros((S, 3, 3)))
    A_rows, b_rows = [], []
    for i, s in enumerate(specs):
        tab["type"][i], tab["nh"][i], tab["A_off"][i] = s.type, s.nh, len(b_rows)
        tab["params"][i] = (s.R, s.L, s.H, s.beta)
        tab["r_offset"][i] = s.r_offset
        tab["Q_offset"][i] = np.array(s.Q_offset).reshape(3, 3)
        if s.nh:
            w = 2 if s.type == _lib.POLYGON else 3
            A = np.array(s.A).reshape(s.nh, w)
            for r in range(s.nh):
                A_rows.append(list(A[r]) + [0.0] * (3 - w))
            b_rows += list(s.b)
    tab["A_pool"] = np.array(A_rows, dtype=np.float64).reshape(-1, 3)
    tab["b_pool"] = np.array(b_rows, dtype=np.float64)
    return tab


class OracleField:
    """(knot x obstacle) constraint batches solved by the C oracle."""

    def __init__(self, victim, obstacles, N, tol=1e-6, threads=None):
        self.N, self.n_obs = int(N), len(obstacles)
        self.tab = specs_to_tab([spec_from_object(victim)] + [spec_from_object(o) for o in obstacles])
        self.s1 = np.zeros(self.N * self.n_obs, np.int32)
        self.s2 = np.tile(np.arange(1, self.n_obs + 1, dtype=np.int32), self.N)
        self.pose2 = np.tile(np.array([pose_of(o) for o in obstacles]).reshape(self.n_obs, 6), (self.N, 1))
        self.tol = tol
        self.threads = threads or min(8, os.cpu_count() or 1)

    def _solve(self, p1, grad):
        return c_oracle.run_batch(self.tab, self.s1, self.s2, p1, self.pose2, tol=self.tol, want_grad=grad,
                                  threads=self.threads)

    def evaluate(self, victim_poses, grad, raise_=True):
        """-> (alpha, J), or (alpha, J, status) with raise_=False (ObstacleField.collect)."""
        p1 = np.repeat(np.asarray(victim_poses, dtype=np.float64).reshape(self.N, 6), self.n_obs, axis=0)
        out = self._solve(p1, grad)
        st = out["status"]
        if raise_ and st.any():
            raise_for_status(int(st[np.flatnonzero(st)[0]]))
        alpha = out["alpha"].reshape(self.N, self.n_obs)
        J = out["grad"].reshape(self.N, self.n_obs, 12) if grad else None
        if not raise_:
            return alpha, J, np.asarray(st).reshape(self.N, self.n_obs)
        return alpha, J


class NumpyOracleField(OracleField):
    """Same, solved by the NumPy restatement (bit-exact with the reference; slow)."""

    def _solve(self, p1, grad):
        from oracle import dcol_oracle
        return dcol_oracle.run_batch(self.tab, self.s1, self.s2, p1, self.pose2, tol=self.tol, want_grad=grad)
