"""MRP -> direction-cosine matrix (primitives/problem_matrices.py:213-251).

Provided because the quadrotor dynamics import it (cluttered_hallway_quadrotor.py:7,
:38).  It is NOT used by the proximity path: the conic assembly (problem_matrices()) runs
inside the HIP kernel (csrc/dcol_device.hpp, make_frame / Solver::assemble).
"""
import numpy as np


def dcm_from_mrp(p):
    """Rotation matrix of the modified Rodrigues parameters p (same expanded expression
    as the reference, so results agree bitwise)."""
    p1, p2, p3 = p
    q1, q2, q3 = p1 ** 2, p2 ** 2, p3 ** 2
    den = (q1 + q2 + q3 + 1) ** 2
    a = 4 * q1 + 4 * q2 + 4 * q3 - 4
    diag = lambda u, v: -((8 * u + 8 * v) / den - 1) * den  # noqa: E731
    return np.array([
        [diag(q2, q3), 8 * p1 * p2 + p3 * a, 8 * p1 * p3 - p2 * a],
        [8 * p1 * p2 - p3 * a, diag(q1, q3), 8 * p2 * p3 + p1 * a],
        [8 * p1 * p3 + p2 * a, 8 * p2 * p3 - p1 * a, diag(q1, q2)],
    ]) / den
