"""Seeded random BOX-detector shapes (test infrastructure): 6-row polytopes whose rows 3..5
are the exact negatives of rows 0..2 (DevShape::boxp, dcol_host.hpp digest_shape), which the
engine solves with the axis-pair rows of Solver<..., BOX> (dcol_device.hpp).  Beyond the
bench's centred axis-aligned rect prisms (b = [half, half], so every tested pair had g3 of a
row pair equal): per shape one of
  * an axis-aligned box with six independent offsets b (off-centre: g3 != g3' in every pair),
  * a rotated box A = [R; -R] with asymmetric b,
  * a parallelepiped A = [M; -M], M a random well-conditioned non-orthogonal matrix,
and some with non-identity r_offset / Q_offset; plus control polytopes of 6 rows that are
NOT boxes (a row pair off by a rounding step), which must take the dense rows.
Table layout: tests/golden arrays (type, nh, A_off, A_pool[K, 3], b_pool, params, r_offset,
Q_offset)."""
import numpy as np

from stress_shapes import _rotation


def box_table(rng, n=48, n_control=4):
    A_rows, b_rows, off, r_off, Q_off, boxp = [], [], [], [], [], []
    for k in range(n + n_control):
        kind = k % 3
        if kind == 0:
            M = np.eye(3)
        elif kind == 1:
            M = _rotation(rng)
        else:
            while True:
                M = np.eye(3) + 0.45 * rng.normal(size=(3, 3))
                if np.linalg.cond(M) < 8:
                    break
        A = np.vstack([M, -M])          # exact negatives (negation is exact in floating point)
        if k >= n:                      # control: one row pair off by one ulp -> not a box
            A[4, 1] = np.nextafter(A[4, 1], np.inf)
        b = rng.uniform(0.1, 1.2, 6)    # six independent offsets: off-centre
        off.append(len(b_rows))
        A_rows += list(A)
        b_rows += list(b)
        plain = rng.uniform() < 0.6
        r_off.append(np.zeros(3) if plain else rng.uniform(-0.3, 0.3, 3))
        Q_off.append(np.eye(3) if plain else _rotation(rng))
        boxp.append(k < n)
    S = n + n_control
    tab = {"type": np.zeros(S, np.int32), "nh": np.full(S, 6, np.int32), "A_off": np.array(off, np.int32),
           "A_pool": np.array(A_rows, dtype=np.float64).reshape(-1, 3), "b_pool": np.array(b_rows, dtype=np.float64),
           "params": np.zeros((S, 4)), "r_offset": np.array(r_off).reshape(S, 3),
           "Q_offset": np.array(Q_off).reshape(S, 3, 3)}
    return tab, np.array(boxp)


def box_pairs(rng, tab, B):
    S = len(tab["type"])
    s1 = rng.integers(0, S, B).astype(np.int32)
    s2 = rng.integers(0, S, B).astype(np.int32)
    pose1 = np.hstack([rng.uniform(-3, 3, (B, 3)), rng.uniform(-1, 1, (B, 3))])
    pose2 = np.hstack([rng.uniform(-3, 3, (B, 3)), rng.uniform(-1, 1, (B, 3))])
    return s1, s2, pose1, pose2
