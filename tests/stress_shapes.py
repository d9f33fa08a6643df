"""Seeded random shape tables and pairs for the GPU stress parity test (test infrastructure).

Beyond the bench's fixed mixed table (boxes, pentagons): polytopes with 4-40 faces (the six
axis faces plus random tangent planes, so every bucket from 12 to 128 orthant rows gets
pairs), polygons with 3-12 edges, random radii / lengths / cone angles, non-identity
r_offset / Q_offset, and poses from far apart to overlapping.  Table layout: the
tests/golden arrays (type, nh, A_off, A_pool[K, 3], b_pool, params[S, 4] = (R, L, H, beta),
r_offset[S, 3], Q_offset[S, 3, 3]).
"""
import numpy as np

POLYTOPE, SPHERE, CONE, CAPSULE, CYLINDER, POLYGON = 0, 1, 2, 3, 4, 5


def _rotation(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def random_table(rng, per_kind=24, max_faces=40):
    t, nh, off, prm, A_rows, b_rows, r_off, Q_off = [], [], [], [], [], [], [], []
    axes = np.vstack([np.eye(3), -np.eye(3)])
    for kind in (POLYTOPE, SPHERE, CONE, CAPSULE, CYLINDER, POLYGON):
        for _ in range(per_kind):
            t.append(kind)
            off.append(len(b_rows))
            if kind == POLYTOPE:
                k = int(rng.integers(0, max_faces - 5))
                n = rng.normal(size=(k, 3))
                n /= np.linalg.norm(n, axis=1, keepdims=True)
                A = np.vstack([axes, n])
                half = rng.uniform(0.2, 1.2, 3)
                b = np.concatenate([half, half, rng.uniform(0.15, 1.0, k) * np.linalg.norm(half)])
                A_rows += list(A)
                b_rows += list(b)
                nh.append(6 + k)
                prm.append((0, 0, 0, 0))
            elif kind == POLYGON:
                k = int(rng.integers(3, 13))
                # evenly spaced edge normals, rotated, jittered for k >= 5 (every gap < pi:
                # bounded)
                ang = np.linspace(0, 2 * np.pi, k, endpoint=False) + rng.uniform(0, 2 * np.pi)
                if k >= 5:
                    ang = ang + rng.uniform(-0.25, 0.25, k) * (2 * np.pi / k)
                A = np.stack([np.cos(ang), np.sin(ang), np.zeros(k)], 1)
                A_rows += list(A)
                b_rows += list(rng.uniform(0.3, 1.0, k))
                nh.append(k)
                prm.append((rng.uniform(0.05, 0.4), 0, 0, 0))
            else:
                nh.append(0)
                if kind == SPHERE:
                    prm.append((rng.uniform(0.1, 1.5), 0, 0, 0))
                elif kind == CONE:
                    prm.append((0, 0, rng.uniform(0.3, 2.5), np.deg2rad(rng.uniform(8, 50))))
                else:
                    prm.append((rng.uniform(0.05, 0.8), rng.uniform(0.1, 2.5), 0, 0))
            plain = rng.uniform() < 0.5
            r_off.append(np.zeros(3) if plain else rng.uniform(-0.3, 0.3, 3))
            Q_off.append(np.eye(3) if plain else _rotation(rng))
    S = len(t)
    return {"type": np.array(t, np.int32), "nh": np.array(nh, np.int32), "A_off": np.array(off, np.int32),
            "A_pool": np.array(A_rows, dtype=np.float64).reshape(-1, 3), "b_pool": np.array(b_rows, dtype=np.float64),
            "params": np.array(prm, dtype=np.float64), "r_offset": np.array(r_off).reshape(S, 3),
            "Q_offset": np.array(Q_off).reshape(S, 3, 3)}


def random_pairs(rng, tab, B):
    S = len(tab["type"])
    s1 = rng.integers(0, S, B).astype(np.int32)
    s2 = rng.integers(0, S, B).astype(np.int32)
    # distances from overlapping to far apart (log-uniform scale of the relative position)
    scale = np.exp(rng.uniform(np.log(0.05), np.log(8.0), B))[:, None]
    d = rng.normal(size=(B, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    c = rng.uniform(-3, 3, (B, 3))
    p1 = np.hstack([c, rng.uniform(-1, 1, (B, 3))])
    p2 = np.hstack([c + scale * d, rng.uniform(-1, 1, (B, 3))])
    return s1, s2, p1, p2
