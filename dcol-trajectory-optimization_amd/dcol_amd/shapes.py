"""Primitive objects -> static shape specs -> C-ABI shape descriptors.

The reference dispatches on the primitive's class with isinstance
(primitives/problem_matrices.py:272-349) and reads duck-typed fields
(misc_primitive_constructor.py:4-88).  Here the class is identified by name (so the
reference's own classes, this package's drop-in classes and look-alikes all work), its
static fields are snapshotted into a :class:`ShapeSpec`, and specs are deduplicated by
content so a scene's obstacles are uploaded to the device table once.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib

CLASS_TYPES = {
    "PolytopeMRP": _lib.POLYTOPE,
    "SphereMRP": _lib.SPHERE,
    "ConeMRP": _lib.CONE,
    "CapsuleMRP": _lib.CAPSULE,
    "CylinderMRP": _lib.CYLINDER,
    "PolygonMRP": _lib.POLYGON,
}
TYPE_NAMES = {v: k for k, v in CLASS_TYPES.items()}


def shape_type(obj) -> int:
    for cls in type(obj).__mro__:
        t = CLASS_TYPES.get(cls.__name__)
        if t is not None:
            return t
    # the reference's problem_matrices() returns None for unknown types and the caller's
    # tuple unpacking fails (proximity.py:23)
    raise TypeError("cannot unpack non-iterable NoneType object")


@dataclass(frozen=True)
class ShapeSpec:
    type: int
    A: tuple = ()          # flattened rows (nh*3 for polytope, nh*2 for polygon)
    b: tuple = ()
    R: float = 0.0
    L: float = 0.0
    H: float = 0.0
    beta: float = 0.0
    r_offset: tuple = (0.0, 0.0, 0.0)
    Q_offset: tuple = (1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0)

    @property
    def nh(self) -> int:
        return len(self.b)


def _f(v) -> float:
    return float(v)


def _vec(a, n=None) -> tuple:
    arr = np.asarray(a, dtype=np.float64).reshape(-1)
    if n is not None and arr.size != n:
        raise ValueError(f"expected {n} values, got {arr.size}")
    return tuple(float(v) for v in arr)


def spec_from_object(obj) -> ShapeSpec:
    """Snapshot the static (non-pose) fields of a primitive object."""
    t = shape_type(obj)
    common = dict(r_offset=_vec(getattr(obj, "r_offset", np.zeros(3)), 3),
                  Q_offset=_vec(getattr(obj, "Q_offset", np.eye(3)), 9))
    if t == _lib.POLYTOPE:
        A = np.asarray(obj.A, dtype=np.float64)
        if A.ndim != 2 or A.shape[1] != 3:
            raise ValueError(f"PolytopeMRP.A must be (nh, 3), got {A.shape}")
        b = _vec(obj.b, A.shape[0])
        return ShapeSpec(t, A=_vec(A), b=b, **common)
    if t == _lib.POLYGON:
        A = np.asarray(obj.A, dtype=np.float64)
        if A.ndim != 2 or A.shape[1] != 2:
            raise ValueError(f"PolygonMRP.A must be (nh, 2), got {A.shape}")
        return ShapeSpec(t, A=_vec(A), b=_vec(obj.b, A.shape[0]), R=_f(obj.R), **common)
    if t == _lib.SPHERE:
        return ShapeSpec(t, R=_f(obj.R), **common)
    if t == _lib.CONE:
        return ShapeSpec(t, H=_f(obj.H), beta=_f(obj.beta), **common)
    return ShapeSpec(t, R=_f(obj.R), L=_f(obj.L), **common)   # capsule / cylinder


def spec_from_arrays(tab, k: int) -> ShapeSpec:
    """Shape k of a shape table in array form (the tests/golden/*.npz layout:
    type, nh, A_off, A_pool[K,3], b_pool, params[S,4]=(R,L,H,beta), r_offset, Q_offset)."""
    t = int(tab["type"][k])
    nh = int(tab["nh"][k])
    off = int(tab["A_off"][k])
    R, L, H, beta = (float(v) for v in tab["params"][k])
    common = dict(r_offset=_vec(tab["r_offset"][k], 3), Q_offset=_vec(tab["Q_offset"][k], 9))
    if t == _lib.POLYTOPE:
        return ShapeSpec(t, A=_vec(tab["A_pool"][off:off + nh, :3]), b=_vec(tab["b_pool"][off:off + nh]), **common)
    if t == _lib.POLYGON:
        return ShapeSpec(t, A=_vec(tab["A_pool"][off:off + nh, :2]), b=_vec(tab["b_pool"][off:off + nh]), R=R, **common)
    if t == _lib.SPHERE:
        return ShapeSpec(t, R=R, **common)
    if t == _lib.CONE:
        return ShapeSpec(t, H=H, beta=beta, **common)
    if t in (_lib.CAPSULE, _lib.CYLINDER):
        return ShapeSpec(t, R=R, L=L, **common)
    raise TypeError(f"unknown shape type {t}")


def make_descs(specs):
    """ShapeSpec list -> (ctypes array of dcol_shape_desc, keep-alive buffers)."""
    n = len(specs)
    descs = (_lib.ShapeDesc * max(n, 1))()
    keep = []
    for i, s in enumerate(specs):
        d = descs[i]
        d.type = s.type
        d.nh = s.nh
        if s.nh:
            A = np.ascontiguousarray(np.array(s.A, dtype=np.float64))
            b = np.ascontiguousarray(np.array(s.b, dtype=np.float64))
            keep += [A, b]
            d.A = A.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
            d.b = b.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        d.R, d.L, d.H, d.beta = s.R, s.L, s.H, s.beta
        for k in range(3):
            d.r_offset[k] = s.r_offset[k]
        for k in range(9):
            d.Q_offset[k] = s.Q_offset[k]
    return descs, keep


def pose_of(obj) -> np.ndarray:
    """Current pose [r(3), p(3)] of a primitive object (read at every call, like the
    reference, whose callers overwrite .r/.p before each query)."""
    out = np.empty(6)
    out[:3] = np.asarray(obj.r, dtype=np.float64).reshape(3)
    out[3:] = np.asarray(obj.p, dtype=np.float64).reshape(3)
    return out
