"""Primitive data model, constructor-compatible with the reference
(primitives/misc_primitive_constructor.py:4-164).

Every primitive carries a mutable pose (``r`` position, ``p`` MRP), a body-frame
``r_offset`` and ``Q_offset``, and its shape parameters.  Callers overwrite ``r``/``p``
before each proximity query (e.g. systems/piano_mover.py:60-61); shape parameters are
treated as static and are uploaded once into the device shape table.
"""
import numpy as np


class _Primitive:
    """Common pose/offset fields of every primitive (misc_primitive_constructor.py:7-12)."""

    def __init__(self):
        self.r = np.array([0, 0, 0.0])
        self.p = np.array([0, 0, 0.0])
        self.r_offset = np.array([0, 0, 0.0])
        self.Q_offset = np.eye(3)


class PolygonMRP(_Primitive):
    """Planar polygon {A y <= b} (A: nh x 2) swept by a ball of radius ``radius``."""

    def __init__(self, A, b, radius):
        super().__init__()
        self.A, self.b, self.R = A, b, radius


class ConeMRP(_Primitive):
    """Solid cone of height ``height`` and half-angle ``beta`` (radians)."""

    def __init__(self, height, beta):
        super().__init__()
        self.H, self.beta = height, beta


class CapsuleMRP(_Primitive):
    """Capsule: segment of length ``height`` (without caps) swept by radius ``radius``."""

    def __init__(self, radius, height):
        super().__init__()
        self.R, self.L = radius, height


class CylinderMRP(_Primitive):
    """Cylinder of radius ``radius`` and length ``height``."""

    def __init__(self, radius, height):
        super().__init__()
        self.R, self.L = radius, height


class SphereMRP(_Primitive):
    """Sphere of radius ``radius``."""

    def __init__(self, radius):
        super().__init__()
        self.R = radius


class PolytopeMRP(_Primitive):
    """Convex polytope {A y <= b} (A: nh x 3).  length/width/height are bookkeeping only."""

    def __init__(self, A, b, length=0, width=0, height=0):
        super().__init__()
        self.A, self.b = A, b
        self.length, self.width, self.height = length, width, height


def create_rect_prism(length=20.0, width=20.0, height=2.0, attitude="MRP"):
    """Axis-aligned box centred at the origin as a 6-face polytope
    (misc_primitive_constructor.py:91-142): faces +-x, +-y, +-z at half extents."""
    if attitude != "MRP":
        # the reference's "quat" branch names a class that does not exist
        raise NotImplementedError("only attitude='MRP' primitives are supported")
    half = np.array([length / 2, width / 2, height / 2])
    A = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [-1, 0, 0], [0, -1, 0], [0, 0, -1]], dtype=float)
    b = np.concatenate([half, half])
    return PolytopeMRP(A, b, length=length, width=width, height=height)


def create_n_sided(N, d):
    """Regular N-gon with every side at distance d from the origin
    (misc_primitive_constructor.py:145-164) -> {"A": (N, 2), "b": (N,)}."""
    angles = np.linspace(0, 2 * np.pi, N, endpoint=False)
    A = np.array([[np.cos(t), np.sin(t)] for t in angles])
    return {"A": A, "b": np.full(N, d)}
