"""dcol_amd — MI355X-native batched differentiable proximity (DCOL) engine.

Host-side mirror of the reference's proximity API over the C-ABI of lib/libdcol.so
(include/dcol.h).  The drop-in modules ``proximity.proximity`` and
``proximity.proximity_gradient`` (next to this package) keep the reference signatures.
"""
from . import _lib
from ._lib import DcolLibraryError, device_count, load, status_string
from .engine import (DEFAULT_MAX_ITER, DEFAULT_TOL, Engine, PDIPFailure, Plan, Result, Table,
                     alloc_outputs, cost_order, default_engine, raise_for_status)
from .shapes import ShapeSpec, make_descs, pose_of, shape_type, spec_from_arrays, spec_from_object

__all__ = ["_lib", "DcolLibraryError", "device_count", "load", "status_string", "DEFAULT_MAX_ITER",
           "DEFAULT_TOL", "Engine", "PDIPFailure", "Plan", "Result", "Table", "alloc_outputs", "cost_order",
           "default_engine", "raise_for_status", "ShapeSpec", "make_descs", "pose_of", "shape_type",
           "spec_from_arrays", "spec_from_object"]
