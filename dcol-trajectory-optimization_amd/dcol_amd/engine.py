"""Host-side engine: shape registry + device shape table + plans + batched solves.

Everything numeric happens in lib/libdcol.so (HIP kernels on the GPU).  This module only
marshals primitives into the C-ABI (include/dcol.h) and device buffers:

* host path  -> dcol_prox_batch_host (numpy in / numpy out, synchronous); used by the
  drop-in proximity_mrp / proximity_gradient and by small batches;
* device path -> dcol_plan_run on torch CUDA (HIP) tensors already resident in HBM,
  asynchronous on a stream; used by the batched driver, bench.py and multi-GPU sharding.

torch is only plumbing here (device memory, streams); it is imported lazily so the host
path works without it.
"""
from __future__ import annotations

import ctypes
import threading
from collections import OrderedDict
from dataclasses import dataclass

import numpy as np

from . import _lib
from .shapes import ShapeSpec, make_descs, pose_of, spec_from_object

DEFAULT_TOL = 1e-6        # proximity.py:6, proximity_gradient.py:91
DEFAULT_MAX_ITER = 50     # pdip.py:408 (literal)


class PDIPFailure(Exception):
    """Raised like the reference's bare Exception (pdip.py:470)."""


def _np_ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def grad_flag(grad) -> int:
    if grad in (None, False):
        return 0
    if grad in (True, "fd"):
        return _lib.GRAD_FD
    if grad == "envelope":
        return _lib.GRAD_ENVELOPE
    if grad == "implicit":
        return _lib.GRAD_IMPLICIT
    raise ValueError(f"grad must be None, 'fd', 'envelope' or 'implicit', got {grad!r}")


def raise_for_status(status: int):
    """Map a dcol_status to the exception the reference raises for the same failure."""
    if status == _lib.OK:
        return
    if status == _lib.MAXITER:
        raise PDIPFailure("Maximum number of iterations reached, PDIP failed")   # pdip.py:470
    if status == _lib.UNSUPPORTED:
        raise ValueError("Failed to combine problem matrices.")                  # combine :70
    if status == _lib.NOT_PD:
        raise np.linalg.LinAlgError("Matrix is not positive definite")           # pdip.py:317/:434
    if status == _lib.NONFINITE:
        raise ValueError("array must not contain infs or NaNs")                  # scipy check_finite
    if status == _lib.TOO_LARGE:
        raise ValueError("pair exceeds the engine's orthant-row capacity (128 rows, 64 per primitive)")
    raise RuntimeError(f"unknown dcol status {status}")


@dataclass
class Result:
    alpha: np.ndarray
    contact: np.ndarray | None
    grad: np.ndarray | None
    iters: np.ndarray
    status: np.ndarray


class Table:
    """Owning wrapper of a device shape table (dcol_table)."""

    def __init__(self, specs, device: int = 0):
        lib = _lib.load()
        descs, keep = make_descs(specs)
        h = ctypes.c_void_p()
        _lib.check(lib.dcol_table_create(descs, len(specs), int(device), ctypes.byref(h)), "dcol_table_create")
        del keep
        self.handle = h
        self.n = len(specs)
        self.device = int(device)

    def pair_dims(self, s1: int, s2: int):
        m, n, ns, st = (ctypes.c_int32() for _ in range(4))
        _lib.check(_lib.load().dcol_pair_dims(self.handle, int(s1), int(s2), ctypes.byref(m), ctypes.byref(n),
                                              ctypes.byref(ns), ctypes.byref(st)), "dcol_pair_dims")
        return int(m.value), int(n.value), int(ns.value), int(st.value)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                _lib.load().dcol_table_destroy(h)
            except Exception:  # pragma: no cover - interpreter shutdown
                pass
            self.handle = None


class Plan:
    """Owning wrapper of a dcol_plan: a fixed pairing bucketed by kernel variant."""

    def __init__(self, table: Table, s1, s2, case4: bool = False, fuse: bool = True, suspend: bool = False):
        """case4=True: solve case-4 pairs (DCOL_PLAN_CASE4 extension) instead of reporting
        UNSUPPORTED like the reference.  fuse=False: one launch per variant bucket even for
        a small mixed plan (DCOL_PLAN_NO_FUSE; A/B and tests).  suspend=True: large buckets
        run as a suspend / resume launch pair (DCOL_PLAN_SUSPEND; bitwise the same results;
        the plan owns scratch -- do not run it on two streams at once)."""
        lib = _lib.load()
        self.s1 = np.ascontiguousarray(s1, dtype=np.int32)
        self.s2 = np.ascontiguousarray(s2, dtype=np.int32)
        if self.s1.shape != self.s2.shape or self.s1.ndim != 1:
            raise ValueError("shape id arrays must be 1-D and of equal length")
        self.table = table
        self.B = int(self.s1.size)
        h = ctypes.c_void_p()
        self.case4 = bool(case4)
        opts = (_lib.PLAN_CASE4 if case4 else 0) | (0 if fuse else _lib.PLAN_NO_FUSE) | (
            _lib.PLAN_SUSPEND if suspend else 0)
        _lib.check(lib.dcol_plan_create_ex(table.handle, self.B, _np_ptr(self.s1), _np_ptr(self.s2),
                                           opts, ctypes.byref(h)), "dcol_plan_create_ex")
        self.handle = h
        n = ctypes.c_int32()
        _lib.check(lib.dcol_plan_num_launches(h, ctypes.byref(n)), "dcol_plan_num_launches")
        self.num_launches = int(n.value)       # kernel launches per run
        _lib.check(lib.dcol_plan_num_buckets(h, ctypes.byref(n)), "dcol_plan_num_buckets")
        self.num_buckets = int(n.value)        # variant buckets (incl. rejected pairs)
        _lib.check(lib.dcol_plan_num_streams(h, ctypes.byref(n)), "dcol_plan_num_streams")
        self.num_streams = int(n.value)        # streams a run's launches are spread over
        _lib.check(lib.dcol_plan_launch_form(h, ctypes.byref(n)), "dcol_plan_launch_form")
        # how a run launches its buckets: "buckets" (one launch each), "fused" (small plan),
        # "packed" (mid-size plan; include/dcol.h enum dcol_plan_form)
        self.launch_form = ("buckets", "fused", "packed")[int(n.value)]

    def buckets(self) -> list:
        """The plan's variant buckets (dcol_plan_bucket): one dict per bucket with kind
        ("solve" / "reject"), N, nsoc, omax, lpp (lanes per pair of its launch), oe (extra-row
        slots of a row-partitioned bucket, 0 for dense rows), flags (1 padding-free, 2 ball-SOC
        rows, 4 cone-SOC rows), status (reject buckets) and pairs"""
        lib = _lib.load()
        info = (ctypes.c_int32 * 8)()
        n = ctypes.c_int64()
        out = []
        for i in range(self.num_buckets):
            _lib.check(lib.dcol_plan_bucket(self.handle, i, info, ctypes.byref(n)), "dcol_plan_bucket")
            v = list(info)
            out.append({"kind": "solve" if v[0] == 0 else "reject", "N": v[1], "nsoc": v[2], "omax": v[3],
                        "lpp": v[4], "oe": v[5], "flags": v[6], "status": v[7], "pairs": int(n.value)})
        return out

    def suspended(self) -> int:
        """pairs the last completed run handed to resume launches (synchronise first)"""
        n = ctypes.c_int64()
        _lib.check(_lib.load().dcol_plan_suspended(self.handle, ctypes.byref(n)), "dcol_plan_suspended")
        return int(n.value)

    def run(self, pose1, pose2, tol=DEFAULT_TOL, max_iter=DEFAULT_MAX_ITER, grad="fd", contact=True,
            out=None, stream=None):
        """Solve on the device.  pose1/pose2: torch float64 tensors [6, B] on the table's
        device (structure of arrays).  Returns dict of torch tensors (alpha [B],
        contact [3, B], grad [12, B], iters [B], status [B]); asynchronous on `stream`
        (torch stream or None = current stream)."""
        import torch
        B = self.B
        dev = torch.device("cuda", self.table.device)
        for t in (pose1, pose2):
            if t.dtype != torch.float64 or tuple(t.shape) != (6, B) or not t.is_contiguous() or t.device != dev:
                raise ValueError(f"poses must be contiguous float64 [6, {B}] on {dev}")
        flags = grad_flag(grad) | (_lib.CONTACT if contact else 0)
        if out is None:
            out = alloc_outputs(B, dev, bool(flags & _lib.GRAD_ANY), bool(contact))
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        _lib.check(_lib.load().dcol_plan_run(self.handle, ptr(pose1), ptr(pose2), float(tol), int(max_iter), flags,
                                             ptr(out["alpha"]), ptr(out.get("contact")), ptr(out.get("grad")),
                                             ptr(out["iters"]), ptr(out["status"]), ctypes.c_void_p(stream.cuda_stream)),
                   "dcol_plan_run")
        return out

    def bind(self, pose1, pose2, out, tol=DEFAULT_TOL, max_iter=DEFAULT_MAX_ITER, grad="fd", contact=False,
             stream=None):
        """Pre-convert every argument of dcol_plan_run once; returns a zero-argument callable
        that re-launches the solve on the same device buffers (hot loops: ALTRO phases,
        bench.py).  Validates like run().  `out` without "iters" / "status": those per-pair
        outputs are not written (dcol_plan_run takes NULL for them)."""
        import torch
        B = self.B
        dev = torch.device("cuda", self.table.device)
        for t in (pose1, pose2):
            if t.dtype != torch.float64 or tuple(t.shape) != (6, B) or not t.is_contiguous() or t.device != dev:
                raise ValueError(f"poses must be contiguous float64 [6, {B}] on {dev}")
        flags = grad_flag(grad) | (_lib.CONTACT if contact else 0)
        if (flags & _lib.GRAD_ANY) and "grad" not in out:
            raise ValueError("out has no 'grad' buffer")
        if contact and "contact" not in out:
            raise ValueError("out has no 'contact' buffer")
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        args = (self.handle, ptr(pose1), ptr(pose2), ctypes.c_double(tol), ctypes.c_int32(max_iter),
                ctypes.c_int32(flags), ptr(out["alpha"]), ptr(out.get("contact")), ptr(out.get("grad")),
                ptr(out.get("iters")), ptr(out.get("status")), ctypes.c_void_p(stream.cuda_stream))
        fn = _lib.load().dcol_plan_run
        keep = (self, pose1, pose2, out)

        def launch():
            rc = fn(*args)
            if rc:
                _lib.check(rc, "dcol_plan_run")
        launch.keep = keep
        return launch

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                _lib.load().dcol_plan_destroy(h)
            except Exception:  # pragma: no cover
                pass
            self.handle = None


def alloc_outputs(B: int, device, want_grad=True, want_contact=True):
    import torch
    out = {"alpha": torch.empty(B, dtype=torch.float64, device=device),
           "iters": torch.empty(B, dtype=torch.int32, device=device),
           "status": torch.empty(B, dtype=torch.int32, device=device)}
    if want_contact:
        out["contact"] = torch.empty((3, B), dtype=torch.float64, device=device)
    if want_grad:
        out["grad"] = torch.empty((12, B), dtype=torch.float64, device=device)
    return out


def cost_order(iters) -> np.ndarray:
    """A listing order for a fixed pairing: pair indices in descending order of their last
    Newton iteration counts (stable).  A wave of a solve launch runs until its slowest pair
    has converged, so pairs listed (and their poses and outputs laid out) in this order fill
    each wave with pairs of similar cost, the slowest first; a plan built on the re-listed
    pairing solves the same pairs with bitwise the same results.  For a trajectory optimiser
    (the same pairs at slowly changing poses) re-list once from a solve's `iters` and keep
    the order -- measured on configs[3] at drifting poses: bench.py `cost_order`,
    tools/order_probe.py.  The plan itself cannot reorder slots for free: a permutation read
    through an index array turns the coalesced pose / output accesses into gathers and
    scatters, which cost more than the order saves."""
    it = np.asarray(iters).reshape(-1)
    return np.argsort(-it.astype(np.int64), kind="stable")


class Engine:
    """Shape registry + lazily (re)built device table.

    Shapes are deduplicated by content; a primitive OBJECT's static fields are snapshotted
    the first time it is seen (its pose .r/.p is read at every call, like the reference).
    Call :meth:`forget` after mutating a primitive's shape parameters in place."""

    def __init__(self, device: int = 0):
        self.device = int(device)
        # iteration cap of the object-level calls (solve_objects and the drop-in
        # proximity_mrp / proximity_gradient): the reference's literal 50 (pdip.py:408,
        # quirk Q4); an attribute so a caller or test can lower it for one engine
        self.max_iter = DEFAULT_MAX_ITER
        self._specs: list[ShapeSpec] = []
        self._ids: dict[ShapeSpec, int] = {}
        self._obj_ids: dict[int, tuple[object, int]] = {}
        self._table: Table | None = None
        self._plans: OrderedDict = OrderedDict()
        self._lock = threading.RLock()
        self._pair = None        # solve_pair's staging (buffers + their addresses), made once

    # ---------------------------------------------------------------- registry
    def register(self, spec: ShapeSpec) -> int:
        with self._lock:
            i = self._ids.get(spec)
            if i is None:
                i = len(self._specs)
                self._specs.append(spec)
                self._ids[spec] = i
                self._table = None
                self._plans.clear()
            return i

    def register_object(self, obj) -> int:
        key = id(obj)
        hit = self._obj_ids.get(key)
        if hit is not None and hit[0] is obj:
            return hit[1]
        i = self.register(spec_from_object(obj))
        self._obj_ids[key] = (obj, i)     # strong ref keeps id(obj) from being reused
        return i

    def forget(self, obj):
        self._obj_ids.pop(id(obj), None)

    @property
    def table(self) -> Table:
        with self._lock:
            if self._table is None:
                self._table = Table(self._specs, self.device)
            return self._table

    def plan(self, s1, s2, cache=True, case4=False, fuse=True, suspend=False) -> Plan:
        s1 = np.ascontiguousarray(s1, dtype=np.int32)
        s2 = np.ascontiguousarray(s2, dtype=np.int32)
        if not cache or suspend:   # suspend plans own scratch: never shared through the cache
            return Plan(self.table, s1, s2, case4, fuse, suspend)
        key = (s1.tobytes(), s2.tobytes(), bool(case4), bool(fuse))
        with self._lock:
            p = self._plans.get(key)
            if p is None or p.table is not self.table:
                p = Plan(self.table, s1, s2, case4, fuse)
                self._plans[key] = p
                if len(self._plans) > 32:
                    self._plans.popitem(last=False)
            else:
                self._plans.move_to_end(key)
            return p

    # ---------------------------------------------------------------- solves
    def solve_host(self, s1, s2, pose1, pose2, tol=DEFAULT_TOL, max_iter=DEFAULT_MAX_ITER, grad="fd",
                   contact=True, case4=False) -> Result:
        """Host arrays in/out: s1, s2 int [B]; pose1, pose2 float64 [B, 6] (r, p).
        case4=True: the DCOL_CASE4 extension (see Plan)."""
        s1 = np.ascontiguousarray(s1, dtype=np.int32).reshape(-1)
        s2 = np.ascontiguousarray(s2, dtype=np.int32).reshape(-1)
        B = s1.size
        p1 = np.ascontiguousarray(pose1, dtype=np.float64).reshape(B, 6)
        p2 = np.ascontiguousarray(pose2, dtype=np.float64).reshape(B, 6)
        flags = grad_flag(grad) | (_lib.CONTACT if contact else 0) | (_lib.CASE4 if case4 else 0)
        alpha = np.empty(B)
        cp = np.empty((B, 3)) if contact else None
        g = np.empty((B, 12)) if flags & _lib.GRAD_ANY else None
        iters = np.empty(B, dtype=np.int32)
        status = np.empty(B, dtype=np.int32)
        table = self.table
        _lib.check(_lib.load().dcol_prox_batch_host(table.handle, B, _np_ptr(s1), _np_ptr(s2), _np_ptr(p1), _np_ptr(p2),
                                                    float(tol), int(max_iter), flags, _np_ptr(alpha), _np_ptr(cp),
                                                    _np_ptr(g), _np_ptr(iters), _np_ptr(status)),
                   "dcol_prox_batch_host")
        return Result(alpha, cp, g, iters, status)

    def solve_objects(self, prims1, prims2, tol=DEFAULT_TOL, max_iter=None, grad="fd",
                      contact=True, case4=False) -> Result:
        """Batched form of the drop-in: two equal-length sequences of primitive objects,
        each at its current pose.  max_iter=None: the engine's cap (self.max_iter)."""
        if max_iter is None:
            max_iter = self.max_iter
        s1 = np.fromiter((self.register_object(o) for o in prims1), dtype=np.int32)
        s2 = np.fromiter((self.register_object(o) for o in prims2), dtype=np.int32)
        if s1.size != s2.size:
            raise ValueError("prims1 and prims2 must have equal length")
        p1 = np.array([pose_of(o) for o in prims1]).reshape(-1, 6)
        p2 = np.array([pose_of(o) for o in prims2]).reshape(-1, 6)
        return self.solve_host(s1, s2, p1, p2, tol, max_iter, grad, contact, case4)

    def solve_pair(self, prim1, prim2, tol=DEFAULT_TOL, grad="fd", contact=True):
        """One pair at its current poses -> (alpha, contact [3] | None, grad [12] | None,
        iters, status): the drop-in's per-call path (dcol_prox_pair: a cached one-pair plan
        and device-mapped pinned staging, one kernel launch, no copy commands).  The returned
        arrays are fresh copies.  Thread-safe: the engine's one staging set is held under the
        engine lock from the pose writes to the output copies (two threads on the default
        engine would otherwise overwrite each other's poses or outputs)."""
        flags = grad_flag(grad) | (_lib.CONTACT if contact else 0)
        # fast path (csrc/fastpair.c): both objects known and the table built -- the poses,
        # the library call and the outputs in one C function, no engine lock needed (the
        # library serialises calls per table; `table` keeps this table alive for the call)
        table = self._table
        if table is not None:   # (the library is loaded only once a table exists)
            h1 = self._obj_ids.get(id(prim1))
            h2 = self._obj_ids.get(id(prim2))
            fast = _fastpair()
            # (an id past this table's size belongs to the next table, which another thread's
            # register_object has just invalidated this one for: the locked path rebuilds)
            if (fast is not None and h1 is not None and h2 is not None and h1[0] is prim1 and h2[0] is prim2
                    and h1[1] < table.n and h2[1] < table.n):
                r = fast[0](fast[1], table.handle.value, h1[1], h2[1], prim1.r, prim1.p, prim2.r, prim2.p, tol,
                            self.max_iter, flags, contact)
                if r is not None:
                    if r[0]:
                        _lib.check(r[0], "dcol_prox_pair")
                    return r[1:]
        with self._lock:
            s1 = self.register_object(prim1)
            s2 = self.register_object(prim2)
            table = self.table
            st = self._pair
            if st is None:
                bufs = (np.empty(12), np.empty(1), np.empty(3), np.empty(12), np.empty(2, dtype=np.int32))
                st = self._pair = (bufs, [ctypes.c_void_p(b.ctypes.data) for b in bufs], _lib.load().dcol_prox_pair)
            (pose, alpha, cp, g, ints), (a_pose, a_alpha, a_cp, a_g, a_ints), fn = st
            pose[0:3] = np.reshape(prim1.r, 3)     # read at every call, like the reference (pose_of)
            pose[3:6] = np.reshape(prim1.p, 3)
            pose[6:9] = np.reshape(prim2.r, 3)
            pose[9:12] = np.reshape(prim2.p, 3)
            rc = fn(table.handle, s1, s2, a_pose, ctypes.c_void_p(a_pose.value + 48), tol, self.max_iter, flags,
                    a_alpha, a_cp, a_g, a_ints, ctypes.c_void_p(a_ints.value + 4))
            if rc:
                _lib.check(rc, "dcol_prox_pair")
            return (np.float64(alpha[0]), cp.copy() if contact else None, g.copy() if flags & _lib.GRAD_ANY else None,
                    int(ints[0]), int(ints[1]))

    def stop_pair_server(self):
        """dcol_table_stop_pair_server: the table's resident pair server leaves now (the next
        solve_pair starts a new one)"""
        with self._lock:
            if self._table is not None:
                _lib.check(_lib.load().dcol_table_stop_pair_server(self._table.handle), "dcol_table_stop_pair_server")

    def pair_server_running(self) -> bool:
        with self._lock:
            if self._table is None:
                return False
            v = ctypes.c_int32()
            _lib.check(_lib.load().dcol_table_pair_server_running(self._table.handle, ctypes.byref(v)),
                       "dcol_table_pair_server_running")
            return bool(v.value)

    def pair_stats(self):
        """dcol_table_pair_stats of the current table: {"served": calls the one-pair server
        answered, "launched": calls that launched their own kernel, "server_starts",
        "server_solve_us" / "server_solve_cycles": device time from request to answer summed
        over the served calls, "server_xcd": the XCD the last server started on}."""
        with self._lock:
            v = [ctypes.c_int64() for _ in range(3)] + [ctypes.c_double() for _ in range(2)] + [ctypes.c_int32()]
            _lib.check(_lib.load().dcol_table_pair_stats(self.table.handle, *[ctypes.byref(x) for x in v]),
                       "dcol_table_pair_stats")
            keys = ("served", "launched", "server_starts", "server_solve_us", "server_solve_cycles", "server_xcd")
            return {k: x.value for k, x in zip(keys, v)}


_fast = None


def _fastpair():
    """(dcol_amd._fastpair.solve, address of dcol_prox_pair) or None when the extension is
    not built (Engine.solve_pair then stages through ctypes: same library call)"""
    global _fast
    if _fast is None:
        try:
            from . import _fastpair as fp
            _fast = (fp.solve, ctypes.cast(_lib.load().dcol_prox_pair, ctypes.c_void_p).value)
        except ImportError:
            _fast = False
    return _fast or None


_default: Engine | None = None
_default_lock = threading.Lock()


def default_engine() -> Engine:
    global _default
    with _default_lock:
        if _default is None:
            _default = Engine(device=0)
        return _default
