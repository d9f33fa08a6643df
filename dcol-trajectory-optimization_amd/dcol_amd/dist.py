"""Data-parallel sharding of a pair batch over GPUs (one process per GPU).

Every (knot x primitive-pair) problem is independent, so a batch is split
into per-rank shards with NO data-path collective.  Results are returned per shard; when a
caller needs the whole batch on every rank (e.g. one driver process consuming all alphas
and gradients), :meth:`ShardedBatch.gather` performs ONE all-gather (torch.distributed,
backend "nccl" = RCCL over xGMI on MI355X; "gloo" on CPU for tests) of the packed per-pair
record [alpha, grad(12), status, iters] and scatters it back into the caller's pair order.

Sharding: pairs are dealt to ranks round-robin after a stable sort by kernel class and
Newton-cost proxy (m rows), so every rank receives the same mix of pair classes (cost
balance; Newton iteration counts vary 5-22 by class).  A rank's shard keeps its pairs in
batch order within each class.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time

import numpy as np

REC = 14   # packed record per pair: alpha, grad[12] (float64), then (status, iters) as two int32
           # in the last 8-byte slot (include/dcol.h DCOL_REC)


def shard_indices(B: int, rank: int, world: int, cost_key=None) -> np.ndarray:
    """Indices of the pairs owned by `rank`.  With cost_key (int array [B]), pairs are
    stably sorted by it and dealt round-robin; otherwise contiguous blocks."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    if cost_key is None:
        bounds = np.linspace(0, B, world + 1).astype(np.int64)
        return np.arange(bounds[rank], bounds[rank + 1], dtype=np.int64)
    order = np.argsort(np.asarray(cost_key), kind="stable")
    return np.sort(order[rank::world])


def shard_sizes(B: int, world: int, balanced: bool) -> list[int]:
    if balanced:
        return [len(range(r, B, world)) for r in range(world)]
    bounds = np.linspace(0, B, world + 1).astype(np.int64)
    return [int(bounds[r + 1] - bounds[r]) for r in range(world)]


# ---------------------------------------------------------------------------------------
# When does sharding pay?  (BASELINE north star: "the pair batch shards across GPUs ... when
# the batch is large enough")
#
# A sharded step = the rank's own solve of B / N pairs + ONE all-gather of every rank's
# records (REC doubles per pair) so that each rank holds the whole batch.  The solve time of
# b pairs on one MI355X is measured (bench.py mixed1m.shards: rank 0's class-balanced shard of
# the configs[4] batch solved alone, the plan policy of the library -- packed launches for
# mid-size plans); the all-gather is MODELLED, because this pool has no multi-GPU node to
# time RCCL on: each rank receives (N - 1) / N of the gathered bytes, at a bus bandwidth of
# GATHER_BUS_GBPS (RCCL's all-gather bus bandwidth on an 8-GPU xGMI node is of the order of
# 300 GB/s for messages of this size -- a stated assumption, not a measurement here) plus a
# fixed GATHER_LAT_MS per collective; GATHER_IDEAL_GBPS is the 7 xGMI links x ~153 GB/s
# ingress bound of one MI355X.
GATHER_BUS_GBPS = 300.0
GATHER_IDEAL_GBPS = 7 * 153.0
GATHER_LAT_MS = 0.03

# one-GPU solve time of b configs[4] pairs (ms): rank 0's class-balanced shard of the 1M
# mixed batch at world 1M / b, solved alone on one MI355X with the round-6 plan policy (packed
# launches for mid-size plans, fused ones for small plans), K steps back to back on one stream
# (tools/shard_bench.py, profiles/r06_d/sweep.log)
SOLVE_CURVE_MS = ((245, 0.043), (1_954, 0.045), (7_813, 0.048), (15_625, 0.081), (31_250, 0.093),
                  (62_500, 0.099), (125_000, 0.1435), (250_000, 0.268), (500_000, 0.507), (1_000_000, 0.874))


def gather_ms(B: int, world: int, bus_gbps: float = GATHER_BUS_GBPS, lat_ms: float = GATHER_LAT_MS) -> float:
    """Modelled time of the step's all-gather of B records over `world` ranks (ms)."""
    if world <= 1:
        return 0.0
    cap = -(-int(B) // world)
    total = world * cap * REC * 8.0
    return lat_ms + total * (world - 1) / world / (bus_gbps * 1e9) * 1e3


def solve_ms(b: float, curve=SOLVE_CURVE_MS) -> float:
    """One-GPU solve time of b pairs (ms): log-log interpolation of the measured curve,
    linear extrapolation past its ends (the time per pair of the last / first segment)."""
    pts = sorted(curve)
    xs = np.log([p[0] for p in pts])
    ys = np.log([p[1] for p in pts])
    x = np.log(max(float(b), 1.0))
    if x <= xs[0]:
        return float(np.exp(ys[0]))            # below the curve: a latency floor
    if x >= xs[-1]:
        return float(pts[-1][1] * b / pts[-1][0])   # beyond it: throughput-bound
    return float(np.exp(np.interp(x, xs, ys)))


def sharded_step_ms(B: int, world: int, curve=SOLVE_CURVE_MS, bus_gbps: float = GATHER_BUS_GBPS) -> float:
    """Projected step of B pairs over `world` GPUs: the largest shard's solve + the all-gather."""
    return solve_ms(-(-int(B) // max(world, 1)), curve) + gather_ms(B, world, bus_gbps)


def shard_crossover(world: int, curve=SOLVE_CURVE_MS, bus_gbps: float = GATHER_BUS_GBPS,
                    lo: int = 1_000, hi: int = 1 << 27) -> int | None:
    """B*: the batch size from which on `world` GPUs (shards + one all-gather) beat one GPU on
    every larger batch, from the solve curve and the gather model (the gain need not be
    monotone below it: the one-GPU curve has a latency floor and a step where plans change
    form); None if they lose at `hi`.  Scan on a log grid, then bisection between the last
    loss and the next gain."""
    if world <= 1:
        return None

    def gain(b):
        return solve_ms(b, curve) - sharded_step_ms(b, world, curve, bus_gbps)
    grid = np.unique(np.geomspace(lo, hi, 400).astype(np.int64))
    wins = [gain(int(b)) > 0 for b in grid]
    if not wins[-1]:
        return None
    last_loss = max((i for i, w in enumerate(wins) if not w), default=-1)
    if last_loss < 0:
        return int(grid[0])
    a, b0 = int(grid[last_loss]), int(grid[last_loss + 1])
    while b0 - a > max(1, a // 1000):
        m = (a + b0) // 2
        if gain(m) > 0:
            b0 = m
        else:
            a = m
    return b0


def should_shard(B: int, world: int, curve=SOLVE_CURVE_MS, bus_gbps: float = GATHER_BUS_GBPS) -> bool:
    """True if sharding B pairs over `world` GPUs (one all-gather) is projected to beat
    solving them on one GPU -- the caller's decision before dcol_prox_batch_multi_gpu."""
    return world > 1 and sharded_step_ms(B, world, curve, bus_gbps) < solve_ms(B, curve)


def _ints(rec):
    """[n, REC] float64 records -> [n, 2] int32 (status, iters) of the last slot"""
    return np.ascontiguousarray(rec[:, 13]).view(np.int32).reshape(-1, 2)


def pack(alpha, grad, status, iters):
    """Per-pair results -> [n, REC] float64 record (status / iters bit-packed, exact)."""
    n = len(alpha)
    rec = np.empty((n, REC), dtype=np.float64)
    rec[:, 0] = alpha
    rec[:, 1:13] = grad if grad is not None else np.nan
    ints = np.empty((n, 2), dtype=np.int32)
    ints[:, 0] = status
    ints[:, 1] = iters
    rec[:, 13] = ints.view(np.float64).reshape(n)
    return rec


def unpack(rec):
    ints = _ints(rec)
    return {"alpha": rec[:, 0].copy(), "grad": rec[:, 1:13].copy(),
            "status": ints[:, 0].copy(), "iters": ints[:, 1].copy()}


class ShardedBatch:
    """One rank's view of a sharded batch.

    solve_fn(indices) -> dict with numpy arrays alpha [n], grad [n,12], status [n], iters [n]
    for the given global pair indices (default: the GPU engine; tests inject the oracle)."""

    def __init__(self, B: int, rank: int, world: int, cost_key=None):
        self.B, self.rank, self.world = int(B), int(rank), int(world)
        self.balanced = cost_key is not None
        self.idx = shard_indices(self.B, self.rank, self.world, cost_key)
        self.all_idx = [shard_indices(self.B, r, self.world, cost_key) for r in range(self.world)]

    def solve(self, solve_fn):
        return solve_fn(self.idx)

    def gather(self, local: dict, group=None, device=None):
        """All-gather every rank's packed records; returns full-batch arrays in pair order."""
        import torch
        import torch.distributed as dist
        sizes = [len(i) for i in self.all_idx]
        cap = max(sizes) if sizes else 0
        rec = pack(local["alpha"], local.get("grad"), local["status"], local["iters"])
        buf = np.full((cap, REC), np.nan)
        buf[:len(rec)] = rec
        t = torch.from_numpy(buf)
        if device is not None:
            t = t.to(device)
        out = torch.empty((self.world * cap, REC), dtype=torch.float64, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=group)
        allrec = out.cpu().numpy().reshape(self.world, cap, REC)
        full = np.empty((self.B, REC))
        for r, ids in enumerate(self.all_idx):
            full[ids] = allrec[r, :len(ids)]
        return unpack(full)


def engine_solve_fn(engine, s1, s2, pose1, pose2, tol=1e-6, grad="fd"):
    """Default per-rank solver: the HIP engine on this rank's device (host arrays)."""
    def fn(idx):
        res = engine.solve_host(s1[idx], s2[idx], pose1[idx], pose2[idx], tol=tol, grad=grad, contact=False)
        return {"alpha": res.alpha, "grad": res.grad, "status": res.status, "iters": res.iters}
    return fn


class NativeComm:
    """The C-ABI multi-GPU path (include/dcol.h: dcol_comm_*, dcol_prox_batch_multi_gpu):
    an RCCL communicator owned by libdcol.so, for hosts that do not run torch.distributed.
    Rank 0 creates the id (``NativeComm.unique_id()``) and ships it to the other ranks by
    any means; every rank then builds ``NativeComm(id, world, rank, device)``."""

    def __init__(self, uid: bytes, world: int, rank: int, device: int = 0):
        import ctypes
        from . import _lib
        if len(uid) != _lib.COMM_ID_BYTES:
            raise ValueError(f"communicator id must be {_lib.COMM_ID_BYTES} bytes")
        self.world, self.rank, self.device = int(world), int(rank), int(device)
        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        _lib.check(_lib.load().dcol_comm_create(ctypes.cast(buf, ctypes.c_void_p), self.world, self.rank,
                                                self.device, ctypes.byref(h)), "dcol_comm_create")
        self.handle = h

    @staticmethod
    def unique_id() -> bytes:
        import ctypes
        from . import _lib
        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
        _lib.check(_lib.load().dcol_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)), "dcol_comm_unique_id")
        return bytes(buf)

    def solve_gather(self, plan, pose1, pose2, cap: int, tol=1e-6, max_iter=50, grad="fd", out=None,
                     stream=None, rec_local=None, rec_all=None, in_place=False, soa=True, gather=True):
        """Solve this rank's shard (``plan`` over its pairs; torch float64 [6, n] poses on the
        device) and all-gather the packed records: returns (out, rec_all) with rec_all a
        torch float64 [world * cap, REC] tensor (rank r's shard at rows r * cap), asynchronous
        on ``stream``.  Same record layout as :meth:`ShardedBatch.gather`.

        in_place: the kernels write the records straight into this rank's rows of rec_all and
        the all-gather runs in place (include/dcol.h, rec_local == NULL); rows past the shard
        are all-ones bytes (NaN, int pair (-1, -1)).  soa=False (in place only): no per-pair
        output arrays, records only (out is returned as None).  gather=False (in place only,
        DCOL_NO_GATHER): everything but the all-gather -- issue it with :meth:`all_gather`
        (e.g. on a stream of its own), or time the step without its collective."""
        import ctypes

        import torch

        from . import _lib
        from .engine import alloc_outputs, grad_flag
        if in_place and rec_local is not None:
            raise ValueError("in_place writes into rec_all: pass no rec_local")
        if not soa and not in_place:
            raise ValueError("soa=False needs in_place=True (the pack pass reads the per-pair arrays)")
        if not gather and not in_place:
            raise ValueError("gather=False needs in_place=True")
        n = plan.B
        dev = torch.device("cuda", self.device)
        for t in (pose1, pose2):
            if t.dtype != torch.float64 or tuple(t.shape) != (6, n) or not t.is_contiguous() or t.device != dev:
                raise ValueError(f"poses must be contiguous float64 [6, {n}] on {dev}")
        if cap < n:
            raise ValueError("cap must be >= the shard size")
        flags = grad_flag(grad) | (0 if gather else _lib.NO_GATHER)
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        # Buffers allocated here belong to `stream` in torch's caching allocator (allocated
        # under it): rec_local dies when this call returns while the pack kernel and the
        # all-gather still read it on `stream`, so its block may only be handed out again to
        # later work on that same stream (ordered after them).  rec_local / rec_all / out may
        # also be passed in (hot loops reuse them; then the caller owns their lifetime).
        with torch.cuda.stream(stream):
            if out is None and soa:
                out = alloc_outputs(n, dev, bool(flags & _lib.GRAD_ANY), False)
            if rec_local is None and not in_place:
                rec_local = torch.empty((cap, REC), dtype=torch.float64, device=dev)
            if rec_all is None:
                rec_all = torch.empty((self.world * cap, REC), dtype=torch.float64, device=dev)
        bufs = [(rec_all, (self.world * cap, REC))] + ([] if in_place else [(rec_local, (cap, REC))])
        for t, shape in bufs:
            if t.dtype != torch.float64 or tuple(t.shape) != shape or not t.is_contiguous() or t.device != dev:
                raise ValueError(f"record buffers must be contiguous float64 {shape} on {dev}")
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        o = out if soa else {}
        _lib.check(_lib.load().dcol_prox_batch_multi_gpu(
            plan.handle, self.handle, ptr(pose1), ptr(pose2), float(tol), int(max_iter), flags, int(cap),
            ptr(o.get("alpha")), ptr(o.get("grad")), ptr(o.get("iters")), ptr(o.get("status")), ptr(rec_local),
            ptr(rec_all), ctypes.c_void_p(stream.cuda_stream)), "dcol_prox_batch_multi_gpu")
        return (out if soa else None), rec_all

    def all_gather(self, cap: int, rec_all, stream=None):
        """The in-place all-gather alone (dcol_comm_all_gather): every rank's rows
        [rank * cap, (rank + 1) * cap) of rec_all (torch float64 [world * cap, REC] on this
        rank's device) to every rank, asynchronous on ``stream``.  Follows a
        ``solve_gather(..., in_place=True, gather=False)`` whose stream the caller orders
        before ``stream`` (an event)."""
        import ctypes

        import torch

        from . import _lib
        dev = torch.device("cuda", self.device)
        shape = (self.world * int(cap), REC)
        if (rec_all.dtype != torch.float64 or tuple(rec_all.shape) != shape or not rec_all.is_contiguous()
                or rec_all.device != dev):
            raise ValueError(f"rec_all must be contiguous float64 {shape} on {dev}")
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        _lib.check(_lib.load().dcol_comm_all_gather(self.handle, int(cap), ctypes.c_void_p(rec_all.data_ptr()),
                                                    ctypes.c_void_p(stream.cuda_stream)), "dcol_comm_all_gather")
        return rec_all

    def close(self):
        from . import _lib
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            _lib.load().dcol_comm_destroy(h)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class StepWatchdog:
    """Host-side deadline for one rank of a multi-rank run (bench.py --gpus N > 1).

    The main thread names what it is about to wait for -- ``arm(phase, step)`` before a
    collective, a barrier or a wait for a step's completion event -- and ``disarm()`` after.
    A daemon thread that finds an armed deadline passed prints ONE JSON line to stderr
    ({"dcol_deadline": true, "rank", "world", "phase", "step", "waited_s", "deadline_s"}) and
    ends the process with ``exit_code`` through os._exit: no interpreter teardown, which could
    itself block in the collective that hung.  The launcher (torchrun) then stops the other
    ranks.  It never re-executes anything.  A hang in a native call (RCCL, a HIP stream wait)
    is caught as well as one in Python, since every such call releases the GIL."""

    def __init__(self, rank: int, world: int, deadline_s: float = 120.0, exit_code: int = 3, poll_s: float = 0.05):
        self.rank, self.world = int(rank), int(world)
        self.deadline_s = float(deadline_s)
        self.exit_code = int(exit_code)
        self._poll = float(poll_s)
        self._lock = threading.Lock()
        self._armed = None          # (phase, step, t0, seconds)
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._watch, name="dcol-step-watchdog", daemon=True)
        self._thread.start()

    def arm(self, phase: str, step=None, seconds=None):
        with self._lock:
            self._armed = (str(phase), None if step is None else int(step), time.monotonic(),
                           self.deadline_s if seconds is None else float(seconds))

    def disarm(self):
        with self._lock:
            self._armed = None

    def guard(self, phase: str, step=None, seconds=None):
        """context manager: arm on entry, disarm on exit"""
        wd = self

        class _G:
            def __enter__(self_):
                wd.arm(phase, step, seconds)

            def __exit__(self_, *exc):
                wd.disarm()
                return False
        return _G()

    def wait_event(self, event, phase: str, step=None, seconds=None):
        """wait for a torch.cuda.Event (polling query(), so the wait itself never blocks
        the interpreter) under the deadline"""
        self.arm(phase, step, seconds)
        while not event.query():
            time.sleep(0)
        self.disarm()

    def close(self):
        self._stop.set()
        self._thread.join(timeout=1.0)

    def _watch(self):
        while not self._stop.wait(self._poll):
            with self._lock:
                a = self._armed
            if a is None:
                continue
            phase, step, t0, seconds = a
            waited = time.monotonic() - t0
            if waited > seconds:
                self._fire(phase, step, waited, seconds)

    def _fire(self, phase, step, waited, seconds):
        line = {"dcol_deadline": True, "rank": self.rank, "world": self.world, "phase": phase, "step": step,
                "waited_s": round(waited, 3), "deadline_s": seconds,
                "note": "this rank waited past its deadline; exiting non-zero (the launcher stops the other ranks)"}
        try:
            sys.stderr.write(json.dumps(line) + "\n")
            sys.stderr.flush()
            sys.stdout.flush()
        finally:
            os._exit(self.exit_code)
