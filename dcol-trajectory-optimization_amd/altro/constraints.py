"""Collision constraints of a whole trajectory as ONE device batch per optimizer phase.

The reference evaluates them knot by knot and obstacle by obstacle: every knot of a
backward pass calls proximity_mrp then proximity_gradient once per obstacle
(piano_mover.py:49-97, cluttered_hallway_quadrotor.py:116-171, cone_through_wall.py:
118-172), and compute_total_cost repeats the alpha solves (ALTRO.py:103-145).  Given the
trajectory X the N x n_obs problems are independent, so ObstacleField
puts all of them into one fixed pairing (a dcol_plan, pair index = knot * n_obs + obstacle)
and solves a phase with one dcol_plan_run:

    victim pose per knot (host, [N, 6]) --H2D--> pose1 [6, B] --kernel--> alpha, d alpha
                                             (obstacle poses pose2 stay resident)

Alpha-only phases (line-search trials) launch without the gradient flag.  The gradient
solve also returns alpha, which the driver reuses for the cost of the same trajectory.
The outputs live in ONE device buffer [alpha | status, iters | grad] mirrored by one pinned
host buffer, so a phase is one H2D copy, one (fused) launch and one D2H copy.
"""
from __future__ import annotations

import os

import numpy as np

from dcol_amd.engine import DEFAULT_TOL, PDIPFailure, default_engine, raise_for_status
from dcol_amd.shapes import pose_of


class ObstacleField:
    """Fixed (knot x obstacle) pairing of one victim against static obstacles, on the GPU."""

    def __init__(self, victim, obstacles, N, engine=None, tol=DEFAULT_TOL, grad="fd"):
        import torch
        eng = engine if engine is not None else default_engine()
        self.N, self.n_obs = int(N), len(obstacles)
        B = self.N * self.n_obs
        self.B = B
        vid = eng.register_object(victim)
        oids = np.array([eng.register_object(o) for o in obstacles], dtype=np.int32)
        s1 = np.full(B, vid, dtype=np.int32)
        s2 = np.tile(oids, self.N)
        self.plan = eng.plan(s1, s2, cache=False)
        dev = torch.device("cuda", eng.device)
        obs_pose = np.array([pose_of(o) for o in obstacles], dtype=np.float64).reshape(self.n_obs, 6)
        self.pose2 = torch.from_numpy(np.ascontiguousarray(np.tile(obs_pose, (self.N, 1)).T)).to(dev)
        self.pose1 = torch.empty((6, B), dtype=torch.float64, device=dev)
        # packed outputs: [alpha B | status B int32, iters B int32 | grad 12 x B] (float64 slots)
        self.d_out = torch.empty(14 * B, dtype=torch.float64, device=dev)
        self.out = self._views(self.d_out, B)
        self.stream = torch.cuda.current_stream(dev)
        self._launch = {True: self.plan.bind(self.pose1, self.pose2, self.out, tol=tol, grad=grad, stream=self.stream),
                        False: self.plan.bind(self.pose1, self.pose2, self.out, tol=tol, grad=None,
                                              stream=self.stream)}
        pin = dict(pin_memory=True)
        self.h_pose1 = torch.empty((6, B), dtype=torch.float64, **pin)
        self.h_out = torch.empty(14 * B, dtype=torch.float64, **pin)
        h = self._views(self.h_out, B)
        self.h_alpha, self.h_status, self.h_grad = h["alpha"], h["status"], h["grad"]
        # numpy views of the pinned buffers, made once (phases are latency-bound)
        self._hp3 = self.h_pose1.numpy().reshape(6, self.N, self.n_obs)
        self._np_alpha, self._np_status, self._np_grad = (t.numpy() for t in (self.h_alpha, self.h_status, self.h_grad))
        self.batches = 0
        self.pairs = 0
        self._pending = None
        self._warm(pose_of(victim))
        # How a phase reaches the GPU (DCOL_ALTRO_PHASE=zero_copy|graph|eager for A/B runs):
        #  zero_copy (default where the pinned buffers are device-mapped): ONE kernel launch
        #    that reads the victim poses from, and writes the packed outputs to, the pinned
        #    host buffers directly (a few KB over PCIe inside the kernel, no copy commands);
        #  graph: H2D of the poses -> solve -> D2H of the outputs as one hipGraph replay;
        #  eager: the same three calls issued one by one.
        mode = os.environ.get("DCOL_ALTRO_PHASE", "eager" if os.environ.get("DCOL_ALTRO_NO_GRAPH") else "zero_copy")
        self._graphs, self._direct = {}, {}
        if mode == "zero_copy":
            self._direct = self._map_host(tol, grad)
            if not self._direct:
                mode = "graph"
        if mode == "graph":
            self._graphs = self._capture(tol, grad)
        self.mode = mode

    def _map_host(self, tol, grad):
        """Launchers whose pose1 / output pointers are the device addresses of the pinned
        host buffers ({} if the allocations are not device-mapped)."""
        import ctypes

        from dcol_amd import _lib
        from dcol_amd.engine import grad_flag
        p_pose = _lib.host_device_pointer(self.h_pose1.data_ptr())
        p_out = _lib.host_device_pointer(self.h_out.data_ptr())
        if p_pose is None or p_out is None:
            return {}
        B = self.B
        fn = _lib.load().dcol_plan_run
        launchers = {}
        for g in (True, False):
            args = (self.plan.handle, ctypes.c_void_p(p_pose), ctypes.c_void_p(self.pose2.data_ptr()),
                    ctypes.c_double(tol), ctypes.c_int32(50), ctypes.c_int32(grad_flag(grad if g else None)),
                    ctypes.c_void_p(p_out), None, ctypes.c_void_p(p_out + 16 * B) if g else None,
                    ctypes.c_void_p(p_out + 12 * B), ctypes.c_void_p(p_out + 8 * B),
                    ctypes.c_void_p(self.stream.cuda_stream))

            def launch(args=args):
                rc = fn(*args)
                if rc:
                    _lib.check(rc, "dcol_plan_run")
            launchers[g] = launch
        return launchers

    def _capture(self, tol, grad):
        import torch
        dev = self.pose1.device
        cs = torch.cuda.Stream(dev)
        graphs = {}
        for g in (True, False):
            launch = self.plan.bind(self.pose1, self.pose2, self.out, tol=tol, grad=grad if g else None, stream=cs)
            n = 14 * self.B if g else 2 * self.B
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=cs):
                self.pose1.copy_(self.h_pose1, non_blocking=True)
                launch()
                self.h_out[:n].copy_(self.d_out[:n], non_blocking=True)
            graphs[g] = graph
        torch.cuda.synchronize(dev)
        return graphs

    @staticmethod
    def _views(flat, B):
        import torch
        ints = flat[B:2 * B].view(torch.int32)
        return {"alpha": flat[:B], "status": ints[:B], "iters": ints[B:2 * B], "grad": flat[2 * B:].view(12, B)}

    def _warm(self, pose):
        """Launch both variants once (loads the code objects; outputs discarded)."""
        hp = self.h_pose1.numpy()
        hp[:] = np.asarray(pose, dtype=np.float64).reshape(6, 1)
        self.pose1.copy_(self.h_pose1, non_blocking=True)
        self._launch[True]()
        self._launch[False]()
        self.stream.synchronize()

    def submit(self, victim_poses, grad: bool):
        """Start one phase asynchronously: victim_poses [N, 6] (r, p per knot) are staged in
        the pinned buffer and the phase (H2D -> solve -> D2H) is queued on self.stream; the
        host is free until collect().  One phase in flight at a time."""
        import torch
        if self._pending is not None:
            # the running phase may still read h_pose1 (zero_copy) or write h_out
            raise RuntimeError("submit() while a phase is in flight: collect() it first")
        P = np.asarray(victim_poses, dtype=np.float64).reshape(self.N, 6)
        self._hp3[:] = P.T[:, :, None]          # pose of knot t for each of its n_obs pairs
        direct = self._direct.get(bool(grad))
        if direct is not None:                  # explicit stream, no copies
            direct()
            self._pending = bool(grad)
            return
        graph = self._graphs.get(bool(grad))
        # replay() and the eager copies go to the CURRENT stream: pin it to self.stream (the
        # stream synchronised in collect) whatever stream context the caller is in
        with torch.cuda.stream(self.stream):
            if graph is not None:
                graph.replay()
            else:
                self.pose1.copy_(self.h_pose1, non_blocking=True)
                self._launch[bool(grad)]()
                n = 14 * self.B if grad else 2 * self.B  # alpha-only phases skip the gradient block
                self.h_out[:n].copy_(self.d_out[:n], non_blocking=True)
        self._pending = bool(grad)

    soa_grad = True   # collect(soa=True): gradients in the engine's [12, N n_obs] layout

    def collect(self, soa=False, raise_=True):
        """Wait for the phase started by submit() -> (alpha [N, n_obs], J [N, n_obs, 12] |
        None), or J [12, N n_obs] with soa=True (no transpose).  Raises like the reference on
        the first failed pair (knot-major order); with raise_=False returns (alpha, J,
        status [N, n_obs]) instead and leaves the decision to the caller (a batch of several
        line-search trials, where only the trials the reference would evaluate count)."""
        grad = self._pending
        self._pending = None
        if grad is None:
            raise RuntimeError("collect() without submit()")
        self.stream.synchronize()
        self.batches += 1
        self.pairs += self.B
        st = self._np_status
        if raise_ and st.any():
            raise_for_status(int(st[np.flatnonzero(st)[0]]))
        alpha = self._np_alpha.reshape(self.N, self.n_obs).copy()
        if not grad:
            J = None
        else:
            J = self._np_grad.copy() if soa else self._np_grad.T.reshape(self.N, self.n_obs, 12).copy()
        if not raise_:
            return alpha, J, st.reshape(self.N, self.n_obs).copy()
        return alpha, J

    def evaluate(self, victim_poses, grad: bool, raise_=True):
        """submit() + collect()."""
        self.submit(victim_poses, grad)
        return self.collect(raise_=raise_)


__all__ = ["ObstacleField", "PDIPFailure"]
