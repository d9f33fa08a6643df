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
        self.batches = 0
        self.pairs = 0
        self._warm(pose_of(victim))
        # Each phase (H2D of the victim poses -> solve -> D2H of the packed outputs) is one
        # hipGraph replay: one submission instead of three per batch (launch-bound at ALTRO
        # sizes).  DCOL_ALTRO_NO_GRAPH=1 keeps the eager three-call path (A/B runs).
        self._graphs = {} if os.environ.get("DCOL_ALTRO_NO_GRAPH") else self._capture(tol, grad)

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

    def evaluate(self, victim_poses, grad: bool):
        """victim_poses [N, 6] (r, p per knot) -> (alpha [N, n_obs], J [N, n_obs, 12] | None).
        Raises like the reference on the first failed pair (knot-major order)."""
        P = np.asarray(victim_poses, dtype=np.float64).reshape(self.N, 6)
        hp = self.h_pose1.numpy()
        hp[:] = np.repeat(P.T, self.n_obs, axis=1)
        import torch
        graph = self._graphs.get(bool(grad))
        # replay() and the eager copies go to the CURRENT stream: pin it to self.stream (the
        # stream synchronised below) whatever stream context the caller is in
        with torch.cuda.stream(self.stream):
            if graph is not None:
                graph.replay()
            else:
                self.pose1.copy_(self.h_pose1, non_blocking=True)
                self._launch[bool(grad)]()
                n = 14 * self.B if grad else 2 * self.B  # alpha-only phases skip the gradient block
                self.h_out[:n].copy_(self.d_out[:n], non_blocking=True)
        self.stream.synchronize()
        self.batches += 1
        self.pairs += self.B
        st = self.h_status.numpy()
        if st.any():
            raise_for_status(int(st[np.flatnonzero(st)[0]]))
        alpha = self.h_alpha.numpy().reshape(self.N, self.n_obs).copy()
        J = self.h_grad.numpy().T.reshape(self.N, self.n_obs, 12).copy() if grad else None
        return alpha, J


__all__ = ["ObstacleField", "PDIPFailure"]
