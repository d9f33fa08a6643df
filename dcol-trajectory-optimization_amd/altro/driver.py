"""Batched AL-iLQR (ALTRO) driver over the GPU proximity engine.

Same algorithm, parameters, dual/penalty schedule, regularisation rule and printout as the
reference optimizer (ALTRO.py:365-488); what changes is how the work is issued:

  reference (per knot, per obstacle, Python)      here
  ---------------------------------------------   ------------------------------------------
  backward_pass: at every knot, N x n_obs alpha    nothing: the accepted line-search trial
    solves + N x n_obs gradient solves              of the previous iteration was solved as
    (ALTRO.py:268-300) and compute_jacobian         ONE batch of N x n_obs pairs WITH
    per knot (ALTRO.py:77-100)                      gradients on the GPU, and the dynamics
                                                    Jacobians of its trajectory were computed
                                                    in the same submission, all knots in one
                                                    launch beside the solves (jacobians.py;
                                                    host fallback: dcol_altro_jacobians);
                                                    only the first iteration launches its
                                                    own batch
  Riccati loop with scipy cho_factor (:304-336)    dcol_altro_backward, native
  forward_pass: old cost recomputed per line-      old cost from the cached alpha; per trial
    search trial, rollout + N x n_obs solves        one native rollout + ONE batch (alpha and
    (:183-239)                                      gradients, overlapped with the Jacobians)
  AL dual update re-solves N x n_obs (:444-470)    reuses the accepted trial's alpha
  cost / AL terms per knot (:103-145, :259-300)    dcol_altro_cost / dcol_altro_stage_terms,
                                                   native, whole trajectory per call

Every reuse is of a value the reference recomputes from identical inputs, so the
iterates are the reference's up to floating-point rounding (tests/test_altro.py pins them
against whole-run fixtures of the reference itself).
"""
from __future__ import annotations

import dataclasses
import inspect
import logging
import os
import time

import numpy as np

from dcol_amd.engine import raise_for_status

from . import _native
from . import jacobians as _jacobians
from . import systems as _systems

log = logging.getLogger("altro")

TRIALS = 4   # line-search step lengths per batch after a rejected full step


@dataclasses.dataclass
class AltroResult:
    X: np.ndarray                      # [N, nx]
    U: np.ndarray                      # [N-1, nu]
    converged: bool
    iterations: int                    # outer iterations run (backward passes)
    J: list = dataclasses.field(default_factory=list)
    delta_J: list = dataclasses.field(default_factory=list)
    kmax: list = dataclasses.field(default_factory=list)
    alpha: list = dataclasses.field(default_factory=list)
    reg: list = dataclasses.field(default_factory=list)      # reg on entry to each iteration
    rho: list = dataclasses.field(default_factory=list)      # rho on entry to each iteration
    convio: list = dataclasses.field(default_factory=list)   # (iteration, violation) at each AL update
    wall_s: float = 0.0                # optimizer loop incl. the initial rollout
    setup_s: float = 0.0               # problem set-up + constraint evaluator construction
    prox_s: float = 0.0                # time inside proximity batches (H2D + kernel + D2H)
    prox_batches: int = 0
    prox_pairs: int = 0
    jacobians: str = "host"            # where the dynamics Jacobians ran ("device" / "host")

    @property
    def ms_per_iter(self) -> float:
        return 1e3 * self.wall_s / max(self.iterations, 1)


class _Timed:
    """Wraps a constraint evaluator: submit() starts a batch, collect() waits for it (an
    evaluator without submit/collect -- e.g. a CPU one -- is evaluated synchronously at
    collect).  Accounts the host time spent blocked in the evaluator."""

    def __init__(self, field):
        self.field = field
        self.async_ = hasattr(field, "submit") and hasattr(field, "collect")
        # evaluators written against the two-value contract (evaluate(poses, grad) ->
        # (alpha, J), raising on a failed pair) have no raise_ keyword: collect(raise_=False)
        # then calls them the old way and reports an all-zero status
        fn = field.collect if self.async_ else field.evaluate
        try:
            self.has_raise = "raise_" in inspect.signature(fn).parameters
        except (TypeError, ValueError):
            self.has_raise = False
        self.seconds = 0.0
        self.batches = 0
        self.pairs = 0
        self._job = None

    def submit(self, poses, grad):
        t0 = time.perf_counter()
        if self.async_:
            self.field.submit(poses, grad)
        self._job = (poses, grad)
        self.seconds += time.perf_counter() - t0

    @property
    def soa(self):
        """the evaluator returns gradients in the engine's component-major layout on request"""
        return self.async_ and getattr(self.field, "soa_grad", False)

    def collect(self, raise_=True):
        """-> (alpha, J), or (alpha, J, status) with raise_=False (see ObstacleField.collect)."""
        t0 = time.perf_counter()
        poses, grad = self._job
        self._job = None
        kw = {} if (raise_ or not self.has_raise) else {"raise_": False}
        if self.soa:
            out = self.field.collect(soa=True, **kw)
        else:
            out = self.field.collect(**kw) if self.async_ else self.field.evaluate(poses, grad, **kw)
        if not raise_ and not kw:       # a two-value evaluator: it raised on a failed pair already
            out = (out[0], out[1], np.zeros(np.shape(out[0]), dtype=np.int32))
        self.seconds += time.perf_counter() - t0
        self.batches += 1
        self.pairs += poses.shape[0] * out[0].shape[1]
        return out


def _masked(dual, h):
    """Active-set mask of the AL penalty: mu > 0 or h > 0 (ALTRO.py:16-31)."""
    return ((dual > 0) | (h > 0)).astype(np.float64)


class _Problem:
    """A reference params dict as native structs (dcol_altro_model / dcol_altro_problem)."""

    def __init__(self, params):
        self.params = params
        self.sys = _systems.get(params["system"])
        self.N, self.nx, self.nu = int(params["N"]), int(params["nx"]), int(params["nu"])
        self.ncx = len(params["P_obs"])
        self.Xref = np.asarray(params["Xref"], dtype=np.float64).reshape(-1, self.nx)[: self.N]
        self.u_max = np.asarray(params["u_max"], dtype=np.float64)
        self.u_min = np.asarray(params["u_min"], dtype=np.float64)
        self.model = self.sys.native_model(params)
        self.prob = _native.make_problem(
            self.N, self.nx, self.nu, self.ncx, params["Q"], params["R"], params["Qf"], self.Xref,
            np.asarray(params["Uref"], dtype=np.float64).reshape(-1, self.nu)[: self.N - 1], self.u_min, self.u_max)

    def hu(self, U):
        return np.concatenate([U - self.u_max, -U + self.u_min], axis=1)

    def cost(self, X, U, hx, mu, mux, lam, rho):
        """compute_total_cost (ALTRO.py:103-145)."""
        return _native.cost(self.prob, X, U, hx, mu, mux, lam, rho)


def _print_iter(itr, J, dJ, kmax, a, reg, rho):
    if itr % 50 == 0:
        print("iter     J           ΔJ        |d|         α        reg         ρ")
        print("---------------------------------------------------------------------")
    print(f"{itr+1:3d}   {J:10.3e}  {dJ:9.2e}  {kmax:9.2e}  {a:6.4f}   {reg:9.2e}   {rho:9.2e}")


def solve(params, X, U, prox=None, engine=None, verbose=True, prox_wide=None) -> AltroResult:
    """Run the batched ALTRO on a reference-style problem.

    params/X/U: as returned by altro.systems.<system>.initialize() (or the reference's own
    initialize_<system>()).  prox: constraint evaluator with
    ``evaluate(victim_poses [N, 6], grad) -> (alpha [N, n_obs], J [N, n_obs, 12] | None)``
    that raises (like the reference) on a failed pair; default: an ObstacleField on the GPU
    (constraints.py).  prox_wide: the same evaluator over TRIALS * N knots (line-search
    retries, TRIALS trajectories per batch); default: an ObstacleField when prox is None,
    else retries go through prox one at a time.  The retries are read with
    ``evaluate(..., raise_=False)`` (or ``collect(raise_=False)``) ->
    ``(alpha, J, status [N, n_obs] int32)`` when the evaluator takes that keyword, so that a
    failed pair raises only if its trial is the one the reference would evaluate; an
    evaluator without it is called the two-value way (it raises on any failed pair of the
    batch, and its status is taken as all zero).
    params['reg'] / ['rho'] /
    ['X_hist'] / ['U_hist'] are updated in place like the reference does."""
    t_setup = time.perf_counter()
    P = _Problem(params)
    N, nx, nu = P.N, P.nx, P.nu
    X = np.array(X, dtype=np.float64).reshape(N, nx)
    U = np.array(U, dtype=np.float64).reshape(N - 1, nu)
    wide = _Timed(prox_wide) if prox_wide is not None else None
    if prox is None:
        from .constraints import ObstacleField
        prox = ObstacleField(params["P_vic"], params["P_obs"], N, engine=engine)
        # the same pairing over TRIALS stacked trajectories: the retries of a line search
        # after a rejected full step, TRIALS step lengths per batch
        wide = _Timed(ObstacleField(params["P_vic"], params["P_obs"], TRIALS * N, engine=engine))
    evaluate = _Timed(prox)
    # dynamics Jacobians: on the GPU beside the constraint batches when those run there
    stream = getattr(prox, "stream", None)
    jac = _jacobians.provider(P.model, N - 1, stream.device.index if stream is not None else None,
                              os.environ.get("DCOL_ALTRO_JAC", "device"))
    t_start = time.perf_counter()          # one-time set-up (shape table, plan, warm-up) excluded
    ncx = P.ncx
    if int(params.get("ncx", ncx)) != ncx or int(params.get("ncu", 2 * nu)) != 2 * nu:
        raise AssertionError("ncx / ncu do not match the problem")

    # initial rollout (ALTRO.py:407-409)
    X, U = _native.rollout(P.model, X, U, np.zeros((N - 1, nu, nx)), np.zeros((N - 1, nu)), 0.0)
    params.setdefault("X_hist", []).append(X)
    params.setdefault("U_hist", []).append(U)

    mu = np.zeros((N - 1, 2 * nu))
    mux = np.zeros((N, ncx))
    lam = np.zeros(nx)
    res = AltroResult(X=X, U=U, converged=False, iterations=0, jacobians=jac.where)
    hx_cur = None            # 1 - alpha at the current X, when known from the last accepted trial
    # (alpha, d alpha, A, B) at the current (X, U): every line-search trial is solved WITH
    # gradients and its dynamics Jacobians are computed on the host while the GPU batch runs,
    # so the accepted trial hands the next backward pass everything it would recompute from
    # the same (X, U) (ALTRO.py:77-100, :268-300)
    at_x = None
    max_iters = int(params["max_iters"])
    for itr in range(max_iters):
        rho, reg = float(params["rho"]), float(params["reg"])   # mutated in place, like the reference
        res.reg.append(reg)
        res.rho.append(rho)
        # ---------------------------------------------------------------- backward pass
        if at_x is None:
            evaluate.submit(_native.victim_poses(P.model, X), True)
            jac.submit(X, U)                                         # beside the batch
            alpha, Jp = evaluate.collect()
            at_x = (alpha, Jp) + jac.collect()
        alpha, Jp, A, B = at_x
        hx = 1 - alpha
        # constraint Jacobian, stage terms, Riccati sweep and the cost of (X, U): one call
        # (gradients in the engine's [12, N ncx] layout when they came from the GPU batch)
        K, k, dJ, old = _native.backward_pass(P.model, P.prob, X, U, alpha, Jp, A, B, mu, mux, lam, rho, reg,
                                              soa=Jp.ndim == 2)
        # ---------------------------------------------------------------- forward pass
        a, J, accepted = 1.0, old, False
        n_ls = int(params["max_linesearch_iters"])
        tried = 0
        while tried < n_ls and not accepted:
            if tried == 0 or wide is None:
                # the full step (accepted in most iterations), or every trial when no wide
                # evaluator exists: one trajectory, Jacobians overlapped with its batch
                Xn, Un, poses = _native.trial(P.model, X, U, K, k, a)
                evaluate.submit(poses, True)
                jac.submit(Xn, Un)                                   # beside the batch
                an, Jn = evaluate.collect()
                An, Bn = jac.collect()
                hxn = 1 - an
                new = P.cost(Xn, Un, hxn, mu, mux, lam, rho)
                tried += 1
                if new < old:
                    X, U, J, accepted, hx_cur = Xn, Un, new, True, hxn
                    at_x = (an, Jn, An, Bn)
                else:
                    a *= 0.5
                continue
            # retries: the next TRIALS step lengths of the reference's halving sequence in
            # one batch; the first one that lowers the cost is taken, exactly as trying them
            # one at a time would (later ones are discarded).  A failed pair raises only when
            # its trial is the one being evaluated: trials after the accepted one, or past
            # max_linesearch_iters, are never looked at by the reference.
            w = min(TRIALS, n_ls - tried)
            steps = [a * 0.5 ** j for j in range(TRIALS)]
            Xs, Us = _native.rollouts(P.model, X, U, K, k, steps)
            wide.submit(_native.victim_poses(P.model, Xs.reshape(-1, nx)), True)
            ans, Jns, sts = wide.collect(raise_=False)
            ans = ans.reshape(TRIALS, N, ncx)
            sts = sts.reshape(TRIALS, N * ncx)
            if not wide.soa:
                Jns = Jns.reshape(TRIALS, N, ncx, 12)
            for j in range(w):
                if sts[j].any():            # knot-major first failure of this trial
                    raise_for_status(int(sts[j][np.flatnonzero(sts[j])[0]]))
                hxn = 1 - ans[j]
                new = P.cost(Xs[j], Us[j], hxn, mu, mux, lam, rho)
                tried += 1
                if new < old:
                    X, U, J, accepted, hx_cur = Xs[j], Us[j], new, True, hxn
                    jac.submit(X, U)
                    Jj = Jns[:, j * N * ncx:(j + 1) * N * ncx] if wide.soa else Jns[j]
                    at_x = (ans[j].copy(), Jj.copy()) + jac.collect()
                    break
                a *= 0.5
        if not accepted:
            log.warning("Forward pass failed to reduce cost after line search, increasing reg")
            a, hx_cur = 0.0, hx
        params["X_hist"].append(X)
        params["U_hist"].append(U)
        # ---------------------------------------------------- regularisation (ALTRO.py:51-74)
        if a == 0.0:
            if reg == params["reg_max"]:
                raise ValueError("Regularization parameter reached maximum value.")
            params["reg"] = min(params["reg_max"], reg * 10)
        elif a == 1.0:
            params["reg"] = max(params["reg_min"], reg / 10)
        kmax = float(np.max(np.linalg.norm(k, axis=1))) if len(k) else 0.0
        kmax = max(0.0, kmax)
        res.J.append(J)
        res.delta_J.append(dJ)
        res.kmax.append(kmax)
        res.alpha.append(a)
        res.iterations = itr + 1
        if verbose:
            _print_iter(itr, J, dJ, kmax, a, params["reg"], rho)
        # ------------------------------------------------------ AL update (ALTRO.py:444-481)
        if a > 0 and kmax < params["atol"]:
            hu = P.hu(U)
            mu = np.maximum(0, mu + rho * (_masked(mu, hu) * hu))
            mux = np.maximum(0, mux + rho * (_masked(mux, hx_cur) * hx_cur))
            g = X[-1] - P.Xref[-1]
            lam = lam + rho * g
            convio = max(float(np.max(np.abs(hu + np.abs(hu)))) if hu.size else 0.0,
                         float(np.max(np.abs(hx_cur + np.abs(hx_cur)))) if hx_cur.size else 0.0,
                         float(np.max(np.abs(g))))
            res.convio.append((itr, convio))
            if convio < params["convio_tol"]:
                log.info(f"Convergence reached in {itr} iterations.")
                res.converged = True
                break
            log.info(f"convio: {convio}, increasing penalty parameter")
            params["rho"] = rho * params["phi"]
    else:
        log.info("iLQR optimization complete without convergence")
    res.X, res.U = X, U
    res.wall_s = time.perf_counter() - t_start
    res.setup_s = t_start - t_setup
    res.prox_s, res.prox_batches, res.prox_pairs = evaluate.seconds, evaluate.batches, evaluate.pairs
    if wide is not None:
        res.prox_s += wide.seconds
        res.prox_batches += wide.batches
        res.prox_pairs += wide.pairs
    return res


def ALTRO(params, X, U, prox=None, engine=None, verbose=True):
    """Drop-in for the reference's ALTRO(params, X, U) (ALTRO.py:365-488): returns the
    optimised (X, U) as lists of per-knot arrays."""
    r = solve(params, X, U, prox=prox, engine=engine, verbose=verbose)
    return [x.copy() for x in r.X], [u.copy() for u in r.U]
