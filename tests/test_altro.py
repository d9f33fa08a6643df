"""Batched ALTRO driver.

CPU: the native host library (lib/libdcol_altro.so) against the NumPy restatement of the
reference's per-knot math (oracle/altro_oracle.py), and whole optimizer runs — driver +
C-oracle constraint evaluator — against runs of the reference itself recorded in
tests/golden/altro/altro_<system>.npz (gen_altro.py).  GPU: the same runs with the constraints
solved by the HIP engine (altro.constraints.ObstacleField).

Whole-run parity criteria.  The iterates pass through forward-difference Jacobians
(delta 1e-6 on the dynamics, sqrt(eps) on the proximity gradient), which amplify
last-bit differences by 1e6-1e8; so bit-exact iterates are not a meaningful target, and
the run is compared on its discrete decisions — number of outer iterations, every
line-search step, the regularisation and penalty schedules, convergence — plus the cost
sequence (rel 1e-6) and the final trajectory (abs 1e-6 on X, 1e-4 on U).
"""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG, REPO, gpu_available

HEADER = os.path.join(REPO, "include", "dcol_altro.h")


def _native():
    from altro import _native
    return _native


def declared_functions():
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(dcol_altro_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    nat = _native()
    lib = nat.load()
    assert set(nat.SIGNATURES) == set(declared_functions())
    out = subprocess.run(["nm", "-D", "--defined-only", nat.LIB_PATH], capture_output=True, text=True).stdout
    assert set(declared_functions()) <= set(re.findall(r" T (dcol_altro_\w+)", out))
    assert lib.dcol_altro_abi_version() == nat.ABI_VERSION


def test_missing_library_fails_loudly(tmp_path):
    nat = _native()
    with pytest.raises(nat.AltroLibraryError):
        nat.load(str(tmp_path / "nope.so"))


# ------------------------------------------------------------------ native host kernels
def _models():
    from altro.systems import cone_through_wall as cone
    from oracle import altro_oracle as ao
    nat = _native()
    mass, J = cone.mass_properties(cone.ConeMRP(height=2.0, beta=np.radians(22)))
    return {
        "piano": (nat.make_model(nat.SYS_PIANO, 6, 3, 0.1, u_scale=100.0), ao.dynamics_piano, 6, 3),
        "quadrotor": (nat.make_model(nat.SYS_QUADROTOR, 12, 4, 0.08, mass=0.5, inertia=np.diag([0.0023, 0.0023, 0.004]),
                                     gravity=(0, 0, -9.81), arm=0.175, kf=1.0, km=0.0245), ao.dynamics_quadrotor, 12, 4),
        "rigid": (nat.make_model(nat.SYS_RIGID, 12, 6, 0.1, mass=mass, inertia=J),
                  lambda x, u: ao.dynamics_rigid(x, u, mass, J), 12, 6),
    }


@pytest.mark.parametrize("name", ["piano", "quadrotor", "rigid"])
def test_dynamics_matches_reference_math(name):
    from oracle import altro_oracle as ao
    model, f, nx, nu = _models()[name]
    rng = np.random.default_rng(7)
    X = rng.normal(size=(64, nx))
    U = rng.normal(size=(64, nu)) * (3 if name == "quadrotor" else 1)
    got = _native().dynamics(model, X, U)
    want = np.array([ao.rk4(f, X[i], U[i], model.dt) for i in range(64)])
    np.testing.assert_allclose(got, want, rtol=1e-13, atol=1e-14)


@pytest.mark.parametrize("name", ["piano", "quadrotor", "rigid"])
def test_fd_jacobians_match_reference_math(name):
    from oracle import altro_oracle as ao
    model, f, nx, nu = _models()[name]
    rng = np.random.default_rng(8)
    T = 9
    X = rng.normal(size=(T + 1, nx)) * 0.5
    U = rng.normal(size=(T, nu))
    A, B = _native().jacobians(model, X, U)
    for t in range(T):
        Aw = ao.fd_jacobian(lambda x_: ao.rk4(f, x_, U[t], model.dt), X[t])
        Bw = ao.fd_jacobian(lambda u_: ao.rk4(f, X[t], u_, model.dt), U[t])
        # forward differences with delta 1e-6: last-bit differences of the dynamics show up
        # at ~1e-10 absolute
        np.testing.assert_allclose(A[t], Aw, rtol=0, atol=1e-8)
        np.testing.assert_allclose(B[t], Bw, rtol=0, atol=1e-8)


def _spd(rng, n, shift):
    M = rng.normal(size=(n, n))
    return M @ M.T + shift * np.eye(n)


@pytest.mark.parametrize("nx,nu,T", [(6, 3, 12), (12, 4, 20), (12, 6, 7), (7, 2, 9)])   # last: generic sizes
def test_riccati_matches_reference_math(nx, nu, T):
    from oracle import altro_oracle as ao
    rng = np.random.default_rng(nx * 100 + nu)
    A = np.eye(nx) + 0.1 * rng.normal(size=(T, nx, nx))
    B = 0.1 * rng.normal(size=(T, nx, nu))
    lx, lu = rng.normal(size=(T, nx)), rng.normal(size=(T, nu))
    lxx = np.array([_spd(rng, nx, 1.0) for _ in range(T)])
    luu = np.array([_spd(rng, nu, 0.5) for _ in range(T)])
    VxT, VxxT = rng.normal(size=nx), _spd(rng, nx, 1.0)
    K, k, dJ = _native().backward(A, B, lx, lu, lxx, luu, VxT, VxxT, 1e-3)
    Kw, kw, dJw = ao.riccati(A, B, lx, lu, lxx, luu, VxT, VxxT, 1e-3)
    np.testing.assert_allclose(K, Kw, rtol=1e-9, atol=1e-11)
    np.testing.assert_allclose(k, kw, rtol=1e-9, atol=1e-11)
    assert abs(dJ - dJw) <= 1e-9 * abs(dJw)


def test_riccati_not_pd_raises_linalgerror():
    nx, nu, T = 6, 3, 4
    A = np.tile(np.eye(nx), (T, 1, 1))
    B = np.zeros((T, nx, nu))
    luu = np.tile(-np.eye(nu), (T, 1, 1))            # Quu = luu: negative definite
    with pytest.raises(np.linalg.LinAlgError, match="knot 3"):
        _native().backward(A, B, np.zeros((T, nx)), np.zeros((T, nu)), np.tile(np.eye(nx), (T, 1, 1)), luu,
                           np.zeros(nx), np.eye(nx), 0.0)


@pytest.mark.parametrize("name", ["piano", "quadrotor", "rigid"])
def test_rollout_matches_reference_math(name):
    from oracle import altro_oracle as ao
    model, f, nx, nu = _models()[name]
    rng = np.random.default_rng(9)
    T = 15
    X = rng.normal(size=(T + 1, nx)) * 0.3
    U = rng.normal(size=(T, nu)) * 0.1 + (1.226 if name == "quadrotor" else 0.0)   # near hover
    K = 0.01 * rng.normal(size=(T, nu, nx))
    k = 0.1 * rng.normal(size=(T, nu))
    Xn, Un = _native().rollout(model, X, U, K, k, 0.5)
    Xw, Uw = ao.rollout(lambda x, u: ao.rk4(f, x, u, model.dt), X, U, K, k, 0.5)
    np.testing.assert_allclose(Xn, Xw, rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(Un, Uw, rtol=1e-12, atol=1e-13)


def test_bad_arguments_rejected():
    nat = _native()
    bad = nat.make_model(nat.SYS_PIANO, 6, 4, 0.1, u_scale=100.0)    # piano has nu = 3
    with pytest.raises(ValueError):
        nat.dynamics(bad, np.zeros((1, 6)), np.zeros((1, 4)))


# ------------------------------------------------------------------ systems set-up
@pytest.mark.parametrize("name", ["piano_mover", "coneThroughWall", "quadrotor"])
def test_initial_problem_matches_reference(name):
    from altro import systems
    g = np.load(os.path.join(GOLDEN, "altro", f"altro_{name}.npz"))
    params, X, U = systems.initialize(name)
    assert np.array_equal(np.array(X), g["X0"])
    assert np.array_equal(np.array(U), g["U0"])
    assert np.array_equal(np.array([np.asarray(o.r, float) for o in params["P_obs"]]), g["obs_r"])
    assert np.array_equal(np.array([np.asarray(o.p, float) for o in params["P_obs"]]), g["obs_p"])


# ------------------------------------------------------------------ whole runs
def check_run(r, g):
    n = int(g["iterations"])
    assert r.converged
    assert r.iterations == n
    assert np.array_equal(np.array(r.alpha), g["alpha"])          # every line-search step
    assert np.array_equal(np.array(r.reg), g["reg"])              # regularisation schedule
    assert np.array_equal(np.array(r.rho), g["rho"])              # penalty schedule
    np.testing.assert_allclose(r.J, g["J"], rtol=1e-6)
    np.testing.assert_allclose(r.X, g["X"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(r.U, g["U"], rtol=0, atol=1e-4)


@pytest.mark.parametrize("name", ["piano_mover", "coneThroughWall", "quadrotor"])
def test_altro_run_matches_reference_cpu_evaluator(name):
    from altro import solve, systems
    from altro_cpu import OracleField
    g = np.load(os.path.join(GOLDEN, "altro", f"altro_{name}.npz"))
    params, X, U = systems.initialize(name)
    r = solve(params, X, U, prox=OracleField(params["P_vic"], params["P_obs"], params["N"]), verbose=False)
    check_run(r, g)
    assert params["rho"] == float(g["rho_final"]) and params["reg"] == float(g["reg_final"])


def test_altro_wide_line_search_matches_reference_cpu_evaluator():
    """Line-search retries batched TRIALS step lengths at a time (prox_wide) take exactly the
    reference's decisions: the quadrotor run (13 iterations with retries, down to a = 1/512)
    against its whole-run fixture."""
    from altro import solve, systems
    from altro.driver import TRIALS
    from altro_cpu import OracleField
    g = np.load(os.path.join(GOLDEN, "altro", "altro_quadrotor.npz"))
    params, X, U = systems.initialize("quadrotor")
    N = params["N"]
    r = solve(params, X, U, prox=OracleField(params["P_vic"], params["P_obs"], N),
              prox_wide=OracleField(params["P_vic"], params["P_obs"], TRIALS * N), verbose=False)
    check_run(r, g)
    trials = np.log2(1 / np.array(r.alpha)) + 1
    assert r.prox_batches == 1 + int(np.sum(1 + np.ceil((trials - 1) / TRIALS)))


def _poisoned_wide(params, N, golden_alpha, poison_accepted):
    """A wide (TRIALS-trajectory) oracle evaluator that marks every pair of the trials the
    reference never evaluates (after the accepted one) as failed (MAXITER); with
    poison_accepted the accepted trial itself fails instead."""
    from altro.driver import TRIALS
    from altro_cpu import OracleField
    from dcol_amd import _lib
    # per retry batch: index of the accepted trial in it (None: all TRIALS tried, none accepted)
    plan = []
    n_ls = int(params["max_linesearch_iters"])
    for a in golden_alpha:
        if a == 0:                          # failed line search: every batch tried, none accepted
            plan += [None] * (-(-(n_ls - 1) // TRIALS))
            continue
        t = int(round(np.log2(1 / a))) + 1
        if t == 1:
            continue
        nb = -(-(t - 1) // TRIALS)
        plan += [None] * (nb - 1) + [(t - 2) % TRIALS]

    class Poisoned(OracleField):
        batch = 0

        def evaluate(self, poses, grad, raise_=True):
            a, J, st = super().evaluate(poses, grad, raise_=False)
            j_acc = plan[Poisoned.batch]
            Poisoned.batch += 1
            st = st.reshape(TRIALS, -1).copy()
            if j_acc is not None:
                if poison_accepted:
                    st[j_acc, 7] = _lib.MAXITER
                else:
                    st[j_acc + 1:] = _lib.MAXITER
            st = st.reshape(a.shape)
            if raise_ and st.any():
                from dcol_amd.engine import raise_for_status
                raise_for_status(int(st.ravel()[np.flatnonzero(st)[0]]))
            return (a, J) if raise_ else (a, J, st)
    return Poisoned(params["P_vic"], params["P_obs"], TRIALS * N)


def test_wide_line_search_ignores_failures_of_unevaluated_trials():
    """a retry batch solves TRIALS step lengths at once; a failure in a trial the
    reference would never evaluate (after the accepted one) must not abort the run, while a
    failure in the accepted trial raises like the reference (PDIPFailure, pdip.py:470)."""
    from altro import solve, systems
    from altro_cpu import OracleField
    from dcol_amd.engine import PDIPFailure
    g = np.load(os.path.join(GOLDEN, "altro", "altro_quadrotor.npz"))
    params, X, U = systems.initialize("quadrotor")
    N = params["N"]
    r = solve(params, X, U, prox=OracleField(params["P_vic"], params["P_obs"], N),
              prox_wide=_poisoned_wide(params, N, g["alpha"], False), verbose=False)
    check_run(r, g)
    params, X, U = systems.initialize("quadrotor")
    with pytest.raises(PDIPFailure):
        solve(params, X, U, prox=OracleField(params["P_vic"], params["P_obs"], N),
              prox_wide=_poisoned_wide(params, N, g["alpha"], True), verbose=False)


def test_wide_two_value_evaluator_contract():
    """a prox_wide evaluator written against the two-value contract
    (evaluate(poses, grad) -> (alpha, J), no raise_ keyword) still drives the batched
    retries -- called the old way, status taken as all zero -- with the reference's decisions."""
    from altro import solve, systems
    from altro.driver import TRIALS
    from altro_cpu import OracleField

    class TwoValue(OracleField):
        def evaluate(self, poses, grad):
            return super().evaluate(poses, grad)
    g = np.load(os.path.join(GOLDEN, "altro", "altro_quadrotor.npz"))
    params, X, U = systems.initialize("quadrotor")
    N = params["N"]
    r = solve(params, X, U, prox=OracleField(params["P_vic"], params["P_obs"], N),
              prox_wide=TwoValue(params["P_vic"], params["P_obs"], TRIALS * N), verbose=False)
    check_run(r, g)


def test_reg_max_raises_like_reference():
    """update_reg (ALTRO.py:51-74): a failed line search at reg == reg_max is a ValueError."""
    from altro import solve, systems
    from altro_cpu import OracleField

    class Worse(OracleField):
        calls = 0

        def evaluate(self, poses, grad):
            a, J = super().evaluate(poses, grad)
            Worse.calls += 1
            return (a if Worse.calls == 1 else a * 0 - 1e6), J       # every trial looks infeasible
    params, X, U = systems.initialize("piano_mover")
    params["reg"] = params["reg_max"]
    params["max_linesearch_iters"] = 2
    with pytest.raises(ValueError, match="maximum value"):
        solve(params, X, U, prox=Worse(params["P_vic"], params["P_obs"], params["N"]), verbose=False)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["piano_mover", "coneThroughWall", "quadrotor"])
def test_altro_run_matches_reference_gpu(name):
    if not gpu_available():
        pytest.skip("no GPU")
    from altro import solve, systems
    g = np.load(os.path.join(GOLDEN, "altro", f"altro_{name}.npz"))
    params, X, U = systems.initialize(name)
    r = solve(params, X, U, verbose=False)
    assert r.jacobians == "device"   # dynamics Jacobians batched over knots on the GPU (section 8 f3)
    check_run(r, g)
    # one batch for the first backward pass, then per iteration one for the full step and one
    # per TRIALS retries after it: every accepted trial's batch (with gradients) serves the
    # next backward pass
    from altro.driver import TRIALS
    trials = np.log2(1 / np.array(r.alpha)) + 1
    assert r.prox_batches == 1 + int(np.sum(1 + np.ceil((trials - 1) / TRIALS)))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["piano_mover", "quadrotor", "coneThroughWall"])
def test_obstacle_field_matches_oracle(name):
    if not gpu_available():
        pytest.skip("no GPU")
    from altro import systems
    from altro.constraints import ObstacleField
    from altro_cpu import OracleField
    from conftest import alpha_close, grad_close
    params, X, U = systems.initialize(name)
    mod = systems.get(name)
    rng = np.random.default_rng(3)
    Xs = np.array(params["Xref"], dtype=np.float64) + 0.05 * rng.normal(size=(params["N"], params["nx"]))
    poses = mod.victim_poses(params, Xs)
    gpu = ObstacleField(params["P_vic"], params["P_obs"], params["N"])
    cpu = OracleField(params["P_vic"], params["P_obs"], params["N"])
    a, J = gpu.evaluate(poses, True)
    aw, Jw = cpu.evaluate(poses, True)
    assert alpha_close(a, aw).all()
    assert grad_close(J.reshape(-1, 12), Jw.reshape(-1, 12)).all()
    a2, none = gpu.evaluate(poses, False)
    assert none is None and np.array_equal(a2, a)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["piano_mover", "quadrotor", "coneThroughWall"])
def test_obstacle_field_phase_modes_bitwise_equal(name, monkeypatch):
    """The three ways a phase reaches the GPU -- zero-copy (kernel reads / writes the pinned
    host buffers), one hipGraph replay of H2D + solve + D2H, and the eager calls -- give the
    same bits, submit/collect split or not."""
    if not gpu_available():
        pytest.skip("no GPU")
    from altro import systems
    from altro.constraints import ObstacleField
    from altro_cpu import OracleField
    from conftest import alpha_close, grad_close
    params, X, U = systems.initialize(name)
    mod = systems.get(name)
    rng = np.random.default_rng(4)
    poses = [mod.victim_poses(params, np.array(params["Xref"], dtype=np.float64)
                              + 0.05 * rng.normal(size=(params["N"], params["nx"]))) for _ in range(3)]
    cpu = OracleField(params["P_vic"], params["P_obs"], params["N"])
    want = [cpu.evaluate(p, True) for p in poses]

    class Counting:
        """graph proxy counting replays (graph mode must replay its captured graph)"""
        def __init__(self, g):
            self.g, self.n = g, 0

        def replay(self):
            self.n += 1
            self.g.replay()

    outs = {}
    for mode in ("zero_copy", "graph", "eager"):
        monkeypatch.setenv("DCOL_ALTRO_PHASE", mode)
        f = ObstacleField(params["P_vic"], params["P_obs"], params["N"])
        f._graphs = {k: Counting(g) for k, g in f._graphs.items()}
        outs[mode] = []
        for i, g in enumerate((True, False, True)):
            f.h_out.fill_(float("nan"))              # stale outputs must never come back
            f.submit(poses[i], g)
            with pytest.raises(RuntimeError, match="in flight"):
                f.submit(poses[i], g)
            outs[mode].append(f.collect())
        assert f.mode == mode or (mode == "zero_copy" and f.mode == "graph")
        if f.mode == "graph":
            assert f._graphs[True].n == 2 and f._graphs[False].n == 1
        for i, (a, J) in enumerate(outs[mode]):      # every mode against the oracle
            assert alpha_close(a, want[i][0]).all(), mode
            if J is not None:
                assert grad_close(J.reshape(-1, 12), want[i][1].reshape(-1, 12)).all(), mode
    for mode in ("graph", "eager"):
        for (a, J), (b, K) in zip(outs["zero_copy"], outs[mode]):
            assert np.array_equal(a, b)
            assert (J is None and K is None) or np.array_equal(J, K)


# ------------------------------------------------------------------ AL objective pieces
def _al_case(name, seed):
    from altro import systems
    rng = np.random.default_rng(seed)
    params, X, U = systems.initialize(name)
    N, nx, nu, nc = params["N"], params["nx"], params["nu"], len(params["P_obs"])
    X = np.array(params["Xref"], dtype=float) + 0.3 * rng.normal(size=(N, nx))
    U = np.array(U, dtype=float) + 0.5 * rng.normal(size=(N - 1, nu))
    hx = rng.normal(size=(N, nc)) * 0.3
    Gx = rng.normal(size=(N, nc, nx))
    mu = np.maximum(0, rng.normal(size=(N - 1, 2 * nu)))
    mux = np.maximum(0, rng.normal(size=(N, nc)))
    lam = rng.normal(size=nx)
    Uref = np.asarray(params["Uref"], dtype=float)[: N - 1]
    args = (np.asarray(params["Q"], float), np.asarray(params["R"], float), np.asarray(params["Qf"], float),
            np.asarray(params["Xref"], float), Uref, params["u_min"], params["u_max"])
    return params, args, X, U, hx, Gx, mu, mux, lam


@pytest.mark.parametrize("name", ["piano_mover", "coneThroughWall", "quadrotor"])
def test_al_cost_and_stage_terms_match_reference_math(name):
    from altro import _native
    from oracle import altro_oracle as ao
    params, args, X, U, hx, Gx, mu, mux, lam = _al_case(name, 11)
    prob = _native.make_problem(params["N"], params["nx"], params["nu"], hx.shape[1], *args)
    for rho in (1.0, 1e4):
        J = _native.cost(prob, X, U, hx, mu, mux, lam, rho)
        Jw = ao.al_cost(*args, X, U, hx, mu, mux, lam, rho)
        assert abs(J - Jw) <= 1e-12 * abs(Jw)
        got = _native.stage_terms(prob, X, U, hx, Gx, mu, mux, lam, rho)
        want = ao.stage_terms(*args, X, U, hx, Gx, mu, mux, lam, rho)
        for a, b in zip(got, want):
            np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12 * max(1.0, np.abs(b).max()))


def test_backward_pass_component_major_gradients_equal():
    """dcol_altro_backward_pass on the engine's [12, N ncx] gradient layout (what the GPU
    batch returns) equals the call on [N, ncx, 12]: same K, k, dJ, J bitwise."""
    from altro import _native as nat
    from altro import systems
    from altro.driver import _Problem
    params, X, U = systems.initialize("quadrotor")
    P = _Problem(params)
    N, nx, nu, ncx = P.N, P.nx, P.nu, P.ncx
    rng = np.random.default_rng(11)
    X = np.asarray(X, dtype=np.float64).reshape(N, nx) + 0.01 * rng.normal(size=(N, nx))
    U = np.asarray(U, dtype=np.float64).reshape(N - 1, nu)
    alpha = 1 + rng.uniform(0.0, 2.0, size=(N, ncx))
    J = rng.normal(size=(N, ncx, 12))
    A, B = nat.jacobians(P.model, X, U)
    args = (np.zeros((N - 1, 2 * nu)), np.zeros((N, ncx)), np.zeros(nx), 1.0, 1e-6)
    r0 = nat.backward_pass(P.model, P.prob, X, U, alpha, J, A, B, *args)
    r1 = nat.backward_pass(P.model, P.prob, X, U, alpha, np.ascontiguousarray(J.reshape(-1, 12).T), A, B, *args,
                           soa=True)
    for a, b in zip(r0, r1):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    with pytest.raises(ValueError):
        nat.backward_pass(P.model, P.prob, X, U, alpha, J.reshape(-1, 12), A, B, *args, soa=True)


@pytest.mark.parametrize("name", ["piano_mover", "quadrotor"])
def test_pose_map_and_constraint_jacobian(name):
    from altro import _native, systems
    from oracle import altro_oracle as ao
    params, X, U = systems.initialize(name)
    rng = np.random.default_rng(5)
    X = np.array(params["Xref"], dtype=float) + 0.4 * rng.normal(size=(params["N"], params["nx"]))
    J = rng.normal(size=(params["N"], len(params["P_obs"]), 12))
    m = systems.get(name).native_model(params)
    P = _native.victim_poses(m, X)
    G = _native.constraint_jacobian(m, X, J)
    if name == "piano_mover":
        np.testing.assert_allclose(P, ao.victim_poses_piano(X), rtol=1e-15, atol=0)
        np.testing.assert_allclose(G, ao.constraint_jacobian_piano(X, J), rtol=1e-14, atol=1e-15)
    else:
        np.testing.assert_array_equal(P, np.concatenate([X[:, :3], X[:, 6:9]], axis=1))
        np.testing.assert_array_equal(G, ao.constraint_jacobian_rigid(J))
    # the system module's NumPy forms (per-knot reference interface) agree too
    mod = systems.get(name)
    np.testing.assert_allclose(mod.victim_poses(params, X), P, rtol=1e-15, atol=0)
    np.testing.assert_allclose(mod.state_jacobian(params, X, J), G, rtol=1e-14, atol=1e-15)
