"""Case-4 pairs (both primitives with extra columns: capsule / cylinder / polygon x capsule /
cylinder / polygon) — an opt-in EXTENSION (DCOL_PLAN_CASE4).  The
reference raises ValueError for them (combine_problem_matrices.py:58-67), so there is no
reference output: the oracle's right-padded assembly (oracle.dcol_oracle.combine(...,
case4=True)) is validated against brute-force geometry (tests/geometry_bruteforce.py),
and the GPU kernel against that oracle.  Parity is therefore pinned to geometry, not to
the reference."""
import numpy as np
import pytest

from conftest import alpha_close, gpu_available, grad_close
from geometry_bruteforce import CAPSULE, CYLINDER, POLYGON, Body, _dcm, min_scaling

KINDS = (CAPSULE, CYLINDER, POLYGON)


def ngon(n, d):
    t = np.linspace(0, 2 * np.pi, n, endpoint=False)
    return np.stack([np.cos(t), np.sin(t)], 1), np.full(n, d)


def case4_table(rng, n_shapes=9):
    """Shape table (tests/golden layout) of capsules, cylinders and polygons, some with
    non-trivial body offsets."""
    tab = {k: [] for k in ("type", "nh", "A_off", "params", "r_offset", "Q_offset")}
    A_rows, b_rows = [], []
    for k in range(n_shapes):
        t = KINDS[k % 3]
        R, L = rng.uniform(0.15, 0.6), rng.uniform(0.4, 2.0)
        tab["type"].append(t)
        tab["A_off"].append(len(b_rows))
        if t == POLYGON:
            A, b = ngon(int(rng.integers(3, 8)), rng.uniform(0.3, 1.0))
            tab["nh"].append(len(b))
            A_rows += [list(a) + [0.0] for a in A]
            b_rows += list(b)
            tab["params"].append((R * 0.5, 0, 0, 0))
        else:
            tab["nh"].append(0)
            tab["params"].append((R, L, 0, 0))
        off = k % 4 == 3
        tab["r_offset"].append(rng.uniform(-0.3, 0.3, 3) if off else np.zeros(3))
        tab["Q_offset"].append(_dcm(rng.uniform(-0.5, 0.5, 3)) if off else np.eye(3))
    out = {k: np.array(v) for k, v in tab.items()}
    out["type"] = out["type"].astype(np.int32)
    out["nh"] = out["nh"].astype(np.int32)
    out["A_off"] = out["A_off"].astype(np.int32)
    out["A_pool"] = np.array(A_rows, dtype=np.float64).reshape(-1, 3)
    out["b_pool"] = np.array(b_rows, dtype=np.float64)
    return out


def body(tab, k, pose):
    t = int(tab["type"][k])
    R, L = tab["params"][k][0], tab["params"][k][1]
    A = b = None
    if t == POLYGON:
        o, n = int(tab["A_off"][k]), int(tab["nh"][k])
        A, b = tab["A_pool"][o:o + n, :2], tab["b_pool"][o:o + n]
    return Body(t, pose, R=R, L=L, A=A, b=b, r_offset=tab["r_offset"][k], Q_offset=tab["Q_offset"][k])


def pairs(rng, tab, B):
    S = len(tab["type"])
    s1 = rng.integers(0, S, B).astype(np.int32)
    s2 = rng.integers(0, S, B).astype(np.int32)
    p1 = np.hstack([rng.uniform(-1.5, 1.5, (B, 3)), rng.uniform(-1, 1, (B, 3))])
    p2 = np.hstack([rng.uniform(-1.5, 1.5, (B, 3)), rng.uniform(-1, 1, (B, 3))])
    return s1, s2, p1, p2


def test_dcm_matches_oracle():
    from oracle import dcol_oracle as O
    rng = np.random.default_rng(0)
    for _ in range(20):
        p = rng.uniform(-1.5, 1.5, 3)
        np.testing.assert_allclose(_dcm(p), O.dcm_from_mrp(p), atol=1e-14)


def test_reference_behaviour_without_option():
    from oracle import dcol_oracle as O
    rng = np.random.default_rng(1)
    tab = case4_table(rng)
    s1, s2, p1, p2 = pairs(rng, tab, 12)
    out = O.run_batch(tab, s1, s2, p1, p2, want_grad=False)
    assert (out["status"] == O.ST_UNSUPPORTED).all()


def test_oracle_case4_matches_bruteforce_geometry():
    """Every ordered combination of capsule / cylinder / polygon once (random poses and
    sizes, some with body offsets)."""
    from oracle import dcol_oracle as O
    rng = np.random.default_rng(2)
    tab = case4_table(rng)
    ids = {t: [k for k in range(len(tab["type"])) if tab["type"][k] == t] for t in KINDS}
    combos = [(a, b) for a in KINDS for b in KINDS]
    s1 = np.array([ids[a][i % len(ids[a])] for i, (a, b) in enumerate(combos)], np.int32)
    s2 = np.array([ids[b][(i + 1) % len(ids[b])] for i, (a, b) in enumerate(combos)], np.int32)
    B = len(combos)
    p1 = np.hstack([rng.uniform(-1.5, 1.5, (B, 3)), rng.uniform(-1, 1, (B, 3))])
    p2 = np.hstack([rng.uniform(-1.5, 1.5, (B, 3)), rng.uniform(-1, 1, (B, 3))])
    # tight pdip_tol: at the default 1e-6 the PDIP exits with a duality gap s'z ~ deg * 1e-6,
    # i.e. alpha above the optimum by up to ~1e-5; the formulation is what is checked here
    out = O.run_batch(tab, s1, s2, p1, p2, tol=1e-11, want_grad=False, case4=True)
    assert (out["status"] == O.ST_OK).all()
    for i in range(B):
        b1, b2 = body(tab, int(s1[i]), p1[i]), body(tab, int(s2[i]), p2[i])
        a = out["alpha"][i]
        c = out["contact"][i]
        # the oracle's point is in both shapes scaled by its alpha ...
        assert max(b1.gauge(c), b2.gauge(c)) <= a * (1 + 1e-9) + 1e-12, i
        # ... and no point needs a smaller scaling (measured agreement ~1e-11)
        a_bf, _ = min_scaling(b1, b2, starts=[c])
        assert abs(a_bf - a) <= 1e-8 * max(1.0, a), (i, combos[i], a_bf, a)


@pytest.mark.gpu
def test_gpu_case4_matches_oracle():
    if not gpu_available():
        pytest.skip("no GPU")
    from dcol_amd import Engine, spec_from_arrays
    from oracle import dcol_oracle as O
    rng = np.random.default_rng(3)
    tab = case4_table(rng, 12)
    s1, s2, p1, p2 = pairs(rng, tab, 400)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    ref = O.run_batch(tab, s1, s2, p1, p2, want_grad=True, case4=True)
    for grad in ("fd", "envelope"):
        res = eng.solve_host(ids[s1], ids[s2], p1, p2, grad=grad, case4=True)
        assert np.array_equal(res.status, ref["status"])
        ok = ref["status"] == O.ST_OK
        assert ok.mean() > 0.95
        assert (res.iters[ok] == ref["iters"][ok]).mean() >= 0.99
        assert alpha_close(res.alpha[ok], ref["alpha"][ok]).all()
        assert grad_close(res.grad[ok], ref["grad"][ok]).all()
    # without the option: the reference's behaviour (ValueError -> UNSUPPORTED)
    res = eng.solve_host(ids[s1], ids[s2], p1, p2, grad=None)
    assert (res.status == 2).all() and np.isnan(res.alpha).all()
    # device-resident plan path gives the same bits as the host path
    import torch
    plan = eng.plan(ids[s1], ids[s2], case4=True)
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).cuda()
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).cuda()
    out = plan.run(d1, d2, grad="fd")
    torch.cuda.synchronize()
    res = eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd", case4=True)
    assert np.array_equal(out["alpha"].cpu().numpy(), res.alpha, equal_nan=True)
