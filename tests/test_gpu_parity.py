"""HIP path (lib/libdcol.so through the C-ABI) against the reference's golden vectors.

Every fixture family: status, Newton iteration count, alpha (1e-6 rel), contact point and
the 12-gradient (1e-5 of max(||g||_inf, 1)) in both gradient modes (FD = the reference's
formulation; envelope = closed form of the same derivative)."""
import numpy as np
import pytest

from conftest import alpha_close, golden_files, grad_close, load_golden

pytestmark = pytest.mark.gpu

FILES = [p for p in golden_files() if not p.endswith("tol0_maxiter.npz")]


def register(engine, d):
    from dcol_amd import spec_from_arrays
    ids = np.array([engine.register(spec_from_arrays(d, k)) for k in range(len(d["type"]))], dtype=np.int32)
    return ids[d["s1"]], ids[d["s2"]]


@pytest.mark.parametrize("mode", ["fd", "envelope"])
@pytest.mark.parametrize("path", FILES, ids=lambda p: p.split("/")[-1][:-4])
def test_golden_parity(engine, path, mode):
    d = load_golden(path)
    s1, s2 = register(engine, d)
    want_grad = not np.all(np.isnan(d["grad"]))
    res = engine.solve_host(s1, s2, d["pose1"], d["pose2"], tol=float(d["tol"]), grad=mode if want_grad else None)
    np.testing.assert_array_equal(res.status, d["status"])
    ok = d["status"] == 0
    # same iterate sequence as the reference (required for 1e-6 alpha parity):
    # Newton iteration counts equal on every pair
    np.testing.assert_array_equal(res.iters[ok], d["iters"][ok])
    assert np.all(alpha_close(res.alpha[ok], d["alpha"][ok]))
    assert np.all(np.abs(res.contact[ok] - d["contact"][ok]) <= 1e-6 * np.maximum(np.abs(d["contact"][ok]), 1.0))
    assert np.all(np.isnan(res.alpha[~ok]))
    if want_grad:
        assert np.all(grad_close(res.grad[ok], d["grad"][ok]))


def test_tol0_degenerate(engine):
    """pdip_tol = 0 can only end in a failure state or mu < 0 (the reference hits a
    non-finite value at mu ~ 1e-300); the engine must terminate with a valid status."""
    d = load_golden([p for p in golden_files() if p.endswith("tol0_maxiter.npz")][0])
    s1, s2 = register(engine, d)
    res = engine.solve_host(s1, s2, d["pose1"], d["pose2"], tol=0.0, grad=None)
    assert set(np.unique(res.status)) <= {0, 1, 3, 4}
    assert np.all(res.iters <= 50)


def test_max_iter_cap(engine):
    d = load_golden([p for p in golden_files() if p.endswith("synthetic_polypoly.npz")][0])
    s1, s2 = register(engine, d)
    res = engine.solve_host(s1[:200], s2[:200], d["pose1"][:200], d["pose2"][:200], max_iter=3, grad="fd")
    assert np.all(res.status == 1) and np.all(res.iters == 3)
    assert np.all(np.isnan(res.alpha)) and np.all(np.isnan(res.grad))


def test_empty_batch(engine):
    res = engine.solve_host(np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros((0, 6)), np.zeros((0, 6)))
    assert res.alpha.shape == (0,)


def test_device_path_matches_host_path(engine):
    """dcol_plan_run on HBM-resident SoA poses == dcol_prox_batch_host, bitwise."""
    import torch
    d = load_golden([p for p in golden_files() if p.endswith("synthetic_mixed.npz")][0])
    s1, s2 = register(engine, d)
    host = engine.solve_host(s1, s2, d["pose1"], d["pose2"], grad="fd")
    plan = engine.plan(s1, s2)
    assert plan.num_buckets > 1           # mixed batch -> several variant buckets
    p1 = torch.from_numpy(np.ascontiguousarray(d["pose1"].T)).cuda()
    p2 = torch.from_numpy(np.ascontiguousarray(d["pose2"].T)).cuda()
    out = plan.run(p1, p2, grad="fd")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["status"].cpu().numpy(), host.status)
    np.testing.assert_array_equal(out["alpha"].cpu().numpy(), host.alpha)
    np.testing.assert_array_equal(out["grad"].cpu().numpy().T, host.grad)
    np.testing.assert_array_equal(out["contact"].cpu().numpy().T, host.contact)
    np.testing.assert_array_equal(out["iters"].cpu().numpy(), host.iters)


@pytest.mark.parametrize("name", ["scene_quad.npz", "synthetic_mixed.npz"])
def test_fused_launch_matches_per_bucket_launches(engine, name):
    """A small mixed plan runs all its buckets in ONE fused launch (dcol_kernels_fused.hip);
    the per-bucket launches (DCOL_PLAN_NO_FUSE) give bitwise the same results."""
    import torch
    d = load_golden([p for p in golden_files() if p.endswith(name)][0])
    s1, s2 = register(engine, d)
    fused = engine.plan(s1, s2, cache=False)
    split = engine.plan(s1, s2, cache=False, fuse=False)
    assert fused.num_buckets == split.num_buckets > 1
    n_reject = int(np.any(d["status"] == 2))          # unsupported pairs: their own launch
    assert fused.num_launches == 1 + n_reject < split.num_launches
    p1 = torch.from_numpy(np.ascontiguousarray(d["pose1"].T)).cuda()
    p2 = torch.from_numpy(np.ascontiguousarray(d["pose2"].T)).cuda()
    a = fused.run(p1, p2, grad="fd")
    b = split.run(p1, p2, grad="fd")
    torch.cuda.synchronize()
    for k in ("status", "iters", "alpha", "grad", "contact"):
        np.testing.assert_array_equal(a[k].cpu().numpy(), b[k].cpu().numpy(), err_msg=k)
    ok = d["status"] == 0
    assert np.all(alpha_close(a["alpha"].cpu().numpy()[ok], d["alpha"][ok]))


def test_large_shape_table_sparse_bucketing():
    """A table of more than 2,048 shapes takes the hashed (shape1, shape2) class cache of
    dcol_capi.cpp: bucket_pairs instead of the dense S x S one; the plan (buckets, slot
    order, variants) and therefore the results must be bitwise those of a small table."""
    from dcol_amd import Engine, ShapeSpec, spec_from_arrays
    d = load_golden([p for p in golden_files() if p.endswith("synthetic_mixed.npz")][0])
    small = Engine()
    a1, a2 = register(small, d)
    big = Engine()
    for k in range(2100):                                   # distinct filler spheres first
        big.register(ShapeSpec(1, R=0.5 + 1e-4 * k))
    ids = np.array([big.register(spec_from_arrays(d, k)) for k in range(len(d["type"]))], dtype=np.int32)
    b1, b2 = ids[d["s1"]], ids[d["s2"]]
    assert len(big._specs) > 2048 and ids.min() >= 2100
    ra = small.solve_host(a1, a2, d["pose1"], d["pose2"], grad="fd")
    rb = big.solve_host(b1, b2, d["pose1"], d["pose2"], grad="fd")
    for k in ("status", "iters", "alpha", "grad", "contact"):
        np.testing.assert_array_equal(getattr(ra, k), getattr(rb, k), err_msg=k)
    ok = d["status"] == 0
    np.testing.assert_array_equal(rb.status, d["status"])
    assert np.all(alpha_close(rb.alpha[ok], d["alpha"][ok]))


def test_host_staging_regrow(engine):
    """dcol_prox_batch_host's pinned staging grows on demand and is reused for smaller
    batches: small -> large -> small again gives the same results as the first call."""
    d = load_golden([p for p in golden_files() if p.endswith("synthetic_polypoly.npz")][0])
    s1, s2 = register(engine, d)
    n = 64
    first = engine.solve_host(s1[:n], s2[:n], d["pose1"][:n], d["pose2"][:n], grad="fd")
    full = engine.solve_host(s1, s2, d["pose1"], d["pose2"], grad="fd")
    again = engine.solve_host(s1[:n], s2[:n], d["pose1"][:n], d["pose2"][:n], grad="fd")
    for k in ("status", "iters", "alpha", "grad", "contact"):
        np.testing.assert_array_equal(getattr(first, k), getattr(again, k), err_msg=k)
    ok = d["status"] == 0
    np.testing.assert_array_equal(full.status, d["status"])
    assert np.all(alpha_close(full.alpha[ok], d["alpha"][ok]))
    assert np.all(grad_close(full.grad[ok], d["grad"][ok]))


def test_native_comm_multi_gpu_world1(engine):
    """C-ABI multi-GPU path (dcol_comm_* + dcol_prox_batch_multi_gpu, RCCL via dlopen) at
    world size 1: the gathered records equal the plan's own outputs bitwise, pad rows NaN.
    (More ranks need more GPUs: RCCL refuses two ranks on one device.)"""
    import torch
    from dcol_amd.dist import REC, NativeComm, unpack
    d = load_golden([p for p in golden_files() if p.endswith("synthetic_mixed.npz")][0])
    s1, s2 = register(engine, d)
    plan = engine.plan(s1, s2)
    p1 = torch.from_numpy(np.ascontiguousarray(d["pose1"].T)).cuda()
    p2 = torch.from_numpy(np.ascontiguousarray(d["pose2"].T)).cuda()
    comm = NativeComm(NativeComm.unique_id(), 1, 0, 0)
    try:
        n = plan.B
        out, rec = comm.solve_gather(plan, p1, p2, cap=n + 7, grad="fd")
        ref = plan.run(p1, p2, grad="fd", contact=False)
        torch.cuda.synchronize()
    finally:
        comm.close()
    rec = rec.cpu().numpy()
    assert rec.shape == (n + 7, REC) and np.all(np.isnan(rec[n:]))
    u = unpack(rec[:n])
    np.testing.assert_array_equal(u["alpha"], ref["alpha"].cpu().numpy())
    np.testing.assert_array_equal(u["grad"], ref["grad"].cpu().numpy().T)
    np.testing.assert_array_equal(u["status"], ref["status"].cpu().numpy())
    np.testing.assert_array_equal(u["iters"], ref["iters"].cpu().numpy())
    np.testing.assert_array_equal(u["status"], d["status"])


@pytest.mark.parametrize("grad", ["fd", "envelope", None])
@pytest.mark.parametrize("fuse", [True, False])
def test_native_comm_in_place_records(engine, grad, fuse):
    """In-place record path of dcol_prox_batch_multi_gpu (rec_local NULL): the solver
    epilogues (and the reject kernel) write the records straight into the gathered buffer.
    Records-only and with the per-pair arrays, fused and per-bucket plans, every gradient
    mode: equal bitwise to the pack-pass path / the plan's own outputs; rows past the shard
    all-ones bytes (NaN, int pair (-1, -1)); gradients NaN without a gradient flag."""
    import torch
    from dcol_amd.dist import REC, NativeComm, unpack
    d = load_golden([p for p in golden_files() if p.endswith("synthetic_mixed.npz")][0])
    s1, s2 = register(engine, d)
    plan = engine.plan(s1, s2, fuse=fuse)
    p1 = torch.from_numpy(np.ascontiguousarray(d["pose1"].T)).cuda()
    p2 = torch.from_numpy(np.ascontiguousarray(d["pose2"].T)).cuda()
    n = plan.B
    comm = NativeComm(NativeComm.unique_id(), 1, 0, 0)
    try:
        _, packed = comm.solve_gather(plan, p1, p2, cap=n + 5, grad=grad)
        junk = torch.full((n + 5, REC), 3.0, dtype=torch.float64, device="cuda")
        none_out, rec_only = comm.solve_gather(plan, p1, p2, cap=n + 5, grad=grad, rec_all=junk.clone(),
                                               in_place=True, soa=False)
        out, rec_soa = comm.solve_gather(plan, p1, p2, cap=n + 5, grad=grad, rec_all=junk.clone(), in_place=True)
        ref = plan.run(p1, p2, grad=grad or None, contact=False)
        torch.cuda.synchronize()
    finally:
        comm.close()
    assert none_out is None
    packed = packed.cpu().numpy()
    for rec in (rec_only.cpu().numpy(), rec_soa.cpu().numpy()):
        assert rec.shape == (n + 5, REC)
        assert np.all(rec[n:].view(np.uint64) == np.uint64(0xFFFFFFFFFFFFFFFF))
        np.testing.assert_array_equal(rec[:n].view(np.uint64), packed[:n].view(np.uint64))
        u = unpack(rec[:n])
        np.testing.assert_array_equal(u["alpha"], ref["alpha"].cpu().numpy())
        np.testing.assert_array_equal(u["status"], ref["status"].cpu().numpy())
        np.testing.assert_array_equal(u["iters"], ref["iters"].cpu().numpy())
        if grad is None:
            assert np.all(np.isnan(u["grad"]))
        else:
            np.testing.assert_array_equal(u["grad"], ref["grad"].cpu().numpy().T)
    np.testing.assert_array_equal(out["alpha"].cpu().numpy(), ref["alpha"].cpu().numpy())
    np.testing.assert_array_equal(out["iters"].cpu().numpy(), ref["iters"].cpu().numpy())
    assert (d["status"] != 0).any()   # the golden set's unsupported pairs: records from the reject kernel
    np.testing.assert_array_equal(unpack(rec_only.cpu().numpy()[:n])["status"], d["status"])


def test_native_comm_in_place_edge_shapes(engine):
    """In-place records with no tail rows (cap == n) and for an empty shard (every row of
    the rank's slice is tail: all-ones bytes)."""
    import torch
    from dcol_amd.dist import NativeComm, unpack
    d = load_golden([p for p in golden_files() if p.endswith("synthetic_polypoly.npz")][0])
    s1, s2 = register(engine, d)
    plan = engine.plan(s1[:300], s2[:300])
    p1 = torch.from_numpy(np.ascontiguousarray(d["pose1"][:300].T)).cuda()
    p2 = torch.from_numpy(np.ascontiguousarray(d["pose2"][:300].T)).cuda()
    empty = engine.plan(s1[:0], s2[:0])
    e1 = torch.zeros((6, 0), dtype=torch.float64, device="cuda")
    comm = NativeComm(NativeComm.unique_id(), 1, 0, 0)
    try:
        _, rec = comm.solve_gather(plan, p1, p2, cap=300, grad="fd", in_place=True, soa=False)
        _, rec0 = comm.solve_gather(empty, e1, e1.clone(), cap=3, grad="fd", in_place=True, soa=False)
        ref = plan.run(p1, p2, grad="fd", contact=False)
        torch.cuda.synchronize()
    finally:
        comm.close()
    u = unpack(rec.cpu().numpy())
    np.testing.assert_array_equal(u["alpha"], ref["alpha"].cpu().numpy())
    np.testing.assert_array_equal(u["grad"], ref["grad"].cpu().numpy().T)
    np.testing.assert_array_equal(u["iters"], ref["iters"].cpu().numpy())
    assert np.all(rec0.cpu().numpy().view(np.uint64) == np.uint64(0xFFFFFFFFFFFFFFFF))


def test_native_comm_side_stream(engine):
    """dcol_prox_batch_multi_gpu on a non-default stream with the buffers allocated by
    NativeComm.solve_gather (they belong to that stream in torch's allocator): the records
    stay intact while later allocations churn on the default stream."""
    import torch
    from dcol_amd.dist import NativeComm, unpack
    d = load_golden([p for p in golden_files() if p.endswith("synthetic_polypoly.npz")][0])
    s1, s2 = register(engine, d)
    plan = engine.plan(s1, s2)
    p1 = torch.from_numpy(np.ascontiguousarray(d["pose1"].T)).cuda()
    p2 = torch.from_numpy(np.ascontiguousarray(d["pose2"].T)).cuda()
    ref = plan.run(p1, p2, grad="fd", contact=False)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    comm = NativeComm(NativeComm.unique_id(), 1, 0, 0)
    try:
        recs = []
        for _ in range(3):
            _, rec = comm.solve_gather(plan, p1, p2, cap=plan.B, grad="fd", stream=side)
            junk = [torch.full((plan.B, 15), 7.0, dtype=torch.float64, device="cuda") for _ in range(4)]
            recs.append(rec)
            del junk
        side.synchronize()
    finally:
        comm.close()
    for rec in recs:
        u = unpack(rec.cpu().numpy())
        np.testing.assert_array_equal(u["alpha"], ref["alpha"].cpu().numpy())
        np.testing.assert_array_equal(u["grad"], ref["grad"].cpu().numpy().T)


def test_pair_plan_cache_bounded(engine):
    """dcol_prox_pair keeps at most DCOL_PAIR_PLANS_MAX one-pair plans (least recently used
    out): 100 distinct shape pairs through it, each result at the parity tolerances against
    the reference's golden values with equal iteration counts, the cache never above the cap,
    and a pair whose plan was evicted solves bitwise as on its first call."""
    import ctypes

    from dcol_amd import _lib
    d = load_golden([p for p in golden_files() if p.endswith("synthetic_mixed.npz")][0])
    s1, s2 = register(engine, d)
    lib = _lib.load()
    table = engine.table
    sel = np.flatnonzero(d["status"] == 0)[:100]
    assert len(set(zip(s1[sel].tolist(), s2[sel].tolist()))) == 100 > _lib.PAIR_PLANS_MAX

    def call(i):
        p1 = np.ascontiguousarray(d["pose1"][i], dtype=np.float64)
        p2 = np.ascontiguousarray(d["pose2"][i], dtype=np.float64)
        a, c, g = np.empty(1), np.empty(3), np.empty(12)
        it, st = ctypes.c_int32(), ctypes.c_int32()
        ptr = lambda x: ctypes.c_void_p(x.ctypes.data)  # noqa: E731
        _lib.check(lib.dcol_prox_pair(table.handle, int(s1[i]), int(s2[i]), ptr(p1), ptr(p2), 1e-6, 50,
                                      _lib.GRAD_FD | _lib.CONTACT, ptr(a), ptr(c), ptr(g), ctypes.byref(it),
                                      ctypes.byref(st)), "dcol_prox_pair")
        return a[0], g.copy(), int(it.value), int(st.value)

    n = ctypes.c_int32()
    first = {}
    for i in sel:
        a, g, it, st = call(i)
        first[i] = (a, g)
        assert st == 0 and it == d["iters"][i]
        assert alpha_close(a, d["alpha"][i]) and grad_close(g, d["grad"][i])
        _lib.check(lib.dcol_table_pair_plans(table.handle, ctypes.byref(n)), "dcol_table_pair_plans")
        assert n.value <= _lib.PAIR_PLANS_MAX
    assert n.value == _lib.PAIR_PLANS_MAX
    a, g, _, _ = call(sel[0])          # evicted long ago: a fresh plan, the same bits
    assert a == first[sel[0]][0] and np.array_equal(g, first[sel[0]][1])


_NO_BALL_SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[2], sys.argv[3]]
from dcol_amd import Engine, spec_from_arrays
d = dict(np.load(sys.argv[4], allow_pickle=False))
K = 100                                   # 150k pairs: a plan that fills the GPU (throughput buckets)
eng = Engine(device=0)
ids = np.array([eng.register(spec_from_arrays(d, k)) for k in range(len(d["type"]))], np.int32)
s1, s2 = np.tile(ids[d["s1"]], K), np.tile(ids[d["s2"]], K)
r = eng.solve_host(s1, s2, np.tile(d["pose1"], (K, 1)), np.tile(d["pose2"], (K, 1)), grad="fd", contact=False)
b = eng.plan(s1, s2).buckets()
np.savez(sys.argv[1], alpha=r.alpha, grad=r.grad, iters=r.iters, status=r.status,
         part=np.array([x["oe"] for x in b]), flags=np.array([x["flags"] for x in b]),
         shape=np.array([(x["N"], x["nsoc"], x["lpp"]) for x in b]))
"""


@pytest.mark.parametrize("var", ["DCOL_NO_BALL", "DCOL_NO_CONE", "DCOL_NO_PART", "DCOL_SPLIT"])
def test_mixed_golden_large_plan_env_variants(tmp_path, var):
    """The documented A/B switches on a plan large enough for the throughput buckets (the
    mixed golden set tiled to 150k pairs): DCOL_NO_BALL (no ball-row kernels: the x polytope
    row-partitioned buckets, compiled with ball rows only, must fall back to the dense rows
    instead of failing the launch), DCOL_NO_CONE, DCOL_NO_PART, DCOL_SPLIT (the {capsule,
    cylinder} x polytope buckets at two lanes per pair with the ball SOC block split over
    both, Solver SPLIT; rounding-level reordered sums) -- status and iteration counts
    equal to the reference's on every pair, alpha and gradient at the parity tolerances."""
    import os
    import subprocess
    import sys

    from conftest import PKG, REPO
    path = [p for p in golden_files() if p.endswith("synthetic_mixed.npz")][0]
    env = {k: v for k, v in os.environ.items()
           if k not in ("DCOL_NO_BALL", "DCOL_NO_CONE", "DCOL_NO_PART", "DCOL_LPP", "DCOL_SPLIT")}
    env[var] = "1"
    f = str(tmp_path / "out.npz")
    subprocess.run([sys.executable, "-c", _NO_BALL_SCRIPT, f, PKG, REPO, path], check=True, env=env, timeout=240)
    r = dict(np.load(f))
    d = load_golden(path)
    K = len(r["alpha"]) // len(d["alpha"])
    st, it = np.tile(d["status"], K), np.tile(d["iters"], K)
    np.testing.assert_array_equal(r["status"], st)
    ok = st == 0
    np.testing.assert_array_equal(r["iters"][ok], it[ok])
    assert np.all(alpha_close(r["alpha"][ok], np.tile(d["alpha"], K)[ok]))
    assert np.all(grad_close(r["grad"][ok], np.tile(d["grad"], (K, 1))[ok]))
    if var == "DCOL_NO_BALL":
        assert not np.any((r["flags"] & 2) != 0)
    if var == "DCOL_NO_PART":
        assert not np.any(r["part"] > 0)
    if var == "DCOL_SPLIT":   # the split copies ran: N = 5, one SOC block, PART, two lanes
        sh = r["shape"]
        assert np.any((sh[:, 0] == 5) & (sh[:, 1] == 1) & (r["part"] > 0) & (sh[:, 2] == 2))
