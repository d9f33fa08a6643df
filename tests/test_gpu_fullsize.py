"""Full-size checks on the benchmark workload (BASELINE.json configs[3]: 100k random
polytope-polytope pairs; and 1M) through size-independent properties of the problem,
plus an exact comparison of EVERY pair with the C oracle (100k here, 1M mixed below).

Properties (exact for the mathematical problem; tolerances cover pdip_tol = 1e-6 and the
FD step):
  * every pair converges, alpha > 0 and finite, iters <= 50;
  * swap symmetry: alpha(A, B) = alpha(B, A) and the gradient halves swap;
  * translation invariance: shifting both poses by t leaves alpha unchanged and
    d alpha / d r1 + d alpha / d r2 = 0;
  * the contact point lies in both primitives scaled by alpha (up to the exit residual);
  * FD and envelope gradients agree; chunked launches equal one launch bitwise.
"""
import os

import numpy as np
import pytest

from conftest import PKG, REPO, alpha_close, grad_close, gpu_available

pytestmark = pytest.mark.gpu

B = 100_000


@pytest.fixture(scope="module")
def batch():
    if not gpu_available():
        pytest.skip("no GPU")
    import bench
    from dcol_amd import Engine, spec_from_arrays
    tab = bench.shape_table()
    s1, s2, p1, p2 = bench.pairs(B, len(tab["type"]), seed=1000)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    res = eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd")
    return dict(tab=tab, s1=s1, s2=s2, p1=p1, p2=p2, eng=eng, ids=ids, res=res)


def test_all_converge(batch):
    r = batch["res"]
    assert (r.status == 0).all()
    assert (r.iters <= 50).all() and (r.iters > 0).all()
    assert np.isfinite(r.alpha).all() and (r.alpha > 0).all()
    assert np.isfinite(r.grad).all()


def test_whole_batch_matches_c_oracle(batch):
    """Every one of the 100k pairs against the C restatement (oracle/dcol_oracle.c, ~2e6
    pair-solves/s on the box's 16 host threads): status and Newton iteration counts equal on
    EVERY pair, alpha within 1e-6 rel, gradient within 1e-5 of max(|g|_inf, 1)."""
    from oracle import c_oracle
    ref = c_oracle.run_batch(batch["tab"], batch["s1"], batch["s2"], batch["p1"], batch["p2"],
                             want_grad=True, threads=16)
    r = batch["res"]
    np.testing.assert_array_equal(r.status, ref["status"])
    np.testing.assert_array_equal(r.iters, ref["iters"])
    assert alpha_close(r.alpha, ref["alpha"]).all()
    assert grad_close(r.grad, ref["grad"]).all()


def test_swap_symmetry(batch):
    b, ids = batch, batch["ids"]
    sw = b["eng"].solve_host(ids[b["s2"]], ids[b["s1"]], b["p2"], b["p1"], grad="fd")
    r = b["res"]
    assert (sw.status == 0).all()
    np.testing.assert_allclose(sw.alpha, r.alpha, rtol=2e-5, atol=1e-9)
    g_sw = np.concatenate([sw.grad[:, 6:], sw.grad[:, :6]], axis=1)
    scale = np.maximum(np.abs(r.grad).max(axis=1), 1.0)
    assert (np.abs(g_sw - r.grad).max(axis=1) <= 1e-3 * scale).all()


def test_translation_invariance(batch):
    b, ids = batch, batch["ids"]
    t = np.array([0.7, -1.3, 2.1])
    q1, q2 = b["p1"].copy(), b["p2"].copy()
    q1[:, :3] += t
    q2[:, :3] += t
    sh = b["eng"].solve_host(ids[b["s1"]], ids[b["s2"]], q1, q2, grad="envelope")
    r = b["res"]
    np.testing.assert_allclose(sh.alpha, r.alpha, rtol=1e-6, atol=1e-12)
    scale = np.maximum(np.abs(sh.grad).max(axis=1), 1.0)
    assert (np.abs(sh.grad[:, 0:3] + sh.grad[:, 6:9]).max(axis=1) <= 1e-6 * scale).all()


def test_contact_point_in_both_scaled_prisms(batch):
    from oracle.dcol_oracle import dcm_from_mrp
    b, r = batch, batch["res"]
    tab = b["tab"]
    half = tab["b_pool"].reshape(-1, 6)[:, :3]            # rect prism half-dims
    idx = np.arange(0, B, 97)
    for i in idx:
        a = r.alpha[i]
        c = r.contact[i]
        for s, p in ((b["s1"][i], b["p1"][i]), (b["s2"][i], b["p2"][i])):
            y = dcm_from_mrp(p[3:]).T @ (c - p[:3])
            # the PDIP stops on mu alone (pdip.py:416-422), so the primal residual G x + s - h
            # at exit is small but not zero (~1e-5 relative here, same as the reference)
            assert (np.abs(y) <= a * half[s] * (1 + 1e-4) + 1e-9).all(), i


def test_fd_matches_envelope(batch):
    b, ids = batch, batch["ids"]
    env = b["eng"].solve_host(ids[b["s1"]], ids[b["s2"]], b["p1"], b["p2"], grad="envelope")
    assert np.array_equal(env.alpha, b["res"].alpha)          # same solve, bitwise
    assert grad_close(env.grad, b["res"].grad).all()


def test_chunked_equals_single_launch_1m():
    """1M pairs (the large configuration): one launch vs ten 100k launches, bitwise."""
    if not gpu_available():
        pytest.skip("no GPU")
    import torch

    import bench
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    tab = bench.shape_table()
    n = 1_000_000
    s1, s2, p1, p2 = bench.pairs(n, len(tab["type"]), seed=7)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    dev = torch.device("cuda", 0)
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    whole = eng.plan(ids[s1], ids[s2], cache=False).run(d1, d2, grad="fd", contact=False)
    alpha = whole["alpha"].cpu().numpy()
    status = whole["status"].cpu().numpy()
    assert (status == 0).all()
    c = 100_000
    for k in range(0, n, c):
        out = alloc_outputs(c, dev, want_grad=True, want_contact=False)
        plan = eng.plan(ids[s1[k:k + c]], ids[s2[k:k + c]], cache=False)
        part = plan.run(d1[:, k:k + c].contiguous(), d2[:, k:k + c].contiguous(), grad="fd", contact=False, out=out)
        assert np.array_equal(part["alpha"].cpu().numpy(), alpha[k:k + c])
        assert torch.equal(part["grad"], whole["grad"][:, k:k + c])


def test_mixed_throughput_variants_match_c_oracle():
    """BASELINE configs[4] workload at full size (1M mixed pairs: every class's bucket is
    large enough for its throughput configuration -- the variants ALTRO-sized and golden
    batches never reach), EVERY pair against the C oracle (~1e6 pair-solves/s on 16 host
    threads): status and Newton iteration counts equal on every pair, alpha within 1e-6 rel
    AND within 1e-9 rel (rounding-level -- the variants differ from the oracle only in
    summation order and reciprocal refinement; the defective 326f844 build drifted to 2.7e-9
    on 0.7 % of its polygon x box pairs), gradient within 1e-5 of max(|g|_inf, 1) AND within
    2e-6 (measured <= 4e-7: the forward-difference noise of the reference's own formulation)."""
    if not gpu_available():
        pytest.skip("no GPU")
    import bench
    from dcol_amd import Engine, spec_from_arrays
    from oracle import c_oracle
    tab = bench.mixed_table()
    s1, s2, p1, p2 = bench.mixed_pairs(tab, 1_000_000, seed=0)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    res = eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd")
    cls = tab["type"][s1] * 8 + tab["type"][s2]
    ref = c_oracle.run_batch(tab, s1, s2, p1, p2, want_grad=True, threads=16)
    np.testing.assert_array_equal(res.status, ref["status"])
    ok = ref["status"] == 0
    bad = np.flatnonzero(res.iters[ok] != ref["iters"][ok])
    assert bad.size == 0, (bad.size, np.unique(cls[ok][bad]).tolist())
    a, ra = res.alpha[ok], ref["alpha"][ok]
    assert np.all(alpha_close(a, ra))
    rel = np.abs(a - ra) / np.abs(ra)
    assert rel.max() <= 1e-9, (rel.max(), int(cls[ok][np.argmax(rel)]))
    assert np.all(grad_close(res.grad[ok], ref["grad"][ok]))
    eg = np.abs(res.grad[ok] - ref["grad"][ok]).max(1) / np.maximum(np.abs(ref["grad"][ok]).max(1), 1.0)
    assert eg.max() <= 2e-6, (eg.max(), int(cls[ok][np.argmax(eg)]))


XCHECK_LIB = os.path.join(PKG, "lib_xcheck", "libdcol.so")
_SOLVE_SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[2], sys.argv[3]]
import bench
from dcol_amd import Engine, spec_from_arrays
tab = bench.mixed_table()
s1, s2, p1, p2 = bench.mixed_pairs(tab, 1_000_000, seed=0)
eng = Engine(device=0)
ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
r = eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd", contact=True)
r2 = eng.solve_host(ids[s1[:100000]], ids[s2[:100000]], p1[:100000], p2[:100000], grad="envelope", contact=False)
# a rank's shard at world 8 (125k pairs): the packed launch (dcol_kernels_packed.hip)
from dcol_amd.dist import shard_indices
m = shard_indices(len(s1), 0, 8, tab["type"][s1] * 8 + tab["type"][s2])
assert eng.plan(ids[s1[m]], ids[s2[m]], cache=False).launch_form == "packed"
r3 = eng.solve_host(ids[s1[m]], ids[s2[m]], p1[m], p2[m], grad="fd", contact=True)
np.savez(sys.argv[1], alpha=r.alpha, grad=r.grad, contact=r.contact, iters=r.iters, status=r.status,
         genv=r2.grad, palpha=r3.alpha, pgrad=r3.grad, pcontact=r3.contact, piters=r3.iters, pstatus=r3.status)
"""


def _mixed_outputs(tmp_path, name, lib=None, env_extra=None):
    import subprocess
    import sys
    env = dict(os.environ)
    for k in ("DCOL_LIB", "DCOL_NO_BALL", "DCOL_NO_CONE", "DCOL_LPP"):
        env.pop(k, None)
    if lib:
        env["DCOL_LIB"] = lib
    env.update(env_extra or {})
    f = str(tmp_path / f"{name}.npz")
    subprocess.run([sys.executable, "-c", _SOLVE_SCRIPT, f, PKG, REPO], check=True, env=env, timeout=300)
    return dict(np.load(f))


def _assert_bitwise(a, b):
    for k in ("status", "iters", "pstatus", "piters"):
        np.testing.assert_array_equal(a[k], b[k])
    for k in ("alpha", "grad", "contact", "genv", "palpha", "pgrad", "pcontact"):
        same = (a[k] == b[k]) | (np.isnan(a[k]) & np.isnan(b[k]))
        assert same.all(), (k, int((~same).sum()))


def test_structured_cone_rows_equal_dense(tmp_path):
    """The CONE kernels (cone blocks as 3 x 3 rotation part + one constant, 3-dim SOC
    arithmetic, no zero padding) compute the dense padded kernels' nonzero terms in the same
    order: bitwise equal over the 1M mixed workload (polytope x cone, cone x polytope and
    cone x cone are the classes that switch kernels; DCOL_NO_CONE=1 keeps the dense rows)."""
    if not gpu_available():
        pytest.skip("no GPU")
    _assert_bitwise(_mixed_outputs(tmp_path, "structured"), _mixed_outputs(tmp_path, "dense", env_extra={"DCOL_NO_CONE": "1"}))


@pytest.mark.skipif(not os.path.exists(XCHECK_LIB), reason="lib_xcheck not built (make -C csrc xcheck)")
def test_codegen_invariance_mixed(tmp_path):
    """The product library and its twin built from the same sources with another machine
    schedule (each unit under the other of default / max-ilp; Makefile target xcheck) must agree BITWISE on
    the whole 1M mixed workload (every throughput variant of configs[4], both gradient
    modes, contact points): FP semantics are fixed in the IR before scheduling, so any
    difference is a machine-code defect -- the class of fault that made the 326f844 build
    of the (6, 1, 12) LPP-2 ball kernel drift."""
    _assert_bitwise(_mixed_outputs(tmp_path, "product"), _mixed_outputs(tmp_path, "xcheck", lib=XCHECK_LIB))


_TWIN_EXTRA_SCRIPT = r"""
import glob, os, sys, numpy as np
sys.path[:0] = [sys.argv[2], sys.argv[3], os.path.join(sys.argv[3], "tests")]
from dcol_amd import Engine, spec_from_arrays
from stress_shapes import random_pairs, random_table
out = {}
eng = Engine(device=0)
# stress shapes: the 48 / 64 / 128-row buckets at 8 / 16 lanes per pair, offsets, polygons
# with 3-12 edges; the same pairs with the case-4 extension (N = 7 / 8 kernels)
rng = np.random.default_rng(2)
tab = random_table(rng)
s1, s2, p1, p2 = random_pairs(rng, tab, 200_000)
ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
for tag, c4 in (("stress", False), ("stress_case4", True)):
    r = eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd", contact=True, case4=c4)
    for k in ("alpha", "grad", "contact", "iters", "status"):
        out[f"{tag}_{k}"] = getattr(r, k)
# small plans (fused / latency configurations): every golden file, FD and envelope, the
# mixed one also with case 4
for path in sorted(glob.glob(os.path.join(sys.argv[3], "tests", "golden", "*.npz"))):
    d = dict(np.load(path, allow_pickle=False))
    if "type" not in d or "tol0" in path:
        continue
    gi = np.array([eng.register(spec_from_arrays(d, k)) for k in range(len(d["type"]))], np.int32)
    name = os.path.basename(path)[:-4]
    for mode in ("fd", "envelope"):
        for c4 in ((False, True) if "mixed" in name else (False,)):
            r = eng.solve_host(gi[d["s1"]], gi[d["s2"]], d["pose1"], d["pose2"], tol=float(d["tol"]), grad=mode,
                               contact=True, case4=c4)
            for k in ("alpha", "grad", "contact", "iters", "status"):
                out[f"{name}_{mode}_{int(c4)}_{k}"] = getattr(r, k)
np.savez(sys.argv[1], **out)
"""


def _twin_outputs(tmp_path, name, lib=None):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("DCOL_LIB", "DCOL_NO_BALL", "DCOL_NO_CONE", "DCOL_LPP")}
    if lib:
        env["DCOL_LIB"] = lib
    f = str(tmp_path / f"{name}.npz")
    subprocess.run([sys.executable, "-c", _TWIN_EXTRA_SCRIPT, f, PKG, REPO], check=True, env=env, timeout=300)
    return dict(np.load(f))


@pytest.mark.skipif(not os.path.exists(XCHECK_LIB), reason="lib_xcheck not built (make -C csrc xcheck)")
def test_codegen_invariance_stress_case4_small_plans(tmp_path):
    """The codegen-invariance twin (see test_codegen_invariance_mixed) beyond the 1M mixed set:
    the stress shapes' 48 / 64 / 128-row buckets at 8 / 16 lanes per pair and non-identity
    offsets (200k pairs), the case-4 N = 7 / 8 kernels on the same pairs, and the small
    fused / latency plans of every golden file (scenes, synthetic sets, edge cases; FD and
    envelope gradients): BITWISE equal between the product library and its twin."""
    if not gpu_available():
        pytest.skip("no GPU")
    a = _twin_outputs(tmp_path, "product")
    b = _twin_outputs(tmp_path, "xcheck", lib=XCHECK_LIB)
    assert set(a) == set(b) and len(a) > 40
    for k in a:
        same = (a[k] == b[k]) | (np.isnan(a[k]) & np.isnan(b[k])) if a[k].dtype.kind == "f" else a[k] == b[k]
        assert np.all(same), (k, int((~same).sum()))
    assert (a["stress_case4_status"] == 0).mean() > (a["stress_status"] == 0).mean()   # case-4 pairs solved


def test_max_size_192m_pairs_position_independent():
    """Maximum-size launch: 192M pairs in ONE plan (192 copies of a 1M batch of the benchmark
    distribution; 18 GB of poses and 18 GB of gradients in HBM, so pose / gradient offsets
    run past 2^31 elements -- int64 indexing end to end).  There is no cross-pair arithmetic, so every copy must equal the
    1M solve bitwise -- status, iteration counts, alpha and gradient -- wherever it sits in
    the batch (compared on the device)."""
    if not gpu_available():
        pytest.skip("no GPU")
    import torch

    import bench
    from dcol_amd import Engine, spec_from_arrays
    tab = bench.shape_table()
    n, K = 1_000_000, 192
    s1, s2, p1, p2 = bench.pairs(n, len(tab["type"]), seed=11)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    dev = torch.device("cuda", 0)
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    base = eng.plan(ids[s1], ids[s2], cache=False).run(d1, d2, grad="fd", contact=False)
    assert bool((base["status"] == 0).all())
    big = eng.plan(np.tile(ids[s1], K), np.tile(ids[s2], K), cache=False).run(
        d1.repeat(1, K).contiguous(), d2.repeat(1, K).contiguous(), grad="fd", contact=False)
    assert big["grad"].shape == (12, n * K) and n * K * 12 > 2 ** 31
    for k in range(K):
        sl = slice(k * n, (k + 1) * n)
        assert torch.equal(big["status"][sl], base["status"]), k
        assert torch.equal(big["iters"][sl], base["iters"]), k
        assert torch.equal(big["alpha"][sl], base["alpha"]), k
        assert torch.equal(big["grad"][:, sl], base["grad"]), k


def test_suspend_resume_bitwise_equal(batch):
    """DCOL_PLAN_SUSPEND (opt-in): the benchmark batch as a main launch that hands each
    wave's last few iterating pairs to a resume launch -- the same iteration sequence
    continued from the saved iterate, so every output equals the one-launch plan bitwise;
    and some pairs were actually suspended."""
    import torch
    b = batch
    dev = torch.device("cuda", 0)
    d1 = torch.from_numpy(np.ascontiguousarray(b["p1"].T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(b["p2"].T)).to(dev)
    plain = b["eng"].plan(b["ids"][b["s1"]], b["ids"][b["s2"]], cache=False)
    susp = b["eng"].plan(b["ids"][b["s1"]], b["ids"][b["s2"]], cache=False, suspend=True)
    a = plain.run(d1, d2, grad="fd", contact=True)
    c = susp.run(d1, d2, grad="fd", contact=True)
    torch.cuda.synchronize()
    assert susp.suspended() > 0
    for k in ("status", "iters", "alpha", "grad", "contact"):
        assert torch.equal(a[k], c[k]), k

