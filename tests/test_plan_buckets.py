"""Plan bucketing through the C-ABI (dcol_plan_bucket): which kernel variant and lane
configuration a plan launches -- the host logic of dcol_capi.cpp bucket_pairs /
bucket_and_fuse.  Plans need a table on the device, so these run on the GPU box; no solve is
launched."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ids(engine, tab):
    from dcol_amd import spec_from_arrays
    return np.array([engine.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)


def _solves(plan):
    return [b for b in plan.buckets() if b["kind"] == "solve"]


def test_benchmark_batch_is_one_padding_free_two_lane_bucket(engine):
    """configs[3] (100k random rectangular-prism pairs, bench.py): one bucket, the padding-free
    (4, 0, 12) box x box (axis-pair, flags 1 | 8) kernel at two lanes per pair -- the kernel the
    roofline line and the rocprofv3 summaries in profiles/ describe; with DCOL_NO_BOX the
    padding-free dense-row one (flags 1, test_box_disabled_by_env)."""
    import bench
    tab = bench.shape_table(64, 0)
    s1, s2 = bench.pairs(100_000, 64, 0)[:2]
    ids = _ids(engine, tab)
    plan = engine.plan(ids[s1], ids[s2], cache=False)
    b = plan.buckets()
    assert len(b) == 1 and plan.num_launches == 1
    assert b[0] == {"kind": "solve", "N": 4, "nsoc": 0, "omax": 12, "lpp": 2, "oe": 0, "flags": 9, "status": 0,
                    "pairs": 100_000}


def test_box_needs_exact_axis_pairs(engine):
    """The BOX bucket takes only pairs of 6-row polytopes whose rows 3..5 are the exact
    negatives of rows 0..2: a prism with one face normal perturbed, or rows in another order,
    stays in the dense-row 12-row bucket (flags 1)."""
    import bench
    tab = bench.shape_table(4, 0)
    tab["A_pool"] = tab["A_pool"].copy()
    tab["A_pool"][6 + 4] = [0.0, -1.0, 1e-12]           # shape 1: face 4 no longer -face 1
    tab["A_pool"][12:18] = tab["A_pool"][12:18][[0, 3, 1, 4, 2, 5]]   # shape 2: pairs interleaved
    ids = _ids(engine, tab)
    s1 = np.array([0, 0, 1, 2, 3], np.int32)
    s2 = np.array([3, 1, 0, 3, 0], np.int32)
    b = {(x["flags"], x["pairs"]) for x in engine.plan(ids[s1], ids[s2], cache=False).buckets() if x["kind"] == "solve"}
    assert b == {(9, 2), (1, 3)}, b


def _polygon_box(engine, B, seed=0):
    import bench
    tab = bench.mixed_table()
    ids = _ids(engine, tab)
    rng = np.random.default_rng(seed)
    poly = np.flatnonzero(tab["type"] == 5)
    box = np.flatnonzero(tab["type"] == 0)
    s1 = rng.choice(poly, B).astype(np.int32)
    s2 = rng.choice(box, B).astype(np.int32)
    return engine.plan(ids[s1], ids[s2], cache=False)


def test_large_polygon_box_plan_takes_the_row_partitioned_bucket(engine):
    """A plan that fills the GPU runs pentagon x box pairs (5 edge rows + 6 faces) in the
    row-partitioned (11, 5) bucket at its throughput configuration, one lane per pair."""
    b = _solves(_polygon_box(engine, 200_000))
    assert len(b) == 1
    assert (b[0]["N"], b[0]["nsoc"], b[0]["omax"], b[0]["oe"], b[0]["lpp"]) == (6, 1, 11, 5, 1)


@pytest.mark.parametrize("B", [1, 1000])
def test_small_polygon_box_plan_skips_one_lane_buckets(engine, B):
    """A plan that cannot fill the GPU never runs a one-lane row-partitioned bucket (one lane
    through all 11 rows: 84 us per 1,000 pairs against 50 us on the dense rows); the pairs take
    the dense (6, 1, 12) ball-row kernel in its latency configuration."""
    b = _solves(_polygon_box(engine, B))
    assert b and all(not (x["oe"] > 0 and x["lpp"] < 2) for x in b)
    assert all(x["oe"] == 0 and x["lpp"] >= 4 for x in b)


def test_bucket_index_checked(engine):
    import bench
    from dcol_amd import DcolLibraryError
    tab = bench.shape_table(8, 0)
    ids = _ids(engine, tab)
    plan = engine.plan(ids[[0, 1]], ids[[2, 3]], cache=False)
    assert len(plan.buckets()) == plan.num_buckets
    import ctypes
    from dcol_amd import _lib
    info = (ctypes.c_int32 * 8)()
    n = ctypes.c_int64()
    with pytest.raises(DcolLibraryError):
        _lib.check(_lib.load().dcol_plan_bucket(plan.handle, plan.num_buckets, info, ctypes.byref(n)), "dcol_plan_bucket")


def test_fanout_width_by_plan_size(engine):
    """How a mixed plan launches, by size: the whole 1M configs[4] plan
    (every bucket fills the GPU by itself) one launch per bucket over the caller's stream + 2
    side streams (three buckets in flight); a mid-size one (150k pairs: a rank's shard at 4-8
    GPUs) one packed launch; a small one with fusing disallowed its latency-configured buckets
    over the caller's + 3; a small one otherwise one fused (or, without fused cases, packed)
    launch; a one-bucket plan the caller's stream alone."""
    import os
    import bench
    if any(os.environ.get(k) for k in ("DCOL_SIDE_STREAMS", "DCOL_SIDE_STREAMS_LARGE", "DCOL_NO_FANOUT",
                                      "DCOL_PACK_LANES", "DCOL_SMALL_FANOUT")):
        pytest.skip("plan policy overridden by the environment")
    tab = bench.mixed_table()
    ids = _ids(engine, tab)
    s1, s2 = bench.mixed_pairs(tab, 1_000_000, seed=3)[:2]
    big = engine.plan(ids[s1], ids[s2], cache=False)
    assert len(_solves(big)) > 4 and big.num_streams == 3 and big.launch_form == "buckets"
    mid = engine.plan(ids[s1[:150_000]], ids[s2[:150_000]], cache=False)
    assert len(_solves(mid)) > 4 and mid.launch_form == "packed" and mid.num_streams == 1 and mid.num_launches == 1
    # the packed plan's buckets are the throughput configurations of the large plan's
    key = lambda b: (b["N"], b["nsoc"], b["omax"], b["lpp"], b["oe"], b["flags"])  # noqa: E731
    assert {key(b) for b in _solves(mid)} <= {key(b) for b in _solves(big)}
    small = engine.plan(ids[s1[:2000]], ids[s2[:2000]], cache=False, fuse=False)
    assert len(_solves(small)) > 4 and small.num_streams == 4 and small.launch_form == "buckets"
    one = engine.plan(ids[s1[:2000]], ids[s2[:2000]], cache=False)
    assert one.launch_form in ("fused", "packed") and one.num_streams == 1 and one.num_launches == 1
    tb = bench.shape_table(64, 0)
    idb = _ids(engine, tb)
    b1, b2 = bench.pairs(100_000, 64, 0)[:2]
    p1 = engine.plan(idb[b1], idb[b2], cache=False)
    assert p1.num_streams == 1 and p1.launch_form == "buckets"


@pytest.mark.parametrize("world", [8, 32])
def test_packed_launch_bitwise_equal_to_bucket_launches(engine, world):
    """The packed launch (dcol_kernels_packed.hip: every bucket of a mid-size plan in one
    launch, each in its throughput configuration, segments longest first) runs the same
    solver copies as the per-bucket kernels: rank 0's class-balanced shard of the configs[4]
    batch at world 8 (125k pairs) and 32 (31k: a small plan the fused kernel cannot take,
    packed instead of fanned out) gives BITWISE the outputs of the same buckets launched one
    by one (fuse=False, world 8), and of the shard's pairs inside the whole 1M plan."""
    import torch
    import bench
    from dcol_amd import alloc_outputs
    from dcol_amd.dist import shard_indices
    tab = bench.mixed_table()
    ids = _ids(engine, tab)
    B = 1_000_000
    s1, s2, p1, p2 = bench.mixed_pairs(tab, B, seed=0)
    mine = shard_indices(B, 0, world, tab["type"][s1] * 8 + tab["type"][s2])
    dev = torch.device("cuda", engine.device)
    d1 = torch.from_numpy(np.ascontiguousarray(p1[mine].T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2[mine].T)).to(dev)
    packed = engine.plan(ids[s1[mine]], ids[s2[mine]], cache=False)
    assert packed.launch_form == "packed" and packed.num_launches == 1
    a = packed.run(d1, d2, grad="fd", contact=True)
    if world == 8:   # a mid-size plan: the same buckets launched one by one
        apart = engine.plan(ids[s1[mine]], ids[s2[mine]], cache=False, fuse=False)
        assert apart.launch_form == "buckets"
        b = apart.run(d1, d2, grad="fd", contact=True)
        torch.cuda.synchronize()
        for k in ("status", "iters", "alpha", "grad", "contact"):
            assert torch.equal(a[k], b[k]), k
    # against the whole batch's plan (one launch per bucket, throughput configurations; a
    # small plan unfused would have taken latency configurations instead)
    whole = engine.plan(ids[s1], ids[s2], cache=False)
    w1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    w2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
    whole.run(w1, w2, grad="fd", contact=False, out=out)
    sel = torch.from_numpy(mine).to(dev)
    for k in ("status", "iters", "alpha"):
        assert torch.equal(out[k][sel], a[k]), k
    assert torch.equal(out["grad"][:, sel], a["grad"])
