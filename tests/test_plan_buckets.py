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
    """A mixed plan that fills the GPU spreads its buckets over the caller's stream + 2 side
    streams (three buckets in flight: DESIGN.md section 5, "Two side streams"); a small one,
    whose buckets run their latency configurations, over the caller's + 3; a fused small plan
    and a one-bucket plan run on the caller's stream alone."""
    import os
    import bench
    if os.environ.get("DCOL_SIDE_STREAMS") or os.environ.get("DCOL_SIDE_STREAMS_LARGE") or os.environ.get("DCOL_NO_FANOUT"):
        pytest.skip("fan-out width overridden by the environment")
    tab = bench.mixed_table()
    ids = _ids(engine, tab)
    s1, s2 = bench.mixed_pairs(tab, 150_000, seed=3)[:2]
    big = engine.plan(ids[s1], ids[s2], cache=False)
    assert len(_solves(big)) > 4 and big.num_streams == 3
    small = engine.plan(ids[s1[:2000]], ids[s2[:2000]], cache=False, fuse=False)
    assert len(_solves(small)) > 4 and small.num_streams == 4
    fused = engine.plan(ids[s1[:2000]], ids[s2[:2000]], cache=False)
    assert fused.num_streams == (1 if fused.num_launches == 1 else 4)
    tb = bench.shape_table(64, 0)
    idb = _ids(engine, tb)
    b1, b2 = bench.pairs(100_000, 64, 0)[:2]
    assert engine.plan(idb[b1], idb[b2], cache=False).num_streams == 1
