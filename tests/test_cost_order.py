"""dcol_amd.cost_order: a fixed pairing re-listed in descending order of its last iteration
counts (waves of similar-cost pairs, the slowest first).  CPU: the order itself.  GPU: a plan
on the re-listed pairing returns, un-permuted, bitwise the outputs of the given listing --
a pair's arithmetic does not depend on its slot -- on configs[3] and on the mixed golden set
tiled to 150k (buckets, rejected case-4 pairs with NaN outputs among them)."""
import numpy as np
import pytest

from conftest import golden_files, load_golden


def test_cost_order_descending_stable():
    from dcol_amd import cost_order
    it = np.array([7, 9, 7, 5, 12, 9, 0, 7], np.int32)
    o = cost_order(it)
    assert o.tolist() == [4, 1, 5, 0, 2, 7, 3, 6]
    assert sorted(o.tolist()) == list(range(len(it)))
    assert cost_order(np.zeros(0, np.int32)).size == 0


def _bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.int64) if a.dtype == np.float64 else a


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["configs3", "mixed150k"])
def test_cost_ordered_plan_bitwise_equal(engine, workload):
    import bench
    from dcol_amd import cost_order, spec_from_arrays
    if workload == "configs3":
        tab = bench.shape_table(64, 0)
        s1, s2, p1, p2 = bench.pairs(100_000, 64, 5)
        ids = np.array([engine.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
        a1, a2 = ids[s1], ids[s2]
    else:
        d = load_golden([p for p in golden_files() if p.endswith("synthetic_mixed.npz")][0])
        ids = np.array([engine.register(spec_from_arrays(d, k)) for k in range(len(d["type"]))], np.int32)
        K = 100
        a1, a2 = np.tile(ids[d["s1"]], K), np.tile(ids[d["s2"]], K)
        p1, p2 = np.tile(d["pose1"], (K, 1)), np.tile(d["pose2"], (K, 1))
    r0 = engine.solve_host(a1, a2, p1, p2, grad="fd", contact=True)
    o = cost_order(r0.iters)
    r1 = engine.solve_host(a1[o], a2[o], p1[o], p2[o], grad="fd", contact=True)
    inv = np.empty_like(o)
    inv[o] = np.arange(len(o))
    for k in ("alpha", "grad", "contact", "iters", "status"):
        a = getattr(r0, k)
        b = getattr(r1, k)[inv]
        np.testing.assert_array_equal(_bits(b), _bits(a), err_msg=k)
    assert np.all(np.diff(r1.iters) <= 0)   # the re-listed solve's counts are sorted
