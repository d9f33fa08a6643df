"""Op-counting build of the C restatement (oracle/dcol_oracle_opcount.cpp)
and the counted flop model bench.py reports (profiles/flop_model.json)."""
import json
import os

import numpy as np

from conftest import REPO, golden_files, load_golden


def test_opcount_build_solves_like_the_oracle():
    """Counting does not change the arithmetic: status and iteration counts equal the C
    oracle's (and so the reference's) on the synthetic and scene goldens."""
    from oracle import c_oracle
    for name in ("synthetic_polypoly.npz", "scene_quad.npz", "synthetic_mixed.npz"):
        d = load_golden([p for p in golden_files() if p.endswith(name)][0])
        oc = c_oracle.op_counts(d, d["s1"], d["s2"], d["pose1"], d["pose2"], float(d["tol"]))
        np.testing.assert_array_equal(oc["status"], d["status"], err_msg=name)
        ok = d["status"] == 0
        np.testing.assert_array_equal(oc["iters"][ok], d["iters"][ok], err_msg=name)
        assert np.all(oc["pdip"][ok] > 0) and np.all(oc["grad"][ok] > 0)


def test_flop_model_reproduces():
    """The committed poly6 x poly6 model matches a fresh count (same seeds as bench.py)."""
    import bench
    from oracle import c_oracle
    model = json.load(open(os.path.join(REPO, "profiles", "flop_model.json")))
    c = model["classes"]["polytope-polytope (bench configs[3])"]
    tab = bench.shape_table()
    s1, s2, p1, p2 = bench.pairs(300, len(tab["type"]), seed=1000)
    oc = c_oracle.op_counts(tab, s1, s2, p1, p2)
    ok = oc["status"] == 0
    assert np.all(oc["assembly"][ok] == c["assembly"]) and np.all(oc["grad"][ok] == c["grad_fd"])
    pred = c["pdip_fixed"] + c["pdip_per_iter"] * oc["iters"][ok]
    assert np.all(np.abs(pred - oc["pdip"][ok]) <= 0.02 * oc["pdip"][ok])
    assert abs(bench.flops_per_pair(oc["iters"][ok]) - (oc["assembly"][ok] + oc["pdip"][ok] + oc["grad"][ok]).mean()) \
        <= 0.005 * c["mean_total"]
