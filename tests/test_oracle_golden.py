"""The NumPy oracle (oracle/dcol_oracle.py) against the reference's golden vectors.

The golden vectors were produced by running the reference itself (tests/golden/
gen_golden.py).  The oracle must reproduce them exactly: same status, same Newton
iteration count, alpha/contact/gradient bit-for-bit (it uses the same LAPACK calls)."""
import numpy as np
import pytest

from conftest import golden_files, load_golden
from oracle import dcol_oracle as O


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.split("/")[-1][:-4])
def test_oracle_matches_reference(path):
    d = load_golden(path)
    tol = float(d["tol"])
    want_grad = not np.all(np.isnan(d["grad"]))
    B = len(d["s1"])
    idx = np.arange(B) if B <= 600 else np.random.default_rng(0).choice(B, 600, replace=False)
    out = O.run_batch(d, d["s1"][idx], d["s2"][idx], d["pose1"][idx], d["pose2"][idx], tol, want_grad)
    np.testing.assert_array_equal(out["status"], d["status"][idx])
    ok = d["status"][idx] == 0
    np.testing.assert_array_equal(out["iters"][ok], d["iters"][idx][ok])
    np.testing.assert_array_equal(out["alpha"][ok], d["alpha"][idx][ok])
    np.testing.assert_array_equal(out["contact"][ok], d["contact"][idx][ok])
    if want_grad:
        np.testing.assert_array_equal(out["grad"][ok], d["grad"][idx][ok])


def test_golden_inventory():
    """Every fixture family the parity suite relies on is present and non-trivial."""
    names = {p.split("/")[-1][:-4] for p in golden_files()}
    for n in ("scene_piano", "scene_quad", "scene_cone", "synthetic_polypoly", "synthetic_mixed",
              "edge_cases", "synthetic_tol1e-9", "synthetic_tol1e-3", "synthetic_tol0_maxiter", "traces"):
        assert n in names, n
    mixed = load_golden([p for p in golden_files() if p.endswith("synthetic_mixed.npz")][0])
    assert (mixed["status"] == 2).any() and (mixed["status"] == 0).any()
