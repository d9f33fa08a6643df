"""The C oracle (oracle/dcol_oracle.c) against the reference's golden vectors: same status,
same Newton iteration count on every pair, alpha within 1e-10 rel, gradient within the
parity tolerance (its FD noise differs from numpy's BLAS summation order)."""
import numpy as np
import pytest

from conftest import alpha_close, golden_files, grad_close, load_golden
from oracle import c_oracle


@pytest.mark.parametrize("path", [p for p in golden_files() if "tol0" not in p], ids=lambda p: p.split("/")[-1][:-4])
def test_c_oracle_matches_reference(path):
    d = load_golden(path)
    want_grad = not np.all(np.isnan(d["grad"]))
    out = c_oracle.run_batch(d, d["s1"], d["s2"], d["pose1"], d["pose2"], float(d["tol"]), want_grad, threads=4)
    np.testing.assert_array_equal(out["status"], d["status"])
    ok = d["status"] == 0
    np.testing.assert_array_equal(out["iters"][ok], d["iters"][ok])
    assert np.all(np.abs(out["alpha"][ok] - d["alpha"][ok]) <= 1e-10 * np.abs(d["alpha"][ok]) + 1e-14)
    assert np.all(alpha_close(out["alpha"][ok], d["alpha"][ok]))
    if want_grad:
        assert np.all(grad_close(out["grad"][ok], d["grad"][ok]))
