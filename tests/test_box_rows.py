"""The BOX kernels' axis-pair rows (Solver<..., BOX>, dcol_device.hpp) on boxes whose two
faces of an axis differ: off-centre boxes (six independent offsets), rotated boxes and
parallelepipeds (A = [M; -M]) -- every shape the detector (DevShape::boxp: rows 3..5 the
exact negatives of rows 0..2) accepts, where the bench's centred rect prisms only ever
exercised g3 == g3'.  Against the C restatement of the reference (status, Newton iteration
counts, alpha, FD gradient) and against the same pairs on the padding-free dense rows
(DCOL_NO_BOX).  Reference: primitives/problem_matrices.py:181-209 (polytope blocks),
combine_problem_matrices.py:3-70, proximity/pdip.py:373-470.

CPU: the x86 build of the device solver (tests/emul, one lane per pair).  GPU: the product
library's LPP-2 BOX kernel on 200k pairs."""
import os
import subprocess
import sys

import numpy as np
import pytest

from box_shapes import box_pairs, box_table
from conftest import PKG, REPO, alpha_close, gpu_available, grad_close

EMUL = os.path.join(REPO, "tests", "emul", "libdcol_emul.so")
LF_BOX = 8


def _check_vs_oracle(res, ref, rel_max):
    np.testing.assert_array_equal(res["status"], ref["status"])
    ok = ref["status"] == 0
    assert ok.mean() > 0.99
    np.testing.assert_array_equal(res["iters"][ok], ref["iters"][ok])
    assert alpha_close(res["alpha"][ok], ref["alpha"][ok]).all()
    rel = np.abs(res["alpha"][ok] - ref["alpha"][ok]) / np.abs(ref["alpha"][ok])
    assert rel.max() <= rel_max, rel.max()
    assert grad_close(res["grad"][ok], ref["grad"][ok]).all()


@pytest.mark.skipif(not os.path.exists(EMUL), reason="tests/emul not built")
def test_emulated_box_rows_asymmetric_match_oracle(monkeypatch):
    from oracle import c_oracle
    from test_emul_golden import emul
    rng = np.random.default_rng(11)
    tab, _ = box_table(rng)
    s1, s2, p1, p2 = box_pairs(rng, tab, 3000)
    d = dict(tab, s1=s1, s2=s2, pose1=p1, pose2=p2)
    monkeypatch.delenv("DCOL_NO_BOX", raising=False)
    al, _, gr, it, st = emul(d, 1e-6, 1 | 4)
    ref = c_oracle.run_batch(tab, s1, s2, p1, p2, want_grad=True, threads=8)
    box = {"alpha": al, "grad": gr, "iters": it, "status": st}
    _check_vs_oracle(box, ref, 1e-9)
    # the same pairs on the dense rows: same iterations, rounding-level alpha
    monkeypatch.setenv("DCOL_NO_BOX", "1")
    al2, _, gr2, it2, st2 = emul(d, 1e-6, 1 | 4)
    np.testing.assert_array_equal(st2, st)
    np.testing.assert_array_equal(it2, it)
    ok = st == 0
    assert (np.abs(al2[ok] - al[ok]) <= 1e-9 * np.abs(al[ok])).all()


_SOLVE = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[2], sys.argv[3], sys.argv[3] + "/tests"]
from box_shapes import box_pairs, box_table
from dcol_amd import Engine, spec_from_arrays
rng = np.random.default_rng(int(sys.argv[4]))
tab, _ = box_table(rng)
s1, s2, p1, p2 = box_pairs(rng, tab, int(sys.argv[5]))
eng = Engine(device=0)
ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
plan = eng.plan(ids[s1], ids[s2], cache=False)
nbox = sum(b["pairs"] for b in plan.buckets() if b["kind"] == "solve" and b["flags"] & 8)
r = eng.solve_host(ids[s1], ids[s2], p1, p2, grad="fd", contact=False)
np.savez(sys.argv[1], alpha=r.alpha, grad=r.grad, iters=r.iters, status=r.status, nbox=nbox)
"""


def _gpu_solve(tmp_path, name, seed, B, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("DCOL_LIB", "DCOL_NO_BOX", "DCOL_LPP")}
    env.update(env_extra or {})
    f = str(tmp_path / f"{name}.npz")
    subprocess.run([sys.executable, "-c", _SOLVE, f, PKG, REPO, str(seed), str(B)], check=True, env=env, timeout=300)
    return dict(np.load(f))


@pytest.mark.gpu
def test_gpu_box_rows_asymmetric_match_oracle(tmp_path):
    """200k pairs of off-centre / rotated / parallelepiped boxes (and 4 non-box controls) on
    the GPU: the box x box pairs run the BOX kernel (its bucket holds exactly them), every
    pair matches the C oracle (status and iteration counts equal, alpha within 1e-6 rel and
    1e-9 rel, gradient within 1e-5 of max(|g|, 0.01)), and the dense-row run of the same
    pairs (DCOL_NO_BOX=1) has the same iteration counts and alpha to 1e-9 rel."""
    if not gpu_available():
        pytest.skip("no GPU")
    from oracle import c_oracle
    seed, B = 12, 200_000
    box = _gpu_solve(tmp_path, "box", seed, B)
    dense = _gpu_solve(tmp_path, "dense", seed, B, {"DCOL_NO_BOX": "1"})
    rng = np.random.default_rng(seed)
    tab, boxp = box_table(rng)
    s1, s2, p1, p2 = box_pairs(rng, tab, B)
    assert int(box["nbox"]) == int((boxp[s1] & boxp[s2]).sum()) > B // 2
    assert int(dense["nbox"]) == 0
    ref = c_oracle.run_batch(tab, s1, s2, p1, p2, want_grad=True, threads=16)
    _check_vs_oracle(box, ref, 1e-9)
    np.testing.assert_array_equal(dense["status"], box["status"])
    np.testing.assert_array_equal(dense["iters"], box["iters"])
    ok = box["status"] == 0
    assert (np.abs(dense["alpha"][ok] - box["alpha"][ok]) <= 1e-9 * np.abs(box["alpha"][ok])).all()
