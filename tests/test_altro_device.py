"""Device dynamics Jacobians (include/dcol_altro_device.h, csrc/altro_device.hip): all knots
of a trajectory in one GPU launch (reference compute_jacobian,
ALTRO.py:77-100, per knot).  The kernel runs the host library's own dynamics source
(csrc/altro_model.hpp) without contraction, so its A, B must equal dcol_altro_jacobians
bitwise -- which the CPU tests pin to the reference's math (tests/test_altro.py)."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO, gpu_available
from test_altro import _models

HEADER = os.path.join(REPO, "include", "dcol_altro_device.h")


def test_header_symbols_exported_by_hip_library():
    from dcol_amd import _lib
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    fns = set(re.findall(r"\b(dcol_altro_[a-z_0-9]+)\s*\(", txt))
    assert fns == {"dcol_altro_jacobians_device"}
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert fns <= set(re.findall(r" T (dcol_altro_\w+)", out))


def test_host_provider_is_the_host_library():
    from altro import _native, jacobians
    model, _, nx, nu = _models()["quadrotor"]
    rng = np.random.default_rng(3)
    X, U = rng.normal(size=(11, nx)) * 0.5, rng.normal(size=(10, nu))
    h = jacobians.provider(model, 10, device=None)
    assert h.where == "host"
    h.submit(X, U)
    A, B = h.collect()
    A0, B0 = _native.jacobians(model, X, U)
    assert np.array_equal(A, A0) and np.array_equal(B, B0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["piano", "quadrotor", "rigid"])
@pytest.mark.parametrize("T", [1, 9, 100])
def test_device_jacobians_bitwise_equal_host(name, T):
    if not gpu_available():
        pytest.skip("no GPU")
    from altro import _native, jacobians
    model, _, nx, nu = _models()[name]
    rng = np.random.default_rng(T * 31 + nx)
    d = jacobians.provider(model, T, 0)
    assert d.where == "device"
    for rep in range(2):   # buffer reuse
        X = rng.normal(size=(T + 1, nx)) * 0.5
        U = rng.normal(size=(T, nu)) * (3 if name == "quadrotor" else 1)
        d.submit(X, U)
        A, B = d.collect()
        A0, B0 = _native.jacobians(model, X, U)
        assert np.array_equal(A, A0), np.abs(A - A0).max()
        assert np.array_equal(B, B0), np.abs(B - B0).max()


@pytest.mark.gpu
def test_device_jacobians_device_memory_and_args():
    """The entry point on plain device buffers (torch tensors), and argument checks."""
    if not gpu_available():
        pytest.skip("no GPU")
    import ctypes

    import torch
    from altro import _native, jacobians
    model, _, nx, nu = _models()["rigid"]
    T = 37
    rng = np.random.default_rng(5)
    X, U = rng.normal(size=(T, nx)) * 0.5, rng.normal(size=(T, nu))
    dev = torch.device("cuda", 0)
    dX, dU = torch.from_numpy(X).to(dev), torch.from_numpy(U).to(dev)
    dA = torch.empty((T, nx, nx), dtype=torch.float64, device=dev)
    dB = torch.empty((T, nx, nu), dtype=torch.float64, device=dev)
    fn = jacobians._device_fn()
    st = torch.cuda.current_stream(dev)
    args = lambda m, t, d: (ctypes.byref(m), t, dX.data_ptr(), dU.data_ptr(), d, dA.data_ptr(), dB.data_ptr(),  # noqa: E731
                            st.cuda_stream)
    assert fn(*args(model, T, 1e-6)) == _native.OK
    torch.cuda.synchronize(dev)
    A0, B0 = _native.jacobians(model, X, U)
    assert np.array_equal(dA.cpu().numpy(), A0) and np.array_equal(dB.cpu().numpy(), B0)
    assert fn(*args(model, T, 0.0)) == _native.ERR_ARG          # delta must be nonzero
    assert fn(*args(model, -1, 1e-6)) == _native.ERR_ARG
    bad = _native.make_model(_native.SYS_PIANO, 12, 3, 0.1, u_scale=100.0)   # piano is nx = 6
    assert fn(*args(bad, T, 1e-6)) == _native.ERR_ARG
    assert fn(*args(model, 0, 1e-6)) == _native.OK
