"""Dynamics Jacobians of a whole trajectory for the ALTRO driver.

The reference differentiates the discrete dynamics knot by knot (compute_jacobian,
ALTRO.py:77-100, per knot at :289-290).  Here every knot of a trajectory goes in one call:

  DeviceJacobians  one GPU launch over all knots (dcol_altro_jacobians_device in libdcol.so,
                   include/dcol_altro_device.h) on a stream of its
                   own, so it runs beside the constraint batch's proximity solves (a phase
                   fills a few CUs), reading the trajectory from and writing A, B to
                   device-mapped pinned host buffers;
  HostJacobians    the host library's dcol_altro_jacobians (OpenMP over knots).

Both give bitwise the same A, B (tests/test_altro_device.py).  The driver picks the device
path when the constraint evaluator runs on the GPU (DCOL_ALTRO_JAC=host forces the host
one).  submit() starts the work, collect() returns (A [T, nx, nx], B [T, nx, nu]).
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, c_double, c_int, c_int64, c_void_p

import numpy as np

from . import _native

DELTA = 1e-6   # ALTRO.py:77 compute_jacobian default


class HostJacobians:
    where = "host"

    def __init__(self, model):
        self.model = model
        self._out = None

    def submit(self, X, U):
        self._out = _native.jacobians(self.model, X, U, DELTA)

    def collect(self):
        out, self._out = self._out, None
        return out


class DeviceUnavailable(RuntimeError):
    pass


def _device_fn():
    from dcol_amd import _lib
    fn = _lib.load().dcol_altro_jacobians_device
    fn.restype = c_int
    fn.argtypes = [POINTER(_native.Model), c_int64, c_void_p, c_void_p, c_double, c_void_p, c_void_p, c_void_p]
    return fn


class DeviceJacobians:
    """Jacobians of trajectories of T + 1 states on the GPU, on a stream of their own on
    `device` (index)."""
    where = "device"

    def __init__(self, model, T, device):
        import torch
        from dcol_amd import _lib
        self.model, self.T = model, int(T)
        self.stream = stream = torch.cuda.Stream(torch.device("cuda", int(device)))
        nx, nu = model.nx, model.nu
        n = self.T * (nx + nu + nx * nx + nx * nu)
        self._buf = torch.empty(max(n, 1), dtype=torch.float64, pin_memory=True)
        h = self._buf.numpy()
        o = np.cumsum([0, self.T * nx, self.T * nu, self.T * nx * nx])
        self._x = h[o[0]:o[1]].reshape(self.T, nx)
        self._u = h[o[1]:o[2]].reshape(self.T, nu)
        self._a = h[o[2]:o[3]].reshape(self.T, nx, nx)
        self._b = h[o[3]:o[3] + self.T * nx * nu].reshape(self.T, nx, nu)
        base = _lib.host_device_pointer(self._buf.data_ptr())
        if base is None:
            raise DeviceUnavailable("pinned buffer is not device-mapped")
        self._args = (ctypes.byref(model), self.T, c_void_p(base + 8 * int(o[0])), c_void_p(base + 8 * int(o[1])),
                      DELTA, c_void_p(base + 8 * int(o[2])), c_void_p(base + 8 * int(o[3])),
                      c_void_p(stream.cuda_stream))
        self._fn = _device_fn()
        self._pending = False
        self.submit(np.zeros((self.T, nx)), np.zeros((self.T, nu)))   # load the code object now
        self.collect()

    def submit(self, X, U):
        if self._pending:   # the kernel reads the pinned inputs this would overwrite
            raise RuntimeError("submit() while the previous batch is in flight: collect() it first")
        self._x[:] = np.asarray(X, dtype=np.float64).reshape(-1, self.model.nx)[: self.T]
        self._u[:] = np.asarray(U, dtype=np.float64).reshape(self.T, self.model.nu)
        _native._check(self._fn(*self._args), "dcol_altro_jacobians_device")
        self._pending = True

    def collect(self):
        if not self._pending:
            raise RuntimeError("collect() without submit()")
        self._pending = False
        self.stream.synchronize()
        return self._a.copy(), self._b.copy()


def provider(model, T, device=None, mode="device"):
    """DeviceJacobians on GPU `device` when mode == "device" and the GPU path is available,
    else HostJacobians."""
    if mode == "device" and device is not None:
        try:
            return DeviceJacobians(model, T, device)
        except DeviceUnavailable:
            pass
    return HostJacobians(model)
