"""ctypes binding of include/dcol_altro.h (lib/libdcol_altro.so, built in-tree by csrc/Makefile).

No NumPy fallback: if the library is missing every call raises AltroLibraryError."""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_int, c_int32, c_int64, c_void_p

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("DCOL_ALTRO_LIB", os.path.join(PKG_ROOT, "lib", "libdcol_altro.so"))

SYS_PIANO, SYS_QUADROTOR, SYS_RIGID = 0, 1, 2
OK, ERR_ARG, ERR_NOT_PD, ERR_DEVICE = 0, -1, -2, -3
ABI_VERSION = 2
MAX_NX, MAX_NU = 16, 8


class AltroLibraryError(RuntimeError):
    pass


class Model(ctypes.Structure):
    """struct dcol_altro_model"""
    _fields_ = [("system", c_int32), ("nx", c_int32), ("nu", c_int32), ("dt", c_double), ("mass", c_double),
                ("inertia", c_double * 9), ("gravity", c_double * 3), ("arm", c_double), ("kf", c_double),
                ("km", c_double), ("u_scale", c_double)]


class Problem(ctypes.Structure):
    """struct dcol_altro_problem (pointers into arrays kept alive by `keep`)"""
    _fields_ = [("N", c_int32), ("nx", c_int32), ("nu", c_int32), ("ncx", c_int32), ("Q", c_void_p),
                ("R", c_void_p), ("Qf", c_void_p), ("Xref", c_void_p), ("Uref", c_void_p), ("u_min", c_void_p),
                ("u_max", c_void_p)]


SIGNATURES = {
    "dcol_altro_abi_version": (c_int32, []),
    "dcol_altro_dynamics": (c_int, [POINTER(Model), c_int64, c_void_p, c_void_p, c_void_p]),
    "dcol_altro_jacobians": (c_int, [POINTER(Model), c_int64, c_void_p, c_void_p, c_double, c_void_p, c_void_p]),
    "dcol_altro_backward": (c_int, [c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_double, c_void_p, c_void_p, POINTER(c_double),
                                    POINTER(c_int64)]),
    "dcol_altro_rollout": (c_int, [POINTER(Model), c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_double,
                                   c_void_p, c_void_p]),
    "dcol_altro_rollouts": (c_int, [POINTER(Model), c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_int32, c_void_p, c_void_p]),
    "dcol_altro_cost": (c_int, [POINTER(Problem), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_double, POINTER(c_double)]),
    "dcol_altro_stage_terms": (c_int, [POINTER(Problem), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_double, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p]),
    "dcol_altro_victim_poses": (c_int, [POINTER(Model), c_int64, c_void_p, c_void_p]),
    "dcol_altro_backward_pass": (c_int, [POINTER(Model), POINTER(Problem), c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_double, c_double,
                                         c_void_p, c_void_p, POINTER(c_double), POINTER(c_double), POINTER(c_int64)]),
    "dcol_altro_trial": (c_int, [POINTER(Model), c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_double, c_void_p,
                                 c_void_p, c_void_p]),
    "dcol_altro_constraint_jacobian": (c_int, [POINTER(Model), c_int64, c_int32, c_void_p, c_void_p, c_void_p]),
}

_lib = None


def load(path: str | None = None):
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:
        raise AltroLibraryError(f"cannot load {p}: {e} (build it: make -C csrc)") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    if lib.dcol_altro_abi_version() != ABI_VERSION:
        raise AltroLibraryError(f"{p}: ABI version {lib.dcol_altro_abi_version()} != {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def _ptr(a):
    """address of a C-contiguous array's data (an int: ctypes converts it for c_void_p); the
    buffer protocol is ~3x cheaper per call than ndarray.ctypes, which matters at ~30 calls
    per optimizer iteration"""
    try:
        return ctypes.addressof(ctypes.c_char.from_buffer(a))
    except (TypeError, ValueError, BufferError):      # read-only, empty or strided arrays
        return a.ctypes.data


def _c(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None and a.shape != tuple(shape):
        a = a.reshape(shape)
    return a


def _check(rc, what):
    if rc == ERR_ARG:
        raise ValueError(f"{what}: invalid argument")
    if rc != OK:
        raise AltroLibraryError(f"{what}: error {rc}")


def make_model(system, nx, nu, dt, mass=0.0, inertia=None, gravity=(0.0, 0.0, 0.0), arm=0.0, kf=0.0, km=0.0,
               u_scale=0.0) -> Model:
    m = Model()
    m.system, m.nx, m.nu, m.dt, m.mass = int(system), int(nx), int(nu), float(dt), float(mass)
    J = np.zeros(9) if inertia is None else np.asarray(inertia, dtype=np.float64).reshape(9)
    for i in range(9):
        m.inertia[i] = J[i]
    for i in range(3):
        m.gravity[i] = float(gravity[i])
    m.arm, m.kf, m.km, m.u_scale = float(arm), float(kf), float(km), float(u_scale)
    return m


def dynamics(model: Model, X, U):
    """RK4 step of every row: X [M, nx], U [M, nu] -> [M, nx]."""
    X = _c(X).reshape(-1, model.nx)
    U = _c(U).reshape(-1, model.nu)
    if X.shape[0] != U.shape[0]:
        raise ValueError("X and U must have the same number of rows")
    out = np.empty_like(X)
    _check(load().dcol_altro_dynamics(ctypes.byref(model), X.shape[0], _ptr(X), _ptr(U), _ptr(out)),
           "dcol_altro_dynamics")
    return out


def jacobians(model: Model, X, U, delta=1e-6):
    """Forward-difference A [T, nx, nx], B [T, nx, nu] at the first T = len(U) knots."""
    U = _c(U).reshape(-1, model.nu)
    T = U.shape[0]
    X = _c(X).reshape(-1, model.nx)[:T]
    X = np.ascontiguousarray(X)
    A = np.empty((T, model.nx, model.nx))
    B = np.empty((T, model.nx, model.nu))
    _check(load().dcol_altro_jacobians(ctypes.byref(model), T, _ptr(X), _ptr(U), float(delta), _ptr(A), _ptr(B)),
           "dcol_altro_jacobians")
    return A, B


def backward(A, B, lx, lu, lxx, luu, VxT, VxxT, reg):
    """Riccati recursion -> (K [T, nu, nx], k [T, nu], dJ).  Raises
    numpy.linalg.LinAlgError (like scipy's cho_factor) when Quu is not positive definite."""
    A = _c(A)
    T, nx, _ = A.shape
    nu = B.shape[2]
    B, lx, lu, lxx, luu = _c(B), _c(lx), _c(lu), _c(lxx), _c(luu)
    VxT, VxxT = _c(VxT), _c(VxxT)
    K = np.empty((T, nu, nx))
    k = np.empty((T, nu))
    dJ = c_double()
    fail = c_int64(-1)
    rc = load().dcol_altro_backward(T, nx, nu, _ptr(A), _ptr(B), _ptr(lx), _ptr(lu), _ptr(lxx), _ptr(luu),
                                    _ptr(VxT), _ptr(VxxT), float(reg), _ptr(K), _ptr(k), ctypes.byref(dJ),
                                    ctypes.byref(fail))
    if rc == ERR_NOT_PD:
        raise np.linalg.LinAlgError(f"Quu is not positive definite at knot {fail.value}")
    _check(rc, "dcol_altro_backward")
    return K, k, dJ.value


def rollout(model: Model, X, U, K, k, a):
    """Closed-loop rollout -> (Xn [T+1, nx], Un [T, nu])."""
    X, U, K, k = _c(X), _c(U), _c(K), _c(k)
    T = U.shape[0]
    if X.shape != (T + 1, model.nx) or K.shape != (T, model.nu, model.nx) or k.shape != (T, model.nu):
        raise ValueError("rollout: inconsistent shapes")
    Xn = np.empty_like(X)
    Un = np.empty_like(U)
    _check(load().dcol_altro_rollout(ctypes.byref(model), T, _ptr(X), _ptr(U), _ptr(K), _ptr(k), float(a), _ptr(Xn),
                                     _ptr(Un)), "dcol_altro_rollout")
    return Xn, Un


def rollouts(model: Model, X, U, K, k, a_list):
    """Closed-loop rollouts at several step lengths (one per host thread) -> (Xn [na, T+1, nx],
    Un [na, T, nu]); Xn[j], Un[j] equal rollout(..., a_list[j]) bitwise."""
    X, U, K, k = _c(X), _c(U), _c(K), _c(k)
    a = np.ascontiguousarray(a_list, dtype=np.float64).reshape(-1)
    T = U.shape[0]
    if X.shape != (T + 1, model.nx) or K.shape != (T, model.nu, model.nx) or k.shape != (T, model.nu):
        raise ValueError("rollouts: inconsistent shapes")
    Xn = np.empty((a.size,) + X.shape)
    Un = np.empty((a.size,) + U.shape)
    _check(load().dcol_altro_rollouts(ctypes.byref(model), T, _ptr(X), _ptr(U), _ptr(K), _ptr(k), _ptr(a), a.size,
                                      _ptr(Xn), _ptr(Un)), "dcol_altro_rollouts")
    return Xn, Un


def make_problem(N, nx, nu, ncx, Q, R, Qf, Xref, Uref, u_min, u_max) -> Problem:
    """struct dcol_altro_problem over contiguous float64 copies (held in .keep)."""
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (Q, R, Qf, Xref, Uref, u_min, u_max)]
    shapes = [(nx, nx), (nu, nu), (nx, nx), (N, nx), (N - 1, nu), (nu,), (nu,)]
    arrs = [a.reshape(sh) for a, sh in zip(arrs, shapes)]
    p = Problem(int(N), int(nx), int(nu), int(ncx), *[_ptr(a) for a in arrs])
    p.keep = arrs
    return p


def cost(prob: Problem, X, U, hx, mu, mux, lam, rho):
    """Augmented-Lagrangian objective (ALTRO.py compute_total_cost)."""
    X, U, hx, mu, mux, lam = (_c(a) for a in (X, U, hx, mu, mux, lam))
    J = c_double()
    _check(load().dcol_altro_cost(ctypes.byref(prob), _ptr(X), _ptr(U), _ptr(hx), _ptr(mu), _ptr(mux), _ptr(lam),
                                  float(rho), ctypes.byref(J)), "dcol_altro_cost")
    return J.value


def stage_terms(prob: Problem, X, U, hx, Gx, mu, mux, lam, rho):
    """-> (lx [N-1,nx], lu [N-1,nu], lxx [N-1,nx,nx], luu [N-1,nu,nu], VxT [nx], VxxT [nx,nx])."""
    N, nx, nu = prob.N, prob.nx, prob.nu
    X, U, hx, Gx, mu, mux, lam = (_c(a) for a in (X, U, hx, Gx, mu, mux, lam))
    lx = np.empty((N - 1, nx))
    lu = np.empty((N - 1, nu))
    lxx = np.empty((N - 1, nx, nx))
    luu = np.empty((N - 1, nu, nu))
    VxT = np.empty(nx)
    VxxT = np.empty((nx, nx))
    _check(load().dcol_altro_stage_terms(ctypes.byref(prob), _ptr(X), _ptr(U), _ptr(hx), _ptr(Gx), _ptr(mu),
                                         _ptr(mux), _ptr(lam), float(rho), _ptr(lx), _ptr(lu), _ptr(lxx), _ptr(luu),
                                         _ptr(VxT), _ptr(VxxT)), "dcol_altro_stage_terms")
    return lx, lu, lxx, luu, VxT, VxxT


def victim_poses(model: Model, X):
    X = _c(X).reshape(-1, model.nx)
    P = np.empty((X.shape[0], 6))
    _check(load().dcol_altro_victim_poses(ctypes.byref(model), X.shape[0], _ptr(X), _ptr(P)),
           "dcol_altro_victim_poses")
    return P


def constraint_jacobian(model: Model, X, dalpha):
    X = _c(X).reshape(-1, model.nx)
    N = X.shape[0]
    D = _c(dalpha).reshape(N, -1, 12)
    G = np.empty((N, D.shape[1], model.nx))
    _check(load().dcol_altro_constraint_jacobian(ctypes.byref(model), N, D.shape[1], _ptr(X), _ptr(D), _ptr(G)),
           "dcol_altro_constraint_jacobian")
    return G


def backward_pass(model: Model, prob: Problem, X, U, alpha, dalpha, A, B, mu, mux, lam, rho, reg, soa=False):
    """One backward pass in one call (dcol_altro_backward_pass): hx = 1 - alpha, constraint
    Jacobian, stage terms, Riccati sweep and the AL cost of (X, U) -> (K, k, dJ, J).  dalpha
    [N, ncx, 12], or with soa=True the engine's component-major [12, N ncx] (as the GPU batch
    returns it: no transpose).  Raises numpy.linalg.LinAlgError when Quu is not positive
    definite (like backward())."""
    N, nx, nu = prob.N, prob.nx, prob.nu
    X, U, alpha, dalpha, A, B, mu, mux, lam = (_c(a) for a in (X, U, alpha, dalpha, A, B, mu, mux, lam))
    stride = 0
    if soa:
        if dalpha.ndim != 2 or dalpha.shape[0] != 12 or dalpha.shape[1] != N * prob.ncx:
            raise ValueError("backward_pass: soa dalpha must be [12, N * ncx]")
        stride = dalpha.shape[1]
    K = np.empty((N - 1, nu, nx))
    k = np.empty((N - 1, nu))
    dJ, J, fail = c_double(), c_double(), c_int64(-1)
    rc = load().dcol_altro_backward_pass(ctypes.byref(model), ctypes.byref(prob), _ptr(X), _ptr(U), _ptr(alpha),
                                         _ptr(dalpha), stride, _ptr(A), _ptr(B), _ptr(mu), _ptr(mux), _ptr(lam), float(rho),
                                         float(reg), _ptr(K), _ptr(k), ctypes.byref(dJ), ctypes.byref(J),
                                         ctypes.byref(fail))
    if rc == ERR_NOT_PD:
        raise np.linalg.LinAlgError(f"Quu is not positive definite at knot {fail.value}")
    _check(rc, "dcol_altro_backward_pass")
    return K, k, dJ.value, J.value


def trial(model: Model, X, U, K, k, a):
    """One line-search trial in one call (dcol_altro_trial): closed-loop rollout at step a
    and the victim poses of the rolled-out states -> (Xn, Un, poses [T+1, 6])."""
    X, U, K, k = _c(X), _c(U), _c(K), _c(k)
    T = U.shape[0]
    Xn = np.empty_like(X)
    Un = np.empty_like(U)
    P = np.empty((T + 1, 6))
    _check(load().dcol_altro_trial(ctypes.byref(model), T, _ptr(X), _ptr(U), _ptr(K), _ptr(k), float(a), _ptr(Xn),
                                   _ptr(Un), _ptr(P)), "dcol_altro_trial")
    return Xn, Un, P
