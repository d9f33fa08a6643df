"""proximity_gradient — drop-in for the reference's proximity/proximity_gradient.py:91-138.

alpha and d alpha / d[r1, p1, r2, p2] (12,) for two primitives at their current poses.
The gradient follows the reference's envelope formulation: forward differences (step
sqrt(eps), scipy approx_fprime semantics) of z'(G(theta) x - h(theta)) at the PDIP
solution (x, z), computed on the GPU next to the solve.
"""
from dcol_amd.engine import DEFAULT_TOL, default_engine, raise_for_status


def proximity_gradient(prim1, prim2, pdip_tol=DEFAULT_TOL, verbose=False):
    """-> (alpha: float64, d_alpha_d_state: ndarray(12)).  Raises like the reference."""
    alpha, _, grad, _, status = default_engine().solve_pair(prim1, prim2, tol=pdip_tol, grad="fd", contact=False)
    raise_for_status(status)
    return alpha, grad


def proximity_gradient_batch(prims1, prims2, pdip_tol=DEFAULT_TOL, grad="fd"):
    """Batched form -> (alpha [B], grad [B, 12], status [B]); grad = 'fd' (reference
    mode), 'envelope' (closed form of the same derivative) or 'implicit' (implicit-function
    derivative of the returned iterate through the PDIP's normal matrix; closer to the true
    d alpha / d pose than the reference's formulation at the same tolerance)."""
    res = default_engine().solve_objects(prims1, prims2, tol=pdip_tol, grad=grad, contact=False)
    return res.alpha, res.grad, res.status
