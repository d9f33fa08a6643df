"""proximity_mrp — drop-in for the reference's proximity/proximity.py:6-54.

Minimum uniform scaling alpha at which two primitives (at their current .r/.p poses)
touch, and the contact point x[0:3] of the scaled problem.  The conic assembly
(problem_matrices + combine_problem_matrices) and the PDIP solve run on the GPU.
"""
from dcol_amd.engine import DEFAULT_TOL, default_engine, raise_for_status


def proximity_mrp(prim1, prim2, pdip_tol=DEFAULT_TOL, verbose=False):
    """-> (alpha: float64, contact_point: ndarray(3)).  Raises like the reference:
    Exception after 50 PDIP iterations, ValueError for unsupported pairs,
    numpy.linalg.LinAlgError for a non-PD normal matrix."""
    alpha, contact, _, _, status = default_engine().solve_pair(prim1, prim2, tol=pdip_tol, grad=None, contact=True)
    raise_for_status(status)
    return alpha, contact


def proximity_mrp_batch(prims1, prims2, pdip_tol=DEFAULT_TOL):
    """Batched form: equal-length sequences of primitives -> (alpha [B], contact [B, 3],
    status [B]).  No exception per pair: inspect status (dcol_amd._lib.OK == 0)."""
    res = default_engine().solve_objects(prims1, prims2, tol=pdip_tol, grad=None, contact=True)
    return res.alpha, res.contact, res.status
