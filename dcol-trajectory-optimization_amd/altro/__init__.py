"""altro — batched AL-iLQR trajectory optimizer over the MI355X proximity engine.

Mirrors the reference's ALTRO.py entry point and its three systems:

    from altro import ALTRO, systems
    params, X, U = systems.initialize("piano_mover")
    X, U = ALTRO(params, X, U)

All N x n_obs collision constraints of an optimizer phase are solved as one GPU batch
(constraints.ObstacleField over dcol_amd); dynamics Jacobians, the Riccati recursion and
the closed-loop rollout run in the native host library lib/libdcol_altro.so.
"""
from . import systems
from .driver import ALTRO, AltroResult, solve

__all__ = ["ALTRO", "AltroResult", "solve", "systems"]
