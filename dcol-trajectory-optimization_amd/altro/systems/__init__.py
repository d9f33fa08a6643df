"""Trajectory-optimization problems of the reference (systems/*.py), set up for the
batched driver.  ``get(name)`` maps the reference's params['system'] names
(ALTRO.py:341-362) to the modules here."""
import importlib

_MODULES = {"piano_mover": "piano_mover", "quadrotor": "cluttered_hallway_quadrotor",
            "coneThroughWall": "cone_through_wall"}


def get(name: str):
    try:
        mod = _MODULES[name]
    except KeyError:
        raise ValueError(f"System '{name}' is not recognized. Must be 'piano_mover', 'quadrotor' or "
                         f"'coneThroughWall'.") from None
    return importlib.import_module(f"{__name__}.{mod}")


def initialize(name: str):
    """-> (params, X, U) exactly as the reference's initialize_<system>()."""
    m = get(name)
    return m.initialize()
