"""Experiment inputs the reference hard-codes (initial control guesses taken from the
original Julia runs, piano_mover.py:223 and cluttered_hallway_quadrotor.py:375) and the
decoded systems/polytopes.jld2 arrays (cluttered_hallway_quadrotor.py:271-279), stored as
data by tests/golden/gen_altro.py."""
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "initial_guess.npz")
_cache = None


def load():
    global _cache
    if _cache is None:
        with np.load(_PATH) as d:
            _cache = {k: d[k].copy() for k in d.files}
    return _cache
