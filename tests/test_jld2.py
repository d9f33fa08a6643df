"""JLD2/HDF5 reader for the scene format: the reference's own data file
tests/golden/polytopes.jld2 (copied from systems/polytopes.jld2, read by the reference
through h5py at cluttered_hallway_quadrotor.py:271-279) decodes to the arrays the
quadrotor scene ships, and the reader rejects what it does not support."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

PATH = os.path.join(GOLDEN, "polytopes.jld2")


def test_reads_reference_file():
    from altro.systems import _data, jld2
    d = jld2.read(PATH)
    assert sorted(d) == ["A1", "A2", "b1", "b2"]
    assert d["A1"].shape == (3, 14) and d["A2"].shape == (3, 8)
    ref = _data.load()
    for k, v in d.items():
        assert np.array_equal(v, ref["jld2_" + k])
    # a polytope the engine accepts: the origin is inside (b > 0)
    assert (d["b1"] > 0).all() and (d["b2"] > 0).all()


def test_scene_from_file_equals_packaged():
    from altro.systems import cluttered_hallway_quadrotor as quad
    a = quad.obstacles()[4]
    b = quad.obstacles(PATH)[4]
    assert np.array_equal(a.A, b.A) and np.array_equal(a.b, b.b)


def test_rejects_non_hdf5(tmp_path):
    from altro.systems import jld2
    p = tmp_path / "x.jld2"
    p.write_bytes(b"not an hdf5 file" * 100)
    with pytest.raises(ValueError):
        jld2.read(str(p))
