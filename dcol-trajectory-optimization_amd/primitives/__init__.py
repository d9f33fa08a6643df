"""Drop-in for the reference's ``primitives`` package (primitive data model + MRP utility).

Only what the proximity boundary and its callers import is provided:
``misc_primitive_constructor`` (the six primitive classes, create_rect_prism,
create_n_sided) and ``problem_matrices.dcm_from_mrp`` (used by the quadrotor dynamics,
cluttered_hallway_quadrotor.py:7).  The conic assembly itself runs on the GPU.
"""
