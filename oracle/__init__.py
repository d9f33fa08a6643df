"""Test infrastructure ONLY: CPU restatements of the reference DCOL proximity path.

Nothing under ``oracle/`` is part of the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker / the timed CPU baseline.  The product path
(``dcol-trajectory-optimization_amd/``) never imports this package.

Parity of these restatements is pinned against golden vectors produced by the
reference itself (``tests/golden/gen_golden.py`` imports ``/root/reference`` in the
build container and records its outputs); see ``tests/test_oracle_golden.py``.
"""
