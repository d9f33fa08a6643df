"""Child process of tests/test_dropin.py::test_pair_server_*_exit: makes drop-in calls so the
one-pair server is resident (long idle time), then exits WITHOUT destroying anything.
argv[1]: "python" -- the normal exit (the binding's atexit hook and the library's exit
handler both run); "c" -- the C library's exit() called directly, so Python's own teardown
(atexit hooks, Table.__del__) never runs and only the library's exit handler (registered at
the first server start) can stop the server, as in a C host that exits without destroying
its tables; "reopen" -- a fresh process: create a table and solve pairs (the device must be
usable after the others)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "dcol-trajectory-optimization_amd"), os.path.join(HERE, "..")]

import numpy as np  # noqa: E402


def main():
    mode = sys.argv[1]
    from dcol_amd.engine import default_engine
    from primitives.misc_primitive_constructor import SphereMRP, create_rect_prism
    from proximity.proximity import proximity_mrp
    from proximity.proximity_gradient import proximity_gradient
    box = create_rect_prism(1.0, 2.0, 0.5)
    ball = SphereMRP(0.4)
    box.r, box.p = np.zeros(3), np.array([0.1, -0.2, 0.3])
    alphas = []
    for k in range(20):
        ball.r, ball.p = np.array([2.0, 0.5 + 0.01 * k, -0.3]), np.zeros(3)
        alphas.append(proximity_mrp(ball, box)[0])
        if mode == "reopen":
            alphas.append(proximity_gradient(ball, box)[0])
    eng = default_engine()
    st = eng.pair_stats()
    running = eng.pair_server_running()
    print(f"CHILD_OK mode={mode} served={st['served']} running={int(running)} alpha0={alphas[0]!r}", flush=True)
    if mode == "c":
        import ctypes
        sys.stderr.flush()
        ctypes.CDLL(None).exit(0)      # C exit(): the C exit handlers run, Python's teardown does not
    if mode == "reopen":
        eng.stop_pair_server()
        assert not eng.pair_server_running()


if __name__ == "__main__":
    main()
