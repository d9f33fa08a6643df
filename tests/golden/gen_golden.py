#!/usr/bin/env python3
"""Generate the golden parity vectors by running the REFERENCE implementation.

Runs ONLY in the build container, where /root/reference (CogSP/DCOL-trajectory-optimization)
is mounted read-only.  Imports the reference's own modules (PYTHONDONTWRITEBYTECODE=1 so
nothing is written into it), drives them on fixed, seeded inputs, and writes small .npz
fixtures next to this script.  The fixtures are data only (inputs + the reference's
outputs); no reference source travels with them.

Fixture layout (every file):
  shape table  : type[S] nh[S] A_off[S] A_pool[K,3] b_pool[K] params[S,4]=(R,L,H,beta)
                 r_offset[S,3] Q_offset[S,3,3]
  pairs        : s1[B] s2[B] pose1[B,6] pose2[B,6]  (pose = [r(3), p(3)] MRP)
  reference out: alpha[B] contact[B,3] grad[B,12] iters[B] status[B] x[B,nmax] s[B,mmax]
                 z[B,mmax] m[B] n[B]   (iters = Newton steps = calc_NT_scalings calls - 1)
  tol          : scalar pdip_tol used

Usage:  python tests/golden/gen_golden.py [--only NAME]
"""
import argparse
import os
import sys
import time

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

from primitives import misc_primitive_constructor as mpc  # noqa: E402
from primitives.problem_matrices import problem_matrices  # noqa: E402
from primitives.combine_problem_matrices import combine_problem_matrices  # noqa: E402
from proximity import pdip as ref_pdip  # noqa: E402
from proximity.proximity_gradient import proximity_gradient  # noqa: E402
from proximity.proximity import proximity_mrp  # noqa: E402

POLYTOPE, SPHERE, CONE, CAPSULE, CYLINDER, POLYGON = range(6)
ST_OK, ST_MAXITER, ST_UNSUPPORTED, ST_NOT_PD, ST_NONFINITE = 0, 1, 2, 3, 4


# ------------------------------------------------------------------------------ helpers
class Table:
    """Accumulates reference primitive objects and their array encoding."""

    def __init__(self):
        self.objs, self.type, self.nh, self.A_off, self.params = [], [], [], [], []
        self.r_offset, self.Q_offset, self.A_rows, self.b_rows = [], [], [], []

    def add(self, obj):
        if isinstance(obj, mpc.PolytopeMRP):
            t, A, b = POLYTOPE, np.asarray(obj.A, float), np.asarray(obj.b, float)
            prm = (0, 0, 0, 0)
        elif isinstance(obj, mpc.SphereMRP):
            t, A, b, prm = SPHERE, None, None, (obj.R, 0, 0, 0)
        elif isinstance(obj, mpc.ConeMRP):
            t, A, b, prm = CONE, None, None, (0, 0, obj.H, obj.beta)
        elif isinstance(obj, mpc.CapsuleMRP):
            t, A, b, prm = CAPSULE, None, None, (obj.R, obj.L, 0, 0)
        elif isinstance(obj, mpc.CylinderMRP):
            t, A, b, prm = CYLINDER, None, None, (obj.R, obj.L, 0, 0)
        elif isinstance(obj, mpc.PolygonMRP):
            t, A, b = POLYGON, np.asarray(obj.A, float), np.asarray(obj.b, float)
            prm = (obj.R, 0, 0, 0)
        else:
            raise TypeError(obj)
        self.objs.append(obj)
        self.type.append(t)
        self.params.append(prm)
        self.r_offset.append(np.asarray(obj.r_offset, float))
        self.Q_offset.append(np.asarray(obj.Q_offset, float))
        self.A_off.append(len(self.A_rows))
        if A is not None:
            self.nh.append(A.shape[0])
            for j in range(A.shape[0]):
                row = np.zeros(3)
                row[:A.shape[1]] = A[j]
                self.A_rows.append(row)
                self.b_rows.append(b[j])
        else:
            self.nh.append(0)
        return len(self.objs) - 1

    def arrays(self):
        return dict(type=np.array(self.type, np.int32), nh=np.array(self.nh, np.int32),
                    A_off=np.array(self.A_off, np.int32),
                    A_pool=np.array(self.A_rows, float).reshape(-1, 3),
                    b_pool=np.array(self.b_rows, float),
                    params=np.array(self.params, float).reshape(-1, 4),
                    r_offset=np.array(self.r_offset, float).reshape(-1, 3),
                    Q_offset=np.array(self.Q_offset, float).reshape(-1, 3, 3))


class IterCounter:
    """Counts calc_NT_scalings calls inside the reference's pdip module."""

    def __init__(self):
        self.n = 0
        self.orig = ref_pdip.calc_NT_scalings

    def __enter__(self):
        def wrapped(*a, **k):
            self.n += 1
            return self.orig(*a, **k)
        ref_pdip.calc_NT_scalings = wrapped
        return self

    def __exit__(self, *exc):
        ref_pdip.calc_NT_scalings = self.orig


class Unsupported(Exception):
    pass


def ref_solve(o1, o2, tol):
    """Reference pieces, exactly as proximity_mrp chains them (proximity.py:23-44)."""
    G_o1, h_o1, G_s1, h_s1 = problem_matrices(o1, o1.r, o1.p)
    G_o2, h_o2, G_s2, h_s2 = problem_matrices(o2, o2.r, o2.p)
    if len(G_o1.shape) == 1:
        G_o1 = G_o1.reshape(1, -1)
    if len(G_o2.shape) == 1:
        G_o2 = G_o2.reshape(1, -1)
    try:
        c, G, h, io, i1, i2 = combine_problem_matrices(G_o1, h_o1, G_s1, h_s1, G_o2, h_o2, G_s2, h_s2)
    except ValueError as e:
        raise Unsupported(str(e))
    with IterCounter() as cnt:
        x, s, z = ref_pdip.solve_lp_pdip(c, G, h, io, i1, i2, pdip_tol=tol)
    return x, s, z, cnt.n - 1


def run_pairs(tab, pairs, tol=1e-6, want_grad=True, name=""):
    """pairs: list of (s1, s2, pose1(6), pose2(6)).  Drives the reference."""
    B = len(pairs)
    MM, NN = 136, 8
    out = dict(alpha=np.full(B, np.nan), contact=np.full((B, 3), np.nan),
               grad=np.full((B, 12), np.nan), iters=np.full(B, -1, np.int32),
               status=np.zeros(B, np.int32), x=np.full((B, NN), np.nan),
               s=np.full((B, MM), np.nan), z=np.full((B, MM), np.nan),
               m=np.zeros(B, np.int32), n=np.zeros(B, np.int32))
    t0 = time.time()
    for i, (k1, k2, q1, q2) in enumerate(pairs):
        o1, o2 = tab.objs[k1], tab.objs[k2]
        o1.r, o1.p = np.array(q1[:3], float), np.array(q1[3:], float)
        o2.r, o2.p = np.array(q2[:3], float), np.array(q2[3:], float)
        try:
            x, s, z, it = ref_solve(o1, o2, tol)
            a_mrp, cp = proximity_mrp(o1, o2, pdip_tol=tol)
            assert a_mrp == x[3] and np.array_equal(cp, x[:3])
            if want_grad:
                a_g, g = proximity_gradient(o1, o2, pdip_tol=tol)
                assert a_g == x[3]
                out["grad"][i] = g
            out["alpha"][i] = x[3]
            out["contact"][i] = x[:3]
            out["iters"][i] = it
            out["x"][i, :len(x)] = x
            out["s"][i, :len(s)] = s
            out["z"][i, :len(z)] = z
            out["m"][i], out["n"][i] = len(s), len(x)
        except Unsupported:
            out["status"][i] = ST_UNSUPPORTED
        except ValueError:   # scipy check_finite: non-finite iterate reached a factorisation
            out["status"][i] = ST_NONFINITE
        except np.linalg.LinAlgError:
            out["status"][i] = ST_NOT_PD
        except Exception as e:  # the reference raises a bare Exception at 50 iterations
            if "Maximum number of iterations" in str(e):
                out["status"][i] = ST_MAXITER
            else:
                raise
    dt = time.time() - t0
    ok = out["status"] == 0
    print(f"[{name}] {B} pairs in {dt:.1f}s ({1e3 * dt / max(B, 1):.2f} ms/pair), "
          f"ok={ok.sum()} iters mean={out['iters'][ok].mean() if ok.any() else 0:.2f}", flush=True)
    return out


def save(name, tab, pairs, out, tol, **extra):
    arr = tab.arrays()
    arr.update(s1=np.array([p[0] for p in pairs], np.int32), s2=np.array([p[1] for p in pairs], np.int32),
               pose1=np.array([p[2] for p in pairs], float).reshape(-1, 6),
               pose2=np.array([p[3] for p in pairs], float).reshape(-1, 6), tol=np.float64(tol))
    mm = int(max(out["m"].max(), 1))
    nn = int(max(out["n"].max(), 1))
    out = dict(out)
    out["s"], out["z"], out["x"] = out["s"][:, :mm], out["z"][:, :mm], out["x"][:, :nn]
    arr.update(out)
    arr.update(extra)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **arr)
    print(f"  -> {path} ({os.path.getsize(path) / 1024:.0f} KB)")


# ------------------------------------------------------------------------------ scenes
def jld2_polytopes():
    """Decode systems/polytopes.jld2 (HDF5 compact datasets; no h5py in this image).
    Byte offsets located by inspection: A1 0x276 (3x14), b1 0x407 (14),
    A2 0x4C0 (3x8), b2 0x5C1 (8)."""
    raw = open(os.path.join(REF, "systems", "polytopes.jld2"), "rb").read()

    def f64(off, n):
        return np.frombuffer(raw[off:off + 8 * n], dtype="<f8").copy()
    return dict(A1=f64(0x276, 42).reshape(3, 14), b1=f64(0x407, 14),
                A2=f64(0x4C0, 24).reshape(3, 8), b2=f64(0x5C1, 8))


def scene_piano(rng):
    """piano_mover.py:137-228: thin rect vehicle vs 3 rect walls, N = 80."""
    tab = Table()
    vic = tab.add(mpc.create_rect_prism(2.5, 0.15, 0.01))
    obs = [tab.add(mpc.create_rect_prism(3.0, 3.0, 1.0)), tab.add(mpc.create_rect_prism(4.0, 1.0, 1.0)),
           tab.add(mpc.create_rect_prism(1.0, 5.0, 1.1))]
    opose = [[1.5, 3.5, 0.0, 0, 0, 0], [2, 0.5, 0, 0, 0, 0], [4.5, 2.5, 0, 0, 0, 0]]
    N = 80
    x0 = np.array([1.5, 1.5, 0, 0, 0, 0])
    xg = np.array([3.5, 3.7, 0, 0, np.deg2rad(90), 0])
    pairs = []
    for traj in range(2):
        for k in range(N):
            x = x0 + (xg - x0) * k / (N - 1)
            if traj == 1:
                x = x + rng.normal(0, [0.4, 0.4, 0, 0, 0.5, 0])
            pv = [x[0], x[1], 0, 0, 0, np.tan(x[4] / 4)]         # piano_mover.py:60-61
            for j, o in enumerate(obs):
                pairs.append((vic, o, pv, opose[j]))
    return tab, pairs


def scene_quad(rng):
    """cluttered_hallway_quadrotor.py:227-331: sphere R=0.25 vs 11 obstacles, N = 100."""
    P = jld2_polytopes()
    tab = Table()
    vic = tab.add(mpc.SphereMRP(radius=0.25))
    bot = mpc.create_rect_prism(length=20, width=5, height=0.2)
    top = mpc.create_rect_prism(length=20, width=5, height=0.2)
    poly = mpc.create_n_sided(5, 0.6)
    objs = [mpc.CylinderMRP(radius=0.6, height=3.0), mpc.CapsuleMRP(radius=0.2, height=5.0),
            mpc.SphereMRP(radius=0.8), mpc.ConeMRP(height=2.0, beta=np.deg2rad(22)),
            mpc.PolytopeMRP(P["A2"].T, P["b2"]), mpc.PolygonMRP(poly["A"], poly["b"], 0.2),
            mpc.CylinderMRP(radius=1.1, height=2.3), mpc.CapsuleMRP(radius=0.8, height=1.0),
            mpc.SphereMRP(radius=0.5), bot, top]
    poses = [
        ([-5.0, -0.3597289068234817, 4.087208492428585], [0.9743462834661368, 0.5695654691654629, -0.929297065594203]),
        ([-3.75, 2.0547630560640364, 3.3248927294469155], [0.44432216225861665, -0.8131633664490159, 0.8533462452863487]),
        ([-2.5, 0.01357380155160959, 3.1056516058837307], [-0.7818142467739891, -1.0606493186561021, -0.6997594248738506]),
        ([-1.25, 0.1520302408349855, 2.100626290031169], [0.09970204047057568, -0.6590733218999884, 0.10747184882042882]),
        ([0.0, 0.27038613194550204, 4.579317307027433], [-1.178486073522902, -0.5852806292416908, -0.5104503832374265]),
        ([1.25, -0.20563037602802728, 3.7707031750912097], [1.322242556684692, 1.477962368008582, -0.09186250030835676]),
        ([2.5, 1.724189934074888, 3.1527083547286816], [-1.670756785490579, -1.6504683581003534, 0.9958143390876766]),
        ([3.75, -0.7885513165549604, 2.3533371368422706], [0.40980738483268503, 0.5108420391824778, 0.42272633604120335]),
        ([5.0, 0.32074771862886275, 4.251199978479224], [1.8822143307659809, -0.7779808480817001, 0.8308676764061569]),
        ([0, 0, 0.9], [0, 0, 0]), ([0, 0, 6.0], [0, 0, 0])]
    obs = [tab.add(o) for o in objs]
    N = 100
    pairs = []
    for traj in range(2):
        for k in range(N):
            r = np.array([-8.0, 0, 4]) + np.array([16.0, 0, 0]) * k / (N - 1)
            p = np.zeros(3)
            if traj == 1:
                r = r + rng.normal(0, [0.3, 1.0, 0.8])
                p = rng.uniform(-0.4, 0.4, 3)
            for j, o in enumerate(obs):
                pairs.append((vic, o, list(r) + list(p), list(poses[j][0]) + list(poses[j][1])))
    return tab, pairs


def scene_cone(rng):
    """cone_through_wall.py:209-331: cone H=2, beta=22deg vs 4 rect prisms, N = 60."""
    tab = Table()
    vic = tab.add(mpc.ConeMRP(height=2.0, beta=np.deg2rad(22)))
    objs = [mpc.create_rect_prism(10.0, 10.0, 1.0), mpc.create_rect_prism(10.0, 10.0, 1.0),
            mpc.create_rect_prism(4.1, 4.1, 1.1), mpc.create_rect_prism(4.1, 4.1, 1.1)]
    q = np.array([np.cos(np.pi / 4), np.sin(np.pi / 4), 0, 0])
    pw = list(q[1:4] / (1 + q[0]))                                   # mrp_from_q
    rs = [[-6, 0, 5.0], [6, 0, 5.0], [0, 0, 2.05], [0, 0, 7.96]]
    obs = [tab.add(o) for o in objs]
    N = 60
    pairs = []
    x0, xg = np.array([-4.0, -7, 9]), np.array([-4.5, 7, 3])
    for traj in range(2):
        for k in range(N):
            r = x0 + (xg - x0) * k / (N - 1)
            p = np.zeros(3)
            if traj == 1:
                r = r + rng.normal(0, 0.5, 3)
                p = rng.uniform(-0.5, 0.5, 3)
            for j, o in enumerate(obs):
                pairs.append((vic, o, list(r) + list(p), rs[j] + pw))
    return tab, pairs


def rand_prism(rng):
    d = rng.uniform(0.2, 2.0, 3)
    return mpc.create_rect_prism(d[0], d[1], d[2])


def rand_shape(rng, t):
    if t == POLYTOPE:
        return rand_prism(rng)
    if t == SPHERE:
        return mpc.SphereMRP(rng.uniform(0.2, 1.0))
    if t == CONE:
        return mpc.ConeMRP(rng.uniform(0.5, 2.0), np.deg2rad(rng.uniform(10, 40)))
    if t == CAPSULE:
        return mpc.CapsuleMRP(rng.uniform(0.1, 0.6), rng.uniform(0.3, 2.0))
    if t == CYLINDER:
        return mpc.CylinderMRP(rng.uniform(0.1, 0.6), rng.uniform(0.3, 2.0))
    poly = mpc.create_n_sided(5, 0.6)
    return mpc.PolygonMRP(poly["A"], poly["b"], 0.2)


def rand_pose(rng):
    return list(rng.uniform(-3, 3, 3)) + list(rng.uniform(-1, 1, 3))


def synthetic_polypoly(rng, B):
    """Config 4 distribution: rect prisms dims U(0.2,2)^3, r U(-3,3)^3, p U(-1,1)^3."""
    tab = Table()
    pairs = []
    for _ in range(B):
        a, b = tab.add(rand_prism(rng)), tab.add(rand_prism(rng))
        pairs.append((a, b, rand_pose(rng), rand_pose(rng)))
    return tab, pairs


def synthetic_mixed(rng, B, include_unsupported=True):
    """Config 5 distribution: all 36 ordered type pairs (case-4 ones -> status 2)."""
    tab = Table()
    pairs = []
    for i in range(B):
        t1, t2 = rng.integers(0, 6), rng.integers(0, 6)
        wide = (CAPSULE, CYLINDER, POLYGON)
        if not include_unsupported:
            while t1 in wide and t2 in wide:
                t1, t2 = rng.integers(0, 6), rng.integers(0, 6)
        a, b = tab.add(rand_shape(rng, t1)), tab.add(rand_shape(rng, t2))
        pairs.append((a, b, rand_pose(rng), rand_pose(rng)))
    return tab, pairs


def offsets_and_edges(rng):
    """Edge cases: non-trivial r_offset/Q_offset, odd polytopes (jld2 A1 with 14 faces),
    tetrahedra, coincident poses, far-apart pairs, large MRPs, tiny/huge shapes."""
    P = jld2_polytopes()
    tab = Table()
    pairs = []
    # 14-face polytope from the jld2 file (A1 is unused by the reference scenes)
    a1 = tab.add(mpc.PolytopeMRP(P["A1"].T, P["b1"]))
    a2 = tab.add(mpc.PolytopeMRP(P["A2"].T, P["b2"]))
    tet = tab.add(mpc.PolytopeMRP(np.array([[1.0, 1, 1], [-1, -1, 1], [-1, 1, -1], [1, -1, -1]]) / np.sqrt(3),
                                  np.array([0.5, 0.5, 0.5, 0.5])))
    shapes = [a1, a2, tet]
    # shapes with offsets
    for t in range(6):
        o = rand_shape(rng, t)
        o.r_offset = rng.uniform(-0.5, 0.5, 3)
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        w, v = q[0], q[1:]
        vx = np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])
        o.Q_offset = np.eye(3) + 2 * w * vx + 2 * vx @ vx
        shapes.append(tab.add(o))
    for t in range(6):
        shapes.append(tab.add(rand_shape(rng, t)))
    for i in range(600):
        k1, k2 = rng.choice(shapes, 2, replace=False)  # distinct objects: a shared object
        # would alias its .r/.p between the two roles
        p1, p2 = rand_pose(rng), rand_pose(rng)
        mode = i % 6
        if mode == 1:     # coincident centers
            p2[:3] = p1[:3]
        elif mode == 2:   # far apart
            p2[:3] = list(np.array(p1[:3]) + rng.uniform(20, 50, 3))
        elif mode == 3:   # large MRPs (|p| > 1: shadow set region)
            p1[3:] = list(rng.uniform(-3, 3, 3))
            p2[3:] = list(rng.uniform(-3, 3, 3))
        pairs.append((int(k1), int(k2), p1, p2))
    return tab, pairs


def rand_polytope(rng, k):
    """Bounded random polytope with k faces: the 6 box normals (boundedness) plus k - 6
    random unit normals, offsets U(0.4, 1.3)."""
    A = np.vstack([np.eye(3), -np.eye(3), rng.normal(size=(k - 6, 3))])
    A /= np.linalg.norm(A, axis=1, keepdims=True)
    return mpc.PolytopeMRP(A, rng.uniform(0.4, 1.3, k))


def large_polytopes(rng, B=360):
    """Many-faced primitives (orthant rows 33-64 per pair: the engine's 48- and 64-row
    buckets) against every primitive type, both orders, plus a few pairs above 64 rows
    (the engine's TOO_LARGE)."""
    tab = Table()
    big = [tab.add(rand_polytope(rng, k)) for k in (20, 26, 30, 40, 58)]
    poly40 = mpc.create_n_sided(40, 0.6)
    big.append(tab.add(mpc.PolygonMRP(poly40["A"], poly40["b"], 0.2)))
    small = [tab.add(rand_shape(rng, t)) for t in range(6)] + [tab.add(rand_polytope(rng, 20))]
    pairs = []
    for i in range(B):
        a = big[rng.integers(len(big))]
        b = (small + big)[rng.integers(len(small) + len(big))]
        if a == b:
            b = small[0]
        pr = (a, b) if i % 2 == 0 else (b, a)
        pairs.append((int(pr[0]), int(pr[1]), rand_pose(rng), rand_pose(rng)))
    return tab, pairs


def traces(rng, n=6):
    """Per-iteration (mu, sigma, step) traces of the reference for a few pairs per class."""
    rows = []
    mu_log = []
    orig_nt = ref_pdip.calc_NT_scalings

    tab, pairs = synthetic_mixed(rng, 60, include_unsupported=False)
    sel = pairs[:n * 5]
    for (k1, k2, q1, q2) in sel:
        o1, o2 = tab.objs[k1], tab.objs[k2]
        o1.r, o1.p = np.array(q1[:3]), np.array(q1[3:])
        o2.r, o2.p = np.array(q2[:3]), np.array(q2[3:])
        mus = []

        def wrapped(s, z, *a):
            mus.append(float(np.dot(s, z)))
            return orig_nt(s, z, *a)
        ref_pdip.calc_NT_scalings = wrapped
        try:
            ref_solve(o1, o2, 1e-6)
        finally:
            ref_pdip.calc_NT_scalings = orig_nt
        rows.append((k1, k2, q1, q2))
        mu_log.append(mus + [np.nan] * (51 - len(mus)))
    return tab, rows, np.array(mu_log)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    jobs = {
        "scene_piano": lambda: scene_piano(np.random.default_rng(11)),
        "scene_quad": lambda: scene_quad(np.random.default_rng(12)),
        "scene_cone": lambda: scene_cone(np.random.default_rng(13)),
        "synthetic_polypoly": lambda: synthetic_polypoly(np.random.default_rng(0), 2000),
        "synthetic_mixed": lambda: synthetic_mixed(np.random.default_rng(1), 1500),
        "edge_cases": lambda: offsets_and_edges(np.random.default_rng(2)),
        "large_polytopes": lambda: large_polytopes(np.random.default_rng(5)),
    }
    for name, fn in jobs.items():
        if args.only and name != args.only:
            continue
        tab, pairs = fn()
        out = run_pairs(tab, pairs, 1e-6, True, name)
        save(name, tab, pairs, out, 1e-6)
    if not args.only or args.only == "tolerances":
        # same synthetic pairs at other tolerances (tol is a runtime argument of the path)
        for tol, tag in ((1e-9, "tol1e-9"), (1e-3, "tol1e-3"), (0.0, "tol0_maxiter")):
            tab, pairs = synthetic_mixed(np.random.default_rng(3), 120, include_unsupported=False)
            out = run_pairs(tab, pairs, tol, tol > 0, f"synthetic_{tag}")
            save(f"synthetic_{tag}", tab, pairs, out, tol)
    if not args.only or args.only == "traces":
        tab, rows, mus = traces(np.random.default_rng(4))
        out = run_pairs(tab, rows, 1e-6, False, "traces")
        save("traces", tab, rows, out, 1e-6, sz_trace=mus)


if __name__ == "__main__":
    main()
