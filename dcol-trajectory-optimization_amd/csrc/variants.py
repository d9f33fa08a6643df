#!/usr/bin/env python3
"""Single source of truth for the compiled kernel variants.

A variant is (N, NSOC, OMAX, LPP, WPS): N = primal dimension (4 + extra columns), NSOC =
number of SOC blocks, OMAX = orthant-row capacity bucket, LPP = lanes per pair, WPS =
minimum waves per SIMD requested from the register allocator.  Only (N, NSOC)
combinations that a supported primitive pair can produce are built
(combine_problem_matrices.py cases 1-3; DESIGN.md "Kernel variants").

(LPP, WPS) per shape come from a register sweep (tools/reg_sweep.py): the smallest LPP
that runs spill-free at 2 waves/SIMD, else the smallest spill-free one at 1 wave/SIMD.
The first config listed for a shape is the throughput choice, used when a launch fills
the GPU; a launch too small to fill it (fewer waves than SIMDs) takes the listed config
with the largest LPP instead — more lanes per pair, shorter per-pair latency (ALTRO-sized
batches).  DCOL_LPP=<n> forces an alternative (A/B runs).

FULL variants: a launch whose pairs all have exactly OMAX orthant rows (no padding rows:
box x box = 12 in the 12-row bucket, the benchmark and every reference scene's
polytope-polytope pairs) runs a copy of the kernel with the padding masks folded away.
Built for the polytope x polytope shapes (the only ones whose row count commonly fills
its bucket; a SOC pair's 1-row cone base or sphere's 0 rows never does).

BALL variants: a launch whose SOC blocks are all ball blocks (sphere / capsule / cylinder /
polygon -- no cone) runs a copy of the kernel that holds those blocks in structured form
(radius + extra columns instead of 4 dense G rows; dcol_device.hpp Solver<..., BALL>).
Built for every SOC shape with N <= 6; the host buckets cone pairs apart.

CONE variants: a launch whose SOC blocks are all cone blocks (polytope x cone, cone x cone;
N = 4) runs a copy that holds each cone block as its 3 x 3 rotation part plus the row-0
column-3 constant, unpadded (3-dim SOC arithmetic; dcol_device.hpp Solver<..., CONE>).

FUSED variants: one launch for a whole small plan.  A plan that mixes several variants
and cannot fill the GPU (an ALTRO phase: one victim against spheres, capsules, cylinders,
cones and polytopes) runs every bucket in ONE launch of prox_fused_kernel, whose
workgroups switch on a per-segment variant id (dcol_kernels_fused.hip) — no stream fan-out,
one launch latency.  Each shape's latency configuration (largest LPP) is in the switch,
plus the padding-free copies of the FULL shapes; case-4 shapes (N = 7, 8) are not.

Generates dcol_variants.inc (FL = variant flags: bit 0 FULL, bit 1 BALL, bit 2 CONE, bit 3 BOX):
  DCOL_VARIANTS(X)  X(N, NSOC, OMAX, LPP, WPS, 0) for every compiled kernel
  DCOL_FULL_VARIANTS(X)  X(N, NSOC, OMAX, LPP, WPS, 1) for the padding-free copies
  DCOL_BOX_VARIANTS(X)   X(N, NSOC, OMAX, LPP, WPS, 9) for the box x box axis-pair copies
  DCOL_BOX_FD_VARIANTS(X)  X(N, NSOC, OMAX, LPP, WPS, 73) their FD-only-gradient copies
  DCOL_BALL_VARIANTS(X)  X(N, NSOC, OMAX, LPP, WPS, 2) for the ball-SOC copies
  DCOL_CONE_VARIANTS(X)  X(N, NSOC, OMAX, LPP, WPS, 4) for the structured-cone copies
  DCOL_SHAPES(X)    X(N, NSOC, OMAX) once per shape (used by the test emulator)
  DCOL_FUSED_VARIANTS(X)  X(ID, N, NSOC, OMAX, LPP, FL) the cases of the fused kernel
  DCOL_PART_VARIANTS(X)  X(N, NSOC, OMAX, LPP, WPS, FL, OE) the row-partitioned copies
  DCOL_PART_SHAPES(X)    X(N, NSOC, OMAX, OE) once per PART bucket (host bucketing, emulator)
  DCOL_FUSED_PART_VARIANTS(X)  X(ID, N, NSOC, OMAX, LPP, FL, OE) the PART cases of the fused kernel
  DCOL_SUSP_VARIANTS(X)  X(N, NSOC, OMAX, LPP, WPS, FL, OE) suspend / resume copies (FL bit 4 = 16)
  DCOL_SPLIT_VARIANTS(X)  X(N, NSOC, OMAX, LPP, WPS, FL, OE) split-SOC PART copies (FL bit 5 = 32)
  DCOL_PACKED_VARIANTS(X)  X(ID, N, NSOC, OMAX, LPP, FL, OE) the cases of the packed kernel

SUSP variants (dcol_device.hpp KArgs susp_*, dcol_kernels_susp.hip): a large launch runs as a
main launch in which a wave hands its last few iterating pairs (<= DCOL_SUSPEND_T of 32, after
DCOL_SUSPEND_MIN iterations) to a compact resume launch, instead of running every lane of
the wave until its slowest pair converges.  Results are bitwise those of the one-launch
kernel (the same iteration sequence, continued from the saved iterate).

PART variants (row partition, dcol_device.hpp Solver<..., OE>): N = 5 / 6 pairs of combine
cases 1-3 (one primitive with extra columns) whose pose rows (polytope faces, cone base,
cylinder caps) and extra-column rows (capsule / cylinder segment rows, polygon edges) fit a
bucket (OMAX, OE): OMAX - OE pose-row slots and OE extra-row slots, each slot's column
pattern fixed at compile time.  A pair takes the smallest bucket that holds both counts
(fewest slots, then fewest extra slots); pairs that fit none (many-faced polytopes /
polygons, case 4) stay on the dense-row kernels.  Flavours: BALL (every SOC block a ball:
x polytope, x sphere) or dense SOC rows (x cone), each with its padding-free FULL copy.
"""
import os

OMAX = {
    (4, 0): [4, 8, 12, 16, 24, 32, 48, 64, 128],     # polytope x polytope
    (4, 1): [2, 4, 6, 7, 8, 12, 16, 24, 32, 48, 64, 128],  # polytope x {sphere, cone}; 7: cone x box
    (4, 2): [2],                        # {sphere, cone} x {sphere, cone}
    (5, 1): [8, 10, 12, 16, 24, 32, 48, 64, 128],    # {capsule, cylinder} x polytope
    (5, 2): [2, 4, 6, 8],               # {capsule, cylinder} x {sphere, cone}
    (6, 1): [8, 12, 16, 24, 32, 48, 64, 128],        # polygon x polytope
    (6, 2): [2, 4, 6, 8, 12, 16, 24, 32, 48, 64, 128],  # polygon x {sphere, cone}; case-4 {capsule, cylinder}^2
    (7, 2): [4, 8, 12, 16, 24, 32],     # case-4 extension: {capsule, cylinder} x polygon
    (8, 2): [4, 8, 12, 16, 24, 32],     # case-4 extension: polygon x polygon
}

# (LPP, WPS) choices per shape; default (4, 1) unless listed
CONFIG = {
    (4, 0, 4): [(2, 1)],
    (4, 0, 8): [(2, 1)],
    (4, 0, 12): [(2, 2), (4, 2), (1, 1)],   # the benchmark shape: A/B alternatives kept
    (4, 0, 16): [(4, 2)],
    (4, 0, 24): [(4, 2)],
    (4, 0, 32): [(8, 2)],
    (4, 1, 2): [(2, 1)],
    (4, 1, 4): [(1, 1), (2, 2), (4, 2)],
    (4, 1, 6): [(2, 2), (1, 1)],        # sphere x box: 2 waves/SIMD spill-free with ball rows
    (4, 1, 7): [(1, 1)],                # cone x box (1 + 6 rows): no padding slot at LPP 1
    (4, 1, 8): [(1, 1), (2, 1), (8, 2)],
    (4, 1, 12): [(2, 1), (4, 1)],
    (4, 2, 2): [(2, 2)],
    (5, 1, 8): [(1, 1), (2, 1), (8, 1)],
    (5, 1, 10): [(2, 1)],               # cylinder x box
    (5, 1, 12): [(2, 1), (4, 1)],
    (5, 2, 2): [(2, 2)],
    (5, 2, 4): [(2, 1), (4, 1)],
    (5, 2, 6): [(2, 1)],
    (5, 2, 8): [(2, 1), (8, 1)],
    (6, 1, 8): [(2, 1), (8, 1)],
    (6, 1, 12): [(2, 1), (4, 1)],       # polygon x box (ball rows)
    (6, 2, 6): [(2, 1)],
    (6, 2, 4): [(2, 1), (4, 1)],
    (6, 2, 8): [(2, 1), (8, 1)],
}
# per-flavour overrides for the structured copies (FL 2 = BALL, 4 = CONE): their register
# footprint differs from the dense kernel's, so their spill-free (LPP, WPS) can too
# WPS >= 10: the copy holds its G rows (and CONE rows) in LDS instead of registers
# (dcol_device.hpp Solver GLDS) and runs WPS - 10 waves per SIMD.  The one-lane cone x box
# kernel: 349 VGPRs at one wave -> 256 at two waves with 18 scratch instructions per loop
# (tools/isa_stats.py 4:1:7:1:0:37 --waves 2), bitwise equal; cone x polytope 11.8 -> 12.2e8,
# polytope x cone 11.8 -> 12.1e8 pair-solves/s (profiles/r05_b/cls_*.log, two rounds each).
CONFIG_FL = {(4, 1, 7, 4): [(1, 12)],
             # sphere x box: LDS rows at one lane per pair, two waves per SIMD -- 19.1 loop
             # instructions per pair-iteration against 30.5 for the LPP-2 kernel, whose second
             # lane idles through the SOC block (tools/isa_stats.py 4:1:6:1:0:34 --waves 2: 29
             # scratch instructions per loop); the LPP-2 copy stays for small plans
             (4, 1, 6, 2): [(1, 12), (2, 2)]}
FULL = {(4, 0)}   # shapes with padding-free copies (see module docstring)
# BOX copies (FL 9 = FULL | BOX, dcol_device.hpp Solver BOX): box x box pairs in the 12-row
# bucket, whole axis pairs per lane -- LPP 1 or 2 (an LPP-4 lane holds 3 rows)
# three waves per SIMD: 168 VGPRs, the PDIP loop spill-free (72 B of scratch outside it);
# against two waves (profiles/r05_box3/, interleaved): 100k serial 2.06-2.18e9 = unchanged,
# pipelined 2.59-2.76 -> 3.10-3.15e9, 1M kernel-only 2.87-2.97 -> 2.96-3.05e9
# measured slower, not built (profiles/r05_o/, r05_q/): four waves with LDS rows (4, 0, 12, 2, 14)
# -- 24 scratch accesses per loop, 87 us per 100k; one lane per pair with LDS rows at two
# waves (4, 0, 12, 1, 12) -- spill-free, 64.5 us per 100k, 2.54e9 at 1M
BOX = [(4, 0, 12, 2, 3)]
# FD-only copies of the BOX kernel (FL 73 = FULL | BOX | 64): launched for runs whose gradient
# mode is the reference's FD (or none) -- the headline -- without the envelope / implicit
# code, whose register pressure at 168 VGPRs spilled 124 B per lane to scratch in every mode
BOX_FD = BOX
# padding-free copies of the structured-cone kernels: (N, NSOC, OMAX) whose pairs commonly
# fill the bucket (cone x box: the cone's base row + 6 faces = 7)
FULL_CONE = {(4, 1, 7)}


def ball(n, nsoc):
    """shapes with ball-SOC copies (see module docstring)"""
    return nsoc >= 1 and n <= 6


def cone(n, nsoc, omax=0):
    """shapes with structured-cone copies (see module docstring); the many-faced buckets
    above FUSE_OMAX keep the dense rows only (compile time; rare pairs)"""
    return nsoc >= 1 and n == 4 and omax <= FUSE_OMAX


# (N, NSOC, OMAX, LPP) configurations without a ball copy.  Empty: the (6, 1, 12) ball
# kernel at LPP 2 was excluded once (commit 326f844: alpha 3e-10 / gradient 2e-5 off the C
# oracle on polygon-first x box pairs); that drift was a machine-code defect of that one
# build, not of the source -- the same IR scheduled with -amdgpu-sched-strategy=max-ilp was
# exact, and the variant is exact again at the current source (DESIGN.md section 4,
# "Codegen invariance").  Every throughput variant is now checked against a second build of
# the library with a different machine schedule (tests/test_gpu_fullsize.py).
BALL_SKIP = set()
BIG = 24   # OMAX >= BIG with SOC blocks: 8 lanes per pair
# Row buckets above 32 (48, 64, 128: polytopes / polygons with many faces, up to 128
# orthant rows per pair = two 64-face primitives) run 8 or 16 lanes per pair at one wave per
# SIMD (16 where 8 would spill to scratch) and stay out of the fused kernel (its register
# allocation is the maximum over its cases; plans containing them launch per bucket).
FUSE_OMAX = 32


def configs(n, nsoc, omax):
    if (n, nsoc, omax) in CONFIG:
        return CONFIG[(n, nsoc, omax)]
    if omax >= 128 or (omax >= 64 and (n > 4 or nsoc > 0)):
        return [(16, 1)]
    if omax >= BIG:
        return [(8, 1)]
    return [(4, 1)] if omax % 4 == 0 else [(2, 1)]


def configs_fl(n, nsoc, omax, fl):
    """(LPP, WPS) list of one flavour's copies (fl 0 dense, 1 FULL, 2 BALL, 4 CONE)"""
    return CONFIG_FL.get((n, nsoc, omax, fl), configs(n, nsoc, omax))


# PART buckets: (N, NSOC) -> {(OMAX, OE): [(LPP, WPS), ...]} (first = throughput choice)
PART = {
    # x polytope: one lane per pair (the SOC block would otherwise idle the group's other lane;
    # measured 200k pairs: capsule x box 8.1e8 at LPP 2 -> 9.5e8, cylinder x box 6.6 -> 7.1e8)
    # (LDS rows at one wave per SIMD -- WPS 11, fewer values parked in AGPRs -- measured slower
    # here: capsule x polytope -5 %, cylinder x polytope -10 %, polygon x polytope +-0
    # (profiles/r05_b/cls_*.log); the register rows stay)
    # (two lanes per pair at two waves per SIMD -- (8, 2): 5 scratch accesses per loop, (10, 2): 19
    # -- measured slower too: capsule x polytope -1 %, cylinder x polytope -7 % alone, the 1M
    # mixed step 0.874-0.876 -> 0.879-0.887 ms; profiles/r05_y/, r05_z/)
    (5, 1): {(8, 2): [(1, 1), (2, 1)], (10, 2): [(1, 1), (2, 1)], (14, 2): [(2, 1)], (18, 2): [(2, 1)]},
    # x sphere / cone: both lanes own a SOC block (capsule x sphere 11.2e8 at LPP 2, 9.1e8 at 1)
    # two waves per SIMD where the allocator then spills at most a few scratch accesses per
    # iteration (tools/isa_stats.py --waves 2) -- measured 200k pairs per class
    # (profiles/r04_base/cls_w*.log): capsule x cone 7.82e8 -> 8.68e8, cone x capsule 7.92 -> 8.94e8
    # ((4, 2), 2 scratch accesses per iteration), cylinder x cone 6.88 -> 7.35e8, cone x
    # cylinder 6.78 -> 7.35e8 ((6, 2), 21)
    (5, 2): {(2, 2): [(2, 1), (1, 1)], (4, 2): [(2, 2), (1, 1)], (6, 2): [(2, 2)]},
    (6, 1): {(9, 3): [(1, 1)], (10, 4): [(1, 1), (2, 1)], (11, 5): [(1, 1)], (12, 6): [(1, 1), (2, 1)],
             (14, 8): [(2, 1)]},
    # pentagon x sphere 7.6e8 at LPP 2 (6, 6) against 6.9e8 at LPP 1 (5, 5)
    (6, 2): {(4, 4): [(2, 1)], (6, 4): [(2, 1)], (6, 6): [(2, 1), (1, 1)], (8, 6): [(2, 1)], (8, 8): [(2, 1)]},
}
# per-flavour overrides of PART: (N, NSOC, OMAX, OE, "ball" | "dense") -> [(LPP, WPS), ...].  The
# ball-row copies of the polygon x sphere buckets hold fewer registers than the dense ones and
# run two waves per SIMD (4 / 0 scratch accesses per iteration): pentagon x sphere 7.88e8 ->
# 8.99e8, sphere x pentagon 8.01 -> 9.07e8 ((6, 6)); the dense copies spill far more there
# (polygon x cone in (8, 6) at two waves: 5.98e8 -> 2.77e8), so they keep one wave.
PART_FL = {
    (6, 2, 4, 4, "ball"): [(2, 2)],
    (6, 2, 6, 6, "ball"): [(2, 2), (1, 1)],
    # (cone x polygon / polygon x cone with LDS rows at two waves per SIMD -- WPS 12, 19 scratch
    # instructions per loop against 100 with register rows, tools/isa_stats.py 6:2:8:2:6:32
    # --waves 2 -- measured 1-2 % slower: 6.08 -> 5.97-6.02e8, profiles/r05_lds/i_cls_*.log)
}


def part_flavours(n, nsoc):
    """FL list of a PART shape: BALL (+FULL) always; dense SOC rows (+FULL) when the
    partner can be a cone (NSOC = 2)"""
    return [3, 2] + ([1, 0] if nsoc == 2 else [])


def part_configs(n, s, o, oe, fl):
    """(LPP, WPS) list of one PART bucket's copies of flavour fl (first = throughput choice)"""
    return PART_FL.get((n, s, o, oe, "ball" if fl & 2 else "dense"), PART[(n, s)][(o, oe)])


def part_variants():
    return [(n, s, o, l, w, fl, oe) for (n, s), bl in sorted(PART.items()) for (o, oe) in sorted(bl)
            for fl in part_flavours(n, s) for l, w in part_configs(n, s, o, oe, fl)]


# SPLIT copies (Solver SPLIT, FL bit 5 = 32): {capsule, cylinder} x polytope
# at two lanes per pair with the one ball SOC block split over both lanes (lane q holds its
# coordinates 2q, 2q + 1) instead of lane 1 idling through the SOC work.  Opt-in (DCOL_SPLIT=1,
# A/B: tools/class_bench.py); the buckets' default stays LPP 1 (PART above).
SPLIT = [(5, 1, 8, 2, 1, 35, 2), (5, 1, 8, 2, 1, 34, 2), (5, 1, 8, 2, 2, 35, 2), (5, 1, 8, 2, 2, 34, 2),
         (5, 1, 10, 2, 1, 35, 2), (5, 1, 10, 2, 1, 34, 2)]

# (N, NSOC, OMAX, LPP, WPS, FL without the SUSP bit, OE): the benchmark's poly x poly kernel
SUSP = [(4, 0, 12, 2, 2, 9, 0), (4, 0, 12, 2, 2, 1, 0)]   # the BOX copy first (box x box launches)

FUSE_PART_OMAX = 6   # PART buckets in the fused kernel: the small ones (its compile time grows with its cases)


def fused_part():
    """PART cases of the fused kernel: each small ball-SOC bucket of a victim against
    spheres (the quadrotor hallway's sphere x capsule / cylinder / polygon pairs) in its
    latency configuration (largest LPP)"""
    out = []
    for (n, s), bl in sorted(PART.items()):
        for (o, oe), cf in sorted(bl.items()):
            if s != 2 or o > FUSE_PART_OMAX:
                continue
            for fl in (3, 2):
                out.append((n, s, o, max(l for l, _ in part_configs(n, s, o, oe, fl)), fl, oe))
    return out


def fused():
    out = []
    for (n, s), os_ in sorted(OMAX.items()):
        if n > 6:
            continue
        for o in os_:
            if o > FUSE_OMAX:
                continue
            lpp = max(l for l, _ in configs(n, s, o))
            out.append((n, s, o, lpp, 0))
            if (n, s) in FULL:
                out.append((n, s, o, lpp, 1))
            lb = max(l for l, _ in configs_fl(n, s, o, 2))
            if ball(n, s) and (n, s, o, lb) not in BALL_SKIP:
                out.append((n, s, o, lb, 2))
            if cone(n, s, o):
                out.append((n, s, o, max(l for l, _ in configs_fl(n, s, o, 4)), 4))
    return out


# PACKED variants (dcol_kernels_packed.hip): one launch for a whole mid-size plan -- more
# lanes than a small plan (whose buckets take their latency configurations and the fused
# kernel) but too few for every bucket to fill the GPU by itself (a rank's shard of a mixed
# batch: 125k-250k pairs over ~15 buckets of 8-17k pairs; round-6 measurement: each bucket
# 20-80 us of single-wave latency on 15-30 % of the SIMDs, three in flight -> 0.32 ms per
# 125k step).  Its workgroups switch on a per-segment case id like the fused kernel's, but
# each case is a bucket's THROUGHPUT configuration (the first (LPP, WPS) of its flavour, the
# per-variant kernels' own), and the kernel runs one wave per SIMD with the register rows
# (GLDS off: it has the registers), so the workgroup dispatcher packs every bucket's waves
# onto free SIMDs in segment order.  Cases: the dense shapes and PART buckets up to
# PACK_OMAX rows, every flavour, listed per shape in the per-N launchers' preference order
# (BOX, FULL_CONE, FULL, BALL, CONE, plain; PART: FULL|BALL, BALL, FULL, dense).
PACK_OMAX = 12


def packed():
    """(N, NSOC, OMAX, LPP, FL, OE) per packed case.  (One kernel at one wave per SIMD for every
    case: a split into a one-wave and a two-wave kernel side by side on two streams measured
    slower up to 250k pairs -- 125k 0.144 -> 0.161 ms, 62.5k 0.099 -> 0.111 -- and equal at
    500k: the two kernels' waves compete for the same SIMDs (profiles/r06_f/).)"""
    out = []

    def fam(w):
        return 0
    box = {(n, s, o): (l, w) for n, s, o, l, w in BOX}
    for (n, s), os_ in sorted(OMAX.items()):
        if n > 6:
            continue
        for o in os_:
            if o > PACK_OMAX:
                continue
            if (n, s, o) in box:
                l, w = box[(n, s, o)]
                out.append((n, s, o, l, 9, 0, fam(w)))
            if (n, s, o) in FULL_CONE:
                l, w = configs_fl(n, s, o, 4)[0]
                out.append((n, s, o, l, 5, 0, fam(w)))
            if (n, s) in FULL:
                l, w = configs(n, s, o)[0]
                out.append((n, s, o, l, 1, 0, fam(w)))
            if ball(n, s) and (n, s, o, configs_fl(n, s, o, 2)[0][0]) not in BALL_SKIP:
                l, w = configs_fl(n, s, o, 2)[0]
                out.append((n, s, o, l, 2, 0, fam(w)))
            if cone(n, s, o):
                l, w = configs_fl(n, s, o, 4)[0]
                out.append((n, s, o, l, 4, 0, fam(w)))
            l, w = configs(n, s, o)[0]
            out.append((n, s, o, l, 0, 0, fam(w)))
    for (n, s), bl in sorted(PART.items()):
        for (o, oe) in sorted(bl):
            if o > PACK_OMAX:
                continue
            for fl in part_flavours(n, s):
                l, w = part_configs(n, s, o, oe, fl)[0]
                out.append((n, s, o, l, fl, oe, fam(w)))
    return out


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    shapes = [(n, s, o) for (n, s), os_ in sorted(OMAX.items()) for o in os_]
    lines = ["// generated by variants.py -- do not edit", "#define DCOL_VARIANTS(X) \\"]
    lines += [f"    X({n}, {s}, {o}, {l}, {w}, 0) \\" for n, s, o in shapes for l, w in configs(n, s, o)]
    lines += ["", "#define DCOL_FULL_VARIANTS(X) \\"]
    lines += [f"    X({n}, {s}, {o}, {l}, {w}, 1) \\" for n, s, o in shapes if (n, s) in FULL for l, w in configs(n, s, o)]
    lines += ["", "#define DCOL_BOX_VARIANTS(X) \\"]
    lines += [f"    X({n}, {s}, {o}, {l}, {w}, 9) \\" for n, s, o, l, w in BOX]
    lines += ["", "#define DCOL_BOX_FD_VARIANTS(X) \\"]
    lines += [f"    X({n}, {s}, {o}, {l}, {w}, 73) \\" for n, s, o, l, w in BOX_FD]
    lines += ["", "#define DCOL_FULL_CONE_VARIANTS(X) \\"]
    lines += [f"    X({n}, {s}, {o}, {l}, {w}, 5) \\" for n, s, o in shapes if (n, s, o) in FULL_CONE
              for l, w in configs_fl(n, s, o, 4)]
    lines += ["", "#define DCOL_BALL_VARIANTS(X) \\"]
    lines += [f"    X({n}, {s}, {o}, {l}, {w}, 2) \\" for n, s, o in shapes if ball(n, s)
              for l, w in configs_fl(n, s, o, 2) if (n, s, o, l) not in BALL_SKIP]
    lines += ["", "#define DCOL_CONE_VARIANTS(X) \\"]
    lines += [f"    X({n}, {s}, {o}, {l}, {w}, 4) \\" for n, s, o in shapes if cone(n, s, o)
              for l, w in configs_fl(n, s, o, 4)]
    lines += ["", "#define DCOL_SHAPES(X) \\"]
    lines += [f"    X({n}, {s}, {o}) \\" for n, s, o in shapes]
    lines += ["", "#define DCOL_FUSED_VARIANTS(X) \\"]
    lines += [f"    X({i}, {n}, {s}, {o}, {l}, {f}) \\" for i, (n, s, o, l, f) in enumerate(fused())]
    lines += ["", "#define DCOL_PART_VARIANTS(X) \\"]
    lines += [f"    X({n}, {s}, {o}, {l}, {w}, {fl}, {oe}) \\" for n, s, o, l, w, fl, oe in part_variants()]
    lines += ["", "#define DCOL_PART_SHAPES(X) \\"]
    lines += [f"    X({n}, {s}, {o}, {oe}) \\" for (n, s), bl in sorted(PART.items()) for o, oe in sorted(bl)]
    lines += ["", "#define DCOL_FUSED_PART_VARIANTS(X) \\"]
    base = len(fused())
    lines += [f"    X({base + i}, {n}, {s}, {o}, {l}, {f}, {oe}) \\" for i, (n, s, o, l, f, oe) in enumerate(fused_part())]
    lines += ["", "#define DCOL_PACKED_VARIANTS(X) \\"]
    lines += [f"    X({i}, {n}, {s}, {o}, {l}, {fl}, {oe}) \\" for i, (n, s, o, l, fl, oe, _) in enumerate(packed())]
    lines += ["", "#define DCOL_SPLIT_VARIANTS(X) \\"]
    lines += [f"    X({n}, {s}, {o}, {l}, {w}, {fl}, {oe}) \\" for n, s, o, l, w, fl, oe in SPLIT]
    lines += ["", "#define DCOL_SUSP_VARIANTS(X) \\"]
    lines += [f"    X({n}, {s}, {o}, {l}, {w}, {fl | 16}, {oe}) \\" for n, s, o, l, w, fl, oe in SUSP]
    lines.append("")
    out = os.path.join(here, "dcol_variants.inc")
    txt = "\n".join(lines) + "\n"
    if not os.path.exists(out) or open(out).read() != txt:
        open(out, "w").write(txt)


if __name__ == "__main__":
    main()
