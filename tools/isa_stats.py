#!/usr/bin/env python3
"""ISA statistics of one solver kernel instantiation (gfx950), no GPU needed.

Compiles solve_one<N, NSOC, OMAX, LPP, FULL, BALL, CONE, OE> into a one-kernel code object
(hipcc -S --offload-device-only) and reports, for the longest loop of the kernel (the PDIP
iteration: the largest span between a label and a backward branch to it), the instruction
count and its mix -- FP64 VALU, AGPR moves (v_accvgpr_read/write: values the register
allocator parked in AGPRs), DPP lane moves, selects, scratch traffic -- plus the kernel's
register / scratch totals.  Used for the row-partition work.
Usage: python3 tools/isa_stats.py N:NSOC:OMAX:LPP[:OE[:FL]] [--waves 1] ...
  FL bits: 1 FULL, 2 BALL, 4 CONE, 8 BOX, 64 FD-only (as variants.py), 32 LDS rows (Solver GLDS; WPS >= 10
  in variants.py), 256 split ball SOC block (Solver SPLIT; variants.py FL bit 32)
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

CSRC = os.environ.get("DCOL_ISA_CSRC",   # (another copy of the sources, e.g. an experiment's)
                      os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dcol-trajectory-optimization_amd", "csrc"))

SRC = """#include "dcol_device.hpp"
namespace dcol {{
__global__ void __launch_bounds__(64, {w}) kb(KArgs A) {{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t slot = t / {l}; const int q = (int)(t % {l});
    if (slot >= A.n) return;
    solve_one<{n}, {s}, {o}, {l}, {full}, {ball}, {cone}, {oe}, 0, {glds}, {box}, {fdonly}, {split}>(A, slot, q);
}}
}}
"""

CATS = [("fp64", re.compile(r"^v_(fma|mul|add|fmac|rcp|rsq|sqrt|max|min|ldexp|div_fixup|div_scale|div_fmas|frexp|trig|cmp)\w*_f64")),
        ("agpr_move", re.compile(r"^v_accvgpr_(read|write|mov)")),
        ("select", re.compile(r"^v_cndmask")),
        ("scratch", re.compile(r"^(scratch_|buffer_)")),
        ("salu", re.compile(r"^s_")),
        ("valu", re.compile(r"^v_"))]


def stats(spec, waves, extra=()):
    parts = [int(v) for v in spec.split(":")]
    n, s, o, l = parts[:4]
    oe = parts[4] if len(parts) > 4 else 0
    fl = parts[5] if len(parts) > 5 else 0
    with tempfile.TemporaryDirectory() as tmp:
        src = os.path.join(tmp, "k.hip")
        asm = os.path.join(tmp, "k.s")
        open(src, "w").write(SRC.format(n=n, s=s, o=o, l=l, oe=oe, w=waves, full="true" if fl & 1 else "false",
                                        ball="true" if fl & 2 else "false", cone="true" if fl & 4 else "false",
                                        glds="true" if fl & 32 else "false", box="true" if fl & 8 else "false",
                                        fdonly="true" if fl & 64 else "false", split="true" if fl & 256 else "false"))
        r = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=on", f"-I{CSRC}",
                            *extra, "-S", "--offload-device-only", src, "-o", asm], capture_output=True, text=True)
        if r.returncode:
            sys.exit(r.stderr)
        lines = open(asm).read().splitlines()
    # blocks carry LLVM's loop annotations: "; =>This Inner Loop Header: Depth=1" on a
    # header, "; in Loop: Header=BB0_25 Depth=1" on the other blocks of that loop
    ins, loops = [], {}
    meta = {}
    cur = None
    for ln in lines:
        t = ln.strip()
        m = re.match(r"^\.(vgpr_count|agpr_count|private_segment_fixed_size):\s*(\d+)", t)
        mm = re.match(r"^;\s*(NumVgprs|NumAgprs|ScratchSize|Occupancy):\s*(\d+)", t)
        if mm:
            meta[mm.group(1)] = int(mm.group(2))
        if m:
            meta[m.group(1)] = int(m.group(2))
        lm = re.match(r"^\.LBB(\w+):(.*)$", t)
        if lm:
            rest = lm.group(2)
            h = re.search(r"Header=BB(\w+) Depth=1", rest)
            cur = lm.group(1) if ("Loop Header: Depth=1" in rest) else (h.group(1) if h else None)
            continue
        if not t or t.startswith((";", ".", "//")) or re.match(r"^[.\w$]+:", t):
            continue
        ins.append(t)
        if cur is not None:
            loops.setdefault(cur, []).append(t)
    loop = max(loops.values(), key=len) if loops else []
    cnt = {c: 0 for c, _ in CATS}
    dpp = 0
    for t in loop:
        op = t.split()[0]
        for c, rx in CATS:
            if rx.match(op):
                cnt[c] += 1
                break
        if "dpp" in t or "quad_perm" in t or "row_" in t:
            dpp += 1
    total = len(loop)
    return {"kernel": spec, "waves": waves, "loop_instructions": total, **cnt, "dpp": dpp,
            "agpr_frac": round(cnt["agpr_move"] / max(total, 1), 3), "fp64_frac": round(cnt["fp64"] / max(total, 1), 3),
            "kernel_instructions": len(ins), **meta}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--waves", type=int, default=1)
    ap.add_argument("--flags", default="",
                    help="extra compiler flags (default none, as the library's build; the codegen-invariance "
                         "twin lib_xcheck adds -mllvm -amdgpu-sched-strategy=max-ilp)")
    args = ap.parse_args()
    for sp in args.specs:
        print(stats(sp, args.waves, args.flags.split()), flush=True)


if __name__ == "__main__":
    main()
