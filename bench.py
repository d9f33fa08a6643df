#!/usr/bin/env python3
"""Benchmark: PDIP proximity + gradient pair-solves/sec on MI355X.

Workload (BASELINE.json configs[3], "synthetic 100k random polytope-polytope pairs"):
per GPU, B = 100,000 (knot x primitive-pair) problems; primitives are rect-prism polytopes
(nh = 6) drawn from a 64-entry shape table with dims ~ U(0.2, 2)^3 (shape ids uniform per
pair); poses r ~ U(-3, 3)^3, p (MRP) ~ U(-1, 1)^3; seed 0 (+ rank).  One "step" = one
dcol_plan_run over the whole batch: conic assembly + PDIP (pdip_tol 1e-6) + the 12-gradient
(FD mode = the reference's formulation) + alpha, with poses already resident in HBM.
`value` / `ms_per_step` are the one-stream run: K steps issued back to back on one HIP
stream; `kernel_ms` is the HIP-event time of that same timed region on the launch stream / K
(the per-launch duration of back-to-back launches), so the rooflines come from the same run
and ms_per_step >= kernel_ms.
Beside it, `pipeline`: the same steps issued round-robin on --streams (default 2) streams
with their own output buffers, as a pipelined batch service would (the last, partly-filled
round of one step's waves overlaps the first round of the next) -- an overlap rate, never
`value`.

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) this process is one rank;
`python bench.py --gpus N` without torchrun starts the N ranks itself (torch.distributed.run
as a child process, before this process touches the GPU) and exits with its status.  Every
rank solves its own 100k-pair shard (independent units, no data-path collective) ->
"scaling": "weak"; the timed region is bracketed by barrier + synchronize and the max over
ranks is taken.  The same line carries `mixed1m`: BASELINE configs[4] (1M mixed pairs,
class-balanced shards over the ranks, one RCCL all-gather of the packed records) through
the shipped C-ABI path dcol_prox_batch_multi_gpu (strong scaling).

Also reported: roofline of the solve kernel (HIP-event timed on the launch stream) against
HBM (algorithmic 208 B/pair) and against FP64 vector peak; the CPU baseline = the NumPy
restatement of the reference (oracle/, test infrastructure) on a bounded sample on the
host cores.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "dcol-trajectory-optimization_amd")
for _p in (PKG, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
FP64_VECTOR_PEAK_TFS = 78.6    # MI355X FP64 vector peak (AMD spec)
BYTES_PER_PAIR = 208           # poses 2x6 f64 + 2 int32 ids in; alpha + 12 grad f64 out
# The reference itself (proximity_gradient, NumPy, one core) measured in the survey container:
# random polytope-polytope 1.76-1.93 ms per pair, about 520 pair-solves/s per core (SURVEY.md
# section 6).  The baselines below are restatements ("port"), not the reference, and run
# faster per core; the line states the ratio so neither is mistaken for the reference's speed.
REFERENCE_PER_CORE = 520.0


def shape_table(n_shapes=64, seed=0):
    """Array-form shape table of random rect prisms (tests/golden layout)."""
    rng = np.random.default_rng(seed)
    A = np.array([[1.0, 0, 0], [0, 1, 0], [0, 0, 1], [-1, 0, 0], [0, -1, 0], [0, 0, -1]])
    dims = rng.uniform(0.2, 2.0, (n_shapes, 3))
    b = np.concatenate([dims / 2, dims / 2], axis=1)
    return {"type": np.zeros(n_shapes, np.int32), "nh": np.full(n_shapes, 6, np.int32),
            "A_off": np.arange(n_shapes, dtype=np.int32) * 6, "A_pool": np.tile(A, (n_shapes, 1)),
            "b_pool": b.reshape(-1), "params": np.zeros((n_shapes, 4)),
            "r_offset": np.zeros((n_shapes, 3)), "Q_offset": np.tile(np.eye(3), (n_shapes, 1, 1))}


def pairs(B, n_shapes, seed):
    rng = np.random.default_rng(seed)
    s1 = rng.integers(0, n_shapes, B).astype(np.int32)
    s2 = rng.integers(0, n_shapes, B).astype(np.int32)
    pose1 = np.hstack([rng.uniform(-3, 3, (B, 3)), rng.uniform(-1, 1, (B, 3))])
    pose2 = np.hstack([rng.uniform(-3, 3, (B, 3)), rng.uniform(-1, 1, (B, 3))])
    return s1, s2, pose1, pose2


def _oracle_chunk(args):
    """one single-threaded worker (OMP_NUM_THREADS=1 per process): the
    BLAS / OpenMP pools of the forked worker limited to one thread"""
    tab, s1, s2, p1, p2 = args
    os.environ["OMP_NUM_THREADS"] = "1"
    from threadpoolctl import threadpool_limits
    from oracle import dcol_oracle as O
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        out = O.run_batch(tab, s1, s2, p1, p2, 1e-6, True)
        return time.perf_counter() - t0, out["status"]


def cpu_baseline(tab, s1, s2, p1, p2, sample, workers):
    """NumPy restatement of the reference (oracle/, a 'port'), one process per core."""
    import multiprocessing as mp
    n = min(sample, len(s1))
    chunks = np.array_split(np.arange(n), workers)
    jobs = [(tab, s1[c], s2[c], p1[c], p2[c]) for c in chunks if len(c)]
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(len(jobs)) as pool:
        res = pool.map(_oracle_chunk, jobs)
    wall = time.perf_counter() - t0
    cpu_s = sum(r[0] for r in res)
    return {"value": n / wall, "unit": "pair-solves/s", "cores": len(jobs), "kind": "port",
            "sample": f"{n} of the same synthetic poly-poly pairs, proximity+FD gradient, NumPy oracle "
                      f"(oracle/dcol_oracle.py), {len(jobs)} processes, {cpu_s:.1f} s CPU, {wall:.1f} s wall",
            "per_core": n / cpu_s, **calibration(n / cpu_s)}


def calibration(per_core):
    """the port's per-core rate against the reference's own (REFERENCE_PER_CORE)"""
    return {"reference_per_core": REFERENCE_PER_CORE,
            "reference_per_core_source": "SURVEY.md section 6: the reference's proximity_gradient on one core, "
                                         "random polytope-polytope pairs, 1.76-1.93 ms per pair",
            "port_vs_reference_per_core": per_core / REFERENCE_PER_CORE}


def cpu_baseline_c(tab, s1, s2, p1, p2, threads, seconds=3.0):
    """C restatement of the reference (oracle/dcol_oracle.c, a 'port', OpenMP over `threads`
    host cores; SURVEY.md §8d asks for both restatements): the same pairs, repeated until
    about `seconds` of wall time."""
    from oracle import c_oracle
    n = min(len(s1), 20000)
    c_oracle.run_batch(tab, s1[:256], s2[:256], p1[:256], p2[:256], want_grad=True, threads=threads)  # load/warm
    done, t0 = 0, time.perf_counter()
    while True:
        c_oracle.run_batch(tab, s1[:n], s2[:n], p1[:n], p2[:n], want_grad=True, threads=threads)
        done += n
        wall = time.perf_counter() - t0
        if wall >= seconds:
            break
    return {"value": done / wall, "unit": "pair-solves/s", "cores": threads, "kind": "port",
            "sample": f"{done} solves ({n} distinct synthetic poly-poly pairs), proximity+FD gradient, C oracle "
                      f"(oracle/dcol_oracle.c), OpenMP {threads} threads, {wall:.1f} s wall",
            "per_core": done / wall / threads, **calibration(done / wall / threads)}


def spawn_ranks(n):
    """Run this script as `n` torchrun ranks (127.0.0.1 rendezvous) in a child process and
    return its exit status.  Called before anything initialises the GPU in this process."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def cpu_share(requested=0):
    """(workers, description) for the CPU baselines: every core this process may run on
    (its affinity mask), bounded by the host's OMP_NUM_THREADS when set (the GPU pool pins a
    one-GPU job's CPU share there: os.cpu_count() reports the whole machine)."""
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    share = min(avail, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else avail
    workers = max(1, min(requested, avail) if requested > 0 else share)
    budget = ("; the GPU pool grants a one-GPU job 16 CPUs of a shared host and pins that share in "
              "OMP_NUM_THREADS (its affinity mask and os.cpu_count() show the whole machine, whose other CPUs "
              "belong to other jobs' GPUs) -- so `cores` is the granted budget, one single-threaded worker per "
              "granted CPU, and `per_core` is the figure comparable across hosts") if share < avail else ""
    return workers, (f"{workers} workers; {avail} CPUs in this process's affinity mask, os.cpu_count() "
                     f"{os.cpu_count()}, OMP_NUM_THREADS {omp or 'unset'}" + budget)


def read_traffic(profile_dir, kernel_substr="prox_kernel"):
    """Per-launch HBM bytes of the solve kernel from a committed rocprofv3 PMC pass
    (FETCH_SIZE + WRITE_SIZE in KB; FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM)."""
    path = os.path.join(profile_dir, "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        return d.get("bytes_per_launch")
    except Exception:
        return None


def executed_fp64(kern_ms, B, flops_pair):
    """The FP64 work the solve kernel EXECUTES, beside the counted model: from the committed
    rocprofv3 PMC pass (profiles/pmc_fp64.json, tools/pmc_fp64.py: (ADD + MUL + 2 FMA + TRANS)
    F64 wave-instructions x 64 per launch) over this run's kernel_ms, and the pass's VALU
    issue fraction.  The counted model follows the reference's algorithm op by op (its FD
    gradient re-assembles the rows 13 times, ~8.4 kflop; its NT scalings recompute J(s), J(z)),
    which the kernel does in closed form, so it executes fewer flops per
    pair than it is credited with: executed_frac is the hardware's FP64 utilisation."""
    path = os.path.join(REPO, "profiles", "pmc_fp64.json")
    if not os.path.exists(path):
        return {}
    try:
        d = json.load(open(path))
        per_pair = d["executed_flops_per_pair"]
        tf = per_pair * B / (kern_ms * 1e-3) / 1e12
        return {"executed_flops_per_pair": per_pair, "executed_achieved": tf,
                "executed_frac": tf / FP64_VECTOR_PEAK_TFS, "valu_issue_frac": d["valu_issue_frac"],
                "fp64_share_of_valu": d["fp64_share_of_valu"], "counted_over_executed": flops_pair / per_pair,
                "executed_source": "profiles/pmc_fp64.json (rocprofv3 PMC pass of this kernel, tools/pmc_fp64.py) "
                                   "over this run's kernel_ms"}
    except Exception:
        return {}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500,
                    help="timed steps (0.05-2 ms each; enough for the GPU clocks to settle)")
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--pairs", type=int, default=100_000, help="pairs per GPU")
    ap.add_argument("--grad", choices=["fd", "envelope", "implicit"], default="fd",
                    help="fd: the reference's formulation (the headline); envelope / implicit: the closed-form "
                         "and implicit-function modes (DESIGN.md section 3 \"Gradient modes\")")
    ap.add_argument("--cpu-sample", type=int, default=16000)
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help="host processes / threads for the CPU baselines (0 = every core this process may run on)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check", type=int, default=256, help="pairs re-checked against the oracle")
    ap.add_argument("--max-iter", type=int, default=50, help="PDIP iteration cap (diagnostics only; reference: 50)")
    ap.add_argument("--streams", type=int, default=2,
                    help="steps are issued round-robin on this many HIP streams with their own output buffers "
                         "(a pipelined batch service: one step's tail overlaps the next step's start)")
    ap.add_argument("--no-altro", action="store_true", help="skip the ALTRO wall-clock and scene-batch sections")
    ap.add_argument("--workload", choices=["poly100k", "mixed1m"], default="poly100k",
                    help="poly100k: BASELINE configs[3], 100k poly-poly pairs per GPU (weak scaling, the "
                         "headline); mixed1m: configs[4], 1M mixed pairs sharded over the GPUs + one "
                         "all-gather (strong scaling)")
    ap.add_argument("--backend", default=os.environ.get("DCOL_DIST_BACKEND", "nccl"),
                    help="torch.distributed backend for N > 1 (nccl = RCCL; gloo for rehearsals)")
    ap.add_argument("--mixed-steps", type=int, default=20,
                    help="timed steps of the configs[4] sub-measurement (mixed1m) of the default line; 0 = skip")
    ap.add_argument("--shard-steps", type=int, default=30,
                    help="mixed1m at world 1: timed steps per shard of the configs[4] per-rank regime (`shards`: rank "
                         "0's class-balanced shard at world N solved alone on this GPU); 0 = skip")
    ap.add_argument("--shard-worlds", default="2,3,4,6,8,16,32,64,128,512,4096",
                    help="the world sizes N of the `shards` section (shard = 1M / N pairs)")
    ap.add_argument("--torch-gather", action="store_true",
                    help="mixed1m: all-gather through torch.distributed instead of the C-ABI RCCL path")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process (HIP hardware queues; 0 = leave the environment's)")
    ap.add_argument("--timed-outputs", choices=("reference", "all"), default="reference",
                    help="configs[3]: the outputs the timed steps write -- alpha + gradient, what the reference's "
                         "proximity_gradient returns (default), or also the per-pair status / iteration counts")
    ap.add_argument("--no-cost-order", dest="cost_order", action="store_false",
                    help="skip the `cost_order` section (the pairing re-listed by iteration count, drifting poses)")
    ap.add_argument("--no-kernel-1m", dest="kernel_1m", action="store_false",
                    help="skip the 1M-pair kernel-only steady-state section (kernel_1m)")
    ap.add_argument("--deadline-s", type=float, default=float(os.environ.get("DCOL_BENCH_DEADLINE_S", "180")),
                    help="N > 1: the longest any rank waits for one phase (communicator set-up, a step's solve, its "
                         "all-gather, a barrier) before it prints a JSON diagnostic (rank, step, phase) to stderr and "
                         "exits non-zero (dcol_amd.dist.StepWatchdog)")
    ap.add_argument("--settle-ms", type=float, default=30.0,
                    help="before the warm-up, run the step until this much GPU time has passed (HIP events), so the "
                         "timed steps do not run on the GPU's clock ramp (the clocks settle after ~15 ms of sustained "
                         "load, DESIGN.md section 0); reported in the line as `settle`; 0 = off")
    ap.add_argument("--pack-pass", action="store_true",
                    help="mixed1m: per-pair arrays + pack_records kernel + out-of-place all-gather instead of "
                         "records written by the solver kernels with the all-gather in place (A/B)")
    args = ap.parse_args()
    if args.hw_queues > 0:
        # HIP runtime tunable, read at its initialisation (before any GPU call of this process
        # and inherited by spawned ranks): the pipelined steps run on two caller streams plus
        # the library's three side streams; with the default 4 hardware queues two of those
        # share a queue, and a join barrier of one step then stalls the next step's kernels
        # behind it
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # N ranks requested without a launcher: start them, before this process touches the GPU
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher formed a world of {world} ranks", file=sys.stderr)
        sys.exit(2)

    import torch
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)    # rehearsals may run more ranks than devices (gloo)
    if world > 1 and args.backend == "nccl" and ndev < world:
        print(f"bench.py: {world} RCCL ranks need {world} GPUs, this node shows {ndev}", file=sys.stderr)
        sys.exit(2)
    wd = None
    if world > 1:
        import datetime

        import torch.distributed as dist
        from dcol_amd.dist import StepWatchdog
        wd = StepWatchdog(rank, world, args.deadline_s)
        torch.cuda.set_device(local)
        with guard(wd, "init_process_group"):
            tmo = datetime.timedelta(seconds=args.deadline_s)
            if args.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
            else:
                dist.init_process_group(args.backend, timeout=tmo)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local)
    coll_dev = dev if args.backend == "nccl" else torch.device("cpu")
    if dist is not None and dist.get_world_size() != args.gpus:
        print(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    if args.workload == "mixed1m":
        return run_mixed(args, world, rank, local, dev, coll_dev, dist, wd)

    from dcol_amd import Engine, spec_from_arrays
    tab = shape_table()
    B = args.pairs
    s1, s2, p1, p2 = pairs(B, len(tab["type"]), seed=1000 + rank)
    eng = Engine(device=local)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    plan = eng.plan(ids[s1], ids[s2])
    pose1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    pose2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    from dcol_amd import alloc_outputs
    out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
    stream = torch.cuda.current_stream(dev)

    # the timed steps write what the reference's proximity_gradient returns -- alpha and the
    # gradient (--timed-outputs reference, the default); the per-pair status and Newton
    # iteration counts (optional outputs, 8 B per pair) come from one untimed step after them
    stats_out = ("iters", "status") if args.timed_outputs == "reference" else ()
    out_t = {k: v for k, v in out.items() if k not in stats_out}
    step = plan.bind(pose1, pose2, out_t, grad=args.grad, contact=False, stream=stream, max_iter=args.max_iter)
    # pipelined issue: S streams, each with its own outputs (poses are read-only, shared)
    S = max(1, args.streams)
    lane_streams = [stream] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    lanes = [step] + [plan.bind(pose1, pose2, {k: v for k, v in alloc_outputs(B, dev, want_grad=True,
                                                                            want_contact=False).items()
                                              if k not in stats_out},
                                grad=args.grad, contact=False, stream=st, max_iter=args.max_iter)
                      for st in lane_streams[1:]]

    settle = clock_settle(step, stream, dev, wd, args.settle_ms)
    # the W warm-up steps in the same bracket as the timed steps (timing events, polled end,
    # synchronize): the first such region of a process paid ~40 us more at its end than later
    # ones (tools/region_probe.py), which K = 20 timed steps would otherwise carry
    w_start, w_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w_start.record(stream)
    for k in range(args.warmup):
        step()
    w_end.record(stream)
    wait_event(w_end, wd, "warmup", args.warmup - 1)
    sync(dev, wd, "warmup")

    # value: exactly K steps on ONE stream, barrier + synchronize on both sides.  kernel_ms =
    # the HIP-event time of that same timed region on the launch stream / K: the per-launch
    # duration of the back-to-back launches (one event pair: a pair around every launch costs
    # ~7.5 us of GPU time per step, tools/step_gap.py).  With a deadline (N > 1) every 4th step
    # is followed by an untimed event, so a rank that hangs names the step.
    barrier(dist, wd, "barrier before the timed steps")
    sync(dev, wd, "synchronize before the timed steps")
    e_start, e_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    marks = []
    t0 = time.perf_counter()
    e_start.record(stream)
    for k in range(args.steps):
        step()
        if wd is not None and (k % 4 == 3 or k == args.steps - 1):
            e = torch.cuda.Event()
            e.record(stream)
            marks.append((k, e))
    e_end.record(stream)
    for k, e in marks:
        wait_event(e, wd, "solve", k)
    wait_event(e_end, wd, "solve", args.steps - 1)
    sync(dev, wd, "synchronize after the timed steps")
    elapsed = time.perf_counter() - t0
    barrier(dist, wd, "barrier after the timed steps")
    kern_ms = e_start.elapsed_time(e_end) / args.steps

    # pipeline: the same K steps round-robin on S streams (an overlap rate, reported beside)
    elapsed_pipe = None
    if S > 1:
        for k in range(args.warmup):
            lanes[k % S]()
        sync(dev, wd, "pipeline warmup")
        barrier(dist, wd, "barrier before the pipelined steps")
        sync(dev, wd, "synchronize before the pipelined steps")
        t0 = time.perf_counter()
        done = []
        for k in range(args.steps):
            lanes[k % S]()
            e = torch.cuda.Event()
            e.record(lane_streams[k % S])
            done.append(e)
        for k, e in enumerate(done):
            wait_event(e, wd, "pipelined solve", k)
        sync(dev, wd, "synchronize after the pipelined steps")
        elapsed_pipe = time.perf_counter() - t0
        barrier(dist, wd, "barrier after the pipelined steps")
    # (kernel_1m right after the timed steps, while the clocks are still at their loaded level:
    # after end_to_end's host-side staging the GPU has idled and re-ramps through the first
    # ~10 ms of launches -- measured 0.44 ms per 1M launch there against 0.36 ms)
    k1m = kernel_1m(args, eng, ids, tab, dev) if world == 1 and args.kernel_1m else None
    cord = (cost_order_section(args, eng, ids, s1, s2, p1, p2, dev)
            if world == 1 and args.cost_order and args.max_iter == 50 else None)
    e2e = end_to_end(args, eng, ids, s1, s2, p1, p2, pose1, pose2, out_t, step, dev) if world == 1 else None
    if dist is not None:
        t = torch.tensor([elapsed, kern_ms, elapsed_pipe or 0.0], device=coll_dev, dtype=torch.float64)
        with guard(wd, "all_reduce of the timings"):
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_max = float(t[0]), float(t[1])
        elapsed_pipe = float(t[2]) if elapsed_pipe is not None else None
    else:
        kern_ms_max = kern_ms

    # one untimed step with every output (the timed ones left status / iters unwritten)
    plan.bind(pose1, pose2, out, grad=args.grad, contact=False, stream=stream, max_iter=args.max_iter)()
    sync(dev, wd, "the statistics step")
    status = out["status"].cpu().numpy()
    iters = out["iters"].cpu().numpy()
    alpha = out["alpha"].cpu().numpy()
    grad = out["grad"].cpu().numpy()
    # configs[4] on the same ranks (every rank takes part: one all-gather per step)
    mixed = (mixed_measure(args, world, rank, local, dev, coll_dev, dist, args.mixed_steps, min(args.warmup, 5), wd)
             if args.mixed_steps > 0 else None)

    if rank != 0:
        with guard(wd, "destroy_process_group"):
            dist.destroy_process_group()
        if wd is not None:
            wd.close()
        return

    total = B * world * args.steps
    value = total / elapsed
    achieved_gbs = BYTES_PER_PAIR * B / (kern_ms * 1e-3) / 1e9
    traffic = read_traffic(os.path.join(REPO, "profiles"))
    flops_pair = flops_per_pair(iters[status == 0], args.grad)
    line = {
        "metric": "PDIP proximity+grad pair-solves/sec",
        "value": value,
        "unit": "pair-solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "kernel_ms": kern_ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": "synthetic random polytope-polytope pairs (BASELINE.json configs[3])",
                   "pairs_per_gpu": B, "shape_table": "64 rect prisms, dims U(0.2,2)^3",
                   "poses": "r U(-3,3)^3, p U(-1,1)^3", "pdip_tol": 1e-6, "gradient": args.grad,
                   "parallelism": f"dp{world} (independent pair shards)"},
        "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic},
        "roofline_fp64": {"bound": "fp64-valu", "achieved": flops_pair * B / (kern_ms * 1e-3) / 1e12,
                          "peak": FP64_VECTOR_PEAK_TFS, "unit": "TFLOP/s",
                          "frac": flops_pair * B / (kern_ms * 1e-3) / 1e12 / FP64_VECTOR_PEAK_TFS,
                          "flops_per_pair": flops_pair,
                          "flops_source": "op-counting C restatement, profiles/flop_model.json"
                          if os.path.exists(os.path.join(REPO, "profiles", "flop_model.json")) else "hand model",
                          **executed_fp64(kern_ms, B, flops_pair)},
        "timing": "value = pairs / ms_per_step of K steps on one stream; kernel_ms = the HIP-event time of that same "
                  "timed region on the launch stream / K (the per-launch duration of the back-to-back launches), the "
                  "rooflines' time base",
        "timed_outputs": ("alpha + gradient (the reference's outputs); status / iters from one untimed step after the "
                          "timed ones" if stats_out else "alpha, gradient, status, iters"),
        "pipeline": {"streams": S, "note": "the same K steps issued round-robin on S streams with separate outputs "
                     "(an overlap rate: one step's last round of waves overlaps the next step's first; not value)",
                     "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                     "value": (B * world * args.steps / elapsed_pipe) if elapsed_pipe else None,
                     "ms_per_step": 1e3 * elapsed_pipe / args.steps if elapsed_pipe else None},
        "kernel_ms_max_rank": kern_ms_max,
        "settle": settle,
        "world": {"ranks": world, "process_group_size": dist.get_world_size() if dist is not None else 1,
                  "backend": args.backend if dist is not None else None, "devices_visible": ndev},
        "solve_stats": {"ok_frac": float(np.mean(status == 0)), "iters_mean": float(iters[status == 0].mean()),
                        "iters_max": int(iters.max()),
                        "iters_hist": np.bincount(iters, minlength=int(iters.max()) + 1).tolist()},
    }
    if e2e is not None:
        line["end_to_end"] = e2e
    if k1m is not None:
        line["kernel_1m"] = k1m
    if cord is not None:
        line["cost_order"] = cord
    # spot parity check against the oracle on the first and the last pairs of the timed batch
    # (a graded launch solves its last pairs with the wider lane groups)
    if args.check and args.max_iter == 50:
        from oracle import dcol_oracle as O
        n = min(args.check, B)
        sel = np.unique(np.concatenate([np.arange(n // 2), np.arange(B - (n - n // 2), B)]))
        ref = O.run_batch(tab, s1[sel], s2[sel], p1[sel], p2[sel], 1e-6, True)
        ok = ref["status"] == 0
        if args.grad == "implicit":
            # checked against the oracle's restatement of the implicit mode (the reference
            # has none), on a sub-sample (its dG / dh are central differences)
            sel, ref, ok = implicit_reference(O, tab, s1, s2, p1, p2, sel[:: max(1, sel.size // 64)])
        a_ok = np.all(np.abs(alpha[sel][ok] - ref["alpha"][ok]) <= 1e-6 * np.abs(ref["alpha"][ok]) + 1e-12)
        g_ok = np.all(np.abs(grad[:, sel].T[ok] - ref["grad"][ok]).max(1)
                      <= 1e-5 * np.maximum(np.abs(ref["grad"][ok]).max(1), 1))
        line["parity_check"] = {"pairs": int(sel.size), "status_equal": bool(np.array_equal(status[sel], ref["status"])),
                                "alpha_ok": bool(a_ok), "grad_ok": bool(g_ok)}
    if mixed is not None:
        line["mixed1m"] = mixed
    if world == 1 and not args.no_altro:
        line["altro"] = altro_section()
        line["scene_batches"] = scene_batches(local)
        line["dropin"] = dropin_section()
    if world == 1 and not args.no_cpu:
        workers, host = cpu_share(args.cpu_workers)
        line["cpu_baseline"] = cpu_baseline(tab, s1, s2, p1, p2, args.cpu_sample, workers)
        line["cpu_baseline_c"] = cpu_baseline_c(tab, s1, s2, p1, p2, workers)
        for k in ("cpu_baseline", "cpu_baseline_c"):
            line[k]["host_cpus"] = host
    line["summary"] = summary(line)    # last: the part of the line a truncated tail still shows
    print(json.dumps(line), flush=True)
    if dist is not None:
        with guard(wd, "destroy_process_group"):
            dist.destroy_process_group()
        wd.close()


def summary(line):
    """The headline figures of every section in one short object (printed last)"""
    m = line.get("mixed1m") or {}
    d = line.get("dropin") or {}
    out = {"value": line["value"], "ms_per_step": line["ms_per_step"], "kernel_ms": line["kernel_ms"],
           "fp64_frac": line["roofline_fp64"]["frac"],
           "fp64_executed_frac": line["roofline_fp64"].get("executed_frac"),
           "valu_issue_frac": line["roofline_fp64"].get("valu_issue_frac"), "hbm_frac": line["roofline"]["frac"],
           "pipelined_value": line["pipeline"]["value"]}
    if m:
        out["mixed1m"] = {"value": m["value"], "ms_per_step": m["ms_per_step"], "kernel_ms": m.get("kernel_ms"),
                          "fp64_frac": (m.get("roofline_fp64") or {}).get("frac"),
                          "pipelined_value": m["pipeline"]["value"]}
    sh = m.get("shards") if m else None
    if sh:
        out["mixed1m"]["shards_solve_ms"] = {str(r["world"]): r["solve_ms"] for r in sh["per_world"] if r["world"] in (1, 2, 4, 8)}
        out["mixed1m"]["crossover_pairs"] = sh["crossover_pairs"]
    if "kernel_1m" in line:
        out["kernel_1m"] = {"pair_solves_per_s": line["kernel_1m"]["pair_solves_per_s"],
                            "fp64_frac": line["kernel_1m"]["roofline_fp64"]["frac"]}
    if "cost_order" in line:
        c = line["cost_order"]
        out["cost_order"] = {"given_ms": c["given_order"]["kernel_ms"], "cost_ms": c["cost_order"]["kernel_ms"],
                             "speedup": c["speedup"], "bitwise_equal": c["bitwise_equal"]}
    if d:
        out["dropin_us_per_call"] = {k: d[k]["us_per_call"] for k in ("proximity_mrp", "proximity_gradient") if k in d}
    if "altro" in line:
        out["altro_ms_per_iter"] = {k: v["ms_per_iter"] for k, v in line["altro"]["systems"].items()}
    if "cpu_baseline" in line:
        out["cpu_baseline"] = line["cpu_baseline"]["value"]
    return out


def clock_settle(step, stream, dev, wd, ms):
    """Run `step` in rounds of 10 until `ms` of GPU time (HIP events on its stream) has
    passed: the GPU's clocks ramp up over the first ~15 ms of sustained load
    (profiles/r04_clock/), and a short timed run (the driver's --steps 20) would otherwise be
    measured on the ramp.  Untimed, outside the W warm-up steps and the K timed ones; the
    line reports what it ran."""
    import torch
    done, steps = 0.0, 0
    while done < ms:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(10):
            step()
        e1.record(stream)
        if wd is None:
            e1.synchronize()
        else:
            wd.wait_event(e1, "clock settle")
        done += e0.elapsed_time(e1)
        steps += 10
    return {"gpu_ms": done, "steps": steps,
            "note": "untimed steps before the warm-up until this much GPU time had passed (--settle-ms): the timed "
                    "steps run at settled clocks, not on the ramp"}


def guard(wd, phase, step=None):
    """the rank's deadline around one wait (N > 1); no-op without a watchdog"""
    import contextlib
    return wd.guard(phase, step) if wd is not None else contextlib.nullcontext()


def sync(dev, wd, phase):
    """torch.cuda.synchronize under the rank's deadline (N > 1)"""
    import torch
    if wd is None:
        torch.cuda.synchronize(dev)
        return
    with guard(wd, phase):   # (torch.cuda.synchronize releases the GIL while it waits)
        torch.cuda.synchronize(dev)


def barrier(dist, wd, phase):
    if dist is None:
        return
    with guard(wd, phase):
        dist.barrier()


def wait_event(e, wd, phase, step):
    if wd is None:   # polling, as the deadline's wait does (a blocking wait's wake-up adds
        while not e.query():   # 10-15 us to the timed region, tools/step_latency.py)
            pass
    else:
        wd.wait_event(e, phase, step)


def cost_order_section(args, eng, ids, s1, s2, p1, p2, dev, steps=100, ring=16, sr=0.02, sp=0.01):
    """The listing order of the pairing (dcol_amd.cost_order; not `value`): a wave runs until
    its slowest pair has converged, so pairs listed in descending order of their last
    iteration counts fill waves with pairs of similar cost.  A trajectory optimiser's view:
    the same pairs at poses that drift from step to step -- a random walk from the configs[3]
    poses (r + N(0, sr), p + N(0, sp) per step; a ring of `ring` pose sets walked forth and
    back, so consecutive steps differ by one step) -- solved K steps back to back (HIP events)
    in the given order and in the order of the iteration counts of ONE solve at the first
    poses (re-listed once: pairs, poses and outputs in the new order), with the outputs of
    the last step compared bitwise."""
    import torch
    from dcol_amd import alloc_outputs, cost_order
    rng = np.random.default_rng(17)
    B = len(s1)
    walk = [(p1, p2)]
    for _ in range(ring - 1):
        q1, q2 = walk[-1][0].copy(), walk[-1][1].copy()
        for q in (q1, q2):
            q[:, :3] += rng.normal(0, sr, (B, 3))
            q[:, 3:] += rng.normal(0, sp, (B, 3))
        walk.append((q1, q2))
    seq = list(range(ring)) + list(range(ring - 2, 0, -1))
    stream = torch.cuda.current_stream(dev)
    res = {"poses": f"random walk from the configs[3] poses: r + N(0, {sr}), p + N(0, {sp}) per step, "
                    f"{ring} pose sets forth and back", "steps": steps}
    outs = {}
    first = None
    for name in ("given", "cost"):
        order = np.arange(B) if name == "given" else cost_order(first)
        plan = eng.plan(ids[s1[order]], ids[s2[order]], cache=False)
        dp = [(torch.from_numpy(np.ascontiguousarray(x[order].T)).to(dev),
               torch.from_numpy(np.ascontiguousarray(y[order].T)).to(dev)) for x, y in walk]
        out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
        runs = [plan.bind(d1, d2, out, grad=args.grad, contact=False, stream=stream) for d1, d2 in dp]
        runs[0]()
        torch.cuda.synchronize(dev)
        if first is None:
            first = out["iters"].cpu().numpy()   # the one solve the cost order is taken from
        for k in range(20):
            runs[seq[k % len(seq)]]()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for k in range(steps):
            runs[seq[k % len(seq)]]()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / steps
        inv = np.empty(B, np.int64)
        inv[order] = np.arange(B)
        outs[name] = {k: (v.cpu().numpy()[..., inv]) for k, v in out.items()}
        res[name + "_order"] = {"kernel_ms": ms, "pair_solves_per_s": B / (ms * 1e-3)}
        del runs, dp, out, plan
    res["bitwise_equal"] = all(np.array_equal(outs["given"][k].view(np.int64) if outs["given"][k].dtype == np.float64
                                              else outs["given"][k],
                                              outs["cost"][k].view(np.int64) if outs["cost"][k].dtype == np.float64
                                              else outs["cost"][k]) for k in outs["given"])
    res["speedup"] = res["given_order"]["kernel_ms"] / res["cost_order"]["kernel_ms"]
    return res


def kernel_1m(args, eng, ids, tab, dev, reps=20):
    """The solve kernel's steady state, apart from the 100k launch's quantisation (3,125 waves
    over 2,048 wave slots: 1.53 rounds, the last one partly empty): ONE launch of 1M pairs of
    the same distribution (15.3 rounds), kernel only, HIP events on the launch stream (median
    of `reps` after 40 warm-up launches), with its FP64 roofline fraction (counted flops)."""
    import torch
    from dcol_amd import alloc_outputs
    B = 1_000_000
    s1, s2, p1, p2 = pairs(B, len(tab["type"]), seed=7)
    plan = eng.plan(ids[s1], ids[s2], cache=False)
    d1 = torch.from_numpy(np.ascontiguousarray(p1.T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2.T)).to(dev)
    out = alloc_outputs(B, dev, want_grad=True, want_contact=False)
    stream = torch.cuda.current_stream(dev)
    run = plan.bind(d1, d2, out, grad=args.grad, contact=False, stream=stream)
    for _ in range(40):   # ~16 ms of launches: the clocks settle (profiles/r04_clock/)
        run()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(stream)
        run()
        e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
    st = out["status"].cpu().numpy()
    it = out["iters"].cpu().numpy()
    fl = flops_per_pair(it[st == 0], args.grad)
    tf = fl * B / (ms * 1e-3) / 1e12
    gbs = BYTES_PER_PAIR * B / (ms * 1e-3) / 1e9
    del d1, d2, out, plan
    return {"pairs": B, "kernel_ms": ms, "pair_solves_per_s": B / (ms * 1e-3),
            "roofline_fp64": {"achieved": tf, "peak": FP64_VECTOR_PEAK_TFS, "unit": "TFLOP/s",
                              "frac": tf / FP64_VECTOR_PEAK_TFS, "flops_per_pair": fl},
            "roofline_hbm": {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS},
            "ok_frac": float(np.mean(st == 0)), "iters_mean": float(it[st == 0].mean()),
            "note": "one 1M-pair launch (same shape table and pose distribution, seed 7), kernel only, median of "
                    f"{reps} HIP-event launches: the steady-state rate of the solve kernel without the 100k "
                    "launch's last, partly-filled round of waves"}


def end_to_end(args, eng, ids, s1, s2, p1, p2, pose1, pose2, out, step, dev, reps=20):
    """The same batch with the poses starting in host memory (PCIe-inclusive; never `value`):
    (a) pinned host poses -> H2D, the solve, D2H of alpha / grad / status / iters, on the
    bench stream; (b) the C-ABI host call dcol_prox_batch_host (Engine.solve_host: pageable
    numpy in/out, its own staging).  Median over reps, after one warm-up each."""
    import torch
    B = len(s1)
    h1 = torch.from_numpy(np.ascontiguousarray(p1.T)).pin_memory()
    h2 = torch.from_numpy(np.ascontiguousarray(p2.T)).pin_memory()
    ho = {k: torch.empty(v.shape, dtype=v.dtype).pin_memory() for k, v in out.items()}

    def pinned():
        pose1.copy_(h1, non_blocking=True)
        pose2.copy_(h2, non_blocking=True)
        step()
        for k, v in ho.items():
            v.copy_(out[k], non_blocking=True)
        torch.cuda.synchronize(dev)

    def host():
        eng.solve_host(ids[s1], ids[s2], p1, p2, grad=args.grad, contact=False)

    res = {}
    for name, fn in (("pinned_h2d_solve_d2h", pinned), ("solve_host_pageable", host)):
        fn()
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ms = 1e3 * float(np.median(ts))
        res[name] = {"ms": ms, "pair_solves_per_s": B / (ms * 1e-3)}
    res["bytes_h2d"] = int(2 * 48 * B)
    res["bytes_d2h"] = int(sum(v.numel() * v.element_size() for v in ho.values()))
    return res


MIXED_KINDS = (0, 1, 2, 3, 4, 5)      # polytope sphere cone capsule cylinder polygon


def mixed_table(per_kind=64, seed=0):
    """BASELINE configs[4] shapes: per kind `per_kind` shapes —
    rect prisms U(0.2, 2)^3, spheres R ~ U(.2, 1), cones H ~ U(.5, 2), beta ~ U(10, 40) deg,
    capsules / cylinders R ~ U(.1, .6), L ~ U(.3, 2), pentagons d = 0.6 with R = 0.2."""
    rng = np.random.default_rng(seed)
    t, nh, off, prm, A_rows, b_rows = [], [], [], [], [], []
    ang = np.linspace(0, 2 * np.pi, 5, endpoint=False)
    pent = np.stack([np.cos(ang), np.sin(ang)], 1)
    box = np.array([[1.0, 0, 0], [0, 1, 0], [0, 0, 1], [-1, 0, 0], [0, -1, 0], [0, 0, -1]])
    for kind in MIXED_KINDS:
        for _ in range(per_kind):
            t.append(kind)
            off.append(len(b_rows))
            if kind == 0:
                d = rng.uniform(0.2, 2.0, 3)
                A_rows += list(box)
                b_rows += list(np.concatenate([d / 2, d / 2]))
                nh.append(6)
                prm.append((0, 0, 0, 0))
            elif kind == 5:
                A_rows += [list(a) + [0.0] for a in pent]
                b_rows += [0.6] * 5
                nh.append(5)
                prm.append((0.2, 0, 0, 0))
            else:
                nh.append(0)
                if kind == 1:
                    prm.append((rng.uniform(0.2, 1.0), 0, 0, 0))
                elif kind == 2:
                    prm.append((0, 0, rng.uniform(0.5, 2.0), np.deg2rad(rng.uniform(10, 40))))
                else:
                    prm.append((rng.uniform(0.1, 0.6), rng.uniform(0.3, 2.0), 0, 0))
    S = len(t)
    return {"type": np.array(t, np.int32), "nh": np.array(nh, np.int32), "A_off": np.array(off, np.int32),
            "A_pool": np.array(A_rows, dtype=np.float64).reshape(-1, 3), "b_pool": np.array(b_rows, dtype=np.float64),
            "params": np.array(prm, dtype=np.float64), "r_offset": np.zeros((S, 3)),
            "Q_offset": np.tile(np.eye(3), (S, 1, 1))}


def mixed_pairs(tab, B, seed):
    """Ordered kind pairs uniform over the 27 the reference supports (at least one of
    polytope / sphere / cone), shapes uniform within a kind; poses as configs[3]."""
    rng = np.random.default_rng(seed)
    combos = [(a, b) for a in MIXED_KINDS for b in MIXED_KINDS if a <= 2 or b <= 2]
    by_kind = {k: np.flatnonzero(tab["type"] == k) for k in MIXED_KINDS}
    c = rng.integers(0, len(combos), B)
    ka = np.array([combos[i][0] for i in range(len(combos))])[c]
    kb = np.array([combos[i][1] for i in range(len(combos))])[c]
    s1 = np.empty(B, np.int32)
    s2 = np.empty(B, np.int32)
    for k in MIXED_KINDS:
        m1, m2 = ka == k, kb == k
        s1[m1] = rng.choice(by_kind[k], m1.sum())
        s2[m2] = rng.choice(by_kind[k], m2.sum())
    pose1 = np.hstack([rng.uniform(-3, 3, (B, 3)), rng.uniform(-1, 1, (B, 3))])
    pose2 = np.hstack([rng.uniform(-3, 3, (B, 3)), rng.uniform(-1, 1, (B, 3))])
    return s1, s2, pose1, pose2


def run_mixed(args, world, rank, local, dev, coll_dev, dist, wd=None):
    """--workload mixed1m: BASELINE configs[4] as the bench line itself (strong scaling)."""
    line = mixed_measure(args, world, rank, local, dev, coll_dev, dist, args.steps, args.warmup, wd)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        with guard(wd, "destroy_process_group"):
            dist.destroy_process_group()
        wd.close()


def native_comm(NativeComm, dist, world, rank, local, wd=None):
    """(communicator, error) for the C-ABI RCCL path.  Rank 0 makes the unique id and ALWAYS
    takes part in its broadcast (None when it could not make one), so a failure on rank 0
    never leaves the other ranks in a collective rank 0 skipped; the ranks then all create
    the communicator or all skip it.  (A failure inside ncclCommInitRank itself cannot be
    signalled to the ranks already waiting in it: the rank's deadline (wd) ends that wait;
    the usual failure -- librccl not loadable -- surfaces in the id step.)"""
    uid, err = [None], None
    if rank == 0:
        try:
            uid = [NativeComm.unique_id()]
        except Exception as e:
            err = f"{type(e).__name__}: {e}"
    if dist is not None:
        with guard(wd, "communicator id broadcast"):
            dist.broadcast_object_list(uid, src=0)
    if uid[0] is None:
        return None, err or "rank 0 could not create a communicator id"
    try:
        with guard(wd, "communicator set-up (ncclCommInitRank)"):
            return NativeComm(uid[0], world, rank, local), None
    except Exception as e:   # recorded in the line; the step then uses torch.distributed
        return None, f"{type(e).__name__}: {e}"


def mixed_measure(args, world, rank, local, dev, coll_dev, dist, steps, warmup, wd=None):
    """BASELINE configs[4]: 1M mixed-primitive pairs sharded over the ranks (class-balanced
    round-robin, dcol_amd.dist.shard_indices), each shard solved on its GPU from
    HBM-resident poses, then ONE all-gather of the packed per-pair record [alpha, grad(12),
    status, iters] so every rank holds the whole batch.  The timed step = solve + records +
    all-gather (strong scaling: the batch is fixed as N grows).  With the RCCL backend the
    step is the shipped C-ABI path: dcol_prox_batch_multi_gpu (the solver kernels write the
    records into this rank's rows of the gathered buffer, DCOL_NO_GATHER) then
    dcol_comm_all_gather (ncclAllGather in place), both on the launch stream; gloo rehearsals
    (several ranks on one GPU, which RCCL refuses) and --torch-gather go through
    torch.distributed.  value / ms_per_step: K such steps on ONE stream, each bracketed by
    HIP events on it (start, solved, gathered), so kernel_ms -- the solve's share of each
    step -- comes from the same run; the pipelined rate (solves round-robin on --streams
    streams, all-gathers on one collective stream) is reported beside it.  With a deadline
    (wd, N > 1) every wait names its phase and step.  Returns the line (rank 0) or None."""
    import torch
    from dcol_amd import Engine, alloc_outputs, spec_from_arrays
    from dcol_amd.dist import REC, NativeComm, shard_indices
    B = args.pairs if (args.workload == "mixed1m" and args.pairs != 100_000) else 1_000_000
    tab = mixed_table()
    s1, s2, p1, p2 = mixed_pairs(tab, B, seed=0)
    cost = tab["type"][s1] * 8 + tab["type"][s2]          # class key for balanced dealing
    idx = [shard_indices(B, r, world, cost) for r in range(world)]
    mine = idx[rank]
    cap = max(len(i) for i in idx)
    eng = Engine(device=local)
    ids = np.array([eng.register(spec_from_arrays(tab, k)) for k in range(len(tab["type"]))], np.int32)
    plan = eng.plan(ids[s1[mine]], ids[s2[mine]])
    d1 = torch.from_numpy(np.ascontiguousarray(p1[mine].T)).to(dev)
    d2 = torch.from_numpy(np.ascontiguousarray(p2[mine].T)).to(dev)
    out = alloc_outputs(len(mine), dev, want_grad=True, want_contact=False)
    stream = torch.cuda.current_stream(dev)
    launch = plan.bind(d1, d2, out, grad=args.grad, contact=False, stream=stream)
    n = len(mine)
    comm, path = None, "torch.distributed all_gather_into_tensor" if dist is not None else "local copy (world 1)"
    native_error = None
    if args.backend == "nccl" and not args.torch_gather:
        comm, native_error = native_comm(NativeComm, dist, world, rank, local, wd)
        if dist is not None:     # every rank takes the same path
            ok = torch.tensor([0.0 if comm is None else 1.0], device=coll_dev)
            with guard(wd, "communicator agreement (all_reduce)"):
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if ok.item() < 1.0 and comm is not None:
                comm.close()
                comm, native_error = None, native_error or "another rank could not create its communicator"
        if comm is not None:
            path = ("C-ABI dcol_prox_batch_multi_gpu (pack_records + ncclAllGather, RCCL)" if args.pack_pass else
                    "C-ABI dcol_prox_batch_multi_gpu in place (records written by the solver kernels into the "
                    "gathered buffer, DCOL_NO_GATHER) + dcol_comm_all_gather (ncclAllGather in place, RCCL)")
    rec = torch.full((cap, REC), float("nan"), dtype=torch.float64, device=dev)
    gathered = torch.empty((world * cap, REC), dtype=torch.float64, device=dev if comm is not None else coll_dev)

    # Each step function issues step k on its stream(s) and returns (stream, solved, gathered):
    # events recorded after the step's solve and after its all-gather (None where the
    # all-gather is host-synchronous: torch.distributed with gloo / world 1).
    def ev():
        return torch.cuda.Event(enable_timing=True)

    lanes = []
    if comm is not None and args.pack_pass:
        # the pack kernel + out-of-place all-gather (A/B): one stream, one communicator
        def step(k):
            e = ev()
            comm.solve_gather(plan, d1, d2, cap, grad=args.grad, out=out, stream=stream, rec_local=rec, rec_all=gathered)
            e.record(stream)
            return e, e

        def solve_only():   # its solve: the plan run with the per-pair arrays
            launch()
    elif comm is not None:
        # records written by the solver kernels, all-gather in place.  The pipelined steps are
        # issued round-robin on --streams solve streams, each with its own gathered buffer;
        # every all-gather goes through the ONE communicator on ONE collective stream, in issue
        # order on every rank: step k's solve (DCOL_NO_GATHER) -> event -> its all-gather on the
        # collective stream -> event that step k + S's solve waits for before it overwrites the
        # buffer.  So step k + 1's solve overlaps step k's all-gather (a batch service's steady
        # state) without two communicators or collectives on two streams.
        cstream = torch.cuda.Stream(dev)
        nst = max(1, args.streams)
        bufs = [gathered] + [torch.empty((world * cap, REC), dtype=torch.float64, device=dev) for _ in range(nst - 1)]
        sstreams = [stream] + [torch.cuda.Stream(dev) for _ in range(nst - 1)]
        gdone = [None] * nst

        def lane_fn(j):
            st, g_ = sstreams[j], bufs[j]

            def f(k):
                if gdone[j] is not None:
                    st.wait_event(gdone[j])
                comm.solve_gather(plan, d1, d2, cap, grad=args.grad, stream=st, rec_all=g_, in_place=True, soa=False,
                                  gather=False)
                solved = ev()
                solved.record(st)
                cstream.wait_event(solved)
                comm.all_gather(cap, g_, stream=cstream)
                gd = ev()
                gd.record(cstream)
                gdone[j] = gd
                return solved, gd
            return f
        lanes = [lane_fn(j) for j in range(nst)]

        def step(k):          # one step on the launch stream: the solve, then the all-gather on it
            comm.solve_gather(plan, d1, d2, cap, grad=args.grad, stream=stream, rec_all=gathered, in_place=True,
                              soa=False, gather=False)
            solved = ev()
            solved.record(stream)
            comm.all_gather(cap, gathered, stream=stream)
            gd = ev()
            gd.record(stream)
            return solved, gd

        def solve_only():    # the same solve and record writes without the all-gather (DCOL_NO_GATHER)
            comm.solve_gather(plan, d1, d2, cap, grad=args.grad, stream=stream, rec_all=gathered, in_place=True,
                              soa=False, gather=False)
    else:
        def solve_only():
            launch()
            rec[:n, 0] = out["alpha"]
            rec[:n, 1:13] = out["grad"].T
            # (status, iters) as an int32 pair in the last slot (dcol_amd.dist.REC)
            rec[:n, 13] = ((out["iters"].to(torch.int64) << 32) | (out["status"].to(torch.int64) & 0xFFFFFFFF)).view(
                torch.float64)

        def step(k):
            solve_only()
            solved = ev()
            solved.record(stream)
            if dist is not None:
                src = rec.to(coll_dev)
                with guard(wd, "all-gather", k):
                    dist.all_gather_into_tensor(gathered, src)
            else:
                gathered.copy_(rec)
            gd = ev()
            gd.record(stream)
            return solved, gd

    def settle(phase):
        torch.cuda.synchronize(dev) if wd is None else sync(dev, wd, phase)

    def run_steps(fns, phase):
        """warm-up, then exactly `steps` steps timed between barrier + synchronize pairs;
        (elapsed s max over ranks, per-step [start, solved, gathered] events)"""
        for k in range(warmup):
            fns[k % len(fns)](k)
        settle(phase + " warmup")
        barrier(dist, wd, "barrier before the " + phase + " steps")
        settle("synchronize before the " + phase + " steps")
        marks = []
        t0 = time.perf_counter()
        for k in range(steps):
            st = sstreams[k % len(fns)] if fns is lanes else stream
            e0 = ev()
            e0.record(st)
            marks.append((e0,) + tuple(fns[k % len(fns)](k)))
        for k, (_, solved, gd) in enumerate(marks):   # (a rank that hangs names its step and phase)
            wait_event(solved, wd, phase + " solve", k)
            wait_event(gd, wd, phase + " all-gather", k)
        settle("synchronize after the " + phase + " steps")
        el = time.perf_counter() - t0
        barrier(dist, wd, "barrier after the " + phase + " steps")
        if dist is not None:
            t = torch.tensor([el], device=coll_dev, dtype=torch.float64)
            with guard(wd, "all_reduce of the " + phase + " time"):
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t[0])
        return el, marks

    settle_info = clock_settle(launch, stream, dev, wd, args.settle_ms)
    elapsed, marks = run_steps([step], "serial")
    # the solve's share of each timed step (start -> solved) and the whole step, same run
    kernel_ms = float(np.median([a.elapsed_time(b) for a, b, _ in marks]))
    step_ev_ms = float(np.median([a.elapsed_time(c) for a, _, c in marks]))
    elapsed_pipe = run_steps(lanes, "pipelined")[0] if len(lanes) > 1 else None

    def ev_times(fns, reps=20):
        """HIP-event durations [reps, len(fns)] (ms), the fns interleaved rep by rep (the same
        clock state for all of them)"""
        evs = [[(ev(), ev()) for _ in fns] for _ in range(reps)]
        for row in evs:
            for fn, (e0, e1) in zip(fns, row):
                e0.record(stream)
                fn()
                e1.record(stream)
        settle("step breakdown")
        return np.array([[e0.elapsed_time(e1) for e0, e1 in row] for row in evs])
    # like for like (HIP events on the launch stream, one step at a time, interleaved): solve =
    # the step's own solve and record writes without its collective; step = the same with it;
    # their difference is the communication cost of the step (5-50 %
    # predicted at 8 GPUs).  plan = the plan run with the per-pair arrays.
    tt = ev_times([solve_only, lambda: step(-1), launch])
    solve_ms, step_ms, plan_ms = (float(v) for v in np.median(tt, axis=0))
    comm_d = tt[:, 1] - tt[:, 0]          # paired: each step against the solve just before it
    comm_ms = float(np.median(comm_d))
    comm_iqr = float(np.subtract(*np.percentile(comm_d, [75, 25])))
    my_iters = out["iters"].cpu().numpy()
    my_status = out["status"].cpu().numpy()
    flops_local = mixed_flops(tab, s1[mine], s2[mine], my_iters, my_status, args.grad)
    # per-rank shard figures (load balance): solve ms, step ms, mean Newton iterations
    mine_stats = [solve_ms, step_ms, float(my_iters[my_status == 0].mean()) if (my_status == 0).any() else 0.0, float(n),
                  kernel_ms, plan_ms]
    if dist is not None:
        t = torch.zeros((world, len(mine_stats)), device=coll_dev, dtype=torch.float64)
        t[rank] = torch.tensor(mine_stats, dtype=torch.float64)
        with guard(wd, "all_reduce of the per-rank figures"):
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        ranks_stats = t.cpu().numpy()
    else:
        ranks_stats = np.array([mine_stats])
    solve_ms_max = float(ranks_stats[:, 0].max())
    settle("synchronize before the result copy")
    allrec = gathered.cpu().numpy().reshape(world, cap, REC)
    if comm is not None:
        comm.close()
    if rank != 0:
        return None
    full = np.empty((B, REC))
    for r, ix in enumerate(idx):
        full[ix] = allrec[r, :len(ix)]
    from dcol_amd.dist import unpack
    res_all = unpack(full)
    status = res_all["status"]
    line = {
        "metric": "PDIP proximity+grad pair-solves/sec", "value": B * steps / elapsed, "unit": "pair-solves/s",
        "n_gpus": world, "steps": steps, "warmup": warmup, "ms_per_step": 1e3 * elapsed / steps,
        "kernel_ms": kernel_ms, "step_event_ms": step_ev_ms,
        "timing": "value = pairs / ms_per_step of K steps on one stream (solve, then the all-gather, per step); "
                  "kernel_ms = the median HIP-event time from a step's start to its solve's end, step_event_ms to "
                  "its all-gather's end, in that same run (rank 0); the rooflines use kernel_ms",
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "synthetic 1M mixed-primitive pairs sharded across GPUs + RCCL all-gather "
                               "(BASELINE.json configs[4])", "pairs_total": B, "pairs_per_gpu": cap,
                   "kinds": "polytope sphere cone capsule cylinder polygon; 27 supported ordered kind pairs",
                   "gradient": args.grad, "collective": f"{path}: one all-gather of [alpha, grad(12), (status, iters) int32]",
                   "parallelism": f"dp{world} (class-balanced shards)"},
        "solve_stats": {"ok_frac": float(np.mean(status == 0)), "iters_mean": float(res_all["iters"][status == 0].mean())},
        "solve_ms_rank0": solve_ms, "solve_ms_max_rank": solve_ms_max,
        "step_breakdown": {
            "note": "HIP events on each rank's launch stream, one step at a time (median of 20, the three "
                    "measurements interleaved), like for like: "
                    "solve = the step's own solve and record writes without its collective (" + (
                        "the plan run with the per-pair arrays; the pack pass + all-gather are the comm"
                        if args.pack_pass else "dcol_prox_batch_multi_gpu with DCOL_NO_GATHER") +
                    "); step = the same with the all-gather; comm = the median of the paired per-rep differences "
                    "step - solve (its interquartile range beside it: the measurement's noise)",
            "solve_ms_max_rank": solve_ms_max, "step_ms_max_rank": float(ranks_stats[:, 1].max()),
            "comm_ms_rank0": comm_ms, "comm_frac_rank0": comm_ms / step_ms if step_ms > 0 else None,
            "comm_ms_iqr_rank0": comm_iqr,
            "record_bytes_per_pair": REC * 8,
            "per_rank": {"solve_ms": ranks_stats[:, 0].tolist(), "step_ms": ranks_stats[:, 1].tolist(),
                         "kernel_ms": ranks_stats[:, 4].tolist(), "plan_run_ms": ranks_stats[:, 5].tolist(),
                         "iters_mean": ranks_stats[:, 2].tolist(), "pairs": ranks_stats[:, 3].astype(int).tolist()}},
        "kernel_ms_max_rank": float(ranks_stats[:, 4].max()),
        "settle": settle_info,
        "pipeline": {"streams": max(1, len(lanes)), "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                     "note": "solves round-robin on the streams, all-gathers on one collective stream (an overlap "
                             "rate, not value)",
                     "value": B * steps / elapsed_pipe if elapsed_pipe else None,
                     "ms_per_step": 1e3 * elapsed_pipe / steps if elapsed_pipe else None},
    }
    if comm is not None:
        line["rccl_world_size"] = world
        line["collective_issue"] = ("one communicator, all-gathers in issue order on one collective stream, "
                                    "chained to the solve streams by events" if not args.pack_pass else
                                    "one communicator, one stream")
    if native_error:
        line["native_comm_error"] = native_error
    if flops_local is not None:
        tf = flops_local / (kernel_ms * 1e-3) / 1e12
        line["roofline_fp64"] = {"bound": "fp64-valu", "achieved": tf, "peak": FP64_VECTOR_PEAK_TFS,
                                 "unit": "TFLOP/s", "frac": tf / FP64_VECTOR_PEAK_TFS,
                                 "flops_per_pair": flops_local / max(n, 1),
                                 "note": "rank 0's shard: counted per-class flops (profiles/flop_model.json) at each "
                                         "pair's iteration count / its solve time in the timed run (kernel_ms)"}
    if world == 1 and B == 1_000_000 and args.shard_steps > 0:
        line["shards"] = shards_section(args, eng, ids, tab, s1, s2, p1, p2, cost, dev)
    if args.check:
        from oracle import c_oracle
        k = min(args.check * 8, B)
        ref = c_oracle.run_batch(tab, s1[:k], s2[:k], p1[:k], p2[:k], want_grad=True, threads=cpu_share()[0])
        ok = ref["status"] == 0
        line["parity_check"] = {
            "pairs": int(k), "status_equal": bool(np.array_equal(status[:k], ref["status"])),
            "alpha_ok": bool(np.all(np.abs(full[:k, 0][ok] - ref["alpha"][ok]) <= 1e-6 * np.abs(ref["alpha"][ok]) + 1e-12)),
            "grad_ok": bool(np.all(np.abs(full[:k, 1:13][ok] - ref["grad"][ok]).max(1)
                                   <= 1e-5 * np.maximum(np.abs(ref["grad"][ok]).max(1), 1)))
            if args.grad == "fd" else None}   # the C oracle restates the reference's FD gradient only
    return line


def shards_section(args, eng, ids, tab, s1, s2, p1, p2, cost, dev):
    """configs[4]'s per-rank regime, measured on this one GPU: for each N of --shard-worlds,
    rank 0's class-balanced shard (dcol_amd.dist.shard_indices: the shard bench.py --gpus N
    gives rank 0) solved alone -- K steps back to back on one stream, HIP events around the
    region, the library's plan policy (a packed launch for mid-size plans, DESIGN.md section
    5) -- with its FP64 fraction and its ratio to linear ((1M solve) / N); the all-gather of
    the N-rank step MODELLED (dcol_amd.dist.gather_ms: no multi-GPU node in this pool) and the
    projected strong-scaling step = shard solve + all-gather; B*, the smallest batch for which
    N GPUs beat one, from this run's solve curve."""
    import torch
    from dcol_amd import alloc_outputs
    from dcol_amd import dist as D
    B = len(s1)
    stream = torch.cuda.current_stream(dev)
    worlds = [1] + [int(w) for w in args.shard_worlds.split(",") if int(w) > 1]
    rows, curve = [], []
    for N in worlds:
        mine = D.shard_indices(B, 0, N, cost)
        plan = eng.plan(ids[s1[mine]], ids[s2[mine]], cache=False)
        d1 = torch.from_numpy(np.ascontiguousarray(p1[mine].T)).to(dev)
        d2 = torch.from_numpy(np.ascontiguousarray(p2[mine].T)).to(dev)
        out = alloc_outputs(len(mine), dev, want_grad=True, want_contact=False)
        run = plan.bind(d1, d2, out, grad=args.grad, contact=False, stream=stream)
        clock_settle(run, stream, dev, None, 10.0)   # (as tools/shard_bench.py: each plan from settled clocks)
        for _ in range(10):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.shard_steps):
            run()
        e1.record(stream)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / args.shard_steps
        st, it = out["status"].cpu().numpy(), out["iters"].cpu().numpy()
        fl = mixed_flops(tab, s1[mine], s2[mine], it, st, args.grad)
        r = {"world": N, "pairs": int(len(mine)), "solve_ms": ms, "pair_solves_per_s": len(mine) / (ms * 1e-3),
             "launch_form": plan.launch_form, "launches": plan.num_launches, "buckets": plan.num_buckets}
        if fl is not None:
            r["fp64_frac"] = fl / (ms * 1e-3) / 1e12 / FP64_VECTOR_PEAK_TFS
        curve.append((len(mine), ms))
        rows.append(r)
        del plan, d1, d2, out, run
    full = rows[0]["solve_ms"]
    for r in rows[1:]:
        N = r["world"]
        r["linear_frac"] = full / N / r["solve_ms"]
        g, gi = D.gather_ms(B, N), D.gather_ms(B, N, D.GATHER_IDEAL_GBPS)
        r["gather_model"] = {"bytes_received_per_rank": int((N - 1) * -(-B // N) * D.REC * 8), "ms": g,
                             "ms_at_ideal_xgmi": gi}
        r["projected_step_ms"] = r["solve_ms"] + g
        r["projected_pair_solves_per_s"] = B / ((r["solve_ms"] + g) * 1e-3)
        r["projected_pair_solves_per_s_ideal_xgmi"] = B / ((r["solve_ms"] + gi) * 1e-3)
    return {"note": "rank 0's class-balanced shard of the 1M configs[4] batch at world N, solved alone on this GPU "
                    f"({args.shard_steps} steps back to back on one stream, HIP events); linear_frac = (the 1M solve / N) "
                    "/ the shard's solve; gather_model: the N-rank step's all-gather MODELLED (not measured: no "
                    f"multi-GPU node here) at {D.GATHER_BUS_GBPS:.0f} GB/s RCCL bus bandwidth + {D.GATHER_LAT_MS} ms, "
                    f"and at the {D.GATHER_IDEAL_GBPS:.0f} GB/s xGMI ingress bound; projected_step = shard solve + modelled "
                    "all-gather (the bench's serial mixed1m step)",
            "solve_ms_1m": full, "per_world": rows,
            "crossover_pairs": {str(N): D.shard_crossover(N, curve) for N in (2, 4, 8)},
            "crossover_pairs_ideal_xgmi": {str(N): D.shard_crossover(N, curve, D.GATHER_IDEAL_GBPS) for N in (2, 4, 8)},
            "crossover_note": "B*: the smallest batch for which N GPUs (shards + one all-gather) beat one GPU, from this "
                              "run's solve curve (dcol_amd.dist.shard_crossover / should_shard)"}


def mixed_flops(tab, s1, s2, iters, status, grad="fd"):
    """Counted FP64 flops of a mixed shard: per pair, its class's model
    (profiles/flop_model.json) at its own Newton iteration count; None without the model."""
    path = os.path.join(REPO, "profiles", "flop_model.json")
    if not os.path.exists(path):
        return None
    classes = json.load(open(path))["classes"]
    names = {0: "polytope", 1: "sphere", 2: "cone", 3: "capsule", 4: "cylinder", 5: "polygon"}
    k1, k2 = tab["type"][s1], tab["type"][s2]
    total = 0.0
    for a in range(6):
        for b in range(6):
            m = (k1 == a) & (k2 == b) & (status == 0)
            if not m.any():
                continue
            c = classes[f"{names[a]}-{names[b]}"]
            g = GRAD_OPS.get(grad, c["grad_fd"])   # closed-form modes: the poly x poly hand counts
            total += m.sum() * (c["assembly"] + c["pdip_fixed"] + g) + c["pdip_per_iter"] * iters[m].sum()
    return total


# The reference's quadrotor ALTRO run (quadrotor.prof): 377,311 PDIP solves,
# 66,000 of them through proximity_gradient (one solve each), the rest through proximity_mrp
QUAD_SOLVES, QUAD_GRAD_CALLS = 377_311, 66_000


def dropin_section(reps=3):
    """The drop-in's per-call latency (BASELINE north star: ALTRO.py drops in unchanged):
    the reference's own calling pattern -- for every knot of the quadrotor's reference
    trajectory, overwrite P_vic.r / .p, then call proximity_mrp (inequality_constraints_x,
    cluttered_hallway_quadrotor.py:115-135) or proximity_gradient
    (inequality_constraints_x_grad, :137-171) once per obstacle -- timed on the host clock,
    one call at a time.  Best of `reps` sweeps; projected onto the reference's quadrotor run
    (QUAD_SOLVES solves, QUAD_GRAD_CALLS of them gradient calls)."""
    from altro import systems
    from proximity.proximity import proximity_mrp
    from proximity.proximity_gradient import proximity_gradient
    params, X, U = systems.initialize("quadrotor")
    vic, obs = params["P_vic"], params["P_obs"]
    nx = int(params["nx"])
    Xr = np.asarray(params["Xref"], dtype=np.float64).reshape(-1, nx)
    out = {"pattern": f"{len(Xr)} knots x {len(obs)} obstacles of the quadrotor hallway, one call per pair "
                      "(P_vic.r / .p overwritten per knot)", "calls_per_sweep": len(Xr) * len(obs),
           "path": "dcol_prox_pair: resident one-pair server (DCOL_PAIR_SERVER=0: one launch per call), "
                   "host glue dcol_amd._fastpair"}
    from dcol_amd.engine import default_engine
    for name, fn in (("proximity_mrp", proximity_mrp), ("proximity_gradient", proximity_gradient)):
        for o in obs:                     # first call per pair kind: its plan, code objects
            vic.r, vic.p = np.array(Xr[0, 0:3]), np.array(Xr[0, 6:9])
            fn(vic, o)
        s0 = default_engine().pair_stats()
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            for x in Xr:
                vic.r = np.array(x[0:3])
                vic.p = np.array(x[6:9])
                for o in obs:
                    fn(vic, o)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        s1 = default_engine().pair_stats()
        served = s1["served"] - s0["served"]
        out[name] = {"us_per_call": 1e6 * best / (len(Xr) * len(obs)), "served_by_pair_server": served,
                     "launched": s1["launched"] - s0["launched"]}
        if served:   # the resident one-pair server's request-to-answer time on the device
            out[name]["device_us_per_call"] = (s1["server_solve_us"] - s0["server_solve_us"]) / served
    t_mrp, t_grad = out["proximity_mrp"]["us_per_call"], out["proximity_gradient"]["us_per_call"]
    proj = ((QUAD_SOLVES - QUAD_GRAD_CALLS) * t_mrp + QUAD_GRAD_CALLS * t_grad) * 1e-6
    out["projected_quadrotor_altro"] = {
        "solves": QUAD_SOLVES, "gradient_calls": QUAD_GRAD_CALLS, "proximity_s": proj,
        "reference_altro_wall_s": ALTRO_REFERENCE["quadrotor"]["python_s"],
        "note": "time the unchanged reference ALTRO.py would spend in the drop-in proximity calls on this GPU "
                "(its own Python around them excluded); the batched driver (altro section) is the fast path"}
    return out


def scene_batches(device):
    """Pair-solves/s of the reference's own scene batches (BASELINE configs[1], [2] and the
    piano mover): every (knot, obstacle) pair of the reference trajectory Xref as one
    device-resident batch with FD gradients, repeated; small launches, latency-bound."""
    import torch
    from altro import systems
    from altro.constraints import ObstacleField
    out = {}
    for name in ("quadrotor", "coneThroughWall", "piano_mover"):
        params, X, U = systems.initialize(name)
        mod = systems.get(name)
        f = ObstacleField(params["P_vic"], params["P_obs"], params["N"])
        f.evaluate(mod.victim_poses(params, np.asarray(params["Xref"], dtype=np.float64)), True)
        reps = 200
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(reps):
            f._launch[True]()
        torch.cuda.synchronize(device)
        dt = (time.perf_counter() - t0) / reps
        out[name] = {"pairs_per_batch": f.B, "ms_per_batch": 1e3 * dt, "pair_solves_per_s": f.B / dt,
                     "launches_per_batch": f.plan.num_launches}
    return out


# Whole-run ALTRO wall-clock of the reference on the same problems: the
# Python reference measured in the build container (seconds, outer iterations) and the
# Julia DifferentiableCollisions.jl numbers of Report.pdf Table 5.
ALTRO_REFERENCE = {"piano_mover": {"python_s": 51.76, "iterations": 35, "julia_s": 0.445},
                   "coneThroughWall": {"python_s": 166.04, "iterations": 37, "julia_s": 0.866},
                   "quadrotor": {"python_s": 1887.9, "iterations": 60, "julia_s": 6.98}}


def altro_section():
    """Second metric of BASELINE.json: ALTRO iteration wall-clock.  Each reference problem
    is solved end to end by the batched driver (altro/), constraints on this GPU, three
    times; the median run is reported (all three in runs_ms_per_iter).  The optimizer loop
    is timed (set-up — shape table, plan, code-object load — excluded and reported
    separately)."""
    import logging
    from altro import solve, systems
    logging.getLogger("altro").setLevel(logging.WARNING)
    out = {"metric": "ALTRO iter wall-clock", "unit": "ms/iter", "higher_is_better": False, "systems": {}}
    for name, ref in ALTRO_REFERENCE.items():
        runs = []
        for _ in range(3):               # whole runs repeated: the median run is reported
            params, X, U = systems.initialize(name)
            runs.append(solve(params, X, U, verbose=False))
        runs.sort(key=lambda q: q.wall_s)
        r = runs[1]
        out["systems"][name] = {
            "runs_ms_per_iter": [q.ms_per_iter for q in runs],
            "converged": r.converged, "iterations": r.iterations, "reference_iterations": ref["iterations"],
            "ms_per_iter": r.ms_per_iter, "wall_s": r.wall_s, "setup_s": r.setup_s,
            "prox_ms_per_iter": 1e3 * r.prox_s / max(r.iterations, 1), "prox_batches": r.prox_batches,
            "pairs_per_batch": r.prox_pairs // max(r.prox_batches, 1),
            "reference_python_ms_per_iter": 1e3 * ref["python_s"] / ref["iterations"],
            "julia_ms_per_iter": 1e3 * ref["julia_s"] / ref["iterations"],
            "speedup_vs_python": ref["python_s"] / r.wall_s, "speedup_vs_julia": ref["julia_s"] / r.wall_s}
    return out


def implicit_reference(O, tab, s1, s2, p1, p2, sel):
    """(sel, ref, ok) for the parity check of --grad implicit: alpha / status from the oracle's
    proximity, the gradient from its implicit_gradient restatement at the returned iterate."""
    alpha, grad, status = np.zeros(sel.size), np.zeros((sel.size, 12)), np.zeros(sel.size, np.int32)
    for j, i in enumerate(sel):
        a, b = O.shape_from_table(tab, s1[i]), O.shape_from_table(tab, s2[i])
        alpha[j], _, x, s_, z, _, dims = O.proximity(a, p1[i][:3], p1[i][3:], b, p2[i][:3], p2[i][3:], 1e-6)
        grad[j] = O.implicit_gradient(a, b, x, s_, z, np.concatenate([p1[i], p2[i]]), dims)
    return sel, {"alpha": alpha, "grad": grad, "status": status}, status == 0


def flops_per_pair(iters, grad="fd", cls="polytope-polytope (bench configs[3])"):
    """Algorithmic FP64 operation count per pair (each +, -, *, /, sqrt = 1) at the run's
    mean Newton iteration count.  Official counts: the op-counting build of
    the C restatement, fitted per class into profiles/flop_model.json by
    tests/golden/gen_flop_model.py -- poly6 x poly6: assembly 512 + PDIP 1100 + 1672 per
    iteration + FD gradient 8444 (13 Lagrangian evaluations).  The closed-form envelope
    gradient has no reference counterpart: its 760 ops are the hand count of
    env_grad_prim.  Without the JSON, the hand model of SURVEY.md §8d."""
    it = float(np.mean(iters)) if len(iters) else 7.0
    path = os.path.join(REPO, "profiles", "flop_model.json")
    if os.path.exists(path):
        c = json.load(open(path))["classes"][cls]
        return c["assembly"] + c["pdip_fixed"] + it * c["pdip_per_iter"] + GRAD_OPS.get(grad, c["grad_fd"])
    return 530 + 777 + it * 1682 + 276 + GRAD_OPS.get(grad, 8485)


# hand counts of the closed-form gradient modes for poly6 x poly6 (no reference counterpart,
# so no counted restatement): envelope = env_grad_prim x 2 = 760; implicit (dcol_device.hpp
# Solver::implicit_weights, imp_grad_prim) = normal matrix at the returned iterate 12 rows x
# 28 (336) + 4 x 4 Cholesky (40) + solve v = H^-1 e3 (32) + weights a = -W^-2 G v 12 x 8 (96)
# + two row aggregates per primitive 12 x 2 x 6 (144) + the envelope pass (760) + the dG-only
# pass at v, 2 x 170 (340) = 1,748
GRAD_OPS = {"envelope": 760, "implicit": 1748}


if __name__ == "__main__":
    main()
