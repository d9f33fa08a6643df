"""Multi-rank sharding + all-gather (dcol_amd.dist): world_size 2, gloo backend.

CPU tests: each rank solves its shard with the NumPy oracle (test infrastructure standing in
for the per-rank GPU engine).  GPU test: each rank runs the HIP engine on its shard (two
processes on the one GPU of the box; RCCL refuses two ranks on one device, so the exchange
is gloo).  Either way the gathered full batch must equal a single-process solve of the
whole batch exactly (no cross-pair arithmetic exists)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import golden_files, load_golden


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_fn(d, want_grad=True):
    from oracle import dcol_oracle as O

    def fn(idx):
        out = O.run_batch(d, d["s1"][idx], d["s2"][idx], d["pose1"][idx], d["pose2"][idx], 1e-6, want_grad)
        return {"alpha": out["alpha"], "grad": out["grad"], "status": out["status"], "iters": out["iters"]}
    return fn


def _worker(rank, world, port, path, balanced, q, use_engine=False):
    import sys
    import torch.distributed as dist
    from conftest import PKG, REPO
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    from dcol_amd.dist import ShardedBatch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = load_golden(path)
    B = 120
    d = {k: (v[:B] if k in ("s1", "s2", "pose1", "pose2") else v) for k, v in d.items()}
    cost = (d["nh"][d["s1"]] + d["nh"][d["s2"]]) if balanced else None
    sb = ShardedBatch(B, rank, world, cost_key=cost)
    if use_engine:
        from dcol_amd import Engine, spec_from_arrays
        from dcol_amd.dist import engine_solve_fn
        eng = Engine(device=0)
        ids = np.array([eng.register(spec_from_arrays(d, k)) for k in range(len(d["type"]))], np.int32)
        local = sb.solve(engine_solve_fn(eng, ids[d["s1"]], ids[d["s2"]], d["pose1"], d["pose2"]))
    else:
        local = sb.solve(_oracle_fn(d))
    full = sb.gather(local)
    if rank == 0:
        q.put({k: v for k, v in full.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("balanced", [False, True])
def test_gloo_world2_gather_equals_single(balanced):
    path = [p for p in golden_files() if p.endswith("synthetic_mixed.npz")][0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, path, balanced, q)) for r in range(2)]
    for p in procs:
        p.start()
    full = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    d = load_golden(path)
    ref = _oracle_fn({k: (v[:120] if k in ("s1", "s2", "pose1", "pose2") else v) for k, v in d.items()})(np.arange(120))
    np.testing.assert_array_equal(full["status"], ref["status"])
    np.testing.assert_array_equal(full["iters"], ref["iters"])
    np.testing.assert_array_equal(full["alpha"], ref["alpha"])
    np.testing.assert_array_equal(full["grad"], ref["grad"])


def test_shard_indices_partition():
    from dcol_amd.dist import shard_indices
    rng = np.random.default_rng(0)
    for B in (0, 1, 7, 100, 1001):
        for world in (1, 2, 3, 8):
            for cost in (None, rng.integers(0, 5, B)):
                parts = [shard_indices(B, r, world, cost) for r in range(world)]
                allidx = np.sort(np.concatenate(parts)) if parts else np.zeros(0)
                np.testing.assert_array_equal(allidx, np.arange(B))
                sizes = [len(p) for p in parts]
                assert max(sizes) - min(sizes) <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("balanced", [False, True])
def test_gloo_world2_hip_engine_gather_equals_single(balanced):
    """Two ranks, each solving its shard with the HIP engine (lib/libdcol.so), all-gathered
    over gloo: bitwise equal to one process solving the whole batch with the engine."""
    from dcol_amd import Engine, spec_from_arrays
    path = [p for p in golden_files() if p.endswith("synthetic_mixed.npz")][0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, path, balanced, q, True)) for r in range(2)]
    for p in procs:
        p.start()
    full = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    d = load_golden(path)
    eng = Engine(device=0)
    ids = np.array([eng.register(spec_from_arrays(d, k)) for k in range(len(d["type"]))], np.int32)
    ref = eng.solve_host(ids[d["s1"][:120]], ids[d["s2"][:120]], d["pose1"][:120], d["pose2"][:120], contact=False)
    np.testing.assert_array_equal(full["status"], ref.status)
    np.testing.assert_array_equal(full["iters"], ref.iters)
    np.testing.assert_array_equal(full["alpha"], ref.alpha)
    np.testing.assert_array_equal(full["grad"], ref.grad)
    np.testing.assert_array_equal(full["status"], d["status"][:120])


class _FakeComm:
    """Stand-in for dcol_amd.dist.NativeComm (no RCCL on the CPU): ``fail`` names the step
    that raises -- "id" (rank 0's unique id) or "create" (the constructor on rank 1)."""
    fail = None

    def __init__(self, uid, world, rank, device):
        if _FakeComm.fail == "create" and rank == 1:
            raise RuntimeError("ncclCommInitRank: stand-in failure")
        self.uid, self.rank = uid, rank

    @staticmethod
    def unique_id():
        if _FakeComm.fail == "id":
            raise RuntimeError("librccl not loadable (stand-in)")
        return b"\x07" * 128


def _comm_worker(rank, world, port, fail, q):
    import sys
    import torch.distributed as dist
    from conftest import REPO
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _FakeComm.fail = fail
    c, err = bench.native_comm(_FakeComm, dist, world, rank, 0)
    dist.barrier()                 # reached by both ranks: no collective was left unmatched
    q.put((rank, c is not None, c.uid if c is not None else None, err))
    dist.destroy_process_group()


@pytest.mark.parametrize("fail", [None, "id", "create"])
def test_native_comm_setup_never_splits_collectives(fail):
    """bench.native_comm: rank 0 takes part in the id broadcast even when it cannot make an
    id, so a failure there ends with every rank skipping the C-ABI path instead of one rank
    waiting in a broadcast the other skipped (world 2, gloo)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, 2, port, fail, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if fail is None:
        assert all(ok for _, ok, _, _ in res) and res[0][2] == res[1][2] == b"\x07" * 128
    elif fail == "id":
        assert not any(ok for _, ok, _, _ in res)
        assert "librccl" in res[0][3] and "rank 0" in res[1][3]
    else:   # the caller's all-reduce of the outcome then makes rank 0 drop its communicator
        assert res[0][1] and not res[1][1] and "stand-in" in res[1][3]


def test_native_comm_solve_gather_argument_combinations():
    """NativeComm.solve_gather refuses the combinations the C-ABI cannot honour, before any
    device work: in place with a rec_local, or records-only (soa=False) with the pack pass."""
    from dcol_amd.dist import NativeComm
    comm = object.__new__(NativeComm)          # no communicator: the checks come first
    comm.world, comm.rank, comm.device, comm.handle = 1, 0, 0, None

    class _Plan:
        B = 4
    with pytest.raises(ValueError, match="in_place"):
        comm.solve_gather(_Plan(), None, None, 4, rec_local=object(), in_place=True)
    with pytest.raises(ValueError, match="soa=False"):
        comm.solve_gather(_Plan(), None, None, 4, soa=False)


def _run_deadline(mode, deadline=3.0, timeout=120):
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(here, "deadline_rank.py"), mode, str(deadline)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    diags = []
    for ln in (p.stderr + p.stdout).splitlines():
        i = ln.find('{"dcol_deadline"')
        if i >= 0:
            diags.append(json.loads(ln[i:]))
    return p, diags


def test_deadline_rank_skipping_a_step_exits_nonzero_with_diagnostic():
    """bench.py's N > 1 deadline (dcol_amd.dist.StepWatchdog): rank 1 skips step 2 of the
    all-gather loop and stalls; rank 0, waiting in step 2's all-gather, must print ONE JSON
    diagnostic naming its rank, the phase and the step, and the run must exit non-zero well
    before the backend's own timeout -- instead of hanging until the launcher's limit."""
    import time
    t0 = time.monotonic()
    p, diags = _run_deadline("skip", deadline=3.0)
    took = time.monotonic() - t0
    assert p.returncode != 0, p.stdout + p.stderr
    r0 = [d for d in diags if d["rank"] == 0]
    assert r0, p.stderr[-3000:]
    assert r0[0]["phase"] == "all-gather" and r0[0]["step"] == 2 and r0[0]["world"] == 2
    assert r0[0]["waited_s"] >= 3.0
    assert took < 60, took        # the backend's own timeout is 90 s


def test_deadline_clean_run_exits_zero():
    p, diags = _run_deadline("none", deadline=20.0)
    assert p.returncode == 0, p.stdout + p.stderr
    assert not diags
    assert p.stdout.count("steps done") == 2


def test_gather_model_and_crossover():
    """When sharding pays (dcol_amd.dist): the all-gather model moves
    (N - 1) / N of the N x cap records through each rank; the solve curve interpolates the
    measured points log-log and extrapolates linearly past the largest; B* is where N GPUs
    start winning for good, and should_shard agrees with it on both sides."""
    from dcol_amd import dist as D
    assert D.gather_ms(1_000_000, 1) == 0.0
    g8 = D.gather_ms(1_000_000, 8, bus_gbps=100.0, lat_ms=0.0)
    assert abs(g8 - 8 * 125_000 * D.REC * 8 * 7 / 8 / 100e9 * 1e3) < 1e-12
    pts = ((1000, 0.01), (10_000, 0.1))
    assert abs(D.solve_ms(1000, pts) - 0.01) < 1e-15 and abs(D.solve_ms(10_000, pts) - 0.1) < 1e-15
    assert abs(D.solve_ms(20_000, pts) - 0.2) < 1e-12          # throughput-bound past the curve
    assert D.solve_ms(10, pts) == pytest.approx(0.01, rel=1e-12)   # latency floor below it
    assert D.solve_ms(3000, pts) == pytest.approx(0.03, rel=1e-9)
    for n in (2, 4, 8):
        b = D.shard_crossover(n)
        assert b is not None and 1000 < b < 1_000_000
        assert D.should_shard(1_000_000, n) and D.should_shard(2 * b, n)
        assert not D.should_shard(int(b * 0.98), n) or D.shard_crossover(n) == b
    assert D.shard_crossover(8, bus_gbps=1e-3) is None          # a gather that never pays
    assert not D.should_shard(10 ** 9, 1)
