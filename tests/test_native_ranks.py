"""The C-ABI multi-GPU path at rank != 0 (include/dcol.h dcol_prox_batch_multi_gpu,
dcol_comm_all_gather).

RCCL refuses two ranks on one device, so on the one-GPU box the ranks are host threads of
this process, each with its own communicator, engine, plan, stream and buffers, over the
in-process collective stand-in tests/fake_rccl/ (DCOL_RCCL_LIB).  This executes the
rank-dependent code of the library -- the in-place slice rec_all + rank * cap * DCOL_REC,
the NaN tail memset at a non-zero offset, the all-gather with its send buffer aliased
inside the receive buffer, the pack pass, and the split solve / all-gather on two streams
of the bench's pipelined step -- and checks every rank's gathered buffer bitwise against
the shards solved one by one (plus the reference's golden values for the whole batch).
"""
import os
import threading

import numpy as np
import pytest

from conftest import REPO, alpha_close, golden_files, load_golden

FAKE = os.path.join(REPO, "tests", "fake_rccl", "libdcol_fake_rccl.so")


def test_fake_collective_library_exports():
    """(CPU) the stand-in is built and exports the five entry points libdcol.so resolves"""
    import subprocess
    assert os.path.exists(FAKE), "build it: make -C tests/fake_rccl (done by __graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", FAKE], capture_output=True, text=True).stdout
    for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllGather", "ncclCommDestroy", "ncclGetErrorString"):
        assert f" T {f}" in out, f


def _expected_rows(rec_ref, cap, tail):
    """one rank's slice of the gathered buffer: its shard's records, then `tail` rows"""
    out = np.empty((cap, rec_ref.shape[1]), dtype=np.float64)
    out[:len(rec_ref)] = rec_ref
    out.view(np.uint64)[len(rec_ref):] = tail
    return out


def _run_ranks(world, mode, steps=3):
    """world ranks as threads; returns (per-rank gathered buffers, per-rank shard references,
    shard index lists, cap, golden dict)"""
    import torch
    from dcol_amd import Engine, spec_from_arrays
    from dcol_amd.dist import REC, NativeComm, pack, shard_indices

    d = load_golden([p for p in golden_files() if p.endswith("synthetic_mixed.npz")][0])
    B = len(d["s1"]) - 1                     # odd: unequal shards, so the last ranks have a tail
    cost = d["type"][d["s1"][:B]] * 8 + d["type"][d["s2"][:B]]
    idx = [shard_indices(B, r, world, cost) for r in range(world)]
    cap = max(len(i) for i in idx)
    assert min(len(i) for i in idx) < cap
    uid = NativeComm.unique_id()
    results, refs, errors = [None] * world, [None] * world, []
    barrier = threading.Barrier(world)

    def rank_fn(r):
        try:
            torch.cuda.set_device(0)
            eng = Engine(device=0)
            ids = np.array([eng.register(spec_from_arrays(d, k)) for k in range(len(d["type"]))], np.int32)
            mine = idx[r]
            plan = eng.plan(ids[d["s1"][mine]], ids[d["s2"][mine]])
            p1 = torch.from_numpy(np.ascontiguousarray(d["pose1"][mine].T)).cuda()
            p2 = torch.from_numpy(np.ascontiguousarray(d["pose2"][mine].T)).cuda()
            st = torch.cuda.Stream()
            cs = torch.cuda.Stream()
            comm = NativeComm(uid, world, r, 0)
            try:
                # two buffers used alternately (the bench's pipelined step): a stale buffer
                # or a missing ordering between the streams shows up as a mismatch
                bufs = [torch.full((world * cap, REC), 5.0, dtype=torch.float64, device="cuda") for _ in range(2)]
                gdone = [torch.cuda.Event() for _ in range(2)]
                barrier.wait()
                for k in range(steps):
                    j = k % 2
                    g = bufs[j]
                    if mode == "in_place":
                        comm.solve_gather(plan, p1, p2, cap, grad="fd", stream=st, rec_all=g, in_place=True, soa=False)
                    elif mode == "pack":
                        comm.solve_gather(plan, p1, p2, cap, grad="fd", stream=st, rec_all=g)
                    else:   # split: solve on st, the all-gather on cs, chained by events
                        st.wait_event(gdone[j])
                        comm.solve_gather(plan, p1, p2, cap, grad="fd", stream=st, rec_all=g, in_place=True,
                                          soa=False, gather=False)
                        ev = torch.cuda.Event()
                        ev.record(st)
                        cs.wait_event(ev)
                        comm.all_gather(cap, g, stream=cs)
                        gdone[j].record(cs)
                torch.cuda.synchronize()
                ref = plan.run(p1, p2, grad="fd", contact=False, stream=st)
                st.synchronize()
            finally:
                comm.close()
            results[r] = [b.cpu().numpy() for b in bufs]
            refs[r] = pack(ref["alpha"].cpu().numpy(), ref["grad"].cpu().numpy().T, ref["status"].cpu().numpy(),
                           ref["iters"].cpu().numpy())
        except BaseException as e:   # reported by the main thread
            errors.append(f"rank {r}: {type(e).__name__}: {e}")
            barrier.abort()

    threads = [threading.Thread(target=rank_fn, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in threads), "a rank thread hung"
    assert not errors, errors
    return results, refs, idx, cap, d


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode", ["in_place", "pack", "split"])
def test_native_multi_gpu_ranks(world, mode, monkeypatch):
    """Every rank's gathered buffer == the concatenation of every rank's own shard solve
    (bitwise), tail rows all-ones bytes (in place) or NaN (pack pass); the whole batch
    reassembled from the gathered records matches the reference's golden values."""
    from conftest import gpu_available
    if not gpu_available():
        pytest.skip("no GPU")
    from dcol_amd.dist import unpack
    monkeypatch.setenv("DCOL_RCCL_LIB", FAKE)
    results, refs, idx, cap, d = _run_ranks(world, mode)
    tail = np.uint64(0x7FF8000000000000) if mode == "pack" else np.uint64(0xFFFFFFFFFFFFFFFF)
    expected = np.concatenate([_expected_rows(refs[r], cap, tail) for r in range(world)])
    nsteps = 3
    for r in range(world):
        for j, buf in enumerate(results[r]):
            if j >= nsteps:
                continue
            np.testing.assert_array_equal(buf.view(np.uint64), expected.view(np.uint64),
                                          err_msg=f"rank {r} buffer {j} ({mode}, world {world})")
    # the whole batch from rank world-1's gathered records vs the reference's golden values
    allrec = results[world - 1][0].reshape(world, cap, -1)
    B = sum(len(i) for i in idx)
    full = np.empty((B, allrec.shape[2]))
    for r, ix in enumerate(idx):
        full[ix] = allrec[r, :len(ix)]
    u = unpack(full)
    np.testing.assert_array_equal(u["status"], d["status"][:B])
    ok = d["status"][:B] == 0
    np.testing.assert_array_equal(u["iters"][ok], d["iters"][:B][ok])
    assert np.all(alpha_close(u["alpha"][ok], d["alpha"][:B][ok]))
