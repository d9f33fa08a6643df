"""One rank of the deadline test (tests/test_dist.py::test_deadline_*): gloo on the CPU, a
few all-gather steps under dcol_amd.dist.StepWatchdog, the way bench.py's N > 1 path arms
it.  Rank 1 misbehaves per argv[1]:
  skip  -- skips step 2 and then stalls (a rank stuck outside the collective);
  none  -- every rank takes every step (the run must end cleanly, exit 0).
Launched by torch.distributed.run (127.0.0.1 rendezvous)."""
import datetime
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "dcol-trajectory-optimization_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from dcol_amd.dist import StepWatchdog  # noqa: E402


def main():
    mode, steps, deadline = sys.argv[1], 5, float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    wd = StepWatchdog(rank, world, deadline)
    with wd.guard("init_process_group"):
        # the backend's own timeout well past the deadline: the watchdog must be what ends it
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=10 * deadline + 60))
    for k in range(steps):
        if mode == "skip" and rank == 1 and k == 2:
            # (its own deadline longer: the rank waiting in the collective must fire first)
            with wd.guard("stalled (test: rank 1 skipped step 2)", k, seconds=5 * deadline):
                time.sleep(20 * deadline)
        src = torch.full((4,), float(rank * 100 + k), dtype=torch.float64)
        out = torch.empty(4 * world, dtype=torch.float64)
        with wd.guard("all-gather", k):
            dist.all_gather_into_tensor(out, src)
        assert out.view(world, 4)[:, 0].tolist() == [r * 100.0 + k for r in range(world)]
    with wd.guard("barrier"):
        dist.barrier()
    dist.destroy_process_group()
    wd.close()
    print(f"rank {rank}: {steps} steps done", flush=True)


if __name__ == "__main__":
    main()
