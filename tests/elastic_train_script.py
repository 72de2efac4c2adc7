"""Training script driven by tests/test_elastic_cpu.py through the launcher:
2 gloo ranks, data-parallel SGD on a tiny regression, checkpoint every 2 steps,
fault injection + watchdog, resume from the newest complete checkpoint."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.distributed.elastic import CheckpointManager, Watchdog, maybe_inject_fault  # noqa: E402
from paddle_amd.parallel import comm  # noqa: E402


def main():
    root, out, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    wd_timeout = float(os.environ.get("TEST_WATCHDOG_S", "60"))
    rank, world = comm.init_parallel_env("gloo")
    torch.manual_seed(0)
    w = torch.zeros(4, 1)
    mgr = CheckpointManager(root, max_num_checkpoints=2)
    start = 0
    serial, state = mgr.load()
    if serial is not None:
        w = state["model"]["w"].clone()
        start = serial + 1
    dog = Watchdog(wd_timeout, name=f"rank{rank}")
    for step in range(start, steps):
        maybe_inject_fault(step, rank)
        g = torch.Generator().manual_seed(1000 * step + rank)
        x = torch.randn(8, 4, generator=g)
        y = x @ torch.tensor([[1.0], [-2.0], [0.5], [3.0]])
        grad = 2 * x.t() @ (x @ w - y) / x.shape[0]
        dist.all_reduce(grad)
        w -= 0.05 * grad / world
        if step % 2 == 1:
            mgr.save(step, {"model": {"w": w}}, rank=rank)
            dist.barrier()
        dog.beat(step)
    dog.stop()
    if rank == 0:
        torch.save(w, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
