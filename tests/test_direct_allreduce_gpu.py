"""Direct (IPC / peer-mapped) all-reduce, parallel/direct.py + csrc/kernels/p2p.hip.

Two ranks on the one GPU of the test box (the IPC mapping, signal barriers and
reduce / gather kernels are the same code an 8-GPU node runs over xGMI); handles
are exchanged over a gloo group on 127.0.0.1.  Checked against the exact sum for
fp32 and bf16, one-shot and two-shot, odd chunking and repeated calls."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from paddle_amd.parallel.direct import DirectAllReduce

        ar = DirectAllReduce(max_bytes=8 << 20, one_shot_bytes=64 << 10, max_spins=1 << 24)
        res = []
        for dtype in (torch.float32, torch.bfloat16):
            for n in (8, 1000, 4096, 65544, 1 << 20):
                for algo in ("one_shot", "two_shot"):
                    g = torch.Generator().manual_seed(1000 * n + rank)
                    x = torch.randint(-8, 8, (n,), generator=g).to(dtype)  # exact in bf16 sums
                    t = x.cuda()
                    ar.all_reduce(t, algo=algo)
                    torch.cuda.synchronize()
                    ar.check()
                    exp = sum(torch.randint(-8, 8, (n,), generator=torch.Generator().manual_seed(1000 * n + r))
                              .to(torch.float32) for r in range(world))
                    res.append((str(dtype), n, algo, float((t.float().cpu() - exp).abs().max())))
        # a raised barrier-error flag (what a timed-out peer leaves behind) poisons
        # the result with NaN instead of summing stale staging data, and check() raises
        ar._err.fill_(1)
        t = torch.ones(4096, device="cuda")
        ar.all_reduce(t, algo="two_shot")
        torch.cuda.synchronize()
        poisoned = bool(torch.isnan(t).all())
        try:
            ar.check()
            raised = False
        except Exception:
            raised = True
        res.append(("poison", int(poisoned), "raised", 0.0 if raised else 1.0))
        ar.close()
        dist.destroy_process_group()
        q.put((rank, res, None))
    except Exception as e:  # report to the parent instead of hanging it
        q.put((rank, None, repr(e)))


def test_direct_allreduce_two_ranks_one_gpu():
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=240)
            assert err is None, f"rank {rank}: {err}"
            out[rank] = res
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank in range(world):
        for dtype, n, algo, err in out[rank]:
            assert err == 0.0, (rank, dtype, n, algo, err)
            if dtype == "poison":
                assert n == 1, f"rank {rank}: output not NaN-poisoned after a barrier error"
