"""ZeRO-1 training over the direct xGMI collectives (FLAGS_dp_comm=direct:
parallel/direct.py reduce-scatter / all-gather on IPC-mapped peer buffers) against
the process-group path, two ranks on the one GPU of the test box (the same IPC
mapping, signal barriers and kernels an 8-GPU node runs over xGMI).  LLaMA-tiny on
the framework tape, fp32 main grads, bucketed + overlapped comm, 3 steps: same
losses / parameters up to the run-to-run float-atomic noise of the model's own
kernels; the collectives themselves are checked bitwise against the process group
on random data (a two-rank sum is order-free).
Reference counterpart: details/all_reduce_op_handle.cc:48-108 over
platform/nccl_helper.h:49-123 (NCCL only)."""
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


def _train(dp_comm, rank, steps=3, inplace=False):
    from paddle_amd.autograd import tape
    from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    torch.manual_seed(0)
    cfg = LlamaConfig(**LLAMA_CONFIGS["llama-tiny"])
    model = LlamaForCausalLM(cfg, device="cuda")
    os.environ["FLAGS_dp_direct_inplace"] = "1" if inplace else "0"
    try:
        opt = FlatShardedOptimizer(model.named_parameters(), lr=1e-3, weight_decay=0.1, grad_clip=1.0,
                                   grad_dtype=torch.float32, bucket_mb=1, overlap=True, overlap_allgather=True,
                                   dp_comm=dp_comm)
    finally:
        os.environ.pop("FLAGS_dp_direct_inplace", None)
    assert (opt._direct is not None) == (dp_comm == "direct")
    if inplace:
        # the flat gradient is the registered staging region: reduce-scatters skip the copy-in
        assert opt._direct._in_place(opt.flat_grad) is not None
    ids = torch.randint(0, cfg.vocab_size, (2, 129), generator=torch.Generator().manual_seed(10 + rank)).cuda()
    losses = []
    for _ in range(steps):
        with tape.recording() as t:
            loss = model(ids[:, :-1], ids[:, 1:])
        t.backward(loss)
        opt.step()
        opt.zero_grad()
        losses.append(float(loss))
    opt.sync_params()
    torch.cuda.synchronize()
    if opt._direct is not None:
        opt._direct.poll_error()
        opt._direct.check()
    return losses, opt.flat_param.float().cpu(), len(opt.buckets)


def _collectives_exact(rank, world):
    import torch.distributed as dist

    from paddle_amd.parallel import comm
    from paddle_amd.parallel.direct import DirectAllReduce

    d = DirectAllReduce(max_bytes=64 << 20)
    worst = 0.0
    for n in (2048, 1 << 20, 3 << 20):
        g = torch.Generator().manual_seed(7 * n + rank)
        x = torch.randn(n, generator=g).cuda()
        a, b = torch.empty(n // world, device="cuda"), torch.empty(n // world, device="cuda")
        d.reduce_scatter(a, x)
        comm.reduce_scatter(b, x.clone())
        worst = max(worst, float((a - b).abs().max()))
        sh = torch.randn(n // world, generator=g).to(torch.bfloat16).cuda()
        o1, o2 = torch.empty(n, dtype=torch.bfloat16, device="cuda"), torch.empty(n, dtype=torch.bfloat16, device="cuda")
        d.all_gather(o1, sh)
        comm.all_gather(o2, sh)
        worst = max(worst, float((o1.float() - o2.float()).abs().max()))
    torch.cuda.synchronize()
    d.check()
    d.close()
    dist.barrier()
    return worst


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import paddle_amd  # noqa: F401  (installs the default allocator before the first device use)

        torch.cuda.set_device(0)
        exact = _collectives_exact(rank, world)
        l_pg, p_pg, nb = _train("rccl", rank)
        l_dr, p_dr, _ = _train("direct", rank)
        l_ip, p_ip, _ = _train("direct", rank, inplace=True)
        dist.destroy_process_group()
        q.put((rank, (exact, l_pg, l_dr, float((p_pg - p_dr).abs().max()), nb, l_ip,
                      float((p_pg - p_ip).abs().max())), None))
    except Exception as e:  # report to the parent instead of hanging it
        import traceback

        q.put((rank, None, traceback.format_exc()[-2000:] + repr(e)))


def test_zero1_direct_comm_matches_process_group_two_ranks_one_gpu():
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=300)
            assert err is None, f"rank {rank}: {err}"
            out[rank] = res
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank in range(world):
        exact, l_pg, l_dr, pdiff, nb, l_ip, pdiff_ip = out[rank]
        assert exact == 0.0, (rank, exact)
        assert nb > 1, "the test must exercise several buckets"
        assert l_pg[0] == l_dr[0], (rank, l_pg, l_dr)
        for a, b in zip(l_pg, l_dr):
            assert abs(a - b) <= 1e-4 * abs(a), (rank, l_pg, l_dr)
        assert pdiff < 2e-2, (rank, pdiff)
        # in-place staging (FLAGS_dp_direct_inplace): the same training
        assert l_pg[0] == l_ip[0], (rank, l_pg, l_ip)
        for a, b in zip(l_pg, l_ip):
            assert abs(a - b) <= 1e-4 * abs(a), (rank, l_pg, l_ip)
        assert pdiff_ip < 2e-2, (rank, pdiff_ip)
        assert l_pg[-1] < l_pg[0]
