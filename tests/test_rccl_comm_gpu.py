"""Framework-owned RCCL communicators (csrc/runtime/rccl_comm.cc, parallel/rccl.py):
unique-id rendezvous through a TCP store, collectives on the current HIP stream,
the group guard.  One GPU per box: a one-rank clique (the collectives' data path
and error handling run; multi-rank runs are covered by the 8-GPU driver jobs)."""
import datetime

import pytest
import torch
import torch.distributed as dist

from paddle_amd.parallel import rccl

pytestmark = pytest.mark.gpu


def test_one_rank_clique_collectives():
    assert rccl.available()
    assert rccl.enabled()  # FLAGS_comm_backend=auto: the framework layer is the GPU default
    store = dist.TCPStore("127.0.0.1", 0, 1, True, timeout=datetime.timedelta(seconds=30))
    c = rccl.Communicator.rendezvous(store, "pa_rccl/test/0", 1, 0, torch.cuda.current_device())
    x = torch.arange(1000, device="cuda", dtype=torch.float32)
    ref = x.clone()
    c.all_reduce(x)
    torch.testing.assert_close(x, ref)
    out = torch.empty(1000, device="cuda", dtype=torch.bfloat16)
    c.all_gather(out, ref.to(torch.bfloat16))
    torch.testing.assert_close(out.float(), ref.to(torch.bfloat16).float())
    rs = torch.empty(1000, device="cuda")
    c.reduce_scatter(rs, ref)
    torch.testing.assert_close(rs, ref)
    with rccl.group_guard():
        c.all_reduce(x)
        c.broadcast(out, root=0)
    # expert-parallel all-to-all (grouped ncclSend/ncclRecv) and a self send/recv round
    rows = torch.randn(7, 16, device="cuda", dtype=torch.bfloat16)
    got = torch.empty_like(rows)
    c.all_to_all(got, rows, out_splits=[7], in_splits=[7])
    with rccl.group_guard():
        back = torch.empty(5, device="cuda", dtype=torch.int64)
        c.send(torch.arange(5, device="cuda"), 0)
        c.recv(back, 0)
    torch.cuda.synchronize()
    assert torch.equal(got, rows)
    assert torch.equal(back, torch.arange(5, device="cuda"))
    c.check_async()
    with pytest.raises(rccl.RcclError):
        c.all_reduce(x.cpu())
    c.destroy()
