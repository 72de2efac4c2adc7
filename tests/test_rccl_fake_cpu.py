"""The framework RCCL layer with 4 ranks on the CPU.

``tests/native/fake_rccl.cc`` implements the NCCL C ABI that
``csrc/runtime/rccl_comm.cc`` dlopens (``PA_RCCL_LIBRARY``) over shared memory, so
the SAME Python and C++ code that drives librccl on the GPU -- ``parallel/comm.py``
routing, ``parallel/rccl.py`` rendezvous through the job's TCP store
(``CommContextMap``, the gen_nccl_id role), the group guard, the grouped
send/recv all-to-all, the async-error abort path -- runs here with host buffers.
Reference: platform/nccl_helper.h:49-123, operators/gen_nccl_id_op.cc:54-110."""
import ctypes
import os
import subprocess

import pytest
import torch

from dist_util import run_dist

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def fake_lib(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("fake_rccl") / "libfake_rccl.so")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-o", out,
                           os.path.join(HERE, "native", "fake_rccl.cc"), "-lrt", "-pthread"])
    return out


def _setup(lib):
    os.environ["PA_RCCL_LIBRARY"] = lib
    os.environ["FLAGS_comm_backend"] = "pa_rccl"
    from paddle_amd.parallel import comm, rccl

    comm._HOST_RCCL.append(True)
    return comm, rccl


def _log(lib):
    fake = ctypes.CDLL(lib)
    buf = ctypes.create_string_buffer(1 << 16)
    fake.fake_rccl_log(buf, len(buf))
    return buf.value.decode().splitlines()


def _collectives_worker(rank, world, lib):
    comm, rccl = _setup(lib)
    res = {}
    x = torch.full((6,), float(rank + 1))
    comm.all_reduce(x)
    res["all_reduce"] = x
    m = torch.tensor([float(rank), -float(rank)])
    comm.all_reduce(m, op=torch.distributed.ReduceOp.MAX)
    res["all_reduce_max"] = m
    inp = torch.arange(world * 3, dtype=torch.float32) + 100 * rank
    out = torch.empty(3)
    comm.reduce_scatter(out, inp)
    res["reduce_scatter"] = out
    g = torch.empty(world * 2, dtype=torch.bfloat16)
    comm.all_gather(g, torch.tensor([rank, rank + 0.5], dtype=torch.bfloat16))
    res["all_gather"] = g.float()
    b = torch.full((4,), float(rank), dtype=torch.float64)
    comm.broadcast(b, src=2)
    res["broadcast"] = b
    # all-to-all with uneven splits: rank r sends (p + 1) rows of value 10 r + p to peer p
    ins = [p + 1 for p in range(world)]
    rows = torch.cat([torch.full((p + 1, 2), float(10 * rank + p)) for p in range(world)])
    outs = [rank + 1] * world
    a2a = torch.empty(sum(outs), 2)
    comm.all_to_all(a2a, rows, out_splits=outs, in_splits=ins)
    res["all_to_all"] = a2a
    # one fused point-to-point round around the ring (the pipeline / ring-attention path)
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    got = torch.empty(5, dtype=torch.int64)
    comm.batch_p2p([("send", torch.arange(5) + 1000 * rank, nxt), ("recv", got, prv)])
    res["p2p"] = got
    # group guard: queued inside, executed at ncclGroupEnd in issue order
    c = rccl.context_map().get(list(range(world)), rank, device=-1)
    n0 = len(_log(lib))
    y = torch.ones(3)
    with rccl.group_guard():
        c.all_reduce(y)
        c.broadcast(y, root=0)
        inside = _log(lib)[n0:]
    res["group_inside"] = inside
    res["group_after"] = _log(lib)[n0 + len(inside):]
    res["group_value"] = y
    return res


def test_four_rank_collectives_through_framework_rccl(fake_lib):
    W = 4
    for r, res in enumerate(run_dist(_collectives_worker, W, fake_lib)):
        assert torch.equal(res["all_reduce"], torch.full((6,), 10.0))
        assert torch.equal(res["all_reduce_max"], torch.tensor([3.0, 0.0]))
        full = sum(torch.arange(W * 3, dtype=torch.float32) + 100 * q for q in range(W))
        assert torch.equal(res["reduce_scatter"], full[3 * r:3 * r + 3])
        assert torch.equal(res["all_gather"], torch.tensor([q + h for q in range(W) for h in (0.0, 0.5)]))
        assert torch.equal(res["broadcast"], torch.full((4,), 2.0, dtype=torch.float64))
        want = torch.cat([torch.full((r + 1, 2), float(10 * p + r)) for p in range(W)])
        assert torch.equal(res["all_to_all"], want)
        assert torch.equal(res["p2p"], torch.arange(5) + 1000 * ((r - 1) % W))
        # inside the guard the collectives were only enqueued; GroupEnd ran them in order
        assert res["group_inside"] == ["enqueue all_reduce", "enqueue broadcast"]
        assert res["group_after"] == ["exec all_reduce", "exec broadcast"]
        assert torch.equal(res["group_value"], torch.full((3,), 4.0))


def _abort_worker(rank, world, lib):
    comm, rccl = _setup(lib)
    x = torch.ones(2)
    comm.all_reduce(x)  # creates the world communicator
    cmap = rccl.context_map()
    c = cmap.get(list(range(world)), rank, device=-1)
    handle = c._h.value
    cmap.check_health()  # healthy: no error
    torch.distributed.barrier()
    if rank == 1:  # a peer reports a failure (ncclRemoteError on every rank's comm)
        ctypes.CDLL(lib).fake_rccl_inject_async_error(ctypes.c_void_p(handle), 6)
    torch.distributed.barrier()
    try:
        cmap.check_health()
        raised = False
    except rccl.RcclError:
        raised = True
    aborted = ctypes.CDLL(lib).fake_rccl_aborted(ctypes.c_void_p(handle))
    return raised, aborted, len(cmap._comms), "abort" in " ".join(_log(lib))


def test_async_error_aborts_every_communicator(fake_lib):
    for raised, aborted, left, logged in run_dist(_abort_worker, 4, fake_lib):
        assert raised and aborted == 1 and left == 0 and logged


def test_rendezvous_and_enabled_flag(fake_lib, monkeypatch):
    from paddle_amd.parallel import rccl

    monkeypatch.setenv("FLAGS_comm_backend", "torch")
    assert not rccl.enabled()
    monkeypatch.setenv("FLAGS_comm_backend", "pa_rccl")
    assert rccl.enabled()
    # auto (the default) follows whether librccl and a GPU are there
    monkeypatch.setenv("FLAGS_comm_backend", "auto")
    rccl._AUTO.clear()
    assert rccl.enabled() == (torch.cuda.is_available() and rccl.available())


def _watchdog_worker(rank, world, lib):
    import threading

    comm, rccl = _setup(lib)
    from paddle_amd.distributed.elastic import Watchdog

    x = torch.ones(2)
    comm.all_reduce(x)
    c = rccl.context_map().get(list(range(world)), rank, device=-1)
    fired = threading.Event()
    wd = Watchdog(timeout_s=1e9, poll_s=0.05, on_timeout=lambda step: fired.set())
    torch.distributed.barrier()
    if rank == 0:
        ctypes.CDLL(lib).fake_rccl_inject_async_error(ctypes.c_void_p(c._h.value), 6)
    ok = fired.wait(20)
    wd.stop()
    return ok, len(rccl.context_map()._comms)


def test_watchdog_exits_on_peer_failure(fake_lib):
    for ok, left in run_dist(_watchdog_worker, 2, fake_lib):
        assert ok and left == 0


def _zero_row_worker(rank, world, lib):
    """an expert-parallel rank with no routed tokens sends zero rows."""
    comm, _ = _setup(lib)
    # rank 0 sends nothing to anyone; every other rank sends one row to each peer
    ins = [0 if rank == 0 else 1] * world
    inp = torch.full((sum(ins), 3), float(rank))
    outs = [0 if p == 0 else 1 for p in range(world)]
    out = torch.empty(sum(outs), 3)
    comm.all_to_all(out, inp, out_splits=outs, in_splits=ins)
    empty = torch.empty(0, 3)
    comm.all_to_all(torch.empty(0, 3), empty, out_splits=[0] * world, in_splits=[0] * world)
    return out


def test_all_to_all_with_zero_rows(fake_lib):
    W = 3
    for r, out in enumerate(run_dist(_zero_row_worker, W, fake_lib)):
        assert torch.equal(out, torch.cat([torch.full((1, 3), float(p)) for p in range(1, W)]))


def _agree_worker(rank, world, lib, mode):
    """One rank cannot build its communicator: the go / no-go verdict is agreed through
    the store, so EVERY rank takes the same branch -- all fall back to torch.distributed
    under ``auto``, all raise under ``pa_rccl`` -- and nobody hangs in the init."""
    import warnings

    comm, rccl = _setup(lib)
    os.environ["FLAGS_comm_backend"] = mode
    rccl._AUTO[:] = [True]
    if rank == 1:
        rccl._local_ready = lambda dev: False
    x = torch.full((4,), float(rank + 1))
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            comm.all_reduce(x)
        outcome = "ok"
    except rccl.RcclUnavailable:
        outcome = "raised"
    return outcome, x, len(rccl.context_map()._comms), bool(rccl._AUTO and rccl._AUTO[0])


def test_unavailable_rank_gives_one_verdict_for_all(fake_lib):
    W = 3
    for outcome, x, ncomm, auto_on in run_dist(_agree_worker, W, fake_lib, "auto"):
        # every rank fell back together: the sum ran on gloo, no communicator was built
        assert outcome == "ok" and ncomm == 0 and not auto_on
        assert torch.equal(x, torch.full((4,), float(sum(range(1, W + 1)))))
    for outcome, _, ncomm, _ in run_dist(_agree_worker, W, fake_lib, "pa_rccl"):
        assert outcome == "raised" and ncomm == 0
