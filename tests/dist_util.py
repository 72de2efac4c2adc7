"""Spawn ``world`` gloo ranks on 127.0.0.1 running ``fn(rank, world, *args)``; return
the per-rank results (reference test style: parallel_executor_test_base.py:29 --
same model, parallel vs single, compare)."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pack(x):
    import torch

    if torch.is_tensor(x):
        return ("__t__", x.detach().cpu().float().numpy() if x.dtype == torch.bfloat16 else x.detach().cpu().numpy())
    if isinstance(x, dict):
        return {k: _pack(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_pack(v) for v in x)
    return x


def _unpack(x):
    import torch

    if isinstance(x, tuple) and len(x) == 2 and isinstance(x[0], str) and x[0] == "__t__":
        return torch.from_numpy(x[1])
    if isinstance(x, dict):
        return {k: _unpack(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_unpack(v) for v in x)
    return x


def _entry(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    torch.set_num_threads(1)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        res = fn(rank, world, *args)
        q.put((rank, "ok", _pack(res)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        q.put((rank, "err", traceback.format_exc()))


def run_dist(fn, world, *args, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, st, res = q.get(timeout=timeout)
            if st != "ok":
                raise AssertionError(f"rank {r} failed:\n{res}")
            out[r] = _unpack(res)
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    return [out[r] for r in range(world)]


def assert_adam_close(got, want, atol, rtol, lr, steps, name="", max_frac=1e-4):
    """Parameters trained with Adam from the same init must agree elementwise, except
    that Adam divides by sqrt(v)+eps: a gradient that is ~0 in both runs but differs in
    fp32 summation order can move by up to ~lr per step.  Allow a tiny fraction of such
    elements (bounded by steps*lr); everything else must meet atol/rtol."""
    import torch

    got, want = got.float(), want.float()
    bad = (got - want).abs() > atol + rtol * want.abs()
    frac = bad.float().mean().item()
    worst = (got - want).abs().max().item()
    assert frac <= max_frac and worst <= 2 * steps * lr, (name, frac, worst)
