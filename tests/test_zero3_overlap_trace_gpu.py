"""ZeRO-3 communication overlap in TIME: two ranks share the
GPU of the test box, ShardedStage3 runs its unit all-gathers / reduce-scatters on
the direct collectives (parallel/direct.py kernels on the comm stream), and the
in-process rocprofiler-sdk tracer (utils/device_tracer.py) records one training
step.  The prefetched all-gather kernels must run on another hardware queue than
the GEMMs and overlap them in time, and the reduce-scatters of finished units must
overlap the backward GEMMs of the next ones.
Reference counterpart: the per-device streams + events of
framework/details/op_handle_base.cc:42-110 (there only NCCL all-reduce overlaps)."""
import json
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


def _overlap_ns(a, bs):
    """Total time interval a spends overlapping any interval of bs."""
    s, e = a
    tot = 0
    for bs_, be in bs:
        lo, hi = max(s, bs_), min(e, be)
        if hi > lo:
            tot += hi - lo
    return tot


def _worker(rank, world, port, q):
    import sys

    os.environ["FLAGS_device_tracer"] = "1"
    sys.path.insert(0, ROOT)
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import paddle_amd  # noqa: F401
        from paddle_amd.autograd import tape
        from paddle_amd.distributed.sharding import ShardedStage3
        from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM
        from paddle_amd.utils import device_tracer as dt
        from paddle_amd.utils import profiler as P

        torch.cuda.set_device(0)
        assert dt.available(), dt.error()
        torch.manual_seed(0)
        cfg = LlamaConfig(**dict(LLAMA_CONFIGS["llama-tiny"], hidden_size=1024, intermediate_size=2816,
                                 num_attention_heads=8, num_key_value_heads=8, num_hidden_layers=8,
                                 max_position_embeddings=1024))
        model = LlamaForCausalLM(cfg, device="cuda")
        opt = ShardedStage3(model, lr=1e-4, grad_clip=1.0, dp_comm="direct", prefetch=True)
        assert opt._direct is not None
        ids = torch.randint(0, cfg.vocab_size, (4, 513), generator=torch.Generator().manual_seed(rank)).cuda()

        def step():
            with tape.recording() as t:
                loss = model(ids[:, :-1], ids[:, 1:])
            t.backward(loss)
            opt.step()
            opt.zero_grad()
            return loss

        for _ in range(2):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        P.start("All")
        loss = step()
        torch.cuda.synchronize()
        recs = P.kernel_records()
        P.stop(profile_path=None)
        opt._direct.check()
        dist.barrier()
        dist.destroy_process_group()
        gathers = [(r["start_ns"], r["end_ns"], r["queue"]) for r in recs if "p2p_gather" in r["name"]]
        reduces = [(r["start_ns"], r["end_ns"], r["queue"]) for r in recs if "p2p_reduce" in r["name"]]
        # compute: every kernel of the compute queue that is not a collective / copy
        gemms = [(r["start_ns"], r["end_ns"], r["queue"]) for r in recs
                 if "p2p_" not in r["name"] and ("gemm" in r["name"] or "fa_" in r["name"] or "norm" in r["name"])]
        gi = [(a, b) for a, b, _ in gemms]
        res = {
            "rank": rank, "loss": float(loss), "kernels": len(recs),
            "gathers": len(gathers), "reduce_scatters": len(reduces), "gemms": len(gemms),
            "gather_queues": sorted({qq for _, _, qq in gathers}), "gemm_queues": sorted({qq for _, _, qq in gemms}),
            "gathers_overlapping_gemm": sum(1 for a, b, _ in gathers if _overlap_ns((a, b), gi) > 0),
            "reduces_overlapping_gemm": sum(1 for a, b, _ in reduces if _overlap_ns((a, b), gi) > 0),
            "gather_ns": sum(b - a for a, b, _ in gathers),
            "gather_ns_under_gemm": sum(_overlap_ns((a, b), gi) for a, b, _ in gathers),
            "reduce_ns": sum(b - a for a, b, _ in reduces),
            "reduce_ns_under_gemm": sum(_overlap_ns((a, b), gi) for a, b, _ in reduces),
        }
        q.put((rank, res, None))
    except Exception as e:  # report to the parent instead of hanging it
        import traceback

        q.put((rank, None, traceback.format_exc()[-2000:] + repr(e)))


def test_zero3_allgather_and_reduce_scatter_overlap_compute_in_time():
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=240)
            assert err is None, err
            out[rank] = res
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    if os.environ.get("PA_TRACE_OUT"):
        with open(os.environ["PA_TRACE_OUT"], "w") as f:
            json.dump(out, f, indent=1)
    for rank, r in out.items():
        assert r["gathers"] >= 4 and r["reduce_scatters"] >= 4 and r["gemms"] > 0, r
        # the comm stream is its own hardware queue
        assert not set(r["gather_queues"]) & set(r["gemm_queues"]), r
        # prefetched all-gathers / reduce-scatters run while compute kernels run
        assert r["gathers_overlapping_gemm"] >= 2 and r["gather_ns_under_gemm"] > 0, r
        assert r["reduces_overlapping_gemm"] >= 1 and r["reduce_ns_under_gemm"] > 0, r
