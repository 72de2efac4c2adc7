#!/usr/bin/env python3
"""Flagship benchmark: LLaMA-7B pre-training step, Fleet-style hybrid parallel.

Metric (BASELINE.json): "tokens/sec (whole node) LLaMA-7B Fleet hybrid-parallel at
1/2/4/8 MI355X".  One process per GPU; for N>1 the driver launches this file with
torch.distributed.run (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in the env).

Per GPU work is fixed (weak scaling): micro_batch x seq_len tokens x accum per step.
Parallelism: data parallel over all ranks with sharding stage-1 (ZeRO-1: fp32 master
weights + Adam moments sharded, bucketed reduce-scatter overlapped with backward,
all-gather of bf16 params) -- Paddle fleet `dp_degree=N, sharding stage 1`.
The timed region contains the full step: forward, backward, gradient
reduce-scatter, fused AdamW on the shard, parameter all-gather.
Data: synthetic random token ids; weights: random init (no network here).

``--gpus N`` outside a launcher (no WORLD_SIZE in the env) makes this process a
pure parent: it never touches the GPU, starts ``torch.distributed.run`` with N
ranks on 127.0.0.1 as a CHILD process and exits with its code.  Every rank
asserts WORLD_SIZE == --gpus, so a scaling point can never silently be a 1-GPU
number.  ``--device cpu`` (gloo) is the debug mode the CPU tests use.
Gradients are accumulated and reduce-scattered in fp32 (Fleet ``main_grad``);
``--bf16-grads`` restores the round-1 bf16 gradient buffer.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "tokens/sec (whole node) LLaMA-7B Fleet hybrid-parallel at 1/2/4/8 MI355X"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _self_launch(args, argv) -> int:
    """Parent of an N-rank run: no GPU call happens in this process (it does not
    even import torch); the ranks are a child ``torch.distributed.run``."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(args.master_port or _free_port()),
           os.path.abspath(__file__)] + argv
    log(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="llama-7b")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--micro-batch", type=int, default=8)
    ap.add_argument("--accum", type=int, default=2,
                    help="gradient accumulation micro-steps per optimizer step (Fleet accumulate_steps)")
    ap.add_argument("--layers", type=int, default=None, help="debug only: override layer count (result INVALID)")
    ap.add_argument("--recompute", action="store_true")
    ap.add_argument("--bucket-mb", type=int, default=256)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--tuned-gemm", action="store_true",
                    help="also replay stored hipBLASLt solutions for any library GEMM left in the step "
                         "(the LLaMA projections run on the hand-written gemm.hip either way)")
    ap.add_argument("--bf16-grads", action="store_true",
                    help="accumulate / reduce-scatter gradients in bf16 instead of fp32 main_grad")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = gloo debug mode for tests (tiny models only)")
    ap.add_argument("--master-port", type=int, default=0)
    ap.add_argument("--autograd", default="tape", choices=["tape", "torch"],
                    help="tape: the framework's own reverse pass (torch autograd off); torch: torch.autograd")
    ap.add_argument("--dtype", default=None, choices=["bfloat16", "float32"],
                    help="debug only (CPU tests): override the model dtype; GPU results must stay bf16")
    argv = sys.argv[1:]
    args = ap.parse_args(argv)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(args, argv))

    import torch

    from paddle_amd.autograd import tape
    from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM, llama_flops_per_token
    from paddle_amd.parallel import comm
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    rank, world, local = comm.env_rank_world()
    if world != args.gpus:
        raise SystemExit(f"[bench] rank {rank}: WORLD_SIZE={world} but --gpus {args.gpus}")
    cuda = args.device == "cuda"
    if world > 1:
        # GPU: every device collective on the framework's own RCCL communicators; the c10d
        # default group is gloo (store + host barriers only), so no ProcessGroupNCCL
        # communicators exist and a communicator that cannot be built fails the run
        comm.init_parallel_env("pa_rccl" if cuda else "gloo")
        log(f"[bench] {comm.backend_name()} world={world} rank={rank} local={local}")
    if cuda:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    sync = torch.cuda.synchronize if cuda else (lambda *a: None)
    torch.manual_seed(1234)  # identical init on every rank (DP replicas)
    tuned = False
    if cuda and args.tuned_gemm:
        from paddle_amd.utils import gemm_tuning

        tuned = gemm_tuning.enable(args.model, verbose=rank == 0)

    cfgd = dict(LLAMA_CONFIGS[args.model])
    if args.layers:
        cfgd["num_hidden_layers"] = args.layers
    cfgd["max_position_embeddings"] = max(args.seq_len, cfgd.get("max_position_embeddings", 2048))
    if args.dtype:
        cfgd["dtype"] = args.dtype
    cfg = LlamaConfig(**cfgd, recompute=args.recompute)
    t0 = time.time()
    model = LlamaForCausalLM(cfg, device=dev)
    model.train()
    opt = FlatShardedOptimizer(model.named_parameters(), lr=3e-4, betas=(0.9, 0.95), eps=1e-8,
                               weight_decay=0.1, grad_clip=1.0, bucket_mb=args.bucket_mb,
                               overlap=not args.no_overlap, overlap_allgather=not args.no_overlap,
                               overlap_update=cuda and not args.no_overlap,
                               grad_dtype=None if args.bf16_grads else torch.float32)
    nparams = sum(p.numel() for p in model.parameters())
    from paddle_amd import platform as _plat

    mem = (lambda: _plat.memory_allocated(local) / 2**30) if cuda else (lambda: 0.0)
    peak = (lambda: _plat.max_memory_allocated(local) / 2**30) if cuda else (lambda: 0.0)
    if cuda and os.environ.get("FLAGS_allocator_strategy") == "buddy":
        # torch's pluggable-allocator hook keeps no statistics: ask the buddy allocator
        from paddle_amd import runtime as _rt

        mem = lambda: _rt.torch_allocator_stats(dev.index)["used"] / 2**30  # noqa: E731
        peak = lambda: _rt.torch_allocator_stats(dev.index)["peak"] / 2**30  # noqa: E731
    if rank == 0:
        log(f"[bench] model {args.model} params={nparams/1e9:.3f}B layers={cfg.num_hidden_layers} "
            f"world={world} grads={opt.grad_dtype} build {time.time()-t0:.1f}s mem={mem():.1f}GiB")

    mb, S = args.micro_batch, args.seq_len
    # one global synthetic batch pool; rank r trains on rows [r*mb, (r+1)*mb) of every
    # micro-batch, so an N-rank run sees exactly the data of a 1-rank run at N x batch
    gen = torch.Generator().manual_seed(42)
    pool = [torch.randint(0, cfg.vocab_size, (world * mb, S + 1), generator=gen)[rank * mb:(rank + 1) * mb]
            .to(dev) for _ in range(4)]

    # recompute runs on the tape too (tape.checkpoint: the segment's forward is replayed
    # inside the reverse pass)
    use_tape = args.autograd == "tape"

    def micro(x, y):
        if use_tape:
            # forward recorded on the framework tape with torch autograd disabled; the
            # 1/accum loss scale is the seed gradient of the reverse pass
            with tape.recording() as t:
                loss = model(x, y)
            t.backward(loss, torch.full_like(loss, 1.0 / args.accum))
            return loss / args.accum
        loss = model(x, y) / args.accum
        loss.backward()
        return loss

    def train_step(i):
        for a in range(args.accum):
            batch = pool[(i * args.accum + a) % len(pool)]
            x, y = batch[:, :-1], batch[:, 1:]
            if a < args.accum - 1:
                with opt.no_sync():
                    loss = micro(x, y)
            else:
                loss = micro(x, y)
        opt.step()
        opt.zero_grad()
        return loss

    for i in range(args.warmup):
        l = train_step(i)
        sync()
        if rank == 0:
            log(f"[bench] warmup {i} loss={l.item()*args.accum:.4f} mem_peak={peak():.1f}GiB")
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        l = train_step(args.warmup + i)
        if rank == 0 and (i % 2 == 0 or i == args.steps - 1):
            log(f"[bench] step {i} issued")
    comm.barrier()
    sync()
    el = time.perf_counter() - t0
    elt = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        comm.all_reduce(elt, op=torch.distributed.ReduceOp.MAX)
    el = float(elt.item())
    lt = (l.detach().float() * args.accum).reshape(1).contiguous()
    if world > 1:
        comm.all_reduce(lt)
    final_loss = float(lt.item()) / world
    tokens_per_step = world * args.accum * mb * S
    tps = tokens_per_step * args.steps / el
    ms = el / args.steps * 1000
    fpt = llama_flops_per_token(cfg, S)
    mfu = tps / world * fpt / 2.5e15
    if rank == 0:
        log(f"[bench] final loss={final_loss:.4f} tokens/s={tps:.0f} per-gpu={tps/world:.0f} "
            f"ms/step={ms:.1f} MFU(2.5PF bf16 dense)={mfu*100:.1f}% peak_mem={peak():.1f}GiB")
        invalid = args.layers is not None
        out = {
            "metric": METRIC,
            "value": round(tps, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if cfg.dtype in ("bfloat16", "bf16") else str(cfg.dtype),
            "data": "synthetic random token ids, random-init weights",
            "config": {
                "model": args.model + (f"(DEBUG {args.layers} layers: INVALID)" if invalid else ""),
                "global_batch": world * args.accum * mb,
                "seq_len": S,
                "micro_batch": mb,
                "grad_accum": args.accum,
                "parallelism": f"dp{world}+sharding_stage1",
                "params_b": round(nparams / 1e9, 3),
                "mfu_bf16_dense": round(mfu, 4),
                "recompute": bool(args.recompute),
                "gemm": "gemm.hip (hand-written bf16 MFMA)",
                "hipblaslt_tuning_replay": tuned,
                "grad_dtype": str(opt.grad_dtype).replace("torch.", ""),
                "autograd": "tape" if use_tape else "torch",
                "device": args.device,
                "comm_backend": comm.backend_name(),
                "bucket_mb": args.bucket_mb,
                "dp_comm": opt.dp_comm if world > 1 else None,
            },
            "final_loss": round(final_loss, 5),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
