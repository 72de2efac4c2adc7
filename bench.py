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
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "tokens/sec (whole node) LLaMA-7B Fleet hybrid-parallel at 1/2/4/8 MI355X"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


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
    ap.add_argument("--no-tuned-gemm", action="store_true",
                    help="use hipBLASLt's heuristic GEMM pick instead of the stored tuned solutions")
    args = ap.parse_args()

    from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM, llama_flops_per_token
    from paddle_amd.parallel import comm
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    rank, world, local = comm.env_rank_world()
    if world > 1:
        comm.init_parallel_env("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.manual_seed(1234 + rank)
    tuned = False
    if not args.no_tuned_gemm:
        from paddle_amd.utils import gemm_tuning

        tuned = gemm_tuning.enable(args.model, verbose=rank == 0)

    cfgd = dict(LLAMA_CONFIGS[args.model])
    if args.layers:
        cfgd["num_hidden_layers"] = args.layers
    cfgd["max_position_embeddings"] = max(args.seq_len, cfgd.get("max_position_embeddings", 2048))
    cfg = LlamaConfig(**cfgd, recompute=args.recompute)
    t0 = time.time()
    model = LlamaForCausalLM(cfg, device=dev)
    model.train()
    opt = FlatShardedOptimizer(model.named_parameters(), lr=3e-4, betas=(0.9, 0.95), eps=1e-8,
                               weight_decay=0.1, grad_clip=1.0, bucket_mb=args.bucket_mb,
                               overlap=not args.no_overlap, overlap_allgather=not args.no_overlap)
    nparams = sum(p.numel() for p in model.parameters())
    if rank == 0:
        log(f"[bench] model {args.model} params={nparams/1e9:.3f}B layers={cfg.num_hidden_layers} "
            f"world={world} build {time.time()-t0:.1f}s mem={torch.cuda.memory_allocated(dev)/2**30:.1f}GiB")

    mb, S = args.micro_batch, args.seq_len
    gen = torch.Generator(device=dev)
    gen.manual_seed(42 + rank)
    pool = [torch.randint(0, cfg.vocab_size, (mb, S + 1), device=dev, generator=gen) for _ in range(4)]

    def train_step(i):
        for a in range(args.accum):
            batch = pool[(i * args.accum + a) % len(pool)]
            x, y = batch[:, :-1], batch[:, 1:]
            if a < args.accum - 1:
                with opt.no_sync():
                    loss = model(x, y) / args.accum
                    loss.backward()
            else:
                loss = model(x, y) / args.accum
                loss.backward()
        opt.step()
        opt.zero_grad()
        return loss

    for i in range(args.warmup):
        l = train_step(i)
        torch.cuda.synchronize()
        if rank == 0:
            log(f"[bench] warmup {i} loss={l.item()*args.accum:.4f} mem_peak={torch.cuda.max_memory_allocated(dev)/2**30:.1f}GiB")
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        l = train_step(args.warmup + i)
        if rank == 0 and (i % 2 == 0 or i == args.steps - 1):
            log(f"[bench] step {i} issued")
    comm.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    elt = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(elt, op=torch.distributed.ReduceOp.MAX)
    el = float(elt.item())
    tokens_per_step = world * args.accum * mb * S
    tps = tokens_per_step * args.steps / el
    ms = el / args.steps * 1000
    fpt = llama_flops_per_token(cfg, S)
    mfu = tps / world * fpt / 2.5e15
    if rank == 0:
        log(f"[bench] final loss={l.item()*args.accum:.4f} tokens/s={tps:.0f} per-gpu={tps/world:.0f} "
            f"ms/step={ms:.1f} MFU(2.5PF bf16 dense)={mfu*100:.1f}% peak_mem={torch.cuda.max_memory_allocated(dev)/2**30:.1f}GiB")
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
            "dtype": "bf16",
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
                "tuned_gemm": tuned,
            },
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
