#!/usr/bin/env python3
"""Training-throughput benchmark for the other model families on 1..N MI355X
(same timing contract as bench.py: warm-up, barrier + synchronize around exactly
``--steps`` steps, max over ranks, one JSON line from rank 0).

  python benchmarks/train_lm.py --model gpt3-13b --seq-len 2048 --micro-batch 1 --recompute
  python benchmarks/train_lm.py --model ernie-moe-21b-a3b --fp8-experts
  torchrun --nproc-per-node 8 benchmarks/train_lm.py --model gpt3-13b   # dp8 + ZeRO-1 (flat sharded AdamW)

Synthetic token ids, random-init weights, bf16, fused flat sharded AdamW.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(name, device, args):
    if name.startswith("gpt"):
        from paddle_amd.models.gpt import GPT_CONFIGS, GPTConfig, GPTForCausalLM, gpt_flops_per_token

        cfg = GPTConfig(**GPT_CONFIGS[name], recompute=args.recompute, max_position_embeddings=max(2048,
                                                                                                  args.seq_len))
        return GPTForCausalLM(cfg, device), cfg, gpt_flops_per_token(cfg, args.seq_len)
    if name.startswith("ernie"):
        from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM

        cfg = ErnieMoEConfig(**ERNIE_MOE_CONFIGS[name], use_fp8_experts=args.fp8_experts,
                             grouped_experts=args.grouped_experts)
        H, L, V = cfg.hidden_size, cfg.num_hidden_layers, cfg.vocab_size
        kvd = cfg.kv_heads * cfg.head_dim
        active = H * (H + 2 * kvd) + H * H + 3 * H * cfg.moe_intermediate_size * cfg.top_k
        fpt = 3 * (2 * L * active + 2 * 2 * args.seq_len * H / 2 * L + 2 * H * V)
        return ErnieMoEForCausalLM(cfg, device), cfg, fpt
    from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM, llama_flops_per_token

    cfg = LlamaConfig(**LLAMA_CONFIGS[name], recompute=args.recompute)
    return LlamaForCausalLM(cfg, device), cfg, llama_flops_per_token(cfg, args.seq_len)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt3-13b")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--micro-batch", type=int, default=2)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--recompute", action="store_true")
    ap.add_argument("--fp8-experts", action="store_true")
    ap.add_argument("--grouped-experts", action="store_true", help="MoE experts as ragged grouped GEMMs")
    ap.add_argument("--bucket-mb", type=int, default=512)
    ap.add_argument("--accum", type=int, default=1, help="gradient accumulation micro-steps per optimizer step")
    ap.add_argument("--bf16-grads", action="store_true", help="bf16 gradient buffer instead of fp32 main_grad")
    a = ap.parse_args()

    from paddle_amd.parallel import comm
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    rank, world = comm.init_parallel_env()
    dev = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(1234)
    model, cfg, fpt = build(a.model, dev, a)
    opt = FlatShardedOptimizer(model.named_parameters(), lr=1e-4, weight_decay=0.1, grad_clip=1.0,
                               bucket_mb=a.bucket_mb, grad_dtype=None if a.bf16_grads else torch.float32)
    V = cfg.vocab_size
    g = torch.Generator(device=dev).manual_seed(rank)
    ids = torch.randint(0, V, (a.micro_batch, a.seq_len + 1), device=dev, generator=g)

    def step():
        # Fleet accumulate_steps: gradient sync only on the last micro-step
        for m in range(a.accum):
            if m < a.accum - 1:
                with opt.no_sync():
                    loss = model(ids[:, :-1], ids[:, 1:]) / a.accum
                    loss.backward()
            else:
                loss = model(ids[:, :-1], ids[:, 1:]) / a.accum
                loss.backward()
        opt.step()
        opt.zero_grad()
        return loss

    hist = []
    for _ in range(a.warmup):
        hist.append(step().detach())
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
        hist.append(loss.detach())
    torch.cuda.synchronize()
    comm.barrier()
    dt = torch.tensor([time.perf_counter() - t0], device=dev)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    sec = dt.item() / a.steps
    tok = a.accum * a.micro_batch * a.seq_len * world / sec
    if rank == 0:
        print(json.dumps({"metric": f"tokens/sec (whole job) {a.model} training", "value": round(tok, 1),
                          "unit": "tokens/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(1000 * sec, 2), "dtype": "bf16" + ("+fp8 experts" if a.fp8_experts
                                                                                    else ""),
                          "data": "synthetic", "mfu_bf16_dense": round(tok * fpt / world / 2.5e15, 4),
                          "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1),
                          "config": {"model": a.model, "micro_batch": a.micro_batch, "grad_accum": a.accum, "seq_len": a.seq_len,
                                     "recompute": a.recompute, "grouped_experts": a.grouped_experts,
                                     "grad_dtype": str(opt.grad_dtype), "dw_kmajor": os.environ.get("PADDLE_AMD_DW_KMAJ", "1"), "parallelism": f"dp{world}+sharding_stage1"},
                          "loss": float(loss) * a.accum,
                          "losses": [round(float(x) * a.accum, 4) for x in hist]}))


if __name__ == "__main__":
    main()
