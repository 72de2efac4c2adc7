#!/usr/bin/env python3
"""Training-throughput benchmark for the other model families on 1..N MI355X
(same timing contract as bench.py: warm-up, barrier + synchronize around exactly
``--steps`` steps, max over ranks, one JSON line from rank 0).

  python benchmarks/train_lm.py --model gpt3-13b --seq-len 2048 --micro-batch 1 --recompute
  python benchmarks/train_lm.py --model ernie-moe-21b-a3b --fp8-experts
  torchrun --nproc-per-node 8 benchmarks/train_lm.py --model gpt3-13b   # dp8 + ZeRO-1 (flat sharded AdamW)
  python benchmarks/train_lm.py --model gpt3-13b --gpus 8 --tp 2 --pp 2 --sharding 2 --sharding-stage 3
      # BASELINE config 4: Fleet hybrid TP x PP (1F1B) x sharding stage 3; self-launches 8 ranks

Synthetic token ids, random-init weights, bf16, fused flat sharded AdamW.
"""
import argparse
import contextlib
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

        cfgd = dict(GPT_CONFIGS[name])
        cfgd["max_position_embeddings"] = max(cfgd.get("max_position_embeddings", 2048), args.seq_len)
        cfg = GPTConfig(**cfgd, recompute=args.recompute)
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
    ap.add_argument("--gpus", type=int, default=0, help="self-launch this many ranks (torch.distributed.run)")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree (Fleet mp_degree)")
    ap.add_argument("--pp", type=int, default=1, help="pipeline-parallel degree (1F1B)")
    ap.add_argument("--sharding", type=int, default=1, help="sharding degree")
    ap.add_argument("--sharding-stage", type=int, default=3)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"], help="cpu: gloo rehearsal (tiny models)")
    ap.add_argument("--layers", type=int, default=None, help="debug: override layer count (result INVALID)")
    ap.add_argument("--fixed-batch", action="store_true",
                    help="re-feed ONE batch every micro-step (memorisation probe; default: a pool of distinct batches)")
    ap.add_argument("--pool", type=int, default=8, help="distinct synthetic batches cycled through")
    ap.add_argument("--autograd", default="tape", choices=["tape", "torch"],
                    help="tape: the framework's reverse pass (torch autograd off, recompute on the tape)")
    argv = sys.argv[1:]
    a = ap.parse_args(argv)
    if a.gpus and "WORLD_SIZE" not in os.environ:
        import socket
        import subprocess

        sck = socket.socket()
        sck.bind(("127.0.0.1", 0))
        port = sck.getsockname()[1]
        sck.close()
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.call([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                                  f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1", "--master-port",
                                  str(port), os.path.abspath(__file__)] + argv, env=env))
    if a.tp > 1 or a.pp > 1 or a.sharding > 1:
        return hybrid_main(a)

    from paddle_amd.autograd import tape
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
    pool = [torch.randint(0, V, (a.micro_batch, a.seq_len + 1), device=dev, generator=g)
            for _ in range(1 if a.fixed_batch else a.pool)]
    it = [0]
    ce = [0.0]
    ce_hist = []

    def step():
        # Fleet accumulate_steps: gradient sync only on the last micro-step; every
        # micro-step takes the next batch of the pool (distinct random tokens, so the
        # loss cannot fall by memorising one batch)
        tot = 0.0
        ce[0] = 0.0
        for m in range(a.accum):
            ids = pool[it[0] % len(pool)]
            it[0] += 1
            with (opt.no_sync() if m < a.accum - 1 else contextlib.nullcontext()):
                if a.autograd == "tape":
                    # forward recorded on the framework tape, the 1/accum scale is the
                    # seed gradient of its reverse pass (no torch autograd anywhere)
                    with tape.recording() as t:
                        loss = model(ids[:, :-1], ids[:, 1:])
                    t.backward(loss, torch.full_like(loss, 1.0 / a.accum))
                    loss = loss.detach() / a.accum
                else:
                    loss = model(ids[:, :-1], ids[:, 1:]) / a.accum
                    loss.backward()
            tot = tot + loss.detach()
            if getattr(model, "last_ce", None) is not None:
                ce[0] = ce[0] + model.last_ce / a.accum
        opt.step()
        opt.zero_grad()
        return tot

    hist = []
    for _ in range(a.warmup):
        hist.append(step().detach())
        ce_hist.append(ce[0])
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
        hist.append(loss.detach())
        ce_hist.append(ce[0])
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
                          "peak_mem_gib": round(__import__("paddle_amd.platform", fromlist=["x"]).max_memory_allocated(
                              torch.cuda.current_device()) / 2**30, 1),
                          "config": {"model": a.model, "micro_batch": a.micro_batch, "grad_accum": a.accum, "seq_len": a.seq_len,
                                     "recompute": a.recompute, "grouped_experts": a.grouped_experts, "autograd": a.autograd,
                                     "grad_dtype": str(opt.grad_dtype), "dw_kmajor": os.environ.get("PADDLE_AMD_DW_KMAJ", "1"), "parallelism": f"dp{world}+sharding_stage1"},
                          "batches": "fixed" if a.fixed_batch else f"pool of {a.pool}",
                          "loss": float(loss),
                          "losses": [round(float(x), 4) for x in hist],
                          **({"cross_entropy": [round(float(x), 4) for x in ce_hist]}
                             if getattr(model, "last_ce", None) is not None else {})}))


def hybrid_main(a):
    """Fleet hybrid parallel GPT: fleet.init -> PipelineLayer of TP blocks ->
    fleet.distributed_model (1F1B pipeline, ZeRO-3 units on the sharding axis) ->
    fleet.distributed_optimizer; timing contract of bench.py."""
    import paddle_amd
    from paddle_amd.distributed.fleet import DistributedStrategy, TPGroup, fleet
    from paddle_amd.distributed.fleet.pipeline import PipelineLayer
    from paddle_amd.models.gpt import GPT_CONFIGS, GPTConfig, GPTPretrainingCriterion, gpt_flops_per_token, \
        gpt_pipeline_descs
    from paddle_amd.parallel import comm

    if not a.model.startswith("gpt"):
        raise SystemExit("hybrid mode drives the GPT family (BASELINE config 4)")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dp = world // (a.tp * a.pp * a.sharding)
    if dp < 1 or dp * a.tp * a.pp * a.sharding != world:
        raise SystemExit(f"world {world} != tp {a.tp} x pp {a.pp} x sharding {a.sharding} x dp")
    cpu = a.device == "cpu"
    st = DistributedStrategy()
    st.hybrid_configs = {"dp_degree": dp, "mp_degree": a.tp, "pp_degree": a.pp, "sharding_degree": a.sharding}
    st.sharding = a.sharding > 1
    st.sharding_configs = {"stage": a.sharding_stage}
    st.pipeline_configs = {"accumulate_steps": max(a.accum, a.pp), "micro_batch_size": a.micro_batch}
    if cpu:
        comm.init_parallel_env("gloo")
    fleet.init(is_collective=True, strategy=st)
    hcg = fleet.get_hybrid_communicate_group()
    rank = comm.get_rank()
    if cpu:
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dev = torch.device("cuda", torch.cuda.current_device())
    torch.manual_seed(1234)
    cfgd = dict(GPT_CONFIGS[a.model])
    if a.layers:
        cfgd["num_hidden_layers"] = a.layers
    cfgd["max_position_embeddings"] = max(cfgd.get("max_position_embeddings", 2048), a.seq_len)
    if cpu:
        cfgd["dtype"] = "float32"
    cfg = GPTConfig(**cfgd, recompute=a.recompute)
    tp = TPGroup(hcg.get_model_parallel_group())
    layer = PipelineLayer(gpt_pipeline_descs(cfg, dev, tp), hcg=hcg, loss_fn=GPTPretrainingCriterion(tp), seed=7)
    model = fleet.distributed_model(layer)
    inner = paddle_amd.optimizer.AdamW(learning_rate=1e-4, parameters=list(layer.parameters()), weight_decay=0.1,
                                       grad_clip=paddle_amd.optimizer.clip.ClipGradByGlobalNorm(1.0))
    opt = fleet.distributed_optimizer(inner)
    M = st.pipeline_configs["accumulate_steps"]
    gen = torch.Generator(device="cpu").manual_seed(hcg.get_data_parallel_rank() * 131 + hcg.get_sharding_parallel_rank())
    pool = [torch.randint(0, cfg.vocab_size, (M * a.micro_batch, a.seq_len + 1), generator=gen).to(dev)
            for _ in range(1 if a.fixed_batch else a.pool)]
    it = [0]
    sync = (lambda: None) if cpu else torch.cuda.synchronize

    def step():
        ids = pool[it[0] % len(pool)]
        it[0] += 1
        return model.train_batch((ids[:, :-1], ids[:, 1:]), opt)

    hist = [float(step()) for _ in range(a.warmup)]
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    sync()
    comm.barrier()
    dt = torch.tensor([time.perf_counter() - t0], device=dev if not cpu else "cpu")
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    sec = dt.item() / max(a.steps, 1)
    tok = M * a.micro_batch * a.seq_len * dp * a.sharding / sec
    if rank == 0:
        fpt = gpt_flops_per_token(cfg, a.seq_len)
        print(json.dumps({"metric": f"tokens/sec (whole job) {a.model} Fleet hybrid parallel", "value": round(tok, 1),
                          "unit": "tokens/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(1000 * sec, 2), "dtype": "float32" if cpu else "bf16",
                          "data": "synthetic", "mfu_bf16_dense": round(tok * fpt / world / 2.5e15, 4),
                          "config": {"model": a.model + (f"(DEBUG {a.layers} layers: INVALID)" if a.layers else ""),
                                     "parallelism": f"tp{a.tp}xpp{a.pp}xsharding{a.sharding}(stage{a.sharding_stage})"
                                                    f"xdp{dp}", "micro_batch": a.micro_batch,
                                     "accumulate_steps": M, "seq_len": a.seq_len, "device": a.device},
                          "loss": float(loss), "losses": [round(x, 4) for x in hist]}), flush=True)


if __name__ == "__main__":
    main()
