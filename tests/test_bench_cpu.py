"""bench.py contract on CPU (gloo) and fp32 gradient accumulation.

* ``bench.py --gpus 2`` outside a launcher must start 2 ranks itself and report
  ``n_gpus: 2``; its loss must equal a 1-rank run on the 2x micro-batch (same
  global data), in the spirit of the reference's
  parallel_executor_test_base.check_network_convergence
  (python/paddle/fluid/tests/unittests/parallel_executor_test_base.py:29).
* fp32 main_grad: accumulating 8 micro-batches of a bf16 model into the fp32
  flat buffer must match an fp64 sum of the per-micro-batch gradients, and be
  clearly better than the bf16 buffer (Fleet keeps fp32 main_grad for this).
"""
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--model", "llama-tiny",
           "--seq-len", "64", "--accum", "2", "--steps", "3", "--warmup", "1", "--dtype", "float32"] + list(args)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0]), r.stderr


def test_bench_self_launches_two_ranks_and_matches_one():
    two, err = _bench("--gpus", "2", "--micro-batch", "2")
    assert two["n_gpus"] == 2
    assert "world=2 rank=0" in err and "world=2 rank=1" in err
    assert two["config"]["parallelism"].startswith("dp2")
    assert two["config"]["global_batch"] == 2 * 2 * 2
    one, _ = _bench("--gpus", "1", "--micro-batch", "4")
    assert one["n_gpus"] == 1
    assert one["config"]["global_batch"] == two["config"]["global_batch"]
    # fp32 model on the tape: same data, same init, the 2-rank sum of gradients equals
    # the 1-rank batch (reference: parallel_executor_test_base.py:29, 1e-4-level checks)
    assert abs(one["final_loss"] - two["final_loss"]) < 1e-4, (one["final_loss"], two["final_loss"])
    assert two["config"]["autograd"] == "tape" and two["config"]["comm_backend"] == "gloo"


def _model():
    from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM

    torch.manual_seed(0)
    return LlamaForCausalLM(LlamaConfig(**LLAMA_CONFIGS["llama-tiny"]), device="cpu")


def test_fp32_main_grad_accumulation_matches_fp64_oracle():
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    g = torch.Generator().manual_seed(3)
    mbs = [torch.randint(0, 512, (2, 65), generator=g) for _ in range(8)]

    # oracle: per-micro-batch fp32 gradients summed in fp64
    m = _model()
    opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-3, grad_dtype=torch.float32)
    assert opt.flat_grad.dtype == torch.float32
    oracle = torch.zeros(opt.total, dtype=torch.float64)
    for b in mbs:
        opt.zero_grad()
        (m(b[:, :-1], b[:, 1:]) / len(mbs)).backward()
        oracle += opt.flat_grad.double()
    assert all(p.grad is None for p in m.parameters())  # grads live in main_grad only

    def accumulated(grad_dtype):
        mm = _model()
        o = FlatShardedOptimizer(mm.named_parameters(), lr=1e-3, grad_dtype=grad_dtype)
        for b in mbs:
            with o.no_sync():
                (mm(b[:, :-1], b[:, 1:]) / len(mbs)).backward()
        return o.flat_grad.double()

    nrm = oracle.norm()
    e32 = (accumulated(torch.float32) - oracle).norm() / nrm
    e16 = (accumulated(None) - oracle).norm() / nrm
    assert e32 < 1e-5, e32
    assert e16 > 10 * e32, (e16, e32)


def test_lazy_zero_grad_overwrites_stale_main_grad():
    """zero_grad() in fp32 main_grad mode does not fill the buffer: the first write
    of the next backward overwrites each slice (dW GEMM with beta = 0 / copy_)."""
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    g = torch.Generator().manual_seed(4)
    mb1, mb2 = (torch.randint(0, 512, (2, 65), generator=g) for _ in range(2))
    m = _model()
    opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-3, grad_dtype=torch.float32)
    m(mb1[:, :-1], mb1[:, 1:]).backward()
    opt.zero_grad()
    m(mb2[:, :-1], mb2[:, 1:]).backward()
    got = opt.flat_grad.clone()
    m2 = _model()
    opt2 = FlatShardedOptimizer(m2.named_parameters(), lr=1e-3, grad_dtype=torch.float32)
    m2(mb2[:, :-1], mb2[:, 1:]).backward()
    assert torch.equal(got, opt2.flat_grad)
    # a step after zero_grad with no backward at all must see zero gradients
    opt.zero_grad()
    before = opt.master.clone()
    opt.wd = 0.0
    opt.step()
    assert torch.equal(opt.master, before)
