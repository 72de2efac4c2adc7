"""The native buddy allocator installed behind torch (FLAGS_allocator_strategy=buddy,
csrc/runtime/allocator.cc pa_torch_malloc / pa_torch_free) carries a full
LLaMA-tiny training run on the framework tape: same losses as torch's caching
allocator, blocks come from the buddy pools and frees return them.

Reference: memory/detail/buddy_allocator.cc + memory/malloc.cc (the reference's
only device allocator); its tests (buddy_allocator_test / malloc_test) exercise
alloc/free directly, which tests/test_runtime_cpu.py covers on host arenas."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(strategy, steps=4):
    env = dict(os.environ, FLAGS_allocator_strategy=strategy, FLAGS_buddy_chunk_mb="1024")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "llama_tiny_step.py"), str(steps)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_llama_tiny_under_buddy_allocator_matches_caching_allocator():
    ref = _run("torch_caching")
    bud = _run("buddy")
    assert bud["allocator"] == "buddy"
    st = bud["buddy"]
    assert st["reserved"] >= 1 << 30, st          # tensors really came from the buddy arenas
    assert 0 < st["peak"] <= st["reserved"], st
    assert st["used"] < st["peak"], st            # frees were returned (after their events)
    for a, b in zip(ref["losses"], bud["losses"]):
        assert abs(a - b) <= 1e-3 * max(1.0, abs(a)), (ref["losses"], bud["losses"])
    assert bud["losses"][-1] < bud["losses"][0]


def test_buddy_is_default_and_record_stream_defers_reuse():
    """In this (default-configured) process torch allocates from the buddy pools; a
    block used on a side stream (record_stream) is not handed out again until that
    stream has passed the point where the block was freed."""
    code = r"""
import torch, paddle_amd
from paddle_amd import runtime
x = torch.empty(64 << 20, device="cuda")          # 256 MiB, default stream
assert runtime.torch_allocator_stats()["reserved"] > 0, "buddy allocator not active"
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    torch.cuda._sleep(200_000_000)               # keep the side stream busy
    y = x * 2
x.record_stream(s)
p = x.data_ptr()
del x
assert runtime.torch_deferred_frees() == 1
z = torch.empty(64 << 20, device="cuda")
assert z.data_ptr() != p                          # the pending block was not reused
s.synchronize()
w = torch.empty(16, device="cuda")                # next malloc drains completed frees
assert runtime.torch_deferred_frees() == 0
print("ok")
"""
    env = dict(os.environ)
    env.pop("FLAGS_allocator_strategy", None)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120,
                       cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-3000:]
