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
