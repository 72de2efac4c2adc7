"""Bucketed gradient all-reduce fired from grad-ready hooks (data-parallel axis of
hybrid parallelism), overlapped with the rest of the reverse pass.

Reference: the ParallelExecutor's all-reduce op handles run as soon as the
gradients they read are produced, on their own stream, while later backward ops
keep computing (framework/details/multi_devices_graph_pass.cc:419-427 inserts one
AllReduceOpHandle per gradient; threaded_ssa_graph_executor.cc:93-129 schedules by
readiness).  Here gradients are grouped into buckets of ``bucket_mb`` in backward
order; when the last gradient of a bucket is produced (the framework's eager
engine / tape grad-ready hooks or torch's post-accumulate hook) the bucket is
flattened and its all-reduce is issued asynchronously (RCCL runs it on its own
stream); :meth:`finish` issues what never completed (unused parameters), waits,
and writes the averaged gradients back.

``armed`` gates the hooks: with gradient accumulation (1F1B micro-batches) only
the LAST micro-batch's reverse pass may launch buckets."""
from __future__ import annotations

import torch

from ...parallel import comm


class GradBucketAllReduce:
    def __init__(self, params, group, world, bucket_mb=64):
        self.group, self.W = group, world
        self.params = [p for p in params if p.requires_grad]
        limit = max(1, int(bucket_mb * 2**20) // 4)
        self.buckets, cur, n = [], [], 0
        for p in reversed(self.params):  # backward produces gradients roughly in reverse order
            cur.append(p)
            n += p.numel()
            if n >= limit:
                self.buckets.append(cur)
                cur, n = [], 0
        if cur:
            self.buckets.append(cur)
        self.bucket_of = {id(p): i for i, b in enumerate(self.buckets) for p in b}
        self.ready = [set() for _ in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.pending = []
        self.armed = True
        self.launch_count = 0  # buckets issued from hooks (observability / tests)
        for p in self.params:
            p.register_post_accumulate_grad_hook(self._on_grad)
            p.__dict__.setdefault("_pa_grad_ready_hooks", []).append(self._on_grad)

    def _on_grad(self, p):
        if not self.armed or self.W <= 1:
            return
        b = self.bucket_of.get(id(p))
        if b is None or self.launched[b]:
            return
        self.ready[b].add(id(p))
        if len(self.ready[b]) == len(self.buckets[b]):
            self._launch(b)
            self.launch_count += 1

    def _launch(self, b):
        self.launched[b] = True
        ps = [q for q in self.buckets[b] if q.grad is not None]
        if not ps:
            return
        flat = torch.cat([q.grad.reshape(-1).float() for q in ps])
        work = comm.all_reduce(flat, group=self.group, async_op=True)
        self.pending.append((ps, flat, work))

    @torch.no_grad()
    def finish(self):
        """Issue the buckets that never completed, wait for all, write back mean grads."""
        if self.W > 1:
            for b in range(len(self.buckets)):
                if not self.launched[b]:
                    self._launch(b)
            for ps, flat, work in self.pending:
                if work is not None:
                    work.wait()
                flat /= self.W
                o = 0
                for q in ps:
                    n = q.numel()
                    q.grad.copy_(flat[o:o + n].view_as(q.grad))
                    o += n
        self.pending = []
        self.ready = [set() for _ in self.buckets]
        self.launched = [False] * len(self.buckets)
