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

Correctness rules (the reduction must describe the gradients as they are when
the optimizer consumes them):

* every launched bucket records the identity and version counter of each
  gradient it read; :meth:`finish` re-reduces, from the CURRENT gradients, any
  bucket whose gradients were replaced or modified in place after its launch
  (a second ``backward()`` before ``step()``, AMP ``unscale_``, user clipping);
* a gradient-ready hook on an already launched bucket means a later reverse pass
  (gradient accumulation) is producing new values: the in-flight reduction is
  dropped (waited for, never written back) and the bucket relaunches when it
  completes again, so the LAST pass still overlaps its reduction;
* :meth:`reset` (called by ``clear_grad``) discards everything a skipped step
  (AMP found inf) left behind.

``armed`` gates the hooks: with gradient accumulation (1F1B micro-batches) only
the LAST micro-batch's reverse pass may launch buckets."""
from __future__ import annotations

import torch
import torch.distributed

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
        self.armed = True
        self.launch_count = 0  # buckets issued from hooks (observability / tests)
        self.redo_count = 0    # buckets re-reduced in finish() because grads changed after launch
        self.reset()
        for p in self.params:
            p.register_post_accumulate_grad_hook(self._on_grad)
            p.__dict__.setdefault("_pa_grad_ready_hooks", []).append(self._on_grad)

    def reset(self):
        """Forget every launched / pending bucket (their reductions are waited for)."""
        for ent in getattr(self, "pending", {}).values():
            if ent[2] is not None:
                ent[2].wait()
        for w in getattr(self, "stale", []):
            if w is not None:
                w.wait()
        self.ready = [set() for _ in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.pending = {}   # bucket -> (params, flat, work, signature)
        self.stale = []     # works of dropped launches (waited, never written back)
        self.synced = False  # finish() ran and no gradient changed since

    def _on_grad(self, p):
        if self.W <= 1:
            return
        self.synced = False
        if not self.armed:
            return
        b = self.bucket_of.get(id(p))
        if b is None:
            return
        if self.launched[b]:
            # a later reverse pass is re-producing this bucket's gradients
            ent = self.pending.pop(b, None)
            if ent is not None:
                self.stale.append(ent[2])
            self.launched[b] = False
            self.ready[b] = set()
        self.ready[b].add(id(p))
        if len(self.ready[b]) == len(self.buckets[b]):
            self._launch(b)
            self.launch_count += 1

    @staticmethod
    def _signature(ps):
        return [(id(q.grad), q.grad._version) for q in ps]

    def _launch(self, b, async_op=True):
        self.launched[b] = True
        ps = [q for q in self.buckets[b] if q.grad is not None]
        if not ps:
            return
        flat = torch.cat([q.grad.reshape(-1).float() for q in ps])
        work = comm.all_reduce(flat, group=self.group, async_op=async_op)
        self.pending[b] = (ps, flat, work, self._signature(ps))

    @torch.no_grad()
    def finish(self):
        """Issue the buckets that never completed, wait for all, write back mean grads
        (re-reducing any bucket whose gradients changed after it was launched)."""
        if self.W > 1 and not self.synced:
            for b in range(len(self.buckets)):
                if not self.launched[b]:
                    self._launch(b)
            for w in self.stale:
                if w is not None:
                    w.wait()
            self.stale = []
            order = sorted(self.pending)
            changed = []
            for b in order:
                ps, flat, work, sig = self.pending[b]
                if work is not None:
                    work.wait()
                cur = [q for q in self.buckets[b] if q.grad is not None]
                changed.append(int([id(q) for q in cur] != [id(q) for q in ps] or self._signature(cur) != sig))
            if order:
                # the redo decision is collective (every rank re-reduces the same buckets
                # in the same order, whatever changed locally)
                dev = self.pending[order[0]][1].device
                flags = torch.tensor(changed, dtype=torch.int32, device=dev)
                comm.all_reduce(flags, op=torch.distributed.ReduceOp.MAX, group=self.group)
                changed = flags.tolist()
            for b, ch in zip(order, changed):
                ps, flat, work, sig = self.pending[b]
                if ch:
                    # gradients replaced / modified after launch: reduce what is there now
                    cur = [q for q in self.buckets[b] if q.grad is not None]
                    self.redo_count += 1
                    ps = cur
                    if not ps:
                        continue
                    flat = torch.cat([q.grad.reshape(-1).float() for q in ps])
                    comm.all_reduce(flat, group=self.group)
                flat /= self.W
                o = 0
                for q in ps:
                    n = q.numel()
                    q.grad.copy_(flat[o:o + n].view_as(q.grad))
                    o += n
            self.pending = {}
            self.ready = [set() for _ in self.buckets]
            self.launched = [False] * len(self.buckets)
            self.synced = True
        elif self.W <= 1:
            self.synced = True
