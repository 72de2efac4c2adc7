"""The two single-process multi-device strategies of the reference's legacy engine,
re-designed for one MI355X node:

* :class:`ParallelNeuralNetwork` -- model parallelism by layer placement
  (``--parallel_nn``): every layer carries a device; one compute thread per
  device runs the forward tasks dispatched to it, activations move device to
  device (peer copies over xGMI on a multi-GPU node).  No micro-batching: it is a
  placement strategy for models bigger than one device, not a pipeline (use
  ``fleet.pipeline`` for 1F1B).  The backward runs on the autograd engine, which
  already keeps one worker thread per device.
  Reference: legacy/gserver/gradientmachines/ParallelNeuralNetwork.h:20-80,
  ParallelNeuralNetwork.cpp:34-118.

* :class:`MultiGradientMachine` -- data parallelism over the devices of one
  process: one trainer thread per device computes forward / backward on its slice
  of the batch; gradients are summed with a ring (reduce-scatter then all-gather,
  N - 1 steps each, chunk i travelling device j -> j + 1), so every link carries
  1/N of the gradient per step -- the per-link-bound pattern that suits xGMI's
  point-to-point topology -- and the optimizer runs on every replica with the
  same summed gradient (replicas stay bit-identical).
  Reference: legacy/gserver/gradientmachines/MultiGradientMachine.h:40-167,
  MultiGradientMachine.cpp:410,469-475,619-700.

Devices are torch device strings ("cuda:0", "cuda:1", ... or "cpu" for tests).
"""
from __future__ import annotations

import copy
import queue
import threading

import torch


class _DeviceWorker:
    """One compute thread bound to a device; runs submitted callables in order."""

    def __init__(self, device):
        self.device = torch.device(device)
        self._q: queue.Queue = queue.Queue()
        self._t = threading.Thread(target=self._loop, name=f"pnn-{device}", daemon=True)
        self._t.start()

    def _loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while True:
            item = self._q.get()
            if item is None:
                return
            fn, box, ev = item
            try:
                box["out"] = fn()
            except BaseException as e:  # propagate to the submitter
                box["err"] = e
            ev.set()

    def run(self, fn):
        box, ev = {}, threading.Event()
        self._q.put((fn, box, ev))
        ev.wait()
        if "err" in box:
            raise box["err"]
        return box["out"]

    def close(self):
        self._q.put(None)
        self._t.join(timeout=5)


class ParallelNeuralNetwork(torch.nn.Module):
    """Sequential model whose layers live on given devices.

    ``layers``: list of modules; ``devices``: one device per layer (the layer's
    ``device`` attribute in the reference config).  ``forward`` dispatches each
    layer's task to its device's thread and copies the activation to the next
    layer's device (gradients flow back through the same copies)."""

    def __init__(self, layers, devices):
        super().__init__()
        if len(layers) != len(devices):
            raise ValueError("one device per layer")
        self.layers = torch.nn.ModuleList(layers)
        self.devices = [torch.device(d) for d in devices]
        for m, d in zip(self.layers, self.devices):
            m.to(d)
        self._workers = {str(d): _DeviceWorker(d) for d in dict.fromkeys(self.devices)}
        self.trace = []  # (layer index, device, thread name) of the last forward

    def forward(self, x):
        self.trace = []
        grad_on = torch.is_grad_enabled()
        for i, (m, d) in enumerate(zip(self.layers, self.devices)):
            w = self._workers[str(d)]

            def task(m=m, d=d, x=x, i=i):
                with torch.set_grad_enabled(grad_on):
                    y = m(x.to(d, non_blocking=False))
                if d.type == "cuda":
                    torch.cuda.current_stream(d).synchronize()  # hand the activation over complete
                self.trace.append((i, str(d), threading.current_thread().name))
                return y

            x = w.run(task)
        return x

    def close(self):
        for w in self._workers.values():
            w.close()


def ring_allreduce_(tensors):
    """In-place sum of same-shape tensors living on different devices with a ring:
    N - 1 reduce-scatter steps then N - 1 all-gather steps over N chunks."""
    n = len(tensors)
    if n == 1:
        return tensors
    flats = [t.view(-1) for t in tensors]
    chunks = [list(f.tensor_split(n)) for f in flats]
    # reduce-scatter: at step s, device j sends chunk (j - s) mod n to device j + 1
    for s in range(n - 1):
        sends = [(j, (j - s) % n) for j in range(n)]
        moved = [chunks[j][c].to(tensors[(j + 1) % n].device, copy=True) for j, c in sends]
        for (j, c), m in zip(sends, moved):
            chunks[(j + 1) % n][c].add_(m)
    # device j now owns the full sum of chunk (j + 1) mod n; all-gather around the ring
    for s in range(n - 1):
        sends = [(j, (j + 1 - s) % n) for j in range(n)]
        moved = [chunks[j][c].to(tensors[(j + 1) % n].device, copy=True) for j, c in sends]
        for (j, c), m in zip(sends, moved):
            chunks[(j + 1) % n][c].copy_(m)
    return tensors


class MultiGradientMachine:
    """Single-process multi-device data parallelism with ring gradient exchange.

    ``model_fn()`` builds one replica; ``loss_fn(model, batch_slice)`` returns the
    replica's loss; ``optimizer_fn(params)`` builds a replica's optimizer.  ``step``
    splits the batch along dim 0 over the devices, runs one trainer thread per
    device, ring-sums the gradients, scales them by 1 / N (the mean over the whole
    batch when each replica's loss is a mean) and steps every replica."""

    def __init__(self, model_fn, loss_fn, optimizer_fn, devices):
        self.devices = [torch.device(d) for d in devices]
        base = model_fn()
        self.replicas = [copy.deepcopy(base).to(d) for d in self.devices]
        self.loss_fn = loss_fn
        self.opts = [optimizer_fn(list(r.parameters())) for r in self.replicas]
        self._workers = [_DeviceWorker(d) for d in self.devices]

    def step(self, *batch):
        n = len(self.devices)
        parts = [torch.tensor_split(b, n) for b in batch]
        losses = [None] * n
        threads = []

        def work(j):
            def task():
                r = self.replicas[j]
                for p in r.parameters():
                    p.grad = None
                loss = self.loss_fn(r, *[p[j].to(self.devices[j]) for p in parts])
                loss.backward()
                return loss.detach()
            losses[j] = self._workers[j].run(task)

        for j in range(n):
            t = threading.Thread(target=work, args=(j,))
            t.start()
            threads.append(t)
        for t in threads:
            t.join()
        params = [list(r.parameters()) for r in self.replicas]
        for group in zip(*params):
            grads = [p.grad for p in group]
            if any(g is None for g in grads):
                continue
            ring_allreduce_(grads)
            for g in grads:
                g.div_(n)
        for o in self.opts:
            o.step()
        return sum(float(l.cpu()) for l in losses) / n

    def close(self):
        for w in self._workers:
            w.close()
