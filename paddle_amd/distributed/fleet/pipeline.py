"""Pipeline parallelism: ``PipelineLayer`` + 1F1B ``PipelineParallel``.

North-star component (SURVEY §2.5 row "Pipeline parallel": absent from the
reference; its only model parallelism is the legacy layer->device placement of
``ParallelNeuralNetwork``, paddle/legacy/gserver/gradientmachines/
ParallelNeuralNetwork.cpp:45-98, one thread per device, no micro-batching).

Design (one process per GPU, RCCL point-to-point over xGMI):
  * ``PipelineLayer`` takes a flat list of ``LayerDesc`` and builds ONLY this
    stage's segment (uniform or class-count partition).  Each layer is built
    under its own seed (``seed + index``), so a layer's initial weights do not
    depend on the partition -- pipelined and single-stage models start identical.
  * ``PipelineParallel.train_batch`` runs the 1F1B schedule: ``pp - stage - 1``
    warm-up forwards, steady one-forward-one-backward, cool-down backwards.  Every
    transfer is a batched isend/irecv pair (``send_forward_recv_backward`` etc.),
    so neighbouring stages never deadlock; tensor metadata travels in a small
    int64 header before the payload.
  * activations are tuples of tensors; floating ones carry gradients back.
  * after the schedule: data-parallel gradient all-reduce (dp group), shared-weight
    gradient all-reduce (tied embeddings), then the optimizer step.
"""
from __future__ import annotations

import math

import os

import torch
import torch.distributed as dist

from ...autograd import engine as _eager
from ...autograd import tape as _tape
from ...nn import Layer
from ...parallel import comm

_DTYPES = [torch.float32, torch.bfloat16, torch.float16, torch.int64, torch.int32, torch.bool, torch.float64]
_MAXT, _MAXD = 8, 8


class LayerDesc:
    def __init__(self, layer_cls, *args, **kwargs):
        self.layer_cls, self.args, self.kwargs = layer_cls, args, kwargs

    def build(self):
        return self.layer_cls(*self.args, **self.kwargs)

    def __repr__(self):
        return f"LayerDesc({self.layer_cls.__name__})"


class SharedLayerDesc(LayerDesc):
    """A layer whose parameter ``shared_weight_attr`` is shared (tied) between the
    stages that instantiate ``key`` (e.g. input embedding and LM head)."""

    def __init__(self, key, layer_cls, forward_func=None, shared_weight_attr="weight", *args, **kwargs):
        super().__init__(layer_cls, *args, **kwargs)
        self.key, self.forward_func, self.shared_weight_attr = key, forward_func, shared_weight_attr


class _SharedCall(torch.nn.Module):
    def __init__(self, layer, fn):
        super().__init__()
        self.layer, self.fn = layer, fn

    def forward(self, *a):
        return self.fn(self.layer, *a) if self.fn is not None else self.layer(*a)


def _partition(descs, num_stages, method):
    n = len(descs)
    if method.startswith("layer:"):
        name = method.split(":", 1)[1]
        marks = [i for i, d in enumerate(descs) if getattr(d, "layer_cls", type(d)).__name__ == name]
        per = [len(marks) // num_stages + (1 if s < len(marks) % num_stages else 0) for s in range(num_stages)]
        bounds, c = [0], 0
        for s in range(num_stages - 1):
            c += per[s]
            bounds.append(marks[c] if c < len(marks) else n)
        bounds.append(n)
        return bounds
    per = [n // num_stages + (1 if s < n % num_stages else 0) for s in range(num_stages)]
    bounds = [0]
    for p in per:
        bounds.append(bounds[-1] + p)
    return bounds


class PipelineLayer(Layer):
    def __init__(self, layers, num_stages=None, hcg=None, loss_fn=None, seg_method="uniform", seed=1234,
                 recompute_interval=0):
        super().__init__("pipeline_layer")
        self.hcg = hcg
        self.num_stages = num_stages or (hcg.get_pipe_parallel_world_size() if hcg else 1)
        self.stage_id = hcg.get_stage_id() if hcg else 0
        self.loss_fn = loss_fn
        self.recompute_interval = recompute_interval
        self.bounds = _partition(layers, self.num_stages, seg_method)
        lo, hi = self.bounds[self.stage_id], self.bounds[self.stage_id + 1]
        self.run_function = torch.nn.ModuleList()
        self.shared = {}  # key -> parameter (for tied-weight gradient sync)
        built_shared = {}
        rng = torch.random.get_rng_state()
        for i in range(lo, hi):
            d = layers[i]
            torch.manual_seed(seed + i)
            if isinstance(d, SharedLayerDesc):
                if d.key not in built_shared:
                    # shared layers are seeded by their FIRST occurrence so every stage agrees
                    first = next(j for j, x in enumerate(layers) if isinstance(x, SharedLayerDesc) and x.key == d.key)
                    torch.manual_seed(seed + first)
                    built_shared[d.key] = d.build()
                    self.shared[d.key] = getattr(built_shared[d.key], d.shared_weight_attr)
                self.run_function.append(_SharedCall(built_shared[d.key], d.forward_func))
            elif isinstance(d, LayerDesc):
                self.run_function.append(d.build())
            else:
                self.run_function.append(d)
        torch.random.set_rng_state(rng)
        # which stages hold each shared key (for the tied-gradient all-reduce)
        self.shared_stages = {}
        for s in range(self.num_stages):
            for i in range(self.bounds[s], self.bounds[s + 1]):
                d = layers[i]
                if isinstance(d, SharedLayerDesc):
                    self.shared_stages.setdefault(d.key, set()).add(s)

    def forward(self, x):
        for i, layer in enumerate(self.run_function):
            args = x if isinstance(x, tuple) else (x,)
            if self.recompute_interval and self.training and i % self.recompute_interval == 0 \
                    and _tape.current() is not None:
                x = _tape.checkpoint(layer, *args)  # recomputed on the framework tape
            elif self.recompute_interval and self.training and torch.is_grad_enabled() \
                    and i % self.recompute_interval == 0:
                x = torch.utils.checkpoint.checkpoint(layer, *args, use_reentrant=False)
            else:
                x = layer(*args)
        return x


# ------------------------------------------------------------------ p2p plumbing
def _meta(tensors):
    m = torch.zeros(1 + _MAXT * (2 + _MAXD), dtype=torch.int64)
    m[0] = len(tensors)
    for i, t in enumerate(tensors):
        b = 1 + i * (2 + _MAXD)
        m[b] = _DTYPES.index(t.dtype)
        m[b + 1] = t.dim()
        m[b + 2:b + 2 + t.dim()] = torch.tensor(t.shape, dtype=torch.int64)
    return m


def _unmeta(m, device):
    out = []
    for i in range(int(m[0])):
        b = 1 + i * (2 + _MAXD)
        dt = _DTYPES[int(m[b])]
        shape = [int(x) for x in m[b + 2:b + 2 + int(m[b + 1])]]
        out.append(torch.empty(shape, dtype=dt, device=device))
    return out


class _P2P:
    """Point-to-point activation / gradient exchange between adjacent stages.

    Shapes and dtypes travel as a small metadata message only the first time a
    (peer, direction) pair is used; afterwards both sides reuse the cached
    metadata (static shapes across micro-batches, as in 1F1B steady state), so a
    steady-state exchange is ONE batched isend/irecv round with no host reads.  A
    sender whose tensors no longer match the cached metadata raises, unless the
    exchange was built with ``dynamic_shapes=True`` (metadata every time).
    ``meta_rounds`` / ``host_syncs`` count metadata exchanges and the device->host
    reads they needed (tests assert both stay 0 in steady state)."""

    def __init__(self, hcg, device, dynamic_shapes=None):
        self.hcg, self.device = hcg, device
        self.stage = hcg.get_stage_id()
        self.nst = hcg.get_pipe_parallel_world_size()
        self.prev = hcg.stage_rank(self.stage - 1) if self.stage > 0 else None
        self.next = hcg.stage_rank(self.stage + 1) if self.stage < self.nst - 1 else None
        self.nccl = comm.is_dist() and dist.get_backend() == "nccl"
        if dynamic_shapes is None:
            dynamic_shapes = os.environ.get("FLAGS_pp_dynamic_shapes", "0") == "1"
        self.dynamic = dynamic_shapes
        self._sent = {}   # (peer, "fwd"|"bwd") -> [(dtype, shape)] sent last
        self._recv = {}   # (peer, "fwd"|"bwd") -> [(dtype, shape)] received last
        self.meta_rounds = 0
        self.host_syncs = 0

    def _meta_dev(self):
        return self.device if self.nccl else "cpu"

    @staticmethod
    def _sig(ts):
        return [(t.dtype, tuple(t.shape)) for t in ts]

    def exchange(self, send_next=None, send_prev=None, recv_next=False, recv_prev=False):
        """One batched round: optional sends to next/prev, optional receives from
        next/prev.  Returns (from_next, from_prev) as tensor lists.  Activations flow
        forward (to next, from prev: key "fwd"), gradients backward ("bwd")."""
        mdev = self._meta_dev()
        ops = []
        got_next_m = got_prev_m = None
        # metadata only for pairs not seen yet (both sides decide identically: a
        # pair's first use is the same exchange on the sender and the receiver)
        need_sn = send_next is not None and (self.dynamic or (self.next, "fwd") not in self._sent)
        need_sp = send_prev is not None and (self.dynamic or (self.prev, "bwd") not in self._sent)
        need_rn = recv_next and (self.dynamic or (self.next, "bwd") not in self._recv)
        need_rp = recv_prev and (self.dynamic or (self.prev, "fwd") not in self._recv)
        for lst, key in ((send_next, (self.next, "fwd")), (send_prev, (self.prev, "bwd"))):
            if lst is not None and not self.dynamic and key in self._sent and self._sig(lst) != self._sent[key]:
                raise RuntimeError(f"pipeline p2p: tensors sent to rank {key[0]} changed shape/dtype "
                                   f"({self._sent[key]} -> {self._sig(lst)}); build the pipeline with "
                                   "dynamic_shapes=True (FLAGS_pp_dynamic_shapes=1) for variable shapes")
        if need_sn:
            ops.append(("send", _meta(send_next).to(mdev), self.next))
        if need_sp:
            ops.append(("send", _meta(send_prev).to(mdev), self.prev))
        if need_rn:
            got_next_m = torch.empty(1 + _MAXT * (2 + _MAXD), dtype=torch.int64, device=mdev)
            ops.append(("recv", got_next_m, self.next))
        if need_rp:
            got_prev_m = torch.empty(1 + _MAXT * (2 + _MAXD), dtype=torch.int64, device=mdev)
            ops.append(("recv", got_prev_m, self.prev))
        if ops:
            self.meta_rounds += 1
            self._run(ops)
            ops = []
        if send_next is not None:
            self._sent[(self.next, "fwd")] = self._sig(send_next)
        if send_prev is not None:
            self._sent[(self.prev, "bwd")] = self._sig(send_prev)
        for got, key in ((got_next_m, (self.next, "bwd")), (got_prev_m, (self.prev, "fwd"))):
            if got is not None:
                if got.is_cuda:
                    self.host_syncs += 1
                m = got.cpu()
                self._recv[key] = [(t.dtype, tuple(t.shape)) for t in _unmeta(m, "meta")]
        from_next = [torch.empty(sh, dtype=dt, device=self.device) for dt, sh in self._recv[(self.next, "bwd")]] \
            if recv_next else None
        from_prev = [torch.empty(sh, dtype=dt, device=self.device) for dt, sh in self._recv[(self.prev, "fwd")]] \
            if recv_prev else None
        # gloo moves host memory only: device tensors are staged through the host
        # (the RCCL path sends device buffers directly)
        host = (lambda t: t.detach().cpu()) if not self.nccl else (lambda t: t)
        land = []
        for t in send_next or []:
            ops.append(("send", host(t.contiguous()), self.next))
        for t in send_prev or []:
            ops.append(("send", host(t.contiguous()), self.prev))
        for peer, lst in ((self.next, from_next), (self.prev, from_prev)):
            for t in lst or []:
                buf = t if (self.nccl or not t.is_cuda) else torch.empty(t.shape, dtype=t.dtype)
                if buf is not t:
                    land.append((t, buf))
                ops.append(("recv", buf, peer))
        self._run(ops)
        for t, buf in land:
            t.copy_(buf)
        return from_next, from_prev

    @staticmethod
    def _run(ops):
        # the framework RCCL communicator (one ncclGroupStart/End round of device
        # sends / receives) on GPU ranks, batched isend/irecv otherwise
        comm.batch_p2p(ops)


def _as_tuple(x):
    return x if isinstance(x, tuple) else (x,)


def _needs_grad(t):
    return t.requires_grad or _eager.tracked(t)


def _backward(outs, grads):
    """Reverse pass of one micro-batch: the framework's eager engine for framework
    Tensors (DyGraph layers), torch autograd for raw torch tensors."""
    if not outs:
        return
    if any(isinstance(o, _eager.Tensor) and _eager.tracked(o) for o in outs):
        _eager.backward(outs, grads)
    else:
        torch.autograd.backward(outs, [g for g in grads] if any(g is not None for g in grads) else None)


class PipelineParallel(Layer):
    def __init__(self, layers: PipelineLayer, hcg, strategy=None):
        super().__init__("pipeline_parallel")
        self._layers = layers
        self.hcg = hcg
        cfg = (getattr(strategy, "pipeline_configs", None) or {}) if strategy is not None else {}
        self.accumulate_steps = int(cfg.get("accumulate_steps", 1))
        self.micro_batch_size = cfg.get("micro_batch_size")
        self.stage = hcg.get_stage_id()
        self.nst = hcg.get_pipe_parallel_world_size()
        self.is_first, self.is_last = hcg.is_first_stage(), hcg.is_last_stage()
        self.total_loss = None
        # tied-weight groups: new_group is collective, so every rank creates the group
        # of every pp slice (same order everywhere) and keeps the one it belongs to
        self._shared_groups = {}
        for key, stages in sorted(layers.shared_stages.items()):
            if len(stages) < 2:
                continue
            for sl in hcg.topo.axis_groups("pp"):
                ranks = [sl[s] for s in sorted(stages)]
                g = comm.new_group(ranks) if comm.is_dist() else None
                if hcg.global_rank in ranks:
                    self._shared_groups[key] = g

    def parameters(self, recurse=True):
        return self._layers.parameters(recurse)

    def named_parameters(self, *a, **k):
        return self._layers.named_parameters(*a, **k)

    def forward(self, *a):
        return self._layers(*a)

    # -------------------------------------------------------------------- helpers
    def _split(self, data):
        inputs, labels = data
        M = self.accumulate_steps
        ins = [tuple(x.chunk(M)[i] for x in _as_tuple(inputs)) for i in range(M)]
        labs = [tuple(x.chunk(M)[i] for x in _as_tuple(labels)) for i in range(M)] if labels is not None else [None] * M
        return ins, labs

    def _fwd(self, x, label):
        out = self._layers(x if len(x) > 1 else x[0])
        if self.is_last:
            fn = self._layers.loss_fn
            lab = label if label is None or len(label) > 1 else label[0]
            loss = fn(out, lab) if fn is not None else out
            from ...ops import fused as _F

            return _F.scale(loss, 1.0 / self.accumulate_steps)
        return out

    def _grad_sync_engine(self):
        W = 1 if getattr(self, "_sharded", None) is not None else self.hcg.get_data_parallel_world_size()
        if W <= 1:
            return None
        gs = getattr(self, "_grad_sync", None)
        if gs is None:
            from .grad_sync import GradBucketAllReduce

            gs = self._grad_sync = GradBucketAllReduce(list(self._layers.parameters()),
                                                       self.hcg.get_data_parallel_group(), W)
        return gs

    def _sync_grads(self):
        dp_group = self.hcg.get_data_parallel_group()
        # ZeRO-3 on the stage (fleet.distributed_model): sharded gradients were
        # reduce-scattered during backward; whole (tied) ones are averaged by the
        # HybridParallelOptimizer over dp x sharding
        W = 1 if getattr(self, "_sharded", None) is not None else self.hcg.get_data_parallel_world_size()
        params = [p for p in self._layers.parameters() if p.requires_grad and p.grad is not None]
        gs = getattr(self, "_grad_sync", None)
        if W > 1 and gs is not None:
            gs.finish()  # buckets already in flight since the last micro-batch's backward
            gs.armed = False
        elif W > 1 and params:
            flat = torch.cat([p.grad.reshape(-1).float() for p in params])
            comm.all_reduce(flat, group=dp_group)
            flat /= W
            o = 0
            for p in params:
                n = p.numel()
                p.grad.copy_(flat[o:o + n].view_as(p.grad))
                o += n
        # tied weights: sum the gradients of every stage holding the key
        for key, p in self._layers.shared.items():
            if key in self._shared_groups:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                comm.all_reduce(p.grad, group=self._shared_groups[key])

    # ------------------------------------------------------------------ schedule
    def forward_backward_pipeline(self, data):
        dev = next(self._layers.parameters()).device
        # one exchange object for the life of the engine: its metadata cache makes
        # every steady-state exchange a single batched round with no host reads
        p2p = getattr(self, "_p2p_train", None)
        if p2p is None or p2p.device != dev:
            p2p = self._p2p_train = _P2P(self.hcg, dev)
        ins, labs = self._split(data)
        M = self.accumulate_steps
        warm = min(self.nst - self.stage - 1, M)
        inputs_q, outputs_q = [], []
        losses = []
        # dp all-reduce of this stage's gradients, fired per bucket during the LAST
        # micro-batch's reverse pass (earlier micro-batches only accumulate)
        gs = self._grad_sync_engine()
        if gs is not None:
            gs.armed = False
        nbwd = [0]
        # each micro-batch's forward is recorded on its own framework tape (torch
        # autograd off); its reverse pass is that tape seeded with the next stage's
        # gradients, and the received activations are the tape's watched inputs
        use_tape = os.environ.get("FLAGS_pp_autograd", "tape") == "tape"
        tapes_q = []

        def recv_fwd_input(i):
            if self.is_first:
                return ins[i]
            _, got = p2p.exchange(recv_prev=True)
            return tuple(t.requires_grad_() if (t.is_floating_point() and not use_tape) else t for t in got)

        def run_fwd(i, x):
            if use_tape:
                with _tape.recording() as tp:
                    for t in x:
                        tp.watch(t)
                    out = self._fwd(x, labs[i])
            else:
                tp, out = None, self._fwd(x, labs[i])
            tapes_q.append(tp)
            inputs_q.append(x)
            outputs_q.append(out)
            if self.is_last:
                losses.append(out.detach())
            return out

        def run_bwd(grads):
            x = inputs_q.pop(0)
            out = outputs_q.pop(0)
            tp = tapes_q.pop(0)
            nbwd[0] += 1
            if gs is not None and nbwd[0] == M:
                gs.armed = True
            if tp is not None and not any(isinstance(o, _eager.Tensor) and _eager.tracked(o) for o in _as_tuple(out)):
                if self.is_last:
                    tp.backward_multi([out], [None])
                else:
                    outs = [o for o in _as_tuple(out) if o.is_floating_point()]
                    tp.backward_multi(outs, list(grads))
                if self.is_first:
                    return None
                return tuple(tp.grad(t) if tp.grad(t) is not None else torch.zeros_like(t)
                             for t in x if t.is_floating_point())
            if self.is_last:
                _backward([out], [None])
            else:
                # the next stage returns one gradient per FLOATING activation, in order
                outs = [o for o in _as_tuple(out) if o.is_floating_point()]
                pairs = [(o, g) for o, g in zip(outs, grads) if _needs_grad(o)]
                _backward([o for o, _ in pairs], [g for _, g in pairs])
            return tuple(t.grad if (t.is_floating_point() and t.grad is not None) else torch.zeros_like(t)
                         for t in x if t.is_floating_point()) if not self.is_first else None

        # warm-up
        for i in range(warm):
            x = recv_fwd_input(i)
            out = run_fwd(i, x)
            if not self.is_last:
                p2p.exchange(send_next=[t.detach() for t in _as_tuple(out)])
        # steady 1F1B
        steady = M - warm
        x = recv_fwd_input(warm) if steady > 0 else None
        for j in range(steady):
            i = warm + j
            out = run_fwd(i, x)
            if self.is_last:
                grads = None
            else:
                grads, _ = p2p.exchange(send_next=[t.detach() for t in _as_tuple(out)], recv_next=True)
            gin = run_bwd(grads)
            last = j == steady - 1
            if self.is_first:
                if not last:
                    x = recv_fwd_input(i + 1)
            elif last:
                p2p.exchange(send_prev=list(gin))
            else:
                _, got = p2p.exchange(send_prev=list(gin), recv_prev=True)
                x = tuple(t.requires_grad_() if t.is_floating_point() else t for t in got)
        # cool-down
        for _ in range(warm):
            grads = None
            if not self.is_last:
                grads, _ = p2p.exchange(recv_next=True)
            gin = run_bwd(grads)
            if not self.is_first:
                p2p.exchange(send_prev=list(gin))
        # loss of the batch, visible on every pp rank
        t = torch.stack(losses).sum().float().reshape(1) if self.is_last else torch.zeros(1, device=dev)
        if self.nst > 1:
            comm.all_reduce(t, group=self.hcg.get_pipe_parallel_group())
        self.total_loss = t
        return t

    def train_batch(self, data, optimizer, lr_scheduler=None, scaler=None):
        self._layers.train()
        loss = self.forward_backward_pipeline(data)
        self._sync_grads()
        if hasattr(optimizer, "_dp_sync"):  # HybridParallelOptimizer: dp already synced here
            optimizer._skip_dp_sync = True
        optimizer.step()
        (optimizer.clear_grad if hasattr(optimizer, "clear_grad") else optimizer.zero_grad)()
        if lr_scheduler is not None:
            lr_scheduler.step()
        return loss

    @torch.no_grad()
    def eval_batch(self, data, compute_loss=True):
        self._layers.eval()
        dev = next(self._layers.parameters()).device
        p2p = _P2P(self.hcg, dev)
        ins, labs = self._split(data)
        outs = []
        for i in range(self.accumulate_steps):
            if self.is_first:
                x = ins[i]
            else:
                _, x = p2p.exchange(recv_prev=True)
                x = tuple(x)
            out = self._layers(x if len(x) > 1 else x[0])
            if self.is_last:
                if compute_loss and self._layers.loss_fn is not None:
                    lab = labs[i] if labs[i] is None or len(labs[i]) > 1 else labs[i][0]
                    out = self._layers.loss_fn(out, lab)
                outs.append(out)
            else:
                p2p.exchange(send_next=list(_as_tuple(out)))
        return outs
