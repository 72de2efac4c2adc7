"""Flat-buffer sharded data parallelism ("Fleet sharding stage 1/2") over RCCL.

Parity: the reference's ParallelExecutor offers AllReduce or Reduce+Broadcast
("kReduce": the optimizer runs only on the owner device chosen by
``GetAppropriateDeviceID``) with ONE collective per gradient and no bucketing
(paddle/fluid/framework/details/multi_devices_graph_pass.cc:247,412-452,529;
all_reduce_op_handle.cc:99; reduce_op_handle.cc:155; broadcast_op_handle.cc:100).
The never-used ``FuseVarsOpHandle`` (details/fuse_vars_op_handle.cc:21-47) is the
seed of what is done here, MI355X-first:

* every trainable parameter is a view into ONE flat bf16 buffer, every gradient a
  view into ONE flat gradient buffer.  With ``grad_dtype=torch.float32`` (the
  default for bf16 models, Fleet's fp32 ``main_grad``) that buffer is fp32: the
  fused linear dW GEMMs accumulate into it directly and every other gradient
  is added by a post-accumulate hook, so micro-batch accumulation and the
  reduce-scatter never round through bf16; with ``grad_dtype=None`` it shares the
  parameter dtype and AccumulateGrad adds in place;
* parameters are laid out in reverse forward order, so gradients complete front
  to back during backward; the buffer is cut into buckets (default 256 MB, sized
  for the per-link bound of ring collectives over 7 point-to-point xGMI links);
* a bucket's **reduce-scatter** (ZeRO-1/2 == kReduce generalised) is issued on a
  dedicated HIP stream the moment its last gradient lands, overlapping backward;
* the fp32 master weights and Adam moments exist only for the rank's shard
  (12 B/param / W), updated by ONE fused gfx950 AdamW launch that also writes the
  bf16 parameter shard; an **all-gather** per bucket re-assembles parameters;
* no-weight-decay parameters (norm gains, biases) are placed at the end of the
  buffer so decay is a prefix of every shard (one kernel, no masks);
* global-norm clipping is computed on device (no host sync);
* with ``overlap_allgather`` the parameter all-gathers are issued on the comm
  stream in FORWARD order right after the AdamW launch and each bucket is waited
  for only when the next forward first touches one of its parameters (the fused
  ops call :func:`ops.fused.param_ready`), hiding the all-gather behind the next
  step's forward instead of exposing it after the optimizer.
"""
from __future__ import annotations

import contextlib
import math
import os

import torch

from ..ops import accum as _accum

from ..ops import fused
from ..autograd import tape as _tape
from ..ops import optim as fused_optim
from . import comm


def _no_decay(name, p):
    if getattr(p, "no_weight_decay", False):
        return True
    return p.dim() <= 1 and ("norm" in name or "bias" in name or "ln" in name)


class FlatShardedOptimizer:
    ALIGN = 128  # elements; every parameter view starts 256-B aligned

    def __init__(self, named_params, lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1,
                 group=None, bucket_mb=256, grad_clip=None, overlap=True, stage=1,
                 no_decay_fn=None, overlap_allgather=False, grad_dtype="auto", dp_comm=None,
                 overlap_update=None):
        named = [(n, p) for n, p in named_params if p.requires_grad]
        if not named:
            raise ValueError("no trainable parameters")
        self.group = group
        self.W = comm.get_world_size(group)
        self.r = comm.get_rank(group)
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.grad_clip = grad_clip
        self.stage = stage
        self.step_count = 0
        nd = no_decay_fn or _no_decay
        dev = named[0][1].device
        dt = named[0][1].dtype
        self.device, self.dtype = dev, dt
        if grad_dtype == "auto":
            grad_dtype = torch.float32 if dt in (torch.bfloat16, torch.float16) else dt
        self.grad_dtype = grad_dtype or dt
        # fp32 main-grad mode: gradients live outside p.grad (dtype differs from p)
        self.main_grad = self.grad_dtype != dt
        decay = [(n, p) for n, p in reversed(named) if not nd(n, p)]
        nodec = [(n, p) for n, p in reversed(named) if nd(n, p)]
        order = decay + nodec
        unit = self.W * 256
        bucket_elems = max(unit, int(bucket_mb * 2**20 / torch.empty((), dtype=self.grad_dtype).element_size()))
        # --- assign offsets and buckets
        offs, buckets = [], []
        off = 0
        bstart = 0
        self.decay_end = None
        for i, (n, p) in enumerate(order):
            if i == len(decay):
                self.decay_end = off
            off = (off + self.ALIGN - 1) // self.ALIGN * self.ALIGN
            offs.append(off)
            off += p.numel()
            if off - bstart >= bucket_elems or i == len(order) - 1:
                end = (off + unit - 1) // unit * unit
                buckets.append([bstart, end, []])
                bstart = off = end
        if self.decay_end is None:
            self.decay_end = off
        total = off
        self.total = total
        self.params = [p for _, p in order]
        self.names = [n for n, _ in order]
        self.offsets = offs
        # --- flat buffers; parameters/grads become views
        self.flat_param = torch.zeros(total, dtype=dt, device=dev)
        # FLAGS_dp_comm=direct: reduce-scatter / all-gather over IPC-mapped peer
        # buffers on the xGMI links (parallel/direct.py) instead of RCCL
        self.dp_comm = os.environ.get("FLAGS_dp_comm", "rccl") if dp_comm is None else dp_comm
        self._direct = None
        if self.dp_comm == "direct" and self.W > 1 and dev.type == "cuda":
            from .direct import DirectAllReduce

            ges = torch.empty((), dtype=self.grad_dtype).element_size()
            big = max(be - bs for bs, be, _ in buckets) * max(ges, self.flat_param.element_size())
            # FLAGS_dp_direct_inplace=1: the flat gradient itself lives in the registered
            # staging allocation, so every bucket's reduce-scatter reads it in place
            # (no copy-in pass over the gradients)
            inplace = os.environ.get("FLAGS_dp_direct_inplace", "0") == "1"
            self._direct = DirectAllReduce(group, max_bytes=big, extra_bytes=total * ges if inplace else 0)
        if self._direct is not None and self._direct.extra_bytes:
            self.flat_grad = self._direct.staging_tensor(total, self.grad_dtype)
            self.flat_grad.zero_()
        else:
            self.flat_grad = torch.zeros(total, dtype=self.grad_dtype, device=dev)
        self._bucket_of = {}
        bi = 0
        with torch.no_grad():
            for (n, p), o in zip(order, offs):
                while not (buckets[bi][0] <= o < buckets[bi][1]):
                    bi += 1
                buckets[bi][2].append(p)
                self._bucket_of[id(p)] = bi
                self.flat_param[o:o + p.numel()].copy_(p.data.reshape(-1))
                p.data = self.flat_param[o:o + p.numel()].view(p.shape)
                g = self.flat_grad[o:o + p.numel()].view(p.shape)
                if self.main_grad:
                    p.grad = None
                else:
                    p.grad = g
                # fused-GEMM gradient accumulation target (ops.linear)
                p._pa_main_grad = g
                p._pa_flat_off = o
                p._pa_grad_fresh = False
        self.buckets = buckets
        # --- shard layout: rank r owns slice r of every bucket
        self.shard_slices = []  # (bucket_start + r*L, L, shard_off)
        so = 0
        de = 0
        for bs, be, _ in buckets:
            L = (be - bs) // self.W
            s0 = bs + self.r * L
            self.shard_slices.append((s0, L, so))
            de += min(max(self.decay_end - s0, 0), L)
            so += L
        self.shard_size = so
        self.shard_decay_end = de
        if self.W == 1:
            self.grad_shard = self.flat_grad
            self.param_shard = self.flat_param
        else:
            self.grad_shard = torch.empty(so, dtype=self.grad_dtype, device=dev)
            self.param_shard = torch.empty(so, dtype=dt, device=dev)
        self.master = torch.empty(so, dtype=torch.float32, device=dev)
        for s0, L, sof in self.shard_slices:
            self.master[sof:sof + L].copy_(self.flat_param[s0:s0 + L])
        self.m = torch.zeros(so, dtype=torch.float32, device=dev)
        self.v = torch.zeros(so, dtype=torch.float32, device=dev)
        # --- overlap machinery
        self.overlap = overlap and self.W > 1 and dev.type == "cuda"
        from ..platform import device_context

        dc = device_context(dev) if dev.type == "cuda" else None
        self.comm_stream = ((dc.comm_stream if dc is not None else torch.cuda.Stream(device=dev))
                            if self.overlap else None)
        self._ready = [0] * len(buckets)
        self._launched = [False] * len(buckets)
        self._sync = True
        # deferred all-gathers: [(bucket, cuda event | deferred callable)] in issue order
        self.overlap_allgather = bool(overlap_allgather) and self.W > 1
        self._ag_queue = []
        # overlapped update (one rank): AdamW per bucket on a side stream, forward
        # order, each parameter's first read waits only for its own bucket -- the
        # bandwidth-bound update hides under the next forward's GEMMs
        if overlap_update is None:
            # opt-in: only the fused ops (ops/fused.py param_ready) and the framework
            # tape / eager engine honour the per-bucket waits; plain torch layers and
            # torch autograd would race the side stream
            overlap_update = os.environ.get("FLAGS_overlap_optimizer", "0") == "1"
        self.overlap_update = bool(overlap_update) and self.W == 1 and dev.type == "cuda"
        self.opt_stream = ((dc.aux_stream if dc is not None else torch.cuda.Stream(device=dev))
                           if self.overlap_update else None)
        self._keep = None
        self._hooks = []
        if self.W > 1 or self.main_grad:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
                # the framework tape (autograd/tape.py) fires these at the same point
                p._pa_grad_ready_hooks = [h for h in getattr(p, "_pa_grad_ready_hooks", ())
                                          if getattr(h, "__self__", None) is not self] + [self._on_grad]

    # ------------------------------------------------------------------ comm
    def no_sync(self):
        """Context manager: accumulate micro-batch gradients without communicating.
        Inside it, ops may also defer weight-gradient work to the step's last
        micro-batch (``ops/accum.py``: the experts' dW as one GEMM per step)."""
        opt = self

        class _Ctx:
            def __enter__(self_):
                opt._sync = False
                _accum.set_deferring(True)

            def __exit__(self_, exc_type, *a):
                _accum.set_deferring(False)
                if exc_type is not None:
                    _accum.discard()  # a failed micro-batch: its deferred dW operands are stale
                opt._sync = True
                opt._ready = [0] * len(opt.buckets)

        return _Ctx()

    def _on_grad(self, p):
        if self.main_grad and p.grad is not None:
            # autograd produced a bf16 gradient (non-fused op): fold it into fp32 main_grad
            g, mg = p.grad, p._pa_main_grad
            if (g.is_cuda and g.is_contiguous() and mg.is_contiguous() and g.numel() == mg.numel()
                    and g.dtype in (torch.bfloat16, torch.float32)):
                from ..ops import _native as N

                N.call("pa_fold_grad", N.dt(g), N.ptr(mg), N.ptr(g), g.numel(), int(p._pa_grad_fresh), N.stream())
            elif p._pa_grad_fresh:
                mg.copy_(g)
            else:
                mg.add_(g)
            p._pa_grad_fresh = False
            p.grad = None
        if self.W == 1 or not self._sync:
            return
        b = self._bucket_of[id(p)]
        self._ready[b] += 1
        if self._ready[b] == len(self.buckets[b][2]):
            self._launch(b)

    def _launch(self, b):
        if self._launched[b]:
            return
        self._launched[b] = True
        self._zero_untouched(b)
        if self.device.type == "cuda":
            fused.join_dw_streams(self.device)
        bs, be, _ = self.buckets[b]
        s0, L, so = self.shard_slices[b]
        rs = self._direct.reduce_scatter if self._direct is not None else \
            (lambda o, i: comm.reduce_scatter(o, i, self.group))
        if self.overlap:
            ev = torch.cuda.current_stream(self.device).record_event()
            self.comm_stream.wait_event(ev)
            with torch.cuda.stream(self.comm_stream):
                rs(self.grad_shard[so:so + L], self.flat_grad[bs:be])
        else:
            rs(self.grad_shard[so:so + L], self.flat_grad[bs:be])

    def _finish_comm(self):
        if self.W == 1:
            return
        for b in range(len(self.buckets)):
            if not self._launched[b]:
                self._launch(b)
        if self.overlap:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)
        self._launched = [False] * len(self.buckets)
        self._ready = [0] * len(self.buckets)

    # ------------------------------------------------------------------ step
    def _grad_scale_tensor(self):
        if not self.grad_clip:
            return None
        sq = fused_optim.sumsq(self.grad_shard)
        comm.all_reduce(sq, group=self.group)
        # gradients are sums over W ranks: norm = sqrt(sq) / W
        if sq.is_cuda:
            from ..ops import _native as N

            coef = torch.empty(1, dtype=torch.float32, device=sq.device)
            N.call("pa_clip_coef", N.ptr(sq), 1.0 / self.W, float(self.grad_clip), N.ptr(coef), N.stream())
            return coef
        norm = sq.sqrt() / self.W
        return torch.clamp(self.grad_clip / (norm + 1e-6), max=1.0)

    # ------------------------------------------------------------------ all-gather
    def _gather(self, b):
        bs, be, _ = self.buckets[b]
        s0, L, so = self.shard_slices[b]
        if self._direct is not None:
            self._direct.all_gather(self.flat_param[bs:be], self.param_shard[so:so + L])
        else:
            comm.all_gather(self.flat_param[bs:be], self.param_shard[so:so + L], self.group)

    def _issue_allgathers(self):
        """Queue every bucket's all-gather, forward order first (the last bucket
        holds the embedding, the norms and the first blocks), and mark its
        parameters pending.  On the GPU the gathers run on the comm stream now; on
        the CPU (gloo, tests) they are deferred until first use, which makes a
        missed wait show up as stale parameters."""
        cuda = self.overlap and self.comm_stream is not None
        if cuda:
            self.comm_stream.wait_event(torch.cuda.current_stream(self.device).record_event())
        for b in reversed(range(len(self.buckets))):
            if cuda:
                with torch.cuda.stream(self.comm_stream):
                    self._gather(b)
                h = self.comm_stream.record_event()
            else:
                h = b
            self._ag_queue.append((b, h))
            for p in self.buckets[b][2]:
                p._pa_pending = self._param_wait

    def _param_wait(self, p):
        self._wait_bucket(self._bucket_of[id(p)])

    def _wait_bucket(self, b=None):
        """Complete queued all-gathers up to and including bucket ``b`` (all if None)."""
        if not self._ag_queue:
            return
        last = None
        while self._ag_queue:
            bb, h = self._ag_queue.pop(0)
            if isinstance(h, int):
                self._gather(bb)          # deferred: every rank reaches this in the same order
            else:
                last = h
            for p in self.buckets[bb][2]:
                p._pa_pending = None
            if bb == b:
                break
        if last is not None:
            torch.cuda.current_stream(self.device).wait_event(last)

    def sync_params(self):
        """Make every parameter current (before reading them outside the fused ops,
        e.g. for a checkpoint or an evaluation with plain torch ops)."""
        self._wait_bucket(None)
        self._wait_update()

    def _wait_update(self):
        """The overlapped update also READS grad_shard / m / v / master on the side
        stream: any main-stream write to them must wait for it."""
        if self.opt_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.opt_stream)

    @torch.no_grad()
    def step(self, lr=None):
        if lr is not None:
            self.lr = lr
        _accum.flush()  # weight gradients still deferred (no final micro-batch came)
        if self._direct is not None:
            self._direct.poll_error()  # a peer timeout of the previous step raises here
        self.sync_params()
        if self.device.type == "cuda":
            fused.join_dw_streams(self.device)
        self._finish_fresh()
        self._finish_comm()
        self.step_count += 1
        gst = self._grad_scale_tensor()
        if self.overlap_update:
            self._update_overlapped(gst)
            return
        fused_optim.adamw_flat(self.master, self.grad_shard, self.m, self.v, lr=self.lr,
                               beta1=self.betas[0], beta2=self.betas[1], eps=self.eps,
                               weight_decay=self.wd, step=self.step_count, param_out=self.param_shard,
                               decay_end=self.shard_decay_end, grad_scale=1.0 / self.W,
                               grad_scale_tensor=gst)
        if self.W > 1:
            if self.overlap_allgather:
                self._issue_allgathers()
            else:
                for b in range(len(self.buckets)):
                    self._gather(b)
        if self._direct is not None:
            if self.overlap:
                # the gathers (and their barriers) may have been issued on the main
                # stream: the flag copy must come after them
                self.comm_stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.comm_stream) if self.overlap else contextlib.nullcontext():
                self._direct.error_async()
        fused.bump_weight_epoch()

    def _update_overlapped(self, gst):
        """One-rank step: the update of bucket b runs on ``opt_stream`` after the
        gradients are final, buckets in forward order; each parameter is marked
        pending on its bucket's event (fused.param_ready waits for it at first use),
        and the next reverse pass waits for all of them before it writes gradients."""
        main = torch.cuda.current_stream(self.device)
        self.opt_stream.wait_event(main.record_event())
        if gst is not None:
            gst.record_stream(self.opt_stream)
        self._keep = gst  # read on the side stream: alive until the next step
        for b in reversed(range(len(self.buckets))):
            s0, L, so = self.shard_slices[b]
            if L == 0:
                continue
            de = min(max(self.shard_decay_end - so, 0), L)
            with torch.cuda.stream(self.opt_stream):
                fused_optim.adamw_flat(self.master[so:so + L], self.grad_shard[s0:s0 + L], self.m[so:so + L],
                                       self.v[so:so + L], lr=self.lr, beta1=self.betas[0], beta2=self.betas[1],
                                       eps=self.eps, weight_decay=self.wd, step=self.step_count,
                                       param_out=self.param_shard[s0:s0 + L], decay_end=de, grad_scale=1.0,
                                       grad_scale_tensor=gst)
                ev = self.opt_stream.record_event()
            self._ag_queue.append((b, ev))
            for p in self.buckets[b][2]:
                p._pa_pending = self._param_wait
        _tape.before_next_backward(self.sync_params)
        fused.bump_weight_epoch()

    def zero_grad(self, set_to_none=False):
        _accum.discard()  # deferred dW of an abandoned accumulation must not leak into the next step
        if self.main_grad:
            # lazy zero: the first gradient write of the next step overwrites its
            # slice (fused dW GEMM with beta = 0, or copy_ in the hook); slices that
            # receive no gradient are zeroed in _finish_fresh() before they are read
            for p in self.params:
                p._pa_grad_fresh = True
            self._lazy_zero = True
            return
        self._wait_update()  # an overlapped update may still be reading flat_grad
        self.flat_grad.zero_()

    def _zero_untouched(self, b):
        """Zero the slices of bucket ``b`` that got no gradient this step (lazy zero)."""
        if not getattr(self, "_lazy_zero", False):
            return
        for p in self.buckets[b][2]:
            if p._pa_grad_fresh:
                o = p._pa_flat_off
                self.flat_grad[o:o + p.numel()].zero_()
                p._pa_grad_fresh = False

    def _finish_fresh(self):
        if not getattr(self, "_lazy_zero", False):
            return
        self._lazy_zero = False
        for p, o in zip(self.params, self.offsets):
            if p._pa_grad_fresh:
                self.flat_grad[o:o + p.numel()].zero_()
                p._pa_grad_fresh = False

    clear_grad = zero_grad

    def state_dict(self):
        self.sync_params()
        return {"master": self.master, "m": self.m, "v": self.v, "step": self.step_count,
                "lr": self.lr, "world": self.W, "rank": self.r}

    def set_state_dict(self, sd):
        self.sync_params()
        self.master.copy_(sd["master"])
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.step_count = int(sd["step"])
        self.lr = sd.get("lr", self.lr)
        with torch.no_grad():
            for s0, L, so in self.shard_slices:
                self.param_shard[so:so + L].copy_(self.master[so:so + L])
            if self.W > 1:
                for (bs, be, _), (s0, L, so) in zip(self.buckets, self.shard_slices):
                    comm.all_gather(self.flat_param[bs:be], self.param_shard[so:so + L], self.group)
        fused.bump_weight_epoch()

    def memory_bytes(self):
        es = self.flat_param.element_size()
        return {"flat_param": self.total * es, "flat_grad": self.total * self.flat_grad.element_size(),
                "optimizer_fp32": 3 * self.shard_size * 4}
