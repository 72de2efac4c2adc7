"""ParallelExecutor: data-parallel training of a fluid Program.

Reference: single process, one graph replica per GPU, an SSA-graph
scheduler, one ncclAllReduce per gradient (no bucketing), or Reduce+Broadcast
("kReduce", optimizer on the owner device), loss grad scaled by 1/#devices
(parallel_executor.cc:119-333, multi_devices_graph_pass.cc:320-700).

MI355X design: the primary mode is ONE PROCESS PER GPU (launch with
``python -m paddle_amd.distributed.launch`` / torchrun): each process holds one
replica on its HIP device and gradients are synchronised over RCCL (xGMI) with
bucketed flat all-reduces (fp32/bf16 buckets sized by FLAGS_rccl_bucket_mb).  The
single-process multi-place mode (several CUDAPlaces or CPU_NUM CPU places) is kept
for API parity: replicas run on their own devices and gradients are reduced on
device 0 and broadcast.  Both can combine (places x processes).

Step = [forward+backward ops on every replica] -> gradient sync (AllReduce: sum,
scaled by 1/N; Reduce: reduce to the size-balanced owner replica) -> [optimizer
ops] (AllReduce: every replica; Reduce: owner replica, then parameter broadcast).
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from ..framework import core
from ..framework import registry as R
from ..framework.executor import BlockExecutor
from ..parallel import comm
from ..utils import flags as FLAGS
from .executor import _to_lod_tensor, as_numpy, global_scope
from .framework import Program, Variable, default_main_program


class ExecutionStrategy:
    """details/execution_strategy.h:22."""

    class ExecutorType:
        Default = 0
        Experimental = 1

    def __init__(self):
        self.num_threads = 0
        self.use_cuda = True
        self.allow_op_delay = False
        self.num_iteration_per_drop_scope = 100
        self.type = ExecutionStrategy.ExecutorType.Default
        self.use_experimental_executor = False


class BuildStrategy:
    """details/build_strategy.h:23-58."""

    class ReduceStrategy:
        AllReduce = 0
        Reduce = 1

    class GradientScaleStrategy:
        CoeffNumDevice = 0
        One = 1
        Customized = 2

    def __init__(self):
        self.reduce_strategy = BuildStrategy.ReduceStrategy.AllReduce
        self.gradient_scale_strategy = BuildStrategy.GradientScaleStrategy.CoeffNumDevice
        self.debug_graphviz_path = ""
        self.enable_data_balance = False
        self.fuse_elewise_add_act_ops = False
        self.fuse_all_reduce_ops = True
        self.memory_optimize = False


def _op_role(op):
    return int(op.attrs.get(R.OP_ROLE_ATTR, 0))


def _is_optimize(op):
    r = _op_role(op)
    return (r & 0xFF) == R.OpRole.Optimize or (r & 0xFF) == R.OpRole.RPC


def _sub_program(program, ops):
    p = program.clone()
    keep = set(id(o) for o in ops)
    src = program.global_block().ops
    p.global_block().ops = [nop for nop, op in zip(p.global_block().ops, src) if id(op) in keep]
    return p


class ParallelExecutor:
    def __init__(self, use_cuda, loss_name=None, main_program=None, share_vars_from=None, exec_strategy=None,
                 build_strategy=None, num_trainers=1, trainer_id=0, scope=None, **kwargs):
        self._rank, self._world = comm.get_rank(), comm.get_world_size()
        if self._world > 1:
            places = [core.CUDAPlace(torch.cuda.current_device())] if use_cuda else [core.CPUPlace()]
        elif use_cuda:
            ids = os.environ.get("CUDA_VISIBLE_DEVICES") or os.environ.get("HIP_VISIBLE_DEVICES")
            n = len(ids.split(",")) if ids else core.get_cuda_device_count()
            places = [core.CUDAPlace(i) for i in range(max(1, n))]
        else:
            n = int(os.environ.get("CPU_NUM", max(1, min(4, os.cpu_count() or 1))))
            places = [core.CPUPlace() for _ in range(n)]
        self._places = places
        self._exec_strategy = exec_strategy or ExecutionStrategy()
        self._build_strategy = build_strategy or BuildStrategy()
        self._program = main_program or default_main_program()
        self._loss_name = loss_name
        self._scope = scope or global_scope()
        self._local_scopes = [self._scope] + [self._scope.new_scope() for _ in places[1:]]
        if share_vars_from is not None:
            self._local_scopes = [share_vars_from._local_scopes[0]] + self._local_scopes[1:]
        self._executors = [BlockExecutor(p) for p in places]
        ops = self._program.global_block().ops
        self._fb_ops = [op for op in ops if not _is_optimize(op)]
        self._opt_ops = [op for op in ops if _is_optimize(op)]
        self._fb_prog = _sub_program(self._program, self._fb_ops)
        self._opt_prog = _sub_program(self._program, self._opt_ops)
        # (param, grad) pairs from op_role_var of backward ops
        self._param_grads = []
        seen = set()
        for op in self._fb_ops:
            rv = op.attrs.get(R.OP_ROLE_VAR_ATTR)
            if rv and len(rv) >= 2 and (_op_role(op) & R.OpRole.Backward):
                for i in range(0, len(rv) - 1, 2):
                    if rv[i + 1] not in seen:
                        seen.add(rv[i + 1])
                        self._param_grads.append((rv[i], rv[i + 1]))
        self._owners = self._balance_owners()
        self._persistables = [v.name for v in self._program.list_vars() if v.persistable and
                              v.type not in (core.VT.FEED_MINIBATCH, core.VT.FETCH_LIST, core.VT.RAW)]
        self._bcast_params()
        self._step = 0

    # ---- helpers
    def _balance_owners(self):
        """GetAppropriateDeviceID: assign each param to the least-loaded replica by numel."""
        load = [0] * len(self._places)
        owners = {}
        gb = self._program.global_block()
        for p, g in self._param_grads:
            v = gb._find_var_recursive(p)
            n = int(np.prod([abs(s) for s in v.shape])) if v is not None and v.shape else 1
            i = int(np.argmin(load))
            owners[p] = i
            load[i] += n
        return owners

    def _bcast_params(self):
        """BCastParamsToDevices: copy persistables of replica 0 (and rank 0) to all replicas."""
        src = self._local_scopes[0]
        for name in self._persistables:
            v = src.find_var(name)
            if v is None or not isinstance(v.get(), core.LoDTensor) or v.get().tensor is None:
                continue
            t = v.get().tensor
            if self._world > 1:
                comm.broadcast(t, 0)
            for s, pl in zip(self._local_scopes[1:], self._places[1:]):
                s.var(name).set(core.LoDTensor(t.to(pl.torch_device()).clone(), v.get().lod()))

    def bcast_params(self):
        self._bcast_params()

    @property
    def device_count(self):
        return len(self._places) * self._world

    def _split_feed(self, feed):
        n = len(self._places)
        if isinstance(feed, list):
            return feed
        out = [dict() for _ in range(n)]
        for k, v in feed.items():
            arr = v.tensor if isinstance(v, core.LoDTensor) else (v if isinstance(v, torch.Tensor)
                                                                  else torch.from_numpy(np.asarray(v)))
            lod = v.lod() if isinstance(v, core.LoDTensor) else []
            if n == 1:
                out[0][k] = core.LoDTensor(arr, lod)
                continue
            if lod:
                off = lod[0]
                nseq = len(off) - 1
                per = math.ceil(nseq / n)
                for i in range(n):
                    a, b = min(i * per, nseq), min((i + 1) * per, nseq)
                    sub = [o - off[a] for o in off[a:b + 1]]
                    out[i][k] = core.LoDTensor(arr[off[a]:off[b]], [sub])
            else:
                for i, c in enumerate(torch.chunk(arr, n, 0)):
                    out[i][k] = core.LoDTensor(c)
        return out

    def _grads(self, scope, names):
        res = []
        for g in names:
            v = scope.find_var(g)
            res.append(v.get() if v is not None else None)
        return res

    def _sync_grads(self):
        bs = self._build_strategy
        n_total = self.device_count
        scale = 1.0 / n_total if bs.gradient_scale_strategy == BuildStrategy.GradientScaleStrategy.CoeffNumDevice \
            else 1.0
        names = [g for _, g in self._param_grads]
        per_rep = [self._grads(s, names) for s in self._local_scopes]
        dense_idx = [i for i, v in enumerate(per_rep[0]) if isinstance(v, core.LoDTensor) and v.tensor is not None]
        sparse_idx = [i for i, v in enumerate(per_rep[0]) if isinstance(v, core.SelectedRows)]
        dev0 = self._places[0].torch_device()
        # 1) in-process reduction onto replica 0
        summed = []
        for i in dense_idx:
            t = per_rep[0][i].tensor.clone() if len(self._places) > 1 else per_rep[0][i].tensor
            for r in range(1, len(self._places)):
                t = t + per_rep[r][i].tensor.to(dev0)
            summed.append(t)
        # 2) cross-process bucketed all-reduce over RCCL
        if self._world > 1 and summed:
            bucket = FLAGS.get("rccl_bucket_mb") * (1 << 20)
            groups, cur, cur_b = [], [], 0
            for t in summed:
                cur.append(t)
                cur_b += t.numel() * t.element_size()
                if cur_b >= bucket:
                    groups.append(cur)
                    cur, cur_b = [], 0
            if cur:
                groups.append(cur)
            for grp in groups:
                flat = torch.cat([t.reshape(-1).float() for t in grp])
                comm.all_reduce(flat)
                off = 0
                for t in grp:
                    n = t.numel()
                    t.copy_(flat[off:off + n].view_as(t))
                    off += n
        # 3) sparse grads: gather rows (reference: SelectedRows to device 0, then broadcast)
        for i in sparse_idx:
            rows, vals = [], []
            for r in range(len(self._places)):
                sr = per_rep[r][i]
                rows += sr.rows()
                vals.append(sr.get_tensor().tensor.to(dev0))
            merged = core.SelectedRows(rows, per_rep[0][i].height(), torch.cat(vals, 0) * scale)
            for s in self._local_scopes:
                s.var(names[i]).set(merged)
        # 4) scale + write back
        reduce_mode = bs.reduce_strategy == BuildStrategy.ReduceStrategy.Reduce
        for k, i in enumerate(dense_idx):
            t = summed[k] * scale if scale != 1.0 else summed[k]
            lod = per_rep[0][i].lod()
            p_name = self._param_grads[i][0]
            for r, (s, pl) in enumerate(zip(self._local_scopes, self._places)):
                if reduce_mode and r != self._owners.get(p_name, 0):
                    continue
                s.var(names[i]).set(core.LoDTensor(t if r == 0 else t.to(pl.torch_device()), lod))

    def run(self, fetch_list, feed=None, feed_dict=None, return_numpy=True):
        if feed is None and feed_dict is not None:
            feed = feed_dict
        feed = feed or {}
        fetch_names = [v.name if isinstance(v, Variable) else v for v in fetch_list]
        feeds = self._split_feed(feed)
        for s, ex, fd in zip(self._local_scopes, self._executors, feeds):
            for k, v in fd.items():
                s.var(k).set(_to_lod_tensor(v, ex.place))
            ex.run_block(self._fb_prog, 0, s)
        if self.device_count > 1:
            self._sync_grads()
        if self._build_strategy.reduce_strategy == BuildStrategy.ReduceStrategy.Reduce and len(self._places) > 1:
            owner_ops = {}
            for op in self._opt_ops:
                rv = op.attrs.get(R.OP_ROLE_VAR_ATTR) or []
                owner_ops.setdefault(self._owners.get(rv[0], 0) if rv else 0, []).append(op)
            for r, (s, ex) in enumerate(zip(self._local_scopes, self._executors)):
                ops = owner_ops.get(r, [])
                if ops:
                    ex.run_block(_sub_program(self._program, ops), 0, s)
            # broadcast updated params from owners
            for p, _ in self._param_grads:
                o = self._owners.get(p, 0)
                src = self._local_scopes[o].find_var(p).get()
                for r, (s, pl) in enumerate(zip(self._local_scopes, self._places)):
                    if r != o:
                        s.var(p).set(core.LoDTensor(src.tensor.to(pl.torch_device()), src.lod()))
        else:
            for s, ex in zip(self._local_scopes, self._executors):
                ex.run_block(self._opt_prog, 0, s)
        self._step += 1
        if self._step % max(1, self._exec_strategy.num_iteration_per_drop_scope) == 0:
            for s in self._local_scopes:
                s.drop_kids()
        outs = []
        for n in fetch_names:
            parts = []
            for s in self._local_scopes:
                v = s.find_var(n)
                if v is not None and isinstance(v.get(), core.LoDTensor):
                    parts.append(v.get().tensor.detach().to("cpu"))
            if not parts:
                outs.append(None)
                continue
            t = torch.cat([p.reshape(1) if p.dim() == 0 else p for p in parts], 0)
            outs.append(t.float().numpy() if return_numpy and t.dtype == torch.bfloat16 else
                        (t.numpy() if return_numpy else core.LoDTensor(t)))
        return outs

    def drop_local_exe_scopes(self):
        for s in self._local_scopes:
            s.drop_kids()
