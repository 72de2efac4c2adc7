"""Parameter-server operators: send, recv, send_barrier, fetch_barrier, prefetch,
listen_and_serv, checkpoint_notify, gen_nccl_id, split_selected_rows_by_mod.

Parity: paddle/fluid/operators/{send,recv,send_barrier,fetch_barrier,prefetch,
listen_and_serv,checkpoint_notify,gen_nccl_id}_op.cc.
listen_and_serv keeps the reference's two loops (listen_and_serv_op.cc:102
RunSyncLoop, :178 RunAsyncLoop):

* sync: wait until every trainer sent its SEND_BARRIER (or completed) -> move the
  received ``<grad>.trainer_<k>`` variables into the scope -> run every optimize
  block (each sums the trainers' copies, scales by 1/Fanin and applies the
  optimizer op to its parameter block) -> publish the updated blocks and open the
  GET gate -> wait for every FETCH_BARRIER -> close the gate, next round.
* async: every received gradient immediately runs its own optimize block
  (``grad_to_block_id``) and the parameters stay published.
Sparse distributed tables (``lookup_table`` rows sharded id % n_pservers) are
updated row-wise from SelectedRows gradients and served to ``prefetch``.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..framework import core
from ..framework.registry import register_op


def _client():
    from ..distributed.ps import RPCClient

    return RPCClient.instance()


def _value(v):
    return v if isinstance(v, (core.LoDTensor, core.SelectedRows)) else core.LoDTensor(v)


@register_op("send", ["X*"], ["Out*?"], {"epmap": [], "sync_mode": True, "trainer_id": 0}, grad=None, no_infer=True)
def send(ctx):
    c = _client()
    names = ctx.op.input("X")
    suffix = f".trainer_{ctx.attr('trainer_id')}" if ctx.attr("sync_mode") else ""
    for name, val, ep in zip(names, ctx.input_values("X"), ctx.attr("epmap")):
        c.async_send_var(ep, name + suffix, _value(val))
    c.wait()


@register_op("recv", ["X*?"], ["Out*"], {"epmap": []}, grad=None, no_infer=True)
def recv(ctx):
    c = _client()
    names = ctx.op.output("Out")
    got = {}
    for i, (name, ep) in enumerate(zip(names, ctx.attr("epmap"))):
        c.async_get_var(ep, name, lambda v, i=i: got.__setitem__(i, v))
    c.wait()
    dev = ctx.device
    for i in range(len(names)):
        v = got[i]
        if isinstance(v, core.LoDTensor):
            v = core.LoDTensor(v.tensor.to(dev), v.lod())
        ctx.set_output("Out", v, i=i)


@register_op("send_barrier", ["X*?"], ["Out*?"], {"endpoints": [], "sync_mode": True}, grad=None, no_infer=True)
def send_barrier(ctx):
    if ctx.attr("sync_mode"):
        _client().barrier(ctx.attr("endpoints"), 0)


@register_op("fetch_barrier", ["X*?"], ["Out*?"], {"endpoints": []}, grad=None, no_infer=True)
def fetch_barrier(ctx):
    _client().barrier(ctx.attr("endpoints"), 1)


@register_op("prefetch", ["X*"], ["Out*"], {"epmap": [], "table_names": []}, grad=None, no_infer=True)
def prefetch(ctx):
    c = _client()
    for i, (ids, ep, tbl) in enumerate(zip(ctx.inputs("X"), ctx.attr("epmap"), ctx.attr("table_names"))):
        flat = ids.reshape(-1).long()
        rows = c.prefetch(ep, tbl, flat.cpu().numpy())
        width = rows.size // max(flat.numel(), 1) if flat.numel() else 0
        ctx.set_output("Out", torch.from_numpy(rows.reshape(flat.numel(), width).copy()).to(ctx.device), i=i)


@register_op("checkpoint_notify", ["X*?"], ["Out*?"], {"epmap": [], "dir": ""}, grad=None, no_infer=True)
def checkpoint_notify(ctx):
    _client().checkpoint_notify(ctx.attr("epmap"), ctx.attr("dir"))


@register_op("gen_nccl_id", [], ["NCCLID"], {"trainers": [], "trainer_id": 0}, grad=None, no_infer=True)
def gen_nccl_id(ctx):
    """The reference ships an ncclUniqueId from trainer 0 over gRPC; with RCCL the
    process group rendezvous is a TCP store, so the 'id' is trainer 0's endpoint."""
    eps = ctx.attr("trainers") or ["127.0.0.1:0"]
    ctx.set_output("NCCLID", core.LoDTensor(torch.tensor(list(eps[0].encode()), dtype=torch.uint8)))


@register_op("split_selected_rows_by_mod", ["X"], ["Out*"], {}, grad=None, no_infer=True)
def split_selected_rows_by_mod(ctx):
    """Sparse-table gradient -> one SelectedRows per pserver (rows with id % n == k,
    keeping global ids: the pserver's table is keyed by id)."""
    x = ctx.input_value("X")
    n = len(ctx.output_names("Out"))
    if not isinstance(x, core.SelectedRows):
        ctx.set_outputs("Out", [x] * n)
        return
    rows = torch.tensor(list(x.rows()), dtype=torch.int64)
    val = x.get_tensor().tensor
    outs = []
    for k in range(n):
        sel = torch.nonzero(rows % n == k).reshape(-1)
        o = core.SelectedRows(rows[sel].tolist(), x.height())
        o.get_tensor().set(val[sel.to(val.device)])
        outs.append(o)
    ctx.set_outputs("Out", outs)


# --------------------------------------------------------------- the server loop
def _publish(server, scope, names):
    for n in names:
        v = scope.find_var(n)
        if v is not None and v.get() is not None:
            server.publish(n, _value(v.get()))


def _store(scope, name, value):
    scope.var(name).set(value)


def _apply_sparse(scope, server, tables, name, value, lr_var, scale=1.0):
    """Row-wise SGD on a distributed table shard (the reference's sparse-table update);
    ``scale`` = 1/trainers in sync mode (gradient averaging, as for dense blocks)."""
    tbl = name.split("@GRAD")[0]
    if tbl not in tables:
        return False
    t = tables[tbl]
    lr = float(scope.find_var(lr_var).get().tensor.reshape(-1)[0]) if lr_var and scope.find_var(lr_var) else 0.01
    rows = list(value.rows())
    g = value.get_tensor().tensor.float().cpu().numpy()
    for r, grow in zip(rows, g):
        t.setdefault(r, np.zeros_like(grow))
        t[r] = t[r] - (lr * scale) * grow
    ids = np.array(list(t.keys()), np.int64)
    server.set_table(tbl, ids, np.stack([t[i] for i in ids]) if len(ids) else np.zeros((0, g.shape[1]), np.float32))
    return True


@register_op("listen_and_serv", ["X*?"], [],
             {"endpoint": "127.0.0.1:6174", "Fanin": 1, "sync_mode": True, "optimize_blocks": [],
              "grad_to_block_id": [], "param_names": [], "sparse_tables": [], "lr_var": "", "pserver_id": 0,
              "num_pservers": 1},
             grad=None, no_infer=True)
def listen_and_serv(ctx):
    from ..distributed.ps import RPCServer

    op, scope, exe = ctx.op, ctx.scope, ctx.executor
    ep = ctx.attr("endpoint")
    fanin = ctx.attr("Fanin")
    host, port = ep.rsplit(":", 1)
    server = RPCServer(int(port), fanin, host=os.environ.get("PADDLE_AMD_RPC_BIND", host))
    blocks = ctx.attr("optimize_blocks") or []
    prog = blocks[0].program if blocks else None
    g2b = dict(s.split(":", 1) for s in ctx.attr("grad_to_block_id"))
    params = list(ctx.attr("param_names"))
    lr_var = ctx.attr("lr_var")
    tables = {}
    for t in ctx.attr("sparse_tables"):
        tables[t] = {}
        v = scope.find_var(t)
        if v is not None and isinstance(v.get(), core.LoDTensor):  # dense init rows for ids % n == pserver_id
            init = v.get().tensor.float().cpu().numpy()
            n_ps = ctx.attr("num_pservers") or int(os.environ.get("PADDLE_PSERVERS_NUM", "1"))
            pid = ctx.attr("pserver_id")
            for i in range(pid, init.shape[0], n_ps):
                tables[t][i] = init[i].copy()
        if tables[t]:
            ids = np.array(list(tables[t].keys()), np.int64)
            server.set_table(t, ids, np.stack([tables[t][i] for i in ids]))
    _publish(server, scope, params)
    try:
        if ctx.attr("sync_mode"):
            server.set_ready(False)
            while True:
                done = server.wait(1)
                for name, val in server.pop_all():
                    if not _apply_sparse(scope, server, tables, name.split(".trainer_")[0], val, lr_var, 1.0 / fanin):
                        _store(scope, name, val)
                for d in server.pop_checkpoints():
                    from ..fluid import io as fio

                    fio.save_persistables(exe, d, op.block.program)
                if done == 1:
                    break
                for b in blocks:
                    exe.run_block(prog, b.idx, scope)
                _publish(server, scope, params)
                server.reset(1)
                server.set_ready(True)
                if server.wait(2) == 1:
                    break
                server.set_ready(False)
                server.reset(2)
        else:
            server.set_ready(True)
            while True:
                done = server.wait(3)
                for name, val in server.pop_all():
                    if _apply_sparse(scope, server, tables, name, val, lr_var):
                        continue
                    _store(scope, name, val)
                    bid = g2b.get(name)
                    if bid is not None and prog is not None:
                        exe.run_block(prog, int(bid), scope)
                        _publish(server, scope, params)
                if done == 1:
                    break
    finally:
        server.stop()
