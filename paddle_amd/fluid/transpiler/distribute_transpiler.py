"""DistributeTranspiler: parameter-server data parallelism (sync / async) with
sliced parameters and a distributed (id-sharded) lookup table.

Reference: python/paddle/fluid/transpiler/distribute_transpiler.py:132-1500.
Behaviour kept: parameters (and their gradients) are cut into row blocks of at
least ``min_block_size`` elements (at most one block per pserver), blocks are
assigned by the ``split_method`` dispatcher (RoundRobin / HashName), the trainer
program loses its optimize ops and instead ``split_byref``s gradients,
``send``s them, ``send_barrier``s, ``recv``s the parameter blocks,
``fetch_barrier``s and ``concat``s them back; each pserver program runs a
``listen_and_serv`` whose optimize sub-blocks sum the trainers' gradient copies,
scale by 1/trainers (sync mode) and apply the ORIGINAL optimizer ops (SGD,
Momentum, Adam ... with their accumulators sliced the same way).
``embedding(is_distributed=True)`` tables become ``split_ids`` -> ``prefetch`` ->
``merge_ids`` on trainers, with the table rows held (id % n_pservers) on the
pservers and updated from sparse gradients.

MI355X-era design notes: the transport is the native TCP RPC
(csrc/runtime/rpc.cc), and the pserver start-up runs the trainers' own
initialisers on full shapes before slicing (split_byref), so a transpiled job
starts bit-identical to single-process training.
"""
from __future__ import annotations

import math

from ...framework.registry import OP_ROLE_ATTR, OP_ROLE_VAR_ATTR, OpRole
from ..framework import Program, default_main_program, default_startup_program
from .ps_dispatcher import RoundRobin


class DistributeTranspilerConfig:
    slice_var_up = True
    split_method = RoundRobin
    min_block_size = 8192


def _numel(shape):
    return int(math.prod(int(abs(s)) for s in shape))


def slice_variable(var_list, slice_count, min_block_size):
    """[(var_name, block_id, rows)] -- row blocks of >= min_block_size elements."""
    out = []
    for v in var_list:
        n = _numel(v.shape)
        row = _numel(v.shape[1:]) if len(v.shape) > 1 else 1
        parts = max(1, min(slice_count, n // max(min_block_size, 1)))
        rows_total = int(v.shape[0])
        rows_per = int(math.ceil(rows_total / parts))
        parts = int(math.ceil(rows_total / rows_per))
        for b in range(parts):
            out.append((v.name, b, min(rows_per, rows_total - b * rows_per)))
    return out


class DistributeTranspiler:
    def __init__(self, config=None):
        self.config = config or DistributeTranspilerConfig()

    # ------------------------------------------------------------------ analysis
    def transpile(self, trainer_id, program=None, pservers="127.0.0.1:6174", trainers=1, sync_mode=True,
                  startup_program=None):
        self.trainer_id, self.trainer_num, self.sync_mode = trainer_id, int(trainers), sync_mode
        self.origin_program = program or default_main_program()
        self.origin_startup = startup_program or default_startup_program()
        self.pserver_endpoints = [e.strip() for e in pservers.split(",") if e.strip()]
        gb = self.origin_program.global_block()

        # optimize ops grouped by the parameter they update (op_role_var = [param, grad])
        self.opt_ops, self.params_grads, self.lr_ops = [], [], []
        seen = set()
        for op in gb.ops:
            role = int(op.attrs.get(OP_ROLE_ATTR, 0))
            if role & OpRole.Optimize:
                self.opt_ops.append(op)
                rv = op.attrs.get(OP_ROLE_VAR_ATTR) or []
                if len(rv) >= 2 and rv[0] not in seen:
                    seen.add(rv[0])
                    self.params_grads.append((gb.var(rv[0]), gb.var(rv[1])))
            elif role & OpRole.LRSched:
                self.lr_ops.append(op)
        # distributed lookup tables (embedding(is_distributed=True))
        self.tables = sorted({op.input("W")[0] for op in gb.ops
                              if op.type == "lookup_table" and op.attrs.get("is_distributed")})
        self.params_grads = [(p, g) for p, g in self.params_grads if p.name not in self.tables]
        self.table_grads = {t: t + "@GRAD" for t in self.tables}
        self.lr_var = None
        for op in self.opt_ops:
            if "LearningRate" in op.inputs and op.input("LearningRate"):
                self.lr_var = op.input("LearningRate")[0]
                break

        # param / grad blocks -> endpoints
        n = len(self.pserver_endpoints) if self.config.slice_var_up else 1
        pblocks = slice_variable([p for p, _ in self.params_grads], n, self.config.min_block_size)
        self.blocks = {}  # param -> [(block_var_name, grad_block_name, rows, endpoint)]
        disp = self.config.split_method(self.pserver_endpoints)
        eps = disp.dispatch([f"{name}.block{b}" for name, b, _ in pblocks])
        grad_of = {p.name: g.name for p, g in self.params_grads}
        counts = {}
        for name, _, _ in pblocks:
            counts[name] = counts.get(name, 0) + 1
        for (name, b, rows), ep in zip(pblocks, eps):
            single = counts[name] == 1
            pn = name if single else f"{name}.block{b}"
            gn = grad_of[name] if single else f"{grad_of[name]}.block{b}"
            self.blocks.setdefault(name, []).append((pn, gn, rows, ep))
        self._rewrite_trainer()
        return self

    # ------------------------------------------------------------------ trainer
    def _rewrite_trainer(self):
        prog = self.origin_program
        gb = prog.global_block()
        opt_ids = {id(o) for o in self.opt_ops} | {id(o) for o in self.lr_ops}
        gb.ops = [o for o in gb.ops if id(o) not in opt_ids]
        self._rewrite_tables(gb)
        send_vars, send_eps = [], []
        recv_vars, recv_eps, concats = [], [], []
        for p, g in self.params_grads:
            blks = self.blocks[p.name]
            if len(blks) > 1:
                outs = []
                for pn, gn, rows, ep in blks:
                    gb.create_var(name=gn, shape=[rows] + list(g.shape[1:]), dtype=g.dtype, persistable=False)
                    gb.create_var(name=pn, shape=[rows] + list(p.shape[1:]), dtype=p.dtype, persistable=False)
                    outs.append(gn)
                gb.append_op(type="split_byref", inputs={"X": [g.name]}, outputs={"Out": outs},
                             attrs={"sections": [b[2] for b in blks], OP_ROLE_ATTR: OpRole.RPC})
                concats.append((p.name, [b[0] for b in blks]))
            for pn, gn, rows, ep in blks:
                send_vars.append(gn)
                send_eps.append(ep)
                recv_vars.append(pn)
                recv_eps.append(ep)
        for t in self.tables:  # sparse table gradients: one shard per pserver (ids % n)
            tg = self.table_grads[t]
            shards = [f"{tg}.pserver{k}" for k in range(len(self.pserver_endpoints))]
            for s in shards:
                gb.create_var(name=s, dtype=gb.var(t).dtype)
            gb.append_op(type="split_selected_rows_by_mod", inputs={"X": [tg]}, outputs={"Out": shards},
                         attrs={OP_ROLE_ATTR: OpRole.RPC})
            for k, s in enumerate(shards):
                send_vars.append(s)
                send_eps.append(self.pserver_endpoints[k])
        rpc = {OP_ROLE_ATTR: OpRole.RPC}
        gb.append_op(type="send", inputs={"X": send_vars}, outputs={},
                     attrs=dict(rpc, epmap=send_eps, sync_mode=self.sync_mode, trainer_id=self.trainer_id))
        gb.append_op(type="send_barrier", inputs={}, outputs={},
                     attrs=dict(rpc, endpoints=self.pserver_endpoints, sync_mode=self.sync_mode))
        if recv_vars:
            gb.append_op(type="recv", inputs={}, outputs={"Out": recv_vars}, attrs=dict(rpc, epmap=recv_eps))
        if self.sync_mode:
            gb.append_op(type="fetch_barrier", inputs={}, outputs={},
                         attrs=dict(rpc, endpoints=self.pserver_endpoints))
        for pname, parts in concats:
            gb.append_op(type="concat", inputs={"X": parts}, outputs={"Out": [pname]}, attrs=dict(rpc, axis=0))

    def _rewrite_tables(self, gb):
        if not self.tables:
            return
        n = len(self.pserver_endpoints)
        new_ops = []
        for op in gb.ops:
            if op.type == "lookup_table" and op.input("W")[0] in self.tables:
                t = op.input("W")[0]
                ids, out = op.input("Ids")[0], op.output("Out")[0]
                shards = [f"{ids}.shard{k}" for k in range(n)]
                embs = [f"{out}.shard{k}" for k in range(n)]
                for s in shards:
                    gb.create_var(name=s, dtype="int64")
                for e in embs:
                    gb.create_var(name=e, dtype=gb.var(t).dtype)
                from ..framework import Operator

                new_ops.append(Operator(gb, None, type="split_ids", inputs={"Ids": [ids]}, outputs={"Out": shards}))
                new_ops.append(Operator(gb, None, type="prefetch", inputs={"X": shards}, outputs={"Out": embs},
                                        attrs={"epmap": self.pserver_endpoints, "table_names": [t] * n}))
                new_ops.append(Operator(gb, None, type="merge_ids", inputs={"Ids": [ids], "X": embs},
                                        outputs={"Out": [out]}))
            else:
                new_ops.append(op)
        gb.ops = new_ops

    def get_trainer_program(self, wait_port=True):
        return self.origin_program

    # ------------------------------------------------------------------ pserver
    def _accumulators(self, op, pname):
        """(slot, var) of the optimizer op's per-parameter state (not Param/Grad/LR)."""
        skip = {"Param", "Grad", "LearningRate"}
        out = []
        for slot, names in op.inputs.items():
            if slot in skip:
                continue
            for n in names:
                out.append((slot, n))
        return out

    def get_pserver_program(self, endpoint):
        gb0 = self.origin_program.global_block()
        prog = Program()
        gb = prog.global_block()
        n_tr = self.trainer_num
        my_blocks = [(p, g, blk) for p, g in self.params_grads for blk in self.blocks[p.name] if blk[3] == endpoint]
        if self.lr_var:
            lv = gb0.var(self.lr_var)
            gb.create_var(name=lv.name, shape=lv.shape, dtype=lv.dtype, persistable=True)
        optimize_blocks, g2b, publish = [], [], []
        param_ops = {}
        for op in self.opt_ops:
            rv = op.attrs.get(OP_ROLE_VAR_ATTR) or []
            if rv:
                param_ops.setdefault(rv[0], []).append(op)
        self._acc_plan = []  # (full_acc_name, block_acc_name, rows or None) for the startup program
        if self.lr_ops:  # learning-rate schedule runs once per round, before the optimize blocks
            blk = prog.create_block(0)
            for op in self.lr_ops:
                for names in list(op.inputs.values()) + list(op.outputs.values()):
                    for x in names:
                        ov = gb0._find_var_recursive(x)
                        if ov is not None and not gb.has_var(x):
                            gb.create_var(name=x, shape=ov.shape, dtype=ov.dtype, persistable=ov.persistable)
                blk.append_op(type=op.type, inputs=dict(op.inputs), outputs=dict(op.outputs), attrs=dict(op.attrs))
            prog.rollback()
            optimize_blocks.append(blk)
        for p, g, (pn, gn, rows, ep) in my_blocks:
            gb.create_var(name=pn, shape=[rows] + list(p.shape[1:]), dtype=p.dtype, persistable=True)
            gshape = [rows] + list(p.shape[1:])
            merged = gb.create_var(name=gn, shape=gshape, dtype=g.dtype)
            copies = []
            for k in range(n_tr if self.sync_mode else 1):
                cn = f"{gn}.trainer_{k}" if self.sync_mode else gn
                if cn != gn:
                    gb.create_var(name=cn, shape=gshape, dtype=g.dtype)
                copies.append(cn)
            blk = prog.create_block(0)
            if self.sync_mode:
                blk.append_op(type="sum", inputs={"X": copies}, outputs={"Out": [gn]})
                blk.append_op(type="scale", inputs={"X": [gn]}, outputs={"Out": [gn]},
                              attrs={"scale": 1.0 / n_tr})
            rename = {p.name: pn, g.name: gn}
            for op in param_ops.get(p.name, []):
                for slot, an in self._accumulators(op, p.name):
                    if an in rename:
                        continue
                    av = gb0.var(an)
                    same = list(av.shape) == list(p.shape)
                    bn = f"{an}.{pn}" if pn != p.name else an
                    gb.create_var(name=bn, shape=gshape if same else av.shape, dtype=av.dtype, persistable=True)
                    rename[an] = bn
                    self._acc_plan.append((an, bn, p.name if same else None))
                ins = {s: [rename.get(x, x) for x in v] for s, v in op.inputs.items()}
                outs = {s: [rename.get(x, x) for x in v] for s, v in op.outputs.items()}
                for s, v in list(ins.items()) + list(outs.items()):
                    for x in v:
                        if not blk._find_var_recursive(x) and gb0._find_var_recursive(x) is not None:
                            ov = gb0.var(x)
                            gb.create_var(name=x, shape=ov.shape, dtype=ov.dtype, persistable=ov.persistable)
                attrs = {k: v for k, v in op.attrs.items() if k not in (OP_ROLE_VAR_ATTR,)}
                blk.append_op(type=op.type, inputs=ins, outputs=outs, attrs=attrs)
            prog.rollback()
            optimize_blocks.append(blk)
            g2b += [f"{c}:{blk.idx}" for c in copies]
            publish.append(pn)
        for t in self.tables:
            tv = gb0.var(t)
            gb.create_var(name=t, shape=tv.shape, dtype=tv.dtype, persistable=True)
        self._my_blocks = my_blocks
        gb.append_op(type="listen_and_serv", inputs={}, outputs={},
                     attrs={"endpoint": endpoint, "Fanin": n_tr, "sync_mode": self.sync_mode,
                            "optimize_blocks": optimize_blocks, "grad_to_block_id": g2b, "param_names": publish,
                            "sparse_tables": self.tables, "lr_var": self.lr_var or "",
                            "pserver_id": self.pserver_endpoints.index(endpoint),
                            "num_pservers": len(self.pserver_endpoints), OP_ROLE_ATTR: OpRole.RPC})
        return prog

    def get_startup_program(self, endpoint, pserver_program=None, startup_program=None):
        """Run the trainers' own initialisers on full shapes, then slice out this
        pserver's blocks (identical initial values on every process)."""
        if pserver_program is None:
            pserver_program = self.get_pserver_program(endpoint)
        src = startup_program or self.origin_startup
        sp = src.clone()
        gb = sp.global_block()
        for p, g, (pn, gn, rows, ep) in self._my_blocks:
            if pn == p.name:
                continue
            blks = self.blocks[p.name]
            outs = []
            for bpn, _, brows, _ in blks:
                if not gb.has_var(bpn):
                    gb.create_var(name=bpn, shape=[brows] + list(p.shape[1:]), dtype=p.dtype, persistable=True)
                outs.append(bpn)
            gb.append_op(type="split_byref", inputs={"X": [p.name]}, outputs={"Out": outs},
                         attrs={"sections": [b[2] for b in blks]})
        for full, bn, pname in self._acc_plan:
            if bn == full:
                continue
            if pname is None:  # scalar state (beta pow): every block starts from the same value
                v = self.origin_program.global_block().var(full)
                if not gb.has_var(bn):
                    gb.create_var(name=bn, shape=v.shape, dtype=v.dtype, persistable=True)
                gb.append_op(type="assign", inputs={"X": [full]}, outputs={"Out": [bn]})
            else:
                blks = self.blocks[pname]
                outs = []
                for bpn, _, brows, _ in blks:
                    o = f"{full}.{bpn}"
                    if not gb.has_var(o):
                        v = self.origin_program.global_block().var(full)
                        gb.create_var(name=o, shape=[brows] + list(v.shape[1:]), dtype=v.dtype, persistable=True)
                    outs.append(o)
                gb.append_op(type="split_byref", inputs={"X": [full]}, outputs={"Out": outs},
                             attrs={"sections": [b[2] for b in blks]})
        return sp

    def get_pserver_programs(self, endpoint):
        main = self.get_pserver_program(endpoint)
        return main, self.get_startup_program(endpoint, main)
