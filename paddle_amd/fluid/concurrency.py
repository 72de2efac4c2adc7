"""CSP concurrency API (reference: python/paddle/fluid/concurrency.py -- ``Go``,
``make_channel``, ``channel_send``, ``channel_recv``, ``channel_close``,
``Select``).  Semantics of the runtime objects: operators/concurrency_ops.py."""
from __future__ import annotations

from ..framework import core
from . import unique_name
from .framework import Variable
from .layer_helper import LayerHelper
from .layers.control_flow import BlockGuard, ConditionalBlock
from .layers.tensor import fill_constant
from .layers.control_flow import equal

__all__ = ["Go", "make_channel", "channel_send", "channel_recv", "channel_close", "Select"]


class Go(BlockGuard):
    """``with fluid.Go(): ...`` -- run the block concurrently on a new thread."""

    def __init__(self, name=None):
        self.helper = LayerHelper("go", name=name)
        super().__init__(self.helper.main_program)

    def __exit__(self, exc_type, exc_val, exc_tb):
        if exc_type is not None:
            return False
        prog = self.helper.main_program
        go_block = prog.current_block()
        parent = prog.block(go_block.parent_idx)
        produced, reads = set(), []
        for op in go_block.ops:
            for n in op.input_arg_names:
                if n not in produced and n not in reads and parent._find_var_recursive(n) is not None:
                    reads.append(n)
            produced.update(op.output_arg_names)
        parent.append_op(type="go", inputs={"X": reads}, outputs={}, attrs={"sub_block": go_block})
        return super().__exit__(exc_type, exc_val, exc_tb)


def make_channel(dtype, capacity=0):
    helper = LayerHelper("channel_create", **locals())
    ch = helper.create_variable(name=unique_name.generate("channel"), type=core.VT.CHANNEL, persistable=True)
    helper.main_program.current_block().append_op(
        type="channel_create", outputs={"Out": ch},
        attrs={"data_type": core.convert_dtype(dtype) if isinstance(dtype, str) else dtype,
               "capacity": int(capacity)})
    return ch


def channel_send(channel, value, is_copy=False):
    helper = LayerHelper("channel_send", **locals())
    status = helper.create_variable(name=unique_name.generate("channel_send_status"), dtype=core.VT.BOOL)
    helper.main_program.current_block().append_op(
        type="channel_send", inputs={"Channel": channel, "X": value}, outputs={"Status": status},
        attrs={"is_copy": is_copy})
    return status


def channel_recv(channel, return_value):
    helper = LayerHelper("channel_recv", **locals())
    status = helper.create_variable(name=unique_name.generate("channel_recv_status"), dtype=core.VT.BOOL)
    helper.main_program.current_block().append_op(
        type="channel_recv", inputs={"Channel": channel}, outputs={"Out": return_value, "Status": status})
    return return_value, status


def channel_close(channel):
    helper = LayerHelper("channel_close", **locals())
    helper.main_program.current_block().append_op(type="channel_close", inputs={"Channel": channel})


class SelectCase:
    DEFAULT, SEND, RECEIVE = 0, 1, 2

    def __init__(self, select, idx, action, channel=None, value=None, is_copy=False):
        self.select = select
        self.idx = idx
        self.action = action
        self.channel = channel
        self.value = value
        if action == SelectCase.SEND and is_copy:
            blk = select.parent_block
            cp = blk.create_var(name=unique_name.generate(value.name + "_copy"), dtype=value.dtype,
                                shape=value.shape, lod_level=value.lod_level)
            blk.append_op(type="assign", inputs={"X": value}, outputs={"Out": cp})
            self.value = cp
        self._cb = None

    def __enter__(self):
        idx_var = fill_constant(shape=[1], dtype="int32", value=self.idx)
        cond = equal(self.select.case_to_execute, idx_var)
        self._cb = ConditionalBlock([cond], is_scalar_condition=True)
        self._ctx = self._cb.block()
        self._ctx.__enter__()
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        return self._ctx.__exit__(exc_type, exc_val, exc_tb)

    def serialize(self):
        ch = self.channel.name if self.channel is not None else ""
        val = self.value.name if isinstance(self.value, Variable) else ""
        return f"{self.idx},{self.action},{ch},{val}"


class Select(BlockGuard):
    """``with fluid.Select() as s: with s.case(fluid.channel_send, ch, x): ...``"""

    def __init__(self, name=None):
        self.helper = LayerHelper("select", name=name)
        self.parent_block = self.helper.main_program.current_block()
        self.cases = []
        super().__init__(self.helper.main_program)
        self.case_to_execute = fill_constant(shape=[1], dtype="int32", value=-1)

    def __enter__(self):
        super().__enter__()
        return self

    def case(self, channel_action_fn, channel, value, is_copy=False):
        act = SelectCase.SEND if channel_action_fn.__name__ == "channel_send" else SelectCase.RECEIVE
        c = SelectCase(self, len(self.cases), act, channel, value, is_copy)
        self.cases.append(c)
        return c

    def default(self):
        c = SelectCase(self, len(self.cases), SelectCase.DEFAULT)
        self.cases.append(c)
        return c

    def __exit__(self, exc_type, exc_val, exc_tb):
        if exc_type is not None:
            return False
        prog = self.helper.main_program
        sel_block = prog.current_block()
        parent = prog.block(sel_block.parent_idx)
        reads, outs = [], []
        for op in sel_block.ops:
            for n in op.input_arg_names:
                if parent._find_var_recursive(n) is not None and n not in reads:
                    reads.append(n)
            for n in op.output_arg_names:
                if parent._find_var_recursive(n) is not None and n not in outs:
                    outs.append(n)
        for c in self.cases:
            for v in (c.channel, c.value):
                if isinstance(v, Variable) and v.name not in reads:
                    reads.append(v.name)
        parent.append_op(type="select", inputs={"X": reads, "case_to_execute": [self.case_to_execute]},
                         outputs={"Out": outs},
                         attrs={"sub_block": sel_block, "cases": [c.serialize() for c in self.cases]})
        return super().__exit__(exc_type, exc_val, exc_tb)
