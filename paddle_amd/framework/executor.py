"""Block interpreter (the reference's framework::Executor, executor.cc:125-353).

Differences from the reference, MI355X-first:
  * ops are "prepared" once per (program, block, version) -- kernel lookup, slot
    lists and plain attrs are resolved ahead of time (the reference re-creates
    every op on each ``Run``, executor.cc:294);
  * kernels enqueue on torch's current HIP stream, so a whole block replays
    asynchronously; the only host sync is the fetch;
  * ``FLAGS_check_nan_inf`` / ``FLAGS_benchmark`` keep their reference meaning
    (operator.cc:726-736, 722);
  * control-flow kernels (while / conditional_block / recurrent) re-enter the
    interpreter on a sub-block through ``ctx.executor``.
"""
from __future__ import annotations

import contextlib
import os
import threading

import torch

from ..utils import flags as FLAGS
from ..utils import profiler as prof
from ..utils import stack_trace as _stack_trace


def _traced(run, name):
    def f(info, ctx):
        with _stack_trace.frame(name):
            return run(info, ctx)
    return f
from ..utils import strict as _strict
from . import core
from . import registry as R
from .. import platform as _platform

_LOG_MEM = os.environ.get("FLAGS_log_memory_stats") == "1"


class PreparedBlock:
    def __init__(self, program, block_idx):
        self.program = program
        self.block = program.block(block_idx)
        self.steps = []
        for op in self.block.ops:
            info = R.get_op_info(op.type)
            attrs = {}
            for k, v in op.attrs.items():
                attrs[k] = v
            ins = [(slot, list(names)) for slot, names in op.inputs.items()]
            outs = {slot: list(names) for slot, names in op.outputs.items()}
            self.steps.append((info, op, ins, outs, attrs))
        # forward ops whose auto-VJP grad op is in this program keep their graph
        # (registry.run_kernel_stash) so backward does not re-run them
        grads = _program_grad_types(program)
        self.stash = [FLAGS.get("stash_forward") and (op.type + "_grad") in grads
                      and R.is_auto_grad(op.type + "_grad") for _, op, _, _, _ in self.steps]


_TLS = threading.local()


@contextlib.contextmanager
def no_stash():
    """Run nested blocks without detaching stashed outputs: an op whose kernel
    executes a sub-block (recurrent, parallel_do) is differentiated as a whole by
    its auto-VJP, which needs the autograd graph through the inner ops."""
    prev = getattr(_TLS, "off", False)
    _TLS.off = True
    try:
        yield
    finally:
        _TLS.off = prev


def _program_grad_types(program):
    cached = getattr(program, "_pa_grad_types", None)
    if cached is not None and cached[0] == program._version:
        return cached[1]
    types = {op.type for blk in program.blocks for op in blk.ops if op.type.endswith("_grad")}
    program._pa_grad_types = (program._version, types)
    return types


class BlockExecutor:
    def __init__(self, place=None):
        self.place = place or core.CPUPlace()
        self._cache = {}

    def prepare(self, program, block_idx=0):
        key = (id(program), block_idx, len(program.block(block_idx).ops), program._version)
        pb = self._cache.get(key)
        if pb is None or pb.program is not program:
            pb = PreparedBlock(program, block_idx)
            self._cache[key] = pb
        return pb

    @staticmethod
    def create_variables(program, scope, block_idx):
        """Persistables live in the root scope, temporaries in the local one (executor.cc:88)."""
        root = scope
        while root.parent() is not None:
            root = root.parent()
        for v in program.block(block_idx).vars.values():
            if v.persistable:
                root.var(v.name)
            else:
                var = scope.var(v.name)
                # temporaries start every run empty (the reference drops its local scope
                # after each Run): a tensor array left from the previous batch would
                # otherwise be appended to / accumulated into with stale shapes
                if isinstance(var.get(), core.LoDTensorArray):
                    var.set(core.LoDTensorArray())

    def run_block(self, program, block_idx, scope, create_vars=True):
        if block_idx == 0 and create_vars:
            R.clear_stash()  # graphs of a previous run whose grads never ran
        pb = self.prepare(program, block_idx)
        if create_vars:
            self.create_variables(program, scope, block_idx)
        self.run_prepared(pb, scope)

    def run_prepared(self, pb, scope):
        stash_off = getattr(_TLS, "off", False)
        for k in range(len(pb.steps)):
            self.run_op(pb, k, scope, stash_off)
        if _platform.vlog_level() >= 1 or _LOG_MEM:
            if self.place.torch_device().type == "cuda":
                _platform.log_memory(f"block {pb.block_idx if hasattr(pb, 'block_idx') else 0}",
                                     self.place.torch_device().index or 0)

    def run_op(self, pb, k, scope, stash_off=False):
        """Run step ``k`` of a prepared block (the unit the SSA-graph executor
        schedules: one ComputationOpHandle, details/computation_op_handle.cc)."""
        check_nan = FLAGS.get("check_nan_inf")
        bench = FLAGS.get("benchmark")
        profiling = prof.is_enabled()
        place = self.place
        if True:
            info, op, ins, outs, attrs = pb.steps[k]
            ctx_ins = {}
            for slot, names in ins:
                vals = []
                for n in names:
                    var = scope.find_var(n)
                    vals.append(var.get() if var is not None else None)
                ctx_ins[slot] = vals
            ctx = R.KernelContext(op.type, ctx_ins, outs, attrs, place, scope, op, self)
            if _platform._V >= 3:
                _platform.vlog(3, f"run op {op.type} inputs {dict(ins)} outputs {dict(outs)}")
            run = R.run_kernel_stash if (pb.stash[k] and not stash_off) else R.run_kernel
            if _stack_trace.enabled[0]:
                run = _traced(run, op.type)
            if _strict.watching() and place.torch_device().type == "cuda":
                # framework region: tensor expressions inside the op kernel run on the
                # HIP kernels (ops/aten_native.py); uncovered ATen kernels are counted
                # (and refused under FLAGS_strict_native=1)
                with _strict.region("fluid:" + op.type):
                    if profiling:
                        with prof.RecordEvent(op.type):
                            run(info, ctx)
                    else:
                        run(info, ctx)
            elif profiling:
                with prof.RecordEvent(op.type):
                    run(info, ctx)
            else:
                run(info, ctx)
            for slot, vals in ctx.results.items():
                names = outs.get(slot, [])
                for n, v in zip(names, vals):
                    if v is None or n == R.EMPTY_VAR:
                        continue
                    var = scope.find_var(n)
                    if var is None:
                        var = scope.var(n)
                    var.set(v)
                    if check_nan and isinstance(v, core.LoDTensor) and v.tensor is not None \
                            and v.tensor.is_floating_point():
                        if not torch.isfinite(v.tensor).all():
                            raise RuntimeError(f"Operator {op.type} output {n} contains NaN/Inf")
            if bench and place.torch_device().type == "cuda":
                torch.cuda.synchronize()
