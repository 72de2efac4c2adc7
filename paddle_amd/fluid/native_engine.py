"""The native C++ executor: the default engine behind ``fluid.Executor``.

``fluid.Executor(place)`` (``engine="auto"``, ``FLAGS_executor_engine=auto``) runs
every program the C++ executor can take on it, ``engine="native"`` insists on it,
``engine="python"`` keeps the op interpreter.  It runs a program's block 0 on the C++ executor of ``csrc/native`` (core.cc
Executor::RunBlock, the counterpart of the reference's framework/executor.cc:125-353)
instead of the Python op interpreter: the program is serialised once
(ProgramDesc wire format) and every op dispatches to a registered C++ kernel --
on a HIP place the gfx950 device kernels of ``ops_gpu.hip``, which run the shared
kernel library (GEMM, conv, pool, batch norm, softmax / loss, optimizers), with a
counted host fallback for the few configurations a device kernel declines.

Parameters and optimizer state are NOT copied: each persistable variable of the
Python scope is lent to the native scope (its torch storage pointer), so the
optimizer ops update the very tensors the Python side sees, and a variable whose
native buffer was re-allocated by a kernel is copied back after the run.  Feeds are
copied in; fetches are copied out (the only host syncs of a step).

Scope of the engine: block 0 and the sub-blocks of ``while`` /
``conditional_block`` (run by the C++ executor itself: Executor::RunWhile /
RunConditionalBlock), LoD-carrying feeds, and ANY op type: an op with no C++
kernel is run by its registered Python kernel through the executor's per-op
fallback callback (the op's inputs are zero-copy views of the native buffers, its
outputs are lent back to the native scope), counted in ``py_fallbacks``.  On a HIP
place the native kernels run on torch's current stream, so the two kernel
libraries are ordered without host syncs.  ``while_grad`` / ``conditional_block_grad``
run natively over kept step scopes (core.cc RunWhile / RunWhileGrad), as do
``recurrent`` / ``recurrent_grad`` (RunRecurrent / RunRecurrentGrad), tensor
arrays, rank tables and SelectedRows gradients with the sparse SGD / Adam kernels.
What still goes to the interpreter (``framework/executor.py``): ``parallel_do``,
``go`` / ``select`` and the RPC / pserver ops (``_UNSUPPORTED_CF``, ``_RPC_OPS``).

The engine drives the C++ objects through the ``paddle_amd_core`` CPython
extension (csrc/pybind/core_module.cc, pybind11) when it is built, else through
the ctypes C ABI of ``paddle_amd.native`` (``FLAGS_native_binding=ctypes`` forces
the latter).

Reference: framework/executor.cc:125-353 (Executor::Run), pybind/pybind.cc:507
(the Executor binding the Python layer drives).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from .. import native
from ..framework import core

_TORCH_DT = {torch.float32: 5, torch.int64: 3, torch.int32: 2, torch.float64: 6, torch.bool: 0, torch.uint8: 20,
             torch.float16: 4, torch.int16: 1, torch.int8: 21, torch.bfloat16: 22}
_DT_TORCH = {v: k for k, v in _TORCH_DT.items()}
# control-flow ops the C++ executor runs itself, and the ones it cannot take
_NATIVE_CF = {"while", "while_grad", "conditional_block", "conditional_block_grad", "recurrent", "recurrent_grad"}
_UNSUPPORTED_CF = {"parallel_do",
                   "parallel_do_grad", "go", "select"}


_RPC_OPS = {"send", "recv", "prefetch", "listen_and_serv", "send_barrier", "fetch_barrier", "checkpoint_notify",
            "split_selected_rows", "merge_selected_rows", "split_ids", "merge_ids", "lookup_sparse_table",
            "get_tensor_from_selected_rows", "gen_nccl_id"}


class _CtypesBinding:
    """The C ABI path (paddle_amd.native)."""

    name = "ctypes"

    def __init__(self, device):
        self.exe = native.NativeExecutor(device)

    program = staticmethod(lambda data: native.NativeProgram(data=data))
    scope = staticmethod(native.NativeScope)

    @staticmethod
    def share(ns, name, ptr, dt, shape, device):
        ns.share(name, ptr, dt, shape, device)

    @staticmethod
    def set(ns, name, arr, device):
        ns.set(name, arr, device)

    @staticmethod
    def info(ns, name):
        return ns.info(name)

    @staticmethod
    def get(ns, name):
        return ns.get(name)

    @staticmethod
    def lod(ns, name):
        return None  # the C ABI has no LoD read-back

    def run(self, prog, ns):
        self.exe.run(prog, ns)

    def host_fallbacks(self):
        return self.exe.host_fallbacks()

    supports_fallback = False


class _PybindBinding:
    """The CPython extension path (paddle_amd_core, pybind11 over the C++ classes)."""

    name = "pybind"

    def __init__(self, device, mod):
        self.C = mod
        self.exe = mod.Executor(device)

    def program(self, data):
        return self.C.ProgramDesc(data)

    def scope(self):
        return self.C.Scope()

    def share(self, ns, name, ptr, dt, shape, device):
        ns.var(name).get_tensor().share_external(ptr, self.C.VarType(dt), list(shape), device)

    def set(self, ns, name, arr, device):
        ns.var(name).get_tensor().set(arr, device)

    def info(self, ns, name):
        v = ns.find_var(name)
        if v is None or not v.is_initialized():
            return None
        t = v.get_tensor()
        return int(t.dtype()), tuple(t.shape()), t.data_ptr(), t.device()

    def get(self, ns, name):
        v = ns.find_var(name)
        if v is None or not v.is_initialized():
            raise RuntimeError(f"variable {name} not found or empty")
        return v.get_tensor().numpy()

    def lod(self, ns, name):
        v = ns.find_var(name)
        return [list(level) for level in v.get_tensor().lod()] if v is not None and v.is_initialized() else None

    def run(self, prog, ns):
        self.exe.run(prog, ns)

    def host_fallbacks(self):
        return dict(self.exe.host_fallbacks)

    supports_fallback = True


def _binding(device):
    if os.environ.get("FLAGS_native_binding", "pybind") != "ctypes":
        from .. import core_ext

        mod = core_ext.module()
        if mod is not None:
            return _PybindBinding(device, mod)
    return _CtypesBinding(device)


class NativeEngine:
    def __init__(self, place):
        self.place = place
        self.device = int(place.device_id) if isinstance(place, core.CUDAPlace) else -1
        self._b = _binding(self.device)
        self._progs = {}
        self._scopes = {}  # id(python scope) -> (scope ref, NativeScope, {name: (ptr, shape, dtype, tensor)})
        self._host_ops = set(native.registered_ops(False))
        self._dev_ops = set(native.registered_ops(True)) if self.device >= 0 else set()
        self._bexe = None
        self._wrapped = []
        self._keep = {}
        self._feed_keep = {}
        self.py_fallbacks = {}  # op type -> calls run by the Python op library
        self.py_fallback_types = set()

    # ------------------------------------------------------------------ program
    _VAR_OK = None

    @staticmethod
    def can_run(program, place):
        """Can the C++ executor take ``program`` (engine="auto")?  No control flow
        needing per-step scopes, every variable a dense LoDTensor (or the feed / fetch
        holders), the pybind binding available when some op has no C++ kernel."""
        VT = core.VT
        ok_types = {VT.LOD_TENSOR, VT.FEED_MINIBATCH, VT.FETCH_LIST, VT.LOD_TENSOR_ARRAY, VT.LOD_RANK_TABLE,
                    VT.STEP_SCOPES, VT.SELECTED_ROWS}
        try:
            native.lib()
        except Exception:
            return False
        all_ops = [op for b in program.blocks for op in b.ops]
        for op in all_ops:
            if op.type in _UNSUPPORTED_CF or (any(k in op.attrs for k in ("sub_block", "blocks"))
                                              and op.type not in _NATIVE_CF):
                return False
            # distributed lookup tables and the RPC ops that exchange their SelectedRows
            # stay on the interpreter (local sparse gradients run natively)
            if op.attrs.get("is_distributed") or op.type in _RPC_OPS:
                return False
        for b in program.blocks:
            for v in b.vars.values():
                if v.type not in ok_types:
                    return False
                # fp64 programs (gradient checks) stay on the interpreter: the C++
                # host kernels are fp32 / integer / bool
                if v.type == VT.LOD_TENSOR and getattr(v, "dtype", None) == VT.FP64:
                    return False
        dev = isinstance(place, core.CUDAPlace)
        kern = set(native.registered_ops(False)) | (set(native.registered_ops(True)) if dev else set())
        fallback = [op for op in all_ops if op.type not in kern and op.type not in _NATIVE_CF]
        if fallback:
            from .. import core_ext

            if os.environ.get("FLAGS_native_binding", "") == "ctypes" or core_ext.module() is None:
                return False
            # the per-op Python fallback bridges dense tensors only: an op without a C++
            # kernel that reads or writes a tensor array / rank table / step scopes /
            # SelectedRows keeps the program on the interpreter
            vtype = {n: v.type for b in program.blocks for n, v in b.vars.items()}
            dense = {VT.LOD_TENSOR, VT.FEED_MINIBATCH, VT.FETCH_LIST}
            for op in fallback:
                names = [n for ns in list(op.inputs.values()) + list(op.outputs.values()) for n in ns]
                if any(vtype.get(n, VT.LOD_TENSOR) not in dense for n in names):
                    return False
        return True

    def _program(self, program):
        key = (id(program), program._version)
        ent = self._progs.get(key)
        if ent is not None and ent[0] is program:
            return ent[1], ent[2]
        all_ops = [op for b in program.blocks for op in b.ops]
        cf = sorted({op.type for op in all_ops if op.type in _UNSUPPORTED_CF or (
            any(k in op.attrs for k in ("sub_block", "blocks")) and op.type not in _NATIVE_CF)})
        if cf:
            raise NotImplementedError(f"native engine: control-flow ops needing per-step scopes {cf} "
                                      "(use the default engine)")
        missing = sorted({op.type for op in all_ops if op.type not in self._host_ops and op.type not in self._dev_ops
                          and op.type not in _NATIVE_CF})
        if missing and not self._b.supports_fallback:
            raise NotImplementedError(f"native engine: no C++ kernel for op types {missing}")
        self.py_fallback_types = set(missing)
        src = program
        gb = program.global_block()
        if any(op.type in ("feed", "fetch") for op in gb.ops):
            # a saved program carrying its own feed / fetch ops: feeds are set and
            # fetches read by name here, so run a copy without them
            src = program.clone()
            b0 = src.global_block()
            for i in reversed(range(len(b0.ops))):
                if b0.ops[i].type in ("feed", "fetch"):
                    b0.remove_op(i)
        prog = self._b.program(src.desc.serialize_to_string())
        pers = [v.name for v in program.list_vars()
                if v.persistable and v.name not in ("feed", "fetch") and v.type == core.VT.LOD_TENSOR]
        self._progs[key] = (program, prog, pers, src)
        return prog, pers

    def _scope(self, scope):
        ent = self._scopes.get(id(scope))
        if ent is None or ent[0] is not scope:
            ent = (scope, self._b.scope(), {})
            self._scopes[id(scope)] = ent
        return ent[1], ent[2]

    # ------------------------------------------------------------------ tensors
    def _tdev(self):
        return torch.device("cuda", self.device) if self.device >= 0 else torch.device("cpu")

    def _lend(self, ns, bound, name, lt):
        """Lends the torch storage of LoDTensor ``lt`` to the native scope as ``name``."""
        t = lt._t
        if t is None:
            return
        if t.device != self._tdev() or not t.is_contiguous() or t.dtype not in _TORCH_DT:
            if t.dtype not in _TORCH_DT:
                raise NotImplementedError(f"native engine: {name} has dtype {t.dtype}")
            t = t.to(self._tdev()).contiguous()
            lt._t = t
        sig = (t.data_ptr(), tuple(t.shape), t.dtype)
        if bound.get(name, (None,))[:3] != sig:
            self._b.share(ns, name, t.data_ptr(), _TORCH_DT[t.dtype], tuple(t.shape), self.device)
            bound[name] = sig + (t,)

    def _feed(self, ns, name, data):
        """Lends the feed's storage to the native scope: a tensor already on the
        executor's place (a device tensor on a HIP place) is shared as is, anything
        else is moved there once -- no numpy round trip for device tensors."""
        lod = None
        if isinstance(data, core.LoDTensor):
            lod = data.lod()
            data = data._t
        if not isinstance(data, torch.Tensor):
            data = torch.from_numpy(np.ascontiguousarray(np.asarray(data)))
        t = data.detach()
        if t.dtype not in _TORCH_DT:
            raise NotImplementedError(f"native engine: feed {name} has dtype {t.dtype}")
        t = t.to(self._tdev()).contiguous()
        if t.device.type == "cuda" and data.device.type != "cuda":
            # the host-to-device copy is on torch's stream, the native kernels on ours
            torch.cuda.current_stream(self._tdev()).synchronize()
        self._feed_keep[name] = t  # alive while the native scope references it
        self._b.share(ns, name, t.data_ptr(), _TORCH_DT[t.dtype], tuple(t.shape), self.device)
        if lod:
            if not self._b.supports_fallback:
                raise NotImplementedError(f"native engine: LoD feed {name} needs the pybind binding")
            ns.find_var(name).get_tensor().set_lod([list(map(int, lv)) for lv in lod])

    # ------------------------------------------------------------------ per-op Python fallback
    def _wrap(self, nt):
        """Zero-copy torch view of a native tensor (host or device)."""
        dt, shape, ptr, dev = int(nt.dtype()), tuple(nt.shape()), nt.data_ptr(), nt.device()
        tdt = _DT_TORCH[dt]
        n = int(np.prod(shape)) if shape else 1
        if n == 0 or not ptr:
            return torch.empty(shape, dtype=tdt, device=self._tdev() if dev >= 0 else "cpu")
        esz = torch.empty((), dtype=tdt).element_size()
        self._wrapped.append((ptr, ptr + n * esz))
        if dev < 0:
            buf = (ctypes.c_byte * (n * esz)).from_address(ptr)
            return torch.frombuffer(buf, dtype=tdt).reshape(shape)
        ints = {1: "|i1", 2: "<i2", 4: "<i4", 8: "<i8"}[esz]
        holder = type("_NativeView", (), {"__cuda_array_interface__": {
            "shape": shape, "typestr": ints, "data": (ptr, False), "version": 2, "strides": None}})()
        return torch.as_tensor(holder, device=torch.device("cuda", dev)).view(tdt)

    def _aliases_native(self, t):
        lo = t.data_ptr()
        hi = lo + t.numel() * t.element_size()
        return any(lo < b and a < hi for a, b in self._wrapped)

    def _py_op(self, program, scope, blk, idx, ns):
        """Run op ``idx`` of block ``blk`` with its registered Python kernel on the
        native scope ``ns``."""
        from ..framework import registry as R
        from ..framework.executor import BlockExecutor

        if self._bexe is None:
            self._bexe = BlockExecutor(self.place)
        pb = self._bexe.prepare(program, blk)
        info, op, ins, outs, attrs = pb.steps[idx]
        self._wrapped = []
        ctx_ins = {}
        for slot, names in ins:
            vals = []
            for n in names:
                v = ns.find_var(n)
                if v is None or not v.is_initialized():
                    vals.append(None)
                    continue
                nt = v.get_tensor()
                lt = core.LoDTensor(self._wrap(nt))
                lod = nt.lod()
                if lod:
                    lt.set_lod(lod)
                vals.append(lt)
            ctx_ins[slot] = vals
        in_names = {n for _, names in ins for n in names}
        ent = self._scopes.get(id(scope))
        bound_names = ent[2] if ent is not None and ent[0] is scope else {}
        ctx = R.KernelContext(op.type, ctx_ins, outs, attrs, self.place, scope, op, self._bexe)
        R.run_kernel(info, ctx)
        self.py_fallbacks[op.type] = self.py_fallbacks.get(op.type, 0) + 1
        keep = self._keep.setdefault(id(ns), {})
        for slot, vals in ctx.results.items():
            for n, v in zip(outs.get(slot, []), vals):
                if v is None or n == R.EMPTY_VAR:
                    continue
                if isinstance(v, torch.Tensor):
                    v = core.LoDTensor(v)
                if not isinstance(v, core.LoDTensor):
                    raise NotImplementedError(f"native engine: op {op.type} output {n} is a "
                                              f"{type(v).__name__} (LoDTensor only)")
                t = v.tensor
                if t is None:
                    continue
                if t.device != self._tdev():
                    t = t.to(self._tdev())
                if t.dtype not in _TORCH_DT:
                    raise NotImplementedError(f"native engine: op {op.type} output {n} dtype {t.dtype}")
                if not t.is_contiguous() or self._aliases_native(t):
                    t = t.contiguous() if not t.is_contiguous() and not self._aliases_native(t) else t.clone()
                var = ns.find_var(n)  # an enclosing scope's variable is updated in place
                if var is not None and (n in in_names or n in bound_names) and var.is_initialized():
                    # an in-place op (ParamOut == Param) or a lent persistable: write INTO
                    # its buffer, so every holder of that storage (the Python scope's
                    # parameter, optimizer state) keeps seeing one tensor
                    cur = var.get_tensor()
                    if (int(cur.data_ptr()) and tuple(cur.shape()) == tuple(t.shape)
                            and _DT_TORCH.get(int(cur.dtype())) == t.dtype):
                        dst = self._wrap(cur)
                        if dst.data_ptr() != t.data_ptr():
                            dst.copy_(t)
                        cur.set_lod([list(map(int, lv)) for lv in (v.lod() or [])])
                        continue
                keep[n] = t  # alive while the native scope references it
                nt = (var if var is not None else ns.var(n)).get_tensor()
                nt.share_external(t.data_ptr(), self._b.C.VarType(_TORCH_DT[t.dtype]), list(t.shape),
                                  self.device)
                nt.set_lod([list(map(int, lv)) for lv in (v.lod() or [])])
        self._wrapped = []

    def _write_back(self, scope, ns, bound, name):
        """After a run: a persistable whose native buffer moved is copied into a torch
        tensor of the Python scope (and lent again, so later runs update it in place)."""
        info = self._b.info(ns, name)
        if info is None:
            return
        dt, shape, ptr, dev = info
        b = bound.get(name)
        var = scope.find_var(name) or scope.var(name)
        lt = var.get_tensor()
        if b is not None and b[0] == ptr:
            if tuple(b[1]) != shape and lt._t is not None:
                lt._t = lt._t.view(shape)
                bound[name] = (ptr, shape, b[2], lt._t)
            return
        if dt not in _DT_TORCH:
            return
        t = torch.empty(shape, dtype=_DT_TORCH[dt], device=self._tdev())
        if t.numel():
            native.copy(t.data_ptr(), self.device, ptr, dev, t.numel() * t.element_size())
        lt._t = t
        self._lend(ns, bound, name, lt)

    # ------------------------------------------------------------------ run
    def run(self, program, feed, fetch_names, scope, return_numpy=True):
        prog, pers = self._program(program)
        ns, bound = self._scope(scope)
        for name in pers:
            var = scope.find_var(name)
            val = var.get() if var is not None else None
            if isinstance(val, core.LoDTensor):
                self._lend(ns, bound, name, val)
        for name, data in feed.items():
            self._feed(ns, name, data)
        if self._b.supports_fallback:
            src = self._progs[(id(program), program._version)][3]
            self._b.exe.set_fallback(lambda blk, idx, s, p=src, sc=scope: self._py_op(p, sc, blk, idx, s))
            if self.device >= 0:
                # one stream for both kernel libraries: no host sync between them
                self._b.exe.set_stream(torch.cuda.current_stream(self._tdev()).cuda_stream)
        elif self.device >= 0:
            torch.cuda.current_stream(self._tdev()).synchronize()  # lent tensors written by torch
        try:
            self._b.run(prog, ns)  # ends with a sync of the native stream
        finally:
            if self._b.supports_fallback:
                self._b.exe.set_fallback(None)
        for name in pers:
            self._write_back(scope, ns, bound, name)
        outs = []
        for n in fetch_names:
            a = self._b.get(ns, n)
            if return_numpy:
                outs.append(a)
            else:  # a LoDTensor fetch keeps the variable's LoD
                outs.append(core.LoDTensor(torch.from_numpy(a).to(self._tdev()), self._b.lod(ns, n) or None))
        return outs

    def host_fallbacks(self):
        return self._b.host_fallbacks()

    @property
    def binding(self):
        return self._b.name
