"""Reduced-precision inference transpiler (reference: paddle/contrib/float16/
float16_transpiler.py -- fp16 for V100 tensor cores).  On MI355X the matrix cores'
native 16-bit format for inference and training is bf16 (same MFMA rate as fp16,
fp32 exponent range, no loss scaling), so :class:`ReducedPrecisionTranspiler`
defaults to bfloat16 and :class:`Float16Transpiler` keeps the reference's fp16.

What ``transpile(program, place, scope)`` does (same contract as the reference):
  * after every ``feed`` a ``cast`` to the low precision, so callers still feed fp32;
  * before every ``fetch`` a ``cast`` back to the fetched var's original dtype;
  * every float32 parameter an op reads is converted once into a new
    ``<name>.bf16`` / ``.fp16`` variable in ``scope`` and the op re-pointed to it
    (batch-norm Scale/Bias/Mean/Variance stay fp32, like the reference's
    no-conversion list);
  * intermediate float32 vars are re-typed to the low precision.
"""
from __future__ import annotations

import torch

from ...framework import core

_KEEP_FP32_SLOTS = {"batch_norm": ("Scale", "Bias", "Mean", "Variance"),
                    "layer_norm": ("Scale", "Bias")}


class ReducedPrecisionTranspiler:
    def __init__(self, dtype="bfloat16"):
        self.vt = core.convert_dtype(dtype)
        self.tdtype = core.to_torch_dtype(self.vt)
        self.suffix = ".bf16" if self.vt == core.VT.BF16 else ".fp16"

    def transpile(self, program, place, scope=None):
        from ..framework import Program

        if not isinstance(program, Program):
            raise TypeError("program should be as Program type")
        if not isinstance(place, (core.CPUPlace, core.CUDAPlace)):
            raise TypeError("place should be as CPUPlace/CUDAPlace type")
        self.scope = scope if scope is not None else core.global_scope()
        self.block = program.global_block()
        self._feed_fetch()
        self._params()
        self._retype()
        program._version += 1
        return program

    # ---------------------------------------------------------------- feed / fetch
    def _rename_inputs_after(self, start, old, new):
        for op in self.block.ops[start:]:
            if op.type != "fetch":
                op.rename_input(old, new)

    def _feed_fetch(self):
        ops = self.block.ops
        i = 0
        while i < len(ops):
            op = ops[i]
            if op.type == "feed":
                name = op.output("Out")[0]
                var = self.block.var(name)
                if var.dtype == core.VT.FP32:
                    lp = self.block.create_var(name=name + self.suffix, dtype=self.vt, shape=var.shape,
                                               lod_level=var.lod_level)
                    self._rename_inputs_after(i + 1, name, lp.name)
                    self.block.insert_op(i + 1, type="cast", inputs={"X": [name]}, outputs={"Out": [lp.name]},
                                         attrs={"in_dtype": core.VT.FP32, "out_dtype": self.vt})
                    i += 1
            elif op.type == "fetch":
                name = op.input("X")[0]
                var = self.block.var(name)
                if var.dtype == core.VT.FP32:
                    lp_name = name + self.suffix
                    self.block.create_var(name=lp_name, dtype=self.vt, shape=var.shape, lod_level=var.lod_level)
                    for prev in ops[:i]:
                        prev.rename_output(name, lp_name)
                        if prev.type != "cast" or prev.input("X") != [name]:
                            prev.rename_input(name, lp_name)
                    self.block.insert_op(i, type="cast", inputs={"X": [lp_name]}, outputs={"Out": [name]},
                                         attrs={"in_dtype": self.vt, "out_dtype": core.VT.FP32})
                    i += 1
            ops = self.block.ops
            i += 1

    # ---------------------------------------------------------------- parameters
    def _params(self):
        keep = set()
        for op in self.block.ops:
            for slot in _KEEP_FP32_SLOTS.get(op.type, ()):
                keep.update(op.input(slot))
        converted = {}
        for op in self.block.ops:
            for name in op.input_arg_names:
                v = self.block._find_var_recursive(name)
                if v is None or not v.persistable or v.dtype != core.VT.FP32 or name in keep:
                    continue
                if name not in converted:
                    sv = self.scope.find_var(name)
                    if sv is None or not isinstance(sv.get(), core.LoDTensor):
                        continue
                    t = sv.get()
                    new = name + self.suffix
                    self.block.create_var(name=new, dtype=self.vt, shape=v.shape, persistable=True)
                    self.scope.var(new).set(core.LoDTensor(t.tensor.to(self.tdtype), t.lod()))
                    converted[name] = new
                op.rename_input(name, converted[name])

    def _retype(self):
        for op in self.block.ops:
            if op.type in ("feed", "fetch") or (op.type == "cast" and op.attrs.get("out_dtype") == core.VT.FP32):
                continue
            for name in op.output_arg_names:
                v = self.block._find_var_recursive(name)
                if v is not None and not v.persistable and v.dtype == core.VT.FP32:
                    v.dtype = self.vt


class Float16Transpiler(ReducedPrecisionTranspiler):
    """The reference's fp16 transpiler."""

    def __init__(self):
        super().__init__("float16")


class BF16Transpiler(ReducedPrecisionTranspiler):
    def __init__(self):
        super().__init__("bfloat16")
