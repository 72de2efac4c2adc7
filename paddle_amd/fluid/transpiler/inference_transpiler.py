"""Inference-time graph rewrites (transpiler/inference_transpiler.py:44-388):
fold batch_norm into the preceding conv2d (and its bias), fuse conv2d + bias add."""
from __future__ import annotations

import torch

from ...framework import core


class InferenceTranspiler:
    def transpile(self, program, place, scope=None):
        if scope is None:
            scope = core.global_scope()
        self.scope = scope
        self.block = program.global_block()
        self._fuse_batch_norm()
        program._version += 1

    def _get(self, name):
        return self.scope.find_var(name).get_tensor()

    def _fuse_batch_norm(self):
        ops = self.block.ops
        i = 0
        while i < len(ops) - 1:
            op = ops[i]
            if op.type in ("conv2d", "depthwise_conv2d"):
                nxt = ops[i + 1]
                bias_op = None
                if nxt.type == "elementwise_add" and i + 2 < len(ops) and ops[i + 2].type == "batch_norm":
                    bias_op, bn = nxt, ops[i + 2]
                elif nxt.type == "batch_norm":
                    bn = nxt
                else:
                    i += 1
                    continue
                w = self._get(op.input("Filter")[0])
                sc = self._get(bn.input("Scale")[0]).tensor.float()
                b = self._get(bn.input("Bias")[0]).tensor.float()
                m = self._get(bn.input("Mean")[0]).tensor.float()
                v = self._get(bn.input("Variance")[0]).tensor.float()
                eps = bn.attrs.get("epsilon", 1e-5)
                std = torch.sqrt(v + eps)
                factor = sc / std
                wt = w.tensor.float() * factor.reshape(-1, 1, 1, 1)
                w.set_tensor(wt.to(w.tensor.dtype))
                old_bias = torch.zeros_like(m)
                if bias_op is not None:
                    old_bias = self._get(bias_op.input("Y")[0]).tensor.float().reshape(-1)
                new_bias = (old_bias - m) * factor + b
                bias_name = (bias_op.input("Y")[0] if bias_op is not None else op.output("Output")[0] + "_bn_bias")
                if bias_op is None:
                    self.block.create_var(name=bias_name, shape=list(new_bias.shape), dtype=core.VT.FP32,
                                          persistable=True)
                self.scope.var(bias_name).set(core.LoDTensor(new_bias.to(w.tensor.device)))
                y = bn.output("Y")[0]
                conv_out = op.output("Output")[0]
                # replace [conv, (add), bn] by [conv, add(bias) -> y]
                del_idx = [i + 1, i + 2] if bias_op is not None else [i + 1]
                for j in reversed(del_idx):
                    self.block.remove_op(j)
                self.block.insert_op(i + 1, type="elementwise_add", inputs={"X": [conv_out], "Y": [bias_name]},
                                     outputs={"Out": [y]}, attrs={"axis": 1})
                ops = self.block.ops
            i += 1
