"""Inference-only IR passes that need the parameter scope (graph attr
``__param_scope__``): conv+BN folding (reference inference_transpiler.py:44-388 /
analysis passes) and the bf16 weight conversion (paddle/contrib/float16/
float16_transpiler.py re-targeted to gfx950's bf16 MFMA)."""
from __future__ import annotations

import torch

from ..framework import core
from ..framework import ir


@ir.register_pass("conv_bn_fuse_pass")
class ConvBNFusePass(ir.Pass):
    """conv2d [+ elementwise_add(bias)] + batch_norm(is_test)  ==>  conv2d + elementwise_add
    with the BN scale folded into the filter and the shift into the bias."""

    def apply_impl(self, graph):
        scope = graph.get("__param_scope__")
        if scope is None:
            return graph
        from ..fluid.transpiler.inference_transpiler import InferenceTranspiler

        n_bn = sum(1 for op in graph.block.ops if op.type == "batch_norm")
        # rewrite the op list in the block, then rebuild the SSA graph over it
        graph.block.ops = [n.op for n in ir.topology_sort(graph)]
        t = InferenceTranspiler()
        t.scope, t.block = scope, graph.block
        t._fuse_batch_norm()
        g = ir.Graph(graph.block)
        g._attrs = dict(graph._attrs)
        g.set("conv_bn_fuse_count", n_bn - sum(1 for op in graph.block.ops if op.type == "batch_norm"))
        return g


def convert_params_to_bf16(program, scope):
    """Store every float32 persistable of ``program`` as bfloat16 and mark the vars
    bf16, so GEMM/conv kernels run on bf16 MFMA with fp32 accumulation."""
    n = 0
    for v in program.global_block().vars.values():
        if not v.persistable or v.dtype != core.VT.FP32:
            continue
        var = scope.find_var(v.name)
        if var is None:
            continue
        t = var.get()
        if isinstance(t, core.LoDTensor) and t.tensor is not None and t.tensor.dtype == torch.float32:
            # batch-norm statistics stay fp32 (they are tiny and feed an rsqrt)
            if any(v.name in op.input(s) for op in program.global_block().ops if op.type == "batch_norm"
                   for s in ("Mean", "Variance")):
                continue
            t.set_tensor(t.tensor.to(torch.bfloat16))
            v.dtype = core.VT.BF16
            n += 1
    program._version += 1
    return n
