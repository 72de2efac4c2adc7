"""Small helpers shared by the layer functions."""
from __future__ import annotations

from ..framework import Variable
from ..layer_helper import LayerHelper


def simple_op(op_type, inputs, attrs=None, out_slot="Out", dtype=None, name=None, extra_outputs=(),
              stop_gradient=False):
    """Append one op with a single primary output var; returns that var."""
    helper = LayerHelper(op_type, name=name)
    if dtype is None:
        for v in inputs.values():
            v0 = v[0] if isinstance(v, (list, tuple)) else v
            if isinstance(v0, Variable):
                dtype = v0.dtype
                break
    out = helper.create_variable_for_type_inference(dtype=dtype, stop_gradient=stop_gradient)
    outputs = {out_slot: [out]}
    extras = []
    for slot in extra_outputs:
        e = helper.create_variable_for_type_inference(dtype=dtype, stop_gradient=True)
        outputs[slot] = [e]
        extras.append(e)
    helper.append_op(type=op_type, inputs=inputs, outputs=outputs, attrs=attrs or {})
    if extras:
        return (out,) + tuple(extras)
    return out
