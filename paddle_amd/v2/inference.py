"""v2 inference (reference v2/inference.py): run the forward of ``output_layer`` on a
list of samples with given parameters."""
from __future__ import annotations

import numpy as np

from .. import fluid
from ._core import STATE, executor, place


class Inference:
    def __init__(self, parameters, output_layer=None, fileobj=None):
        self.outputs = output_layer if isinstance(output_layer, (list, tuple)) else [output_layer]
        self.parameters = parameters
        prog = STATE["main"].clone(for_test=True)
        self.program = prog._prune([prog.global_block().var(o.name) for o in self.outputs])
        used = {n for op in self.program.global_block().ops for n in op.input_arg_names}
        self.feed_names = [n for n in STATE["data"] if n in used]

    def infer(self, input, feeding=None, field="value", flatten_result=True, **kw):
        names = self.feed_names
        if feeding is not None:
            names = [n for n, _ in sorted(feeding.items(), key=lambda kv: kv[1]) if n in self.feed_names]
        idx = {n: i for i, n in enumerate(feeding)} if isinstance(feeding, dict) else {n: i for i, n in
                                                                                        enumerate(names)}
        block = self.program.global_block()
        feeder = fluid.DataFeeder(feed_list=[block.var(n) for n in names], place=place(), program=self.program)
        rows = [tuple(s[idx[n]] for n in names) for s in input]
        with fluid.scope_guard(STATE["scope"]):
            outs = executor().run(self.program, feed=feeder.feed(rows), fetch_list=[o.name for o in self.outputs])
        outs = [np.array(o) for o in outs]
        return outs[0] if len(outs) == 1 else outs


def infer(output_layer, parameters, input, feeding=None, field="value"):
    return Inference(parameters, output_layer).infer(input, feeding=feeding, field=field)
