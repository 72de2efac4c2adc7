"""IR graph + pass framework (reference: paddle/fluid/framework/ir/ -- ``Graph``
ir/graph.h:63, ``Node`` ir/node.h:27, ``Pass``/``PassRegistry`` ir/pass.h:32-120,
``GraphPatternDetector`` ir/graph_pattern_detector.h:224, ``graph_helper.cc``
``HasCircle``/``TopologySortOperations``, and the passes ``graph_viz_pass``,
``graph_to_program_pass``, ``infer_clean_graph_pass``, ``fc_fuse_pass``,
``fc_lstm_fuse_pass``, ``seq_concat_fc_fuse_pass``).

A :class:`Graph` is built from one Block of a fluid Program.  Op nodes wrap the
block's ``Operator`` objects; variable nodes are SSA versions (every write of a
name creates a new var node, as in the reference) so dataflow, WAR and WAW
hazards are explicit edges.  Passes rewrite the graph; ``graph_to_program`` writes
the topologically sorted ops back into the block.

MI355X note: the passes that matter on this hardware are the ones that turn
several memory-bound kernels into one (GEMM + bias epilogue of the native MFMA
GEMM behind ``fc``, conv+BN folding, dropout/scale removal at inference): each removed op is
one fewer full pass over HBM.
"""
from __future__ import annotations

import itertools
from collections import OrderedDict, defaultdict

_ids = itertools.count()


class Node:
    OP, VAR = "op", "var"

    def __init__(self, kind, name, op=None, var=None):
        self.id = next(_ids)
        self.kind = kind
        self.name = name
        self.op = op          # fluid Operator (kind == OP)
        self.var = var        # fluid Variable or None (kind == VAR)
        self.inputs: list[Node] = []
        self.outputs: list[Node] = []
        self.order = float(self.id)   # tie-break rank for topology_sort (program order)

    def is_op(self, type=None):
        return self.kind == Node.OP and (type is None or self.op.type == type)

    def is_var(self):
        return self.kind == Node.VAR

    def __repr__(self):
        return f"Node({self.kind}:{self.name}#{self.id})"


class Graph:
    """Dataflow graph of one Block (ir/graph.cc: Graph::Graph(ProgramDesc))."""

    def __init__(self, block):
        self.block = block
        self.program = block.program
        self.nodes: list[Node] = []
        self._attrs: dict = {}
        latest: dict[str, Node] = {}
        for i, op in enumerate(block.ops):
            n = self.create_op_node(op)
            n.order = float(i)
            for name in op.input_arg_names:
                v = latest.get(name)
                if v is None:
                    v = latest[name] = self.create_var_node(name)
                _link(v, n)
            for name in op.output_arg_names:
                v = self.create_var_node(name)   # SSA: a new version per write
                _link(n, v)
                latest[name] = v

    # ------------------------------------------------------------- attributes
    def set(self, key, value):
        self._attrs[key] = value

    def get(self, key, default=None):
        return self._attrs.get(key, default)

    def has(self, key):
        return key in self._attrs

    # ------------------------------------------------------------- nodes
    def create_op_node(self, op):
        n = Node(Node.OP, op.type, op=op)
        self.nodes.append(n)
        return n

    def create_var_node(self, name):
        n = Node(Node.VAR, name, var=self.block._find_var_recursive(name))
        self.nodes.append(n)
        return n

    def op_nodes(self):
        return [n for n in self.nodes if n.kind == Node.OP]

    def var_nodes(self):
        return [n for n in self.nodes if n.kind == Node.VAR]

    def remove_nodes(self, nodes):
        dead = set(id(n) for n in nodes)
        for n in nodes:
            for i in n.inputs:
                i.outputs = [o for o in i.outputs if id(o) not in dead]
            for o in n.outputs:
                o.inputs = [i for i in o.inputs if id(i) not in dead]
        self.nodes = [n for n in self.nodes if id(n) not in dead]

    def consumers(self, var_name):
        return [o for v in self.var_nodes() if v.name == var_name for o in v.outputs]


def _link(a, b):
    a.outputs.append(b)
    b.inputs.append(a)


# ------------------------------------------------------------------ graph helper
def _op_deps(graph):
    """op -> set(ops it depends on) over dataflow plus WAR/WAW hazards on names."""
    deps = defaultdict(set)
    ops = graph.op_nodes()
    for n in ops:
        for v in n.inputs:
            for p in v.inputs:
                if p.is_op():
                    deps[n].add(p)
    # hazards: a writer of name X must follow every earlier reader/writer of X
    order = {n: n.order for n in ops}
    readers, writers = defaultdict(list), defaultdict(list)
    for n in ops:
        for v in n.inputs:
            readers[v.name].append(n)
        for v in n.outputs:
            writers[v.name].append(n)
    for name, ws in writers.items():
        for w in ws:
            for r in readers.get(name, []) + ws:
                if r is not w and order[r] < order[w] and r not in _reachable_from(w, deps):
                    deps[w].add(r)
    return deps


def _reachable_from(n, deps):
    # cheap guard against creating a 2-cycle; full cycle detection in has_circle
    return deps.get(n, ())


def has_circle(graph) -> bool:
    """graph_helper.cc HasCircle over the op dependency relation."""
    deps = _op_deps(graph)
    state = {}

    def dfs(n):
        state[n] = 1
        for d in deps.get(n, ()):
            s = state.get(d, 0)
            if s == 1 or (s == 0 and dfs(d)):
                return True
        state[n] = 2
        return False

    return any(state.get(n, 0) == 0 and dfs(n) for n in graph.op_nodes())


def topology_sort(graph):
    """graph_helper.cc TopologySortOperations: stable (original order breaks ties)."""
    deps = _op_deps(graph)
    ops = graph.op_nodes()
    rank = {n: n.order for n in ops}
    indeg = {n: len(deps.get(n, ())) for n in ops}
    users = defaultdict(list)
    for n, ds in deps.items():
        for d in ds:
            users[d].append(n)
    import heapq

    ready = [(rank[n], n.id, n) for n in ops if indeg[n] == 0]
    heapq.heapify(ready)
    out = []
    while ready:
        _, _, n = heapq.heappop(ready)
        out.append(n)
        for u in users[n]:
            indeg[u] -= 1
            if indeg[u] == 0:
                heapq.heappush(ready, (rank[u], u.id, u))
    if len(out) != len(ops):
        raise RuntimeError("graph has a cycle; cannot topologically sort")
    return out


# ------------------------------------------------------------------ passes
_PASSES: "OrderedDict[str, type]" = OrderedDict()


class Pass:
    """ir/pass.h:32 -- ``apply`` takes and returns a Graph; required graph attrs
    are checked before, declared attrs set after."""

    name = "pass"
    required_graph_attrs: tuple = ()

    def __init__(self, **attrs):
        self.attrs = dict(attrs)

    def apply(self, graph):
        for a in self.required_graph_attrs:
            if not graph.has(a):
                raise ValueError(f"pass {self.name} requires graph attr {a}")
        g = self.apply_impl(graph)
        applied = g.get("__applied_passes__", [])
        g.set("__applied_passes__", applied + [self.name])
        return g

    def apply_impl(self, graph):
        return graph


def register_pass(name):
    def deco(cls):
        cls.name = name
        _PASSES[name] = cls
        return cls

    return deco


def get_pass(name, **attrs) -> Pass:
    if name not in _PASSES:
        raise KeyError(f"pass {name} is not registered")
    return _PASSES[name](**attrs)


def all_passes():
    return list(_PASSES)


class PassBuilder:
    """ir/pass_builder.h: ordered, editable list of passes."""

    def __init__(self, names=()):
        self._passes = [get_pass(n) for n in names]

    def append_pass(self, name, **attrs):
        p = get_pass(name, **attrs)
        self._passes.append(p)
        return p

    def insert_pass(self, idx, name, **attrs):
        p = get_pass(name, **attrs)
        self._passes.insert(idx, p)
        return p

    def remove_pass(self, idx):
        self._passes.pop(idx)

    def all_passes(self):
        return list(self._passes)

    def apply(self, graph):
        for p in self._passes:
            graph = p.apply(graph)
        return graph


# ------------------------------------------------------------------ pattern detector
class PDNode:
    def __init__(self, pattern, name, kind, pred=None):
        self.pattern, self.name, self.kind = pattern, name, kind
        self.preds = [pred] if pred else []

    def assert_op(self, type=None):
        self.kind = Node.OP
        if type is not None:
            self.preds.append(lambda n, t=type: n.is_op(t))
        return self

    def assert_var(self):
        self.kind = Node.VAR
        return self

    def assert_more(self, fn):
        self.preds.append(fn)
        return self

    def assert_is_op_input(self, op_type, slot=None):
        self.kind = Node.VAR

        def f(n):
            return any(o.is_op(op_type) and (slot is None or n.name in o.op.input(slot)) for o in n.outputs)

        self.preds.append(f)
        return self

    def assert_is_op_output(self, op_type, slot=None):
        self.kind = Node.VAR

        def f(n):
            return any(i.is_op(op_type) and (slot is None or n.name in i.op.output(slot)) for i in n.inputs)

        self.preds.append(f)
        return self

    def assert_single_consumer(self):
        self.preds.append(lambda n: len(n.outputs) == 1)
        return self

    def as_input(self, op_pdnode):
        self.pattern.edges.append((self, op_pdnode))
        return self

    def as_output(self, op_pdnode):
        self.pattern.edges.append((op_pdnode, self))
        return self

    def match(self, n):
        return (self.kind is None or n.kind == self.kind) and all(p(n) for p in self.preds)


class PDPattern:
    def __init__(self):
        self.nodes: list[PDNode] = []
        self.edges: list[tuple[PDNode, PDNode]] = []

    def new_node(self, name, kind=None, pred=None):
        n = PDNode(self, name, kind, pred)
        self.nodes.append(n)
        return n


class GraphPatternDetector:
    """graph_pattern_detector.h:224 -- find every injective mapping of pattern nodes
    to graph nodes respecting predicates and edges; matches are non-overlapping
    (first-found wins, as the reference's ``RemoveOverlappedMatch``)."""

    def __init__(self):
        self.pattern = PDPattern()

    def __call__(self, graph, handler):
        matches = self.detect(graph)
        for m in matches:
            handler(m, graph)
        return len(matches)

    def detect(self, graph):
        pat = self.pattern
        cands = {p: [n for n in graph.nodes if p.match(n)] for p in pat.nodes}
        order = sorted(pat.nodes, key=lambda p: len(cands[p]))
        results, used = [], set()

        def consistent(assign):
            for a, b in pat.edges:
                if a in assign and b in assign and assign[b] not in assign[a].outputs:
                    return False
            return True

        def search(i, assign):
            if i == len(order):
                results.append(dict((p.name, n) for p, n in assign.items()))
                return True
            p = order[i]
            for n in cands[p]:
                if n in assign.values() or id(n) in used:
                    continue
                assign[p] = n
                if consistent(assign) and search(i + 1, assign):
                    return True
                del assign[p]
            return False

        while True:
            assign = {}
            before = len(results)
            search(0, assign)
            if len(results) == before:
                break
            used.update(id(n) for n in results[-1].values())
        return results


# ------------------------------------------------------------------ built-in passes
@register_pass("graph_viz_pass")
class GraphVizPass(Pass):
    """Dump graphviz dot (attr ``graph_viz_path``); ops as boxes, vars as ellipses."""

    def apply_impl(self, graph):
        path = self.attrs.get("graph_viz_path") or graph.get("graph_viz_path")
        lines = ["digraph G {", '  rankdir=TB;']
        for n in graph.nodes:
            if n.is_op():
                lines.append(f'  n{n.id} [label="{n.op.type}", shape=box, style=filled, fillcolor="#dfe8f6"];')
            else:
                lines.append(f'  n{n.id} [label="{n.name}", shape=ellipse];')
        for n in graph.nodes:
            for o in n.outputs:
                lines.append(f"  n{n.id} -> n{o.id};")
        lines.append("}")
        dot = "\n".join(lines)
        graph.set("graph_viz_dot", dot)
        if path:
            with open(path, "w") as f:
                f.write(dot)
        return graph


@register_pass("graph_to_program_pass")
class GraphToProgramPass(Pass):
    """Write the topologically sorted op list back into the Block."""

    def apply_impl(self, graph):
        graph.block.ops = [n.op for n in topology_sort(graph)]
        graph.program._version += 1
        return graph


@register_pass("infer_clean_graph_pass")
class InferCleanGraphPass(Pass):
    """Drop feed/fetch ops and variable nodes nothing touches (infer_clean_graph_pass.cc)."""

    def apply_impl(self, graph):
        dead = [n for n in graph.op_nodes() if n.op.type in ("feed", "fetch")]
        graph.remove_nodes(dead)
        graph.remove_nodes([n for n in graph.var_nodes() if not n.inputs and not n.outputs])
        return graph


def _replace_ops(graph, old_op_nodes, new_op, dead_vars=()):
    """Swap ``old_op_nodes`` for ``new_op`` (an Operator) in the graph."""
    n = graph.create_op_node(new_op)
    n.order = min(o.order for o in old_op_nodes)
    ins = {nm for nm in new_op.input_arg_names}
    outs = {nm for nm in new_op.output_arg_names}
    for o in old_op_nodes:
        for v in o.inputs:
            if v.name in ins and v not in n.inputs:
                _link(v, n)
        for v in o.outputs:
            if v.name in outs and v not in n.outputs:
                v.inputs = []
                _link(n, v)
    graph.remove_nodes(list(old_op_nodes) + list(dead_vars))
    return n


def _new_op(block, type, inputs, outputs, attrs):
    from ..fluid.framework import Operator

    return Operator(block, None, type=type, inputs=inputs, outputs=outputs, attrs=attrs)


@register_pass("fc_fuse_pass")
class FCFusePass(Pass):
    """mul(X, W) -> t; elementwise_add(t, b) -> out  ==>  fc(Input=X, W, Bias=b) -> out
    (fc_fuse_pass.cc).  With ``with_relu`` a following relu folds in as the fc
    activation (bias in the native GEMM epilogue, one activation pass)."""

    def apply_impl(self, graph):
        d = GraphPatternDetector()
        p = d.pattern
        x = p.new_node("x").assert_is_op_input("mul", "X")
        w = p.new_node("w").assert_is_op_input("mul", "Y").assert_more(
            lambda n: n.var is not None and n.var.persistable)
        mul = p.new_node("mul").assert_op("mul").assert_more(lambda n: n.op.attrs.get("y_num_col_dims", 1) == 1)
        t = p.new_node("t").assert_is_op_output("mul", "Out").assert_is_op_input("elementwise_add", "X") \
            .assert_single_consumer()
        b = p.new_node("b").assert_is_op_input("elementwise_add", "Y").assert_more(
            lambda n: n.var is not None and n.var.persistable and len(n.var.shape or ()) == 1)
        add = p.new_node("add").assert_op("elementwise_add")
        out = p.new_node("out").assert_is_op_output("elementwise_add", "Out")
        x.as_input(mul)
        w.as_input(mul)
        t.as_output(mul).as_input(add)
        b.as_input(add)
        out.as_output(add)
        fused = [0]

        def handle(m, g):
            mul_op = m["mul"].op
            newop = _new_op(g.block, "fc", {"Input": [m["x"].name], "W": [m["w"].name], "Bias": [m["b"].name]},
                            {"Out": [m["out"].name]},
                            {"in_num_col_dims": mul_op.attrs.get("x_num_col_dims", 1), "activation_type": ""})
            _replace_ops(g, [m["mul"], m["add"]], newop, dead_vars=[m["t"]])
            fused[0] += 1

        d(graph, handle)
        graph.set("fc_fuse_count", fused[0])
        return graph


@register_pass("fc_act_fuse_pass")
class FCActFusePass(Pass):
    """fc -> relu/gelu/tanh/sigmoid (single consumer)  ==>  fc(activation_type=...)."""

    ACTS = ("relu", "gelu", "tanh", "sigmoid")

    def apply_impl(self, graph):
        n_fused = 0
        for act in self.ACTS:
            d = GraphPatternDetector()
            p = d.pattern
            fc = p.new_node("fc").assert_op("fc").assert_more(lambda n: not n.op.attrs.get("activation_type"))
            t = p.new_node("t").assert_is_op_output("fc", "Out").assert_is_op_input(act, "X").assert_single_consumer()
            a = p.new_node("act").assert_op(act)
            o = p.new_node("out").assert_is_op_output(act, "Out")
            t.as_output(fc).as_input(a)
            o.as_output(a)

            def handle(m, g, act=act):
                nonlocal n_fused
                fop = m["fc"].op
                newop = _new_op(g.block, "fc", dict(fop.inputs), {"Out": [m["out"].name]},
                                dict(fop.attrs, activation_type=act))
                _replace_ops(g, [m["fc"], m["act"]], newop, dead_vars=[m["t"]])
                n_fused += 1

            d(graph, handle)
        graph.set("fc_act_fuse_count", n_fused)
        return graph


@register_pass("fc_lstm_fuse_pass")
class FCLstmFusePass(Pass):
    """mul(X, Wx) [+ elementwise_add(bias)] -> lstm  ==>  fusion_lstm (fc_lstm_fuse_pass.cc)."""

    def apply_impl(self, graph):
        d = GraphPatternDetector()
        p = d.pattern
        x = p.new_node("x").assert_is_op_input("mul", "X")
        wx = p.new_node("wx").assert_is_op_input("mul", "Y")
        mul = p.new_node("mul").assert_op("mul")
        t = p.new_node("t").assert_is_op_output("mul", "Out").assert_is_op_input("lstm", "Input") \
            .assert_single_consumer()
        lstm = p.new_node("lstm").assert_op("lstm")
        x.as_input(mul)
        wx.as_input(mul)
        t.as_output(mul).as_input(lstm)
        n = [0]

        def handle(m, g):
            lop = m["lstm"].op
            ins = {"X": [m["x"].name], "WeightX": [m["wx"].name], "WeightH": lop.input("Weight"),
                   "Bias": lop.input("Bias")}
            for s in ("H0", "C0"):
                if lop.input(s):
                    ins[s] = lop.input(s)
            outs = {"Hidden": lop.output("Hidden"), "Cell": lop.output("Cell")}
            attrs = {k: v for k, v in lop.attrs.items() if k in ("use_peepholes", "is_reverse", "gate_activation",
                                                                 "cell_activation", "candidate_activation")}
            newop = _new_op(g.block, "fusion_lstm", ins, outs, attrs)
            _replace_ops(g, [m["mul"], m["lstm"]], newop, dead_vars=[m["t"]])
            n[0] += 1

        d(graph, handle)
        graph.set("fc_lstm_fuse_count", n[0])
        return graph


@register_pass("is_test_pass")
class IsTestPass(Pass):
    """Set ``is_test=True`` on every op that has the attr (inference)."""

    def apply_impl(self, graph):
        for n in graph.op_nodes():
            if "is_test" in n.op.attrs:
                n.op.attrs["is_test"] = True
        return graph


@register_pass("identity_op_clean_pass")
class IdentityOpCleanPass(Pass):
    """Remove ops that are the identity at inference: ``scale`` with scale 1 / bias 0
    and ``dropout`` in upscale_in_train mode with is_test (their consumers are
    rewired to the op's input)."""

    def _is_identity(self, op):
        if op.type == "scale":
            return op.attrs.get("scale", 1.0) == 1.0 and op.attrs.get("bias", 0.0) == 0.0
        if op.type == "dropout":
            return op.attrs.get("is_test", False) and \
                op.attrs.get("dropout_implementation", "downgrade_in_infer") == "upscale_in_train"
        return False

    def apply_impl(self, graph):
        removed = 0
        for n in list(graph.op_nodes()):
            if not self._is_identity(n.op):
                continue
            src = n.inputs[0]
            out_slot = "Out"
            outs = [v for v in n.outputs if v.name in n.op.output(out_slot)]
            if len(outs) != 1:
                continue
            out = outs[0]
            for c in list(out.outputs):
                c.op.rename_input(out.name, src.name)
                c.inputs = [src if i is out else i for i in c.inputs]
                src.outputs.append(c)
            graph.remove_nodes([n] + list(n.outputs))
            removed += 1
        graph.set("identity_removed", removed)
        return graph


def apply_passes(program, names, block_idx=0, **attrs):
    """Build a Graph of ``program.block(block_idx)``, run ``names`` then
    ``graph_to_program_pass``; returns the graph (attrs hold per-pass stats)."""
    g = Graph(program.block(block_idx))
    for k, v in attrs.items():
        g.set(k, v)
    for nme in list(names) + ["graph_to_program_pass"]:
        g = get_pass(nme).apply(g)
    return g


# ------------------------------------------------------------------ sequence / attention fusions
_SEQ_FC_ACTS = ("sigmoid", "tanh", "relu", "identity")


@register_pass("seq_concat_fc_fuse_pass")
class SeqConcatFcFusePass(Pass):
    """concat(X0, sequence_expand(A), sequence_expand(B)) -> mul(W) -> elementwise_add(b)
    -> act  ==>  fusion_seqexpand_concat_fc(X=[X0, A, B], W, b, fc_activation=act)
    (seq_concat_fc_fuse_pass.cc): the expanded copies of A and B, the concat and the
    fc temporaries are never materialised."""

    def apply_impl(self, graph):
        fused = 0
        for cat in list(graph.op_nodes()):
            if cat not in graph.nodes or not cat.is_op("concat") or len(cat.op.input("X")) != 3:
                continue
            xs = cat.op.input("X")
            by_name = {v.name: v for v in cat.inputs}
            exp_ops = []
            for nm in xs[1:]:
                v = by_name.get(nm)
                prod = [p for p in (v.inputs if v is not None else []) if p.is_op("sequence_expand")]
                if not prod or len(v.outputs) != 1:
                    break
                exp_ops.append((prod[0], v))
            if len(exp_ops) != 2:
                continue
            cat_out = [v for v in cat.outputs if v.name in cat.op.output("Out")]
            if len(cat_out) != 1 or len(cat_out[0].outputs) != 1 or not cat_out[0].outputs[0].is_op("mul"):
                continue
            mul = cat_out[0].outputs[0]
            w = [v for v in mul.inputs if v.name in mul.op.input("Y")]
            if not w or w[0].var is None or not w[0].var.persistable:
                continue
            mul_out = [v for v in mul.outputs if v.name in mul.op.output("Out")][0]
            if len(mul_out.outputs) != 1 or not mul_out.outputs[0].is_op("elementwise_add"):
                continue
            add = mul_out.outputs[0]
            b = [v for v in add.inputs if v.name in add.op.input("Y")]
            if not b or b[0].var is None or not b[0].var.persistable:
                continue
            add_out = [v for v in add.outputs if v.name in add.op.output("Out")][0]
            if len(add_out.outputs) != 1 or add_out.outputs[0].op.type not in _SEQ_FC_ACTS:
                continue
            act = add_out.outputs[0]
            fc_out = [v for v in act.outputs if v.name in act.op.output("Out")][0]
            ins = {"X": [xs[0]] + [e.op.input("X")[0] for e, _ in exp_ops], "FCWeight": [w[0].name],
                   "FCBias": [b[0].name]}
            newop = _new_op(graph.block, "fusion_seqexpand_concat_fc", ins, {"Out": [fc_out.name]},
                            {"fc_activation": act.op.type})
            n = _replace_ops(graph, [e for e, _ in exp_ops] + [cat, mul, add, act], newop,
                             dead_vars=[v for _, v in exp_ops] + [cat_out[0], mul_out, add_out])
            # the expanded inputs A and B now feed the fused op directly
            for e, _ in exp_ops:
                for v in e.inputs:
                    if v.name == e.op.input("X")[0] and v not in n.inputs:
                        _link(v, n)
            fused += 1
        graph.set("seq_concat_fc_fuse_count", fused)
        return graph


@register_pass("attention_lstm_fuse_pass")
class AttentionLSTMFusePass(Pass):
    """Replace the while-loop attention-LSTM decoder of the reference's attention
    model with one ``attention_lstm`` op (attention_lstm_fuse_pass.cc).  The loop is
    recognised by the gate parameters its sub-block reads ({forget,input,output,c}
    .{w_0,w_1,b_0}); the pass concatenates them into the fused op's LSTMWeight
    [D + M, 4D] / LSTMBias [1, 4D] (gate order f, i, o, c) in the parameter scope
    (graph attr ``param_scope``), reshapes the attention biases to [1, n], removes
    the loop and the ops only it used, and wires X / C0 / H0 -> Hidden.  Variable
    names default to the reference's and can be overridden by pass attrs."""

    required_graph_attrs = ("param_scope",)
    DEFAULTS = dict(X="concat_0.tmp_0", C0="cell_init", H0="hidden_init", AttentionWeight="attention_fc.w_0",
                    AttentionBias="attention_fc.b_0", AttentionScalar="attention_output.w_0",
                    AttentionScalarBias="attention_output.b_0", LSTMWeight="attention_w.new",
                    LSTMBias="attention_b.new", Hidden="array_to_lod_tensor_0.tmp_0", Cell="at.cell.new",
                    AttentionedX="at.x.new", AttentionFCOut="at.fc.new", LSTMX="at.lstmx.new",
                    LSTMOUT="at.lstmout.new")
    GATES = ("forget", "input", "output", "c")

    def _reads(self, block):
        names = set()
        for op in block.ops:
            names.update(op.input_arg_names)
            sb = op.attrs.get("sub_block")
            if sb is not None:
                names |= self._reads(sb if hasattr(sb, "ops") else block.program.block(sb))
        return names

    def apply_impl(self, graph):
        P = dict(self.DEFAULTS, **{k: v for k, v in self.attrs.items() if k in self.DEFAULTS})
        gate_params = [f"{g}.{s}" for g in self.GATES for s in ("w_0", "w_1", "b_0")]
        loops = []
        for n in graph.op_nodes():
            if n.is_op("while"):
                sb = n.op.attrs.get("sub_block")
                blk = sb if hasattr(sb, "ops") else graph.program.block(sb)
                if set(gate_params) <= self._reads(blk):
                    loops.append(n)
        if not loops:
            graph.set("attention_lstm_fused", 0)
            return graph
        self._prepare_parameters(graph.get("param_scope"), P)
        dead = set(loops)
        hid = [n for n in graph.op_nodes() if P["Hidden"] in n.op.output_arg_names]
        dead.update(hid)
        keep_names = {P["X"], P["C0"], P["H0"]}
        # ops whose results only the removed loop consumed
        changed = True
        while changed:
            changed = False
            for n in graph.op_nodes():
                if n in dead or n.op.type in ("feed", "fetch"):
                    continue
                outs = n.outputs
                if not outs or any(v.name in keep_names for v in outs):
                    continue
                if any(v.var is not None and v.var.persistable for v in outs):
                    continue
                if all(all(c in dead for c in v.outputs) for v in outs) and \
                        any(c in dead for v in outs for c in v.outputs):
                    dead.add(n)
                    changed = True
        ins = {k: [P[k]] for k in ("X", "C0", "H0", "AttentionWeight", "AttentionBias", "AttentionScalar",
                                   "AttentionScalarBias", "LSTMWeight", "LSTMBias")}
        outs = {k: [P[k]] for k in ("Hidden", "Cell", "AttentionedX", "AttentionFCOut", "LSTMX", "LSTMOUT")}
        blk = graph.block
        for nm in ("LSTMWeight", "LSTMBias"):
            if blk._find_var_recursive(P[nm]) is None:
                blk.create_var(name=P[nm], persistable=True)
        for nm in ("Cell", "AttentionedX", "AttentionFCOut", "LSTMX", "LSTMOUT"):
            if blk._find_var_recursive(P[nm]) is None:
                blk.create_var(name=P[nm])
        newop = _new_op(blk, "attention_lstm", ins, outs, {})
        node = graph.create_op_node(newop)
        node.order = min(n.order for n in loops)
        latest = {}
        for v in graph.var_nodes():
            latest[v.name] = v
        for nm in newop.input_arg_names:
            v = latest.get(nm) or graph.create_var_node(nm)
            _link(v, node)
        hidden_vars = [v for n in hid for v in n.outputs if v.name == P["Hidden"]]
        for nm in newop.output_arg_names:
            v = next((hv for hv in hidden_vars if hv.name == nm), None)
            if v is None:
                v = graph.create_var_node(nm)
            v.inputs = []
            _link(node, v)
        graph.remove_nodes([n for n in dead])
        graph.remove_nodes([v for v in graph.var_nodes() if not v.inputs and not v.outputs])
        graph.set("attention_lstm_fused", len(loops))
        return graph

    def _prepare_parameters(self, scope, P):
        import torch

        from . import core

        def get(name):
            v = scope.find_var(name)
            if v is None or v.get() is None:
                raise KeyError(f"attention_lstm_fuse_pass: parameter {name} not in scope")
            return v.get().tensor

        w0 = [get(f"{g}.w_0") for g in self.GATES]   # [D, D] hidden part
        w1 = [get(f"{g}.w_1") for g in self.GATES]   # [M, D] input part
        bs = [get(f"{g}.b_0").reshape(-1) for g in self.GATES]
        W = torch.cat([torch.cat(w0, 1), torch.cat(w1, 1)], 0)
        b = torch.cat(bs).reshape(1, -1)
        scope.var(P["LSTMWeight"]).set(core.LoDTensor(W.contiguous()))
        scope.var(P["LSTMBias"]).set(core.LoDTensor(b.contiguous()))
        for nm in ("AttentionBias", "AttentionScalarBias"):
            v = scope.find_var(P[nm])
            if v is not None and v.get() is not None and v.get().tensor.dim() == 1:
                v.set(core.LoDTensor(v.get().tensor.reshape(1, -1)))
