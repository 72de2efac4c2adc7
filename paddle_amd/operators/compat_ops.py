"""Remaining reference operator types, so ProgramDescs built by the reference's
lower-level APIs (or loaded from its files) run unchanged.

* ``recurrent`` (operators/recurrent_op.cc): the op StaticRNN emits in the
  reference.  Runs the step block once per time step in its own step scope;
  ``ex_states[t] = states[t-1]`` (``initial_states`` at t = 0); ``inputs`` are
  sliced along dim 0 and bound to the same names inside the step block;
  ``outputs`` are stacked along dim 0.  Differentiated by the auto-VJP of the
  whole op (the step blocks run under autograd, see ``executor.no_stash``).
* ``parallel_do`` (parallel_do_op.cc): splits ``inputs`` along dim 0 over the
  ``places`` list, runs the sub-block per split, concatenates ``outputs``.  One
  process drives one GPU here, so the splits run back to back on it.
* ``read`` / ``create_custom_reader`` (reader/read_op.cc,
  create_custom_reader_op.cc): pull the next batch from a reader variable
  (``next_feed()``), optionally through a preprocessing sub-block.
* ``ncclInit`` / ``ncclAllReduce`` / ``ncclReduce`` / ``ncclBcast``
  (nccl_op.cc): the op-level collectives, on RCCL through
  ``torch.distributed`` (one rank per GPU; the communicator variable is a token).
* ``depthwise_conv2d_transpose``, ``max_pool3d_with_index``,
  ``fusion_seqexpand_concat_fc`` (fused/fusion_seqexpand_concat_fc_op.cc),
  ``attention_lstm`` (attention_lstm_op.cc: per-step attention over the whole
  sequence driven by the previous cell, then an LSTM step with gate order
  {forget, input, output, candidate}).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..framework import core
from ..framework import registry as R
from ..framework.registry import register_op
from .nn_ops import _conv_attrs, conv2d_transpose


# ---------------------------------------------------------------- recurrent
def _block_runner(ctx):
    from ..framework import executor as E

    return E


@register_op("recurrent", ["inputs*?", "initial_states*?", "parameters*?"], ["outputs*?", "step_scopes?"],
             {"ex_states": [], "states": [], "sub_block": None, "reverse": False, "is_train": True},
             no_infer=True, share_lod=False)
def recurrent(ctx):
    E = _block_runner(ctx)
    blk = ctx.attr("sub_block")
    op = ctx.op
    in_names = op.input("inputs")
    out_names = op.output("outputs")
    ex_states, states = list(ctx.attr("ex_states")), list(ctx.attr("states"))
    xs = [v.tensor if isinstance(v, core.LoDTensor) else v for v in ctx.input_values("inputs")]
    init = [v.tensor if isinstance(v, core.LoDTensor) else v for v in ctx.input_values("initial_states")]
    T = xs[0].shape[0]
    order = range(T - 1, -1, -1) if ctx.attr("reverse") else range(T)
    prev = list(init)
    outs = {n: [None] * T for n in out_names}
    scopes = []
    with E.no_stash():
        for t in order:
            s = ctx.scope.new_scope()
            scopes.append(s)
            E.BlockExecutor.create_variables(blk.program, s, blk.idx)
            for n, x in zip(in_names, xs):
                s.var(n).set(core.LoDTensor(x[t]))
            for n, v in zip(ex_states, prev):
                s.var(n).set(core.LoDTensor(v))
            # bind the op's own parameter values (autograd leaves under the auto-VJP)
            for n, v in zip(op.input("parameters"), ctx.input_values("parameters")):
                s.var(n).set(v)
            ctx.executor.run_block(blk.program, blk.idx, s, create_vars=False)
            prev = [s.find_var(n).get().tensor for n in states]
            for n in out_names:
                outs[n][t] = s.find_var(n).get().tensor
    for i, n in enumerate(out_names):
        ctx.set_output("outputs", torch.stack(outs[n], 0), None, i)
    if ctx.has_output("step_scopes"):
        ctx.set_output("step_scopes", scopes)



@register_op("recurrent_grad", ["inputs*?", "initial_states*?", "parameters*?", "outputs*?", "outputs@GRAD*?",
                                "step_scopes?"], ["inputs@GRAD*?", "initial_states@GRAD*?", "parameters@GRAD*?"],
             {"ex_states": [], "states": [], "sub_block": None, "reverse": False, "is_train": True},
             grad=None, no_infer=True, share_lod=False)
def recurrent_grad(ctx):
    """recurrent_op.cc RecurrentGradOp::RunImpl: the grad block once per kept step
    scope, last step first; block-local output gradients hold row t of the outer ones
    plus, for states, the ex-state gradient of the later step; input gradient rows are
    stacked, parameter gradients summed, and the first step's ex-state gradients are
    the initial-state gradients (the C++ executor's RunRecurrentGrad does the same)."""
    from .control_flow_grad import _grad_scope_vars

    op, scope, exe = ctx.op, ctx.scope, ctx.executor
    blk = ctx.attr("sub_block")
    program = blk.program
    steps = ctx.input_value("step_scopes") or []
    T = len(steps)
    order = list(range(T - 1, -1, -1)) if ctx.attr("reverse") else list(range(T))
    ex, st = list(ctx.attr("ex_states")), list(ctx.attr("states"))
    xs, inits, params = op.input("inputs"), op.input("initial_states"), op.input("parameters")
    xgs, igs, pgs = op.output("inputs@GRAD"), op.output("initial_states@GRAD"), op.output("parameters@GRAD")
    g = lambda n: n + "@GRAD"  # noqa: E731
    og_outer = {}
    for n in op.input("outputs@GRAD"):
        v = scope.find_var(n)
        val = v.get() if v is not None else None
        if isinstance(val, core.LoDTensor) and val.tensor is not None:
            og_outer[n] = val.tensor
    carry = [None] * len(ex)
    rows = [[None] * T for _ in xs]
    pacc = {}
    for k in range(T - 1, -1, -1):
        t, s = order[k], steps[k]
        gs = s.new_scope()
        _grad_scope_vars(program, gs, blk.idx, set())
        # <name>@GRAD@EXT of every step output / state: row t of its outer gradient
        # plus the later step's ex-state gradient, zeros when neither exists (the
        # grad block adds it to its own contributions: backward.py _recurrent_grad_descs)
        for n in dict.fromkeys(st + list(op.input("outputs"))):
            ext = og_outer[g(n)][t].clone() if g(n) in og_outer else None
            if n in st and carry[st.index(n)] is not None:
                c = carry[st.index(n)]
                ext = c.clone() if ext is None else ext + c
            if ext is None:
                ext = torch.zeros_like(s.find_local_var(n).get().tensor)
            gs.var(g(n) + "@EXT").set(core.LoDTensor(ext))
        exe.run_block(program, blk.idx, gs, create_vars=False)

        def local(n):
            v = gs.find_local_var(n)
            val = v.get() if v is not None else None
            return val.tensor if isinstance(val, core.LoDTensor) and val.tensor is not None else None
        for j, x in enumerate(xs):
            if xgs and j < len(xgs) and xgs[j] != R.EMPTY_VAR:
                rows[j][t] = local(g(x))
        for j, p in enumerate(params):
            if pgs and j < len(pgs) and pgs[j] != R.EMPTY_VAR:
                r = local(g(p))
                if r is not None:
                    pacc[pgs[j]] = r.clone() if pgs[j] not in pacc else pacc[pgs[j]] + r
        carry = [None if local(g(e)) is None else local(g(e)).clone() for e in ex]
        if gs in getattr(s, "_kids", ()):
            s._kids.remove(gs)

    def value(n):
        v = scope.find_var(n)
        val = v.get() if v is not None else None
        return val.tensor if isinstance(val, core.LoDTensor) else val
    for j, x in enumerate(xs):
        if not xgs or j >= len(xgs) or xgs[j] == R.EMPTY_VAR:
            continue
        xv = value(x)
        r = [rows[j][t] if rows[j][t] is not None else torch.zeros_like(xv[t]) for t in range(T)]
        scope.var(xgs[j]).set(core.LoDTensor(torch.stack(r, 0)))
    for j, p in enumerate(params):
        if pgs and j < len(pgs) and pgs[j] != R.EMPTY_VAR:
            scope.var(pgs[j]).set(core.LoDTensor(pacc[pgs[j]] if pgs[j] in pacc else torch.zeros_like(value(p))))
    for i, n in enumerate(inits):
        if igs and i < len(igs) and igs[i] != R.EMPTY_VAR:
            c = carry[i] if i < len(carry) else None
            scope.var(igs[i]).set(core.LoDTensor(c if c is not None else torch.zeros_like(value(n))))

# ---------------------------------------------------------------- parallel_do
@register_op("parallel_do", ["inputs*?", "parameters*?", "places?"], ["outputs*?", "parallel_scopes?"],
             {"sub_block": None, "use_nccl": False}, no_infer=True, share_lod=False)
def parallel_do(ctx):
    E = _block_runner(ctx)
    blk = ctx.attr("sub_block")
    op = ctx.op
    places = ctx.input_value("places")
    n = len(places) if isinstance(places, (list, tuple)) and places else 1
    in_names, out_names = op.input("inputs"), op.output("outputs")
    xs = [v.tensor if isinstance(v, core.LoDTensor) else v for v in ctx.input_values("inputs")]
    splits = [torch.tensor_split(x, n, 0) for x in xs]
    outs = {k: [] for k in out_names}
    scopes = []
    with E.no_stash():
        for r in range(n):
            s = ctx.scope.new_scope()
            scopes.append(s)
            E.BlockExecutor.create_variables(blk.program, s, blk.idx)
            for k, sp in zip(in_names, splits):
                s.var(k).set(core.LoDTensor(sp[r]))
            for k, v in zip(op.input("parameters"), ctx.input_values("parameters")):
                s.var(k).set(v)
            ctx.executor.run_block(blk.program, blk.idx, s, create_vars=False)
            for k in out_names:
                outs[k].append(s.find_var(k).get().tensor)
    for i, k in enumerate(out_names):
        ctx.set_output("outputs", torch.cat(outs[k], 0), None, i)
    if ctx.has_output("parallel_scopes"):
        ctx.set_output("parallel_scopes", scopes)


# ---------------------------------------------------------------- readers
class _CustomReader:
    """A reader whose batches pass through a preprocessing sub-block."""

    def __init__(self, under, blk, sources, sinks, executor, scope):
        self.under, self.blk, self.sources, self.sinks = under, blk, sources, sinks
        self.executor, self.scope = executor, scope

    def next_feed(self):
        item = self.under.next_feed()
        vals = list(item.values()) if isinstance(item, dict) else list(item)
        s = self.scope.new_scope()
        self.executor.create_variables(self.blk.program, s, self.blk.idx)
        for n, v in zip(self.sources, vals):
            s.var(n).set(v if isinstance(v, core.LoDTensor) else core.LoDTensor(torch.as_tensor(v)))
        self.executor.run_block(self.blk.program, self.blk.idx, s, create_vars=False)
        return [s.find_var(n).get() for n in self.sinks]


@register_op("create_custom_reader", ["UnderlyingReader"], ["Out"],
             {"sub_block": None, "source_var_names": [], "sink_var_names": []}, grad=None, no_infer=True,
             share_lod=False)
def create_custom_reader(ctx):
    ctx.set_output("Out", _CustomReader(ctx.input_value("UnderlyingReader"), ctx.attr("sub_block"),
                                        list(ctx.attr("source_var_names")), list(ctx.attr("sink_var_names")),
                                        ctx.executor, ctx.scope))


@register_op("read", ["Reader"], ["Out*"], {"throw_eof_exp": True}, grad=None, no_infer=True, share_lod=False)
def read(ctx):
    from ..fluid.layers.io import EOFException

    reader = ctx.input_value("Reader")
    try:
        item = reader.next_feed()
    except EOFException:
        if ctx.attr("throw_eof_exp"):
            raise
        return
    vals = list(item.values()) if isinstance(item, dict) else list(item)
    dev = ctx.device
    for i, v in enumerate(vals):
        if isinstance(v, core.LoDTensor):
            ctx.set_output("Out", core.LoDTensor(v.tensor.to(dev), v.lod()), None, i)
        else:
            ctx.set_output("Out", torch.as_tensor(v).to(dev), None, i)


# ---------------------------------------------------------------- op-level collectives
_NCCL_OPS = {"ncclSum": "SUM", "ncclProd": "PRODUCT", "ncclMax": "MAX", "ncclMin": "MIN"}


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


@register_op("ncclInit", ["parallel_scopes?"], ["Communicator"], {}, grad=None, no_infer=True, share_lod=False)
def nccl_init(ctx):
    d = _dist()
    ctx.set_output("Communicator", {"world": d.get_world_size() if d else 1, "rank": d.get_rank() if d else 0})


@register_op("ncclAllReduce", ["X", "Communicator?"], ["Out"], {"reduction": "ncclSum"}, grad=None)
def nccl_all_reduce(ctx):
    x = ctx.input("X").clone()
    d = _dist()
    if d is not None:
        d.all_reduce(x, op=getattr(d.ReduceOp, _NCCL_OPS[ctx.attr("reduction")]))
    ctx.set_output("Out", x)


@register_op("ncclReduce", ["X", "Communicator?"], ["Out"], {"reduction": "ncclSum", "root": 0}, grad=None)
def nccl_reduce(ctx):
    x = ctx.input("X").clone()
    d = _dist()
    if d is not None:
        d.reduce(x, dst=int(ctx.attr("root")), op=getattr(d.ReduceOp, _NCCL_OPS[ctx.attr("reduction")]))
    ctx.set_output("Out", x)


@register_op("ncclBcast", ["X", "Communicator?"], ["Out"], {"root": 0}, grad=None)
def nccl_bcast(ctx):
    x = ctx.input("X").clone()
    d = _dist()
    if d is not None:
        d.broadcast(x, src=int(ctx.attr("root")))
    ctx.set_output("Out", x)


# ---------------------------------------------------------------- conv / pool variants
@register_op("depthwise_conv2d_transpose", ["Input", "Filter"], ["Output"], _conv_attrs({"output_size": []}))
def depthwise_conv2d_transpose(ctx):
    conv2d_transpose(ctx)   # groups == channels: the grouped transposed convolution


@register_op("max_pool3d_with_index", ["X"], ["Out", "Mask"], {"ksize": [2, 2, 2], "global_pooling": False,
                                                               "strides": [1, 1, 1], "paddings": [0, 0, 0]})
def max_pool3d_with_index(ctx):
    x = ctx.input("X")
    k, s, p = ctx.attr("ksize"), ctx.attr("strides"), ctx.attr("paddings")
    if ctx.attr("global_pooling"):
        k, p = list(x.shape[2:]), [0, 0, 0]
    from ..ops import convnd as _cnd
    if _cnd.supported_pool(x) and x.dim() == 5:
        y, idx = _cnd.pool_nd(x, "max", k, s, p, return_mask=True)
        ctx.set_output("Out", y)
        ctx.set_output("Mask", idx)
        return
    y, idx = F.max_pool3d(x, k, s, p, return_indices=True)
    ctx.set_output("Out", y)
    ctx.set_output("Mask", idx.to(torch.int32))


# ---------------------------------------------------------------- fused sequence ops
_ACT = {"": lambda t: t, "identity": lambda t: t, "relu": torch.relu, "sigmoid": torch.sigmoid,
        "tanh": torch.tanh}


@register_op("fusion_seqexpand_concat_fc", ["X*", "FCWeight", "FCBias?"], ["Out", "FCOut~"],
             {"fc_activation": "identity"}, share_lod=False)
def fusion_seqexpand_concat_fc(ctx):
    """X[0]: LoD [T, M0] (defines the sequences); X[1..]: [N, Mi], one row per
    sequence, expanded to every step of it; out = act(concat(...) W + b)."""
    xs = ctx.inputs("X")
    lod = ctx.input_lod("X")
    off = lod[-1] if lod else [0, xs[0].shape[0]]
    lens = torch.tensor([off[i + 1] - off[i] for i in range(len(off) - 1)], device=xs[0].device)
    parts = [xs[0]] + [torch.repeat_interleave(x, lens, 0) for x in xs[1:]]
    fc = torch.cat(parts, 1) @ ctx.input("FCWeight")
    if ctx.has_input("FCBias"):
        fc = fc + ctx.input("FCBias").reshape(-1)
    ctx.set_output("FCOut", fc)
    ctx.set_output("Out", _ACT[ctx.attr("fc_activation")](fc), lod)


@register_op("attention_lstm", ["X", "C0", "H0?", "AttentionWeight", "AttentionBias?", "AttentionScalar?",
                                "AttentionScalarBias?", "LSTMWeight", "LSTMBias"],
             ["Hidden", "Cell", "AttentionedX~", "AttentionFCOut~", "LSTMX~", "LSTMOUT~"],
             {"gate_activation": "sigmoid", "cell_activation": "tanh", "candidate_activation": "tanh"},
             share_lod=False)
def attention_lstm(ctx):
    x = ctx.input("X")
    lod = ctx.input_lod("X")
    off = lod[-1]
    N, T, M = len(off) - 1, x.shape[0], x.shape[1]
    W = ctx.input("LSTMWeight")              # [(D + M), 4D]: rows [0, D) hidden, [D, D + M) input
    D = W.shape[1] // 4
    aw = ctx.input("AttentionWeight").reshape(-1)      # [(M + D)]
    ab = ctx.input("AttentionBias").reshape(-1) if ctx.has_input("AttentionBias") else None
    sc = ctx.input("AttentionScalar").reshape(-1) if ctx.has_input("AttentionScalar") else None
    scb = ctx.input("AttentionScalarBias").reshape(-1) if ctx.has_input("AttentionScalarBias") else None
    b = ctx.input("LSTMBias").reshape(-1)
    act_g, act_c, act_cand = (_ACT[ctx.attr(k)] for k in ("gate_activation", "cell_activation",
                                                            "candidate_activation"))
    lens = [off[i + 1] - off[i] for i in range(N)]
    L = max(lens)
    dev = x.device
    idx = torch.full((N, L), -1, dtype=torch.long)
    for i, n in enumerate(lens):
        idx[i, :n] = torch.arange(off[i], off[i] + n)
    idx = idx.to(dev)
    valid = idx >= 0                                     # [N, L]
    xp = x[idx.clamp(min=0)] * valid.unsqueeze(-1)       # [N, L, M]
    ax = x @ aw[:M]
    if ab is not None:
        ax = ax + ab
    axp = ax[idx.clamp(min=0)]                           # [N, L]
    c = ctx.input("C0")
    h = ctx.input("H0") if ctx.has_input("H0") else None
    hs, cs = [], []
    fc = None
    for t in range(L):
        cb = c @ aw[M:]                                  # [N]
        fc = torch.relu(axp + cb.unsqueeze(1))
        if sc is not None:
            fc = fc * sc
            fc = torch.relu(fc + scb) if scb is not None else torch.relu(fc)
        fc = torch.softmax(fc.masked_fill(~valid, float("-inf")), 1)
        lx = torch.einsum("nl,nlm->nm", fc, xp)          # [N, M]
        g = lx @ W[D:]
        if h is not None:
            g = g + h @ W[:D]
        g = g + b
        f, i_, o = act_g(g[:, :D]), act_g(g[:, D:2 * D]), act_g(g[:, 2 * D:3 * D])
        cand = act_cand(g[:, 3 * D:])
        cn = f * c + i_ * cand
        hn = act_c(cn) * o
        alive = (t < torch.tensor(lens, device=dev)).unsqueeze(1)
        c = torch.where(alive, cn, c)
        h = torch.where(alive, hn, h) if h is not None else torch.where(alive, hn, torch.zeros_like(hn))
        hs.append(hn)
        cs.append(cn)
    sel = valid.reshape(-1)
    flat_idx = idx.reshape(-1)[sel]
    H = torch.zeros(T, D, dtype=x.dtype, device=dev).index_copy(0, flat_idx, torch.stack(hs, 1).reshape(-1, D)[sel])
    C = torch.zeros(T, D, dtype=x.dtype, device=dev).index_copy(0, flat_idx, torch.stack(cs, 1).reshape(-1, D)[sel])
    ctx.set_output("Hidden", H, lod)
    ctx.set_output("Cell", C, lod)
    ctx.set_output("AttentionedX", ax.reshape(T, 1).detach())
    ctx.set_output("AttentionFCOut", fc.detach()[-1].reshape(-1, 1))
    ctx.set_output("LSTMX", lx.detach()[-1:].reshape(1, M))
    ctx.set_output("LSTMOUT", g.detach()[-1:].reshape(1, 4 * D))
