"""Programs with step scopes, tensor arrays, rank tables and SelectedRows gradients
for the native-engine tests (CPU and GPU): DynamicRNN training (while / while_grad,
reference tests/unittests/test_dyn_rnn.py), the stacked-LSTM benchmark's DynamicRNN
(benchmark/fluid/models/stacked_dynamic_lstm.py) and book word2vec with a shared
is_sparse embedding (tests/book/test_word2vec.py) under SGD and Adam."""
import numpy as np
import torch

import paddle_amd.fluid as fluid
from paddle_amd.framework import core

D, H = 5, 6
LOD = [0, 3, 5, 9]


def run(build, feeds, engine, place, init=None):
    """Runs ``build``'s program for every feed; returns (fetches per step, initial
    persistables, executor).  ``init`` (from a first run) makes both engines start
    from identical parameters."""
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 7
    with fluid.unique_name.guard(), fluid.program_guard(main, startup):
        fetch = build()
    scope = core.Scope()
    out = []
    with fluid.executor.scope_guard(scope):
        fluid.Executor(place, engine="python").run(startup)
        pers = [v.name for v in main.list_vars() if v.persistable and v.name not in ("feed", "fetch")
                and scope.find_var(v.name) is not None and scope.find_var(v.name).get() is not None]
        if init is None:
            init = {n: np.array(scope.find_var(n).get_tensor().numpy()) for n in pers}
        else:
            for n in pers:
                scope.find_var(n).get_tensor().set(init[n], place)
        exe = fluid.Executor(place, engine=engine)
        for fd in feeds:
            res = exe.run(main, feed=fd, fetch_list=fetch)
            out.append([np.array(r) for r in res])
    return out, init, exe


def drnn_grads():
    """DynamicRNN tanh cell: output, loss, x@GRAD and the parameter gradients."""
    x = fluid.layers.data(name="x", shape=[D], dtype="float32", lod_level=1)
    x.stop_gradient = False
    drnn = fluid.layers.DynamicRNN()
    with drnn.block():
        word = drnn.step_input(x)
        prev = drnn.memory(shape=[H], value=0.0)
        hidden = fluid.layers.fc(input=[word, prev], size=H, act="tanh",
                                 param_attr=[fluid.ParamAttr(name="wx"), fluid.ParamAttr(name="wh")],
                                 bias_attr=fluid.ParamAttr(name="b"))
        drnn.update_memory(prev, hidden)
        drnn.output(hidden)
    out = drnn()
    loss = fluid.layers.mean(out * out)
    pg = fluid.backward.append_backward(loss)
    return [out, loss, "x@GRAD"] + [g for _, g in pg]


def drnn_feeds(steps=2, place=None):
    rng = np.random.RandomState(0)
    return [{"x": core.LoDTensor(torch.from_numpy(rng.randn(LOD[-1], D).astype("float32")), [LOD])}
            for _ in range(steps)]


def drnn_train():
    x = fluid.layers.data(name="x", shape=[D], dtype="float32", lod_level=1)
    y = fluid.layers.data(name="y", shape=[1], dtype="float32", lod_level=1)
    drnn = fluid.layers.DynamicRNN()
    with drnn.block():
        word = drnn.step_input(x)
        prev = drnn.memory(shape=[H], value=0.0)
        hidden = fluid.layers.fc(input=[word, prev], size=H, act="tanh")
        drnn.update_memory(prev, hidden)
        drnn.output(hidden)
    pred = fluid.layers.fc(drnn(), size=1)
    loss = fluid.layers.mean(fluid.layers.square_error_cost(pred, y))
    fluid.optimizer.Adam(learning_rate=0.05).minimize(loss)
    return [loss]


def drnn_train_feeds(steps=8):
    rng = np.random.RandomState(1)
    xv = rng.randn(LOD[-1], D).astype("float32")
    yv = np.cumsum(xv[:, :1], 0).astype("float32") * 0.3
    return [{"x": core.LoDTensor(torch.from_numpy(xv), [LOD]), "y": core.LoDTensor(torch.from_numpy(yv), [LOD])}
            for _ in range(steps)]


def stacked_lstm():
    V, E, Hs = 50, 8, 8
    words = fluid.layers.data(name="words", shape=[1], lod_level=1, dtype="int64")
    label = fluid.layers.data(name="label", shape=[1], dtype="int64")
    sent = fluid.layers.embedding(input=words, size=[V, E])
    sent = fluid.layers.fc(input=sent, size=Hs, act="tanh")
    rnn = fluid.layers.DynamicRNN()
    with rnn.block():
        w = rnn.step_input(sent)
        ph = rnn.memory(value=0.0, shape=[Hs])
        pc = rnn.memory(value=0.0, shape=[Hs])

        def gate(act):
            g = fluid.layers.sums(input=[fluid.layers.fc(input=w, size=Hs),
                                         fluid.layers.fc(input=ph, size=Hs, bias_attr=False)])
            return act(g)

        f, i, o = (gate(fluid.layers.sigmoid) for _ in range(3))
        cg = gate(fluid.layers.tanh)
        c = fluid.layers.sums(input=[fluid.layers.elementwise_mul(f, pc), fluid.layers.elementwise_mul(i, cg)])
        h = fluid.layers.elementwise_mul(o, fluid.layers.tanh(c))
        rnn.update_memory(pc, c)
        rnn.update_memory(ph, h)
        rnn.output(h)
    last = fluid.layers.sequence_pool(rnn(), "last")
    logit = fluid.layers.fc(input=last, size=2, act="softmax")
    loss = fluid.layers.mean(fluid.layers.cross_entropy(input=logit, label=label))
    fluid.optimizer.Adam(learning_rate=1e-2).minimize(loss)
    return [loss]


def stacked_lstm_feeds(steps=4):
    """Batches of different length profiles back to back (arrays / grads must not
    carry over between runs)."""
    out = []
    for seed in range(steps):
        rs = np.random.RandomState(seed)
        lens = rs.randint(1, 12, 5).tolist()
        off = np.concatenate([[0], np.cumsum(lens)]).tolist()
        ids = torch.from_numpy(rs.randint(0, 50, (off[-1], 1)).astype("int64"))
        lab = torch.from_numpy(rs.randint(0, 2, (len(lens), 1)).astype("int64"))
        out.append({"words": core.LoDTensor(ids, [off]), "label": core.LoDTensor(lab)})
    return out


def word2vec(opt):
    def build():
        ws = [fluid.layers.data(name=f"w{i}", shape=[1], dtype="int64") for i in range(5)]
        embs = [fluid.layers.embedding(input=w, size=[64, 16], dtype="float32", is_sparse=True,
                                       param_attr="shared_w") for w in ws[:4]]
        c = fluid.layers.concat(input=embs, axis=1)
        h = fluid.layers.fc(input=c, size=32, act="sigmoid")
        p = fluid.layers.fc(input=h, size=64, act="softmax")
        loss = fluid.layers.mean(fluid.layers.cross_entropy(input=p, label=ws[4]))
        (fluid.optimizer.SGD(learning_rate=0.5) if opt == "sgd" else fluid.optimizer.Adam(learning_rate=0.02)
         ).minimize(loss)
        return [loss]
    return build


def word2vec_feeds(steps=6):
    rs = np.random.RandomState(3)
    out = []
    for _ in range(steps):
        # small vocabulary draws: the 4 context words of a batch repeat ids, so the
        # SelectedRows gradient holds duplicate rows (merged by sum / sparse Adam)
        ids = rs.randint(0, 20, size=(16, 5)).astype("int64")
        out.append({f"w{i}": ids[:, i:i + 1] for i in range(5)})
    return out


CASES = {
    "drnn_grads": (drnn_grads, drnn_feeds),
    "drnn_train": (drnn_train, drnn_train_feeds),
    "stacked_lstm": (stacked_lstm, stacked_lstm_feeds),
    "word2vec_sparse_sgd": (word2vec("sgd"), word2vec_feeds),
    "word2vec_sparse_adam": (word2vec("adam"), word2vec_feeds),
}


def device_ops():
    """The ops that used to have only host kernels (cast, compare / logical,
    increment, assign, arg_max, shape, reduce_prod, elementwise_mul/div grads)."""
    L = fluid.layers
    x = L.data(name="x", shape=[6], dtype="float32")
    y = L.data(name="y", shape=[6], dtype="float32", append_batch_size=False)
    x.stop_gradient = False
    y.stop_gradient = False
    m = L.elementwise_mul(x, y)
    d = L.elementwise_div(x, L.scale(y, scale=1.0, bias=3.0))
    loss = L.mean(L.elementwise_add(m, d))
    pg = fluid.backward.append_backward(loss)
    zero = L.fill_constant([1], "float32", 0.0)
    lt = L.less_than(x, L.scale(y, scale=0.5))
    ge = L.logical_not(lt)
    both = L.logical_and(lt, L.equal(x, x))
    cnt = L.fill_constant([1], "int64", 3)
    L.increment(cnt, value=2.0, in_place=True)
    return [loss, "x@GRAD", "y@GRAD", L.cast(x, "int32"), L.cast(L.cast(x, "float16"), "float32"), lt, ge, both,
            cnt, L.argmax(x, axis=1), L.shape(x), L.reduce_prod(x, dim=1), L.assign(x), zero] + [g for _, g in pg]


def device_ops_feeds(steps=2):
    rs = np.random.RandomState(11)
    return [{"x": rs.randn(5, 6).astype("float32"), "y": (rs.rand(6) + 0.5).astype("float32")} for _ in range(steps)]


CASES_DEVICE_OPS = {"device_ops": (device_ops, device_ops_feeds)}


def cond_block(flag):
    """conditional_block training: fc inside the block, loss outside; the grads
    flow through conditional_block_grad (zeros when the block did not run)."""
    def build():
        L = fluid.layers
        x = L.data(name="x", shape=[4], dtype="float32")
        x.stop_gradient = False
        out = L.fill_constant_batch_size_like(x, [-1, 3], "float32", 0.0)
        out.stop_gradient = False
        cond = L.fill_constant([1], "bool", flag, force_cpu=True)
        cb = L.ConditionalBlock([cond], is_scalar_condition=True)
        with cb.block():
            h = L.fc(x, size=3, act="tanh", param_attr=fluid.ParamAttr(name="cw"),
                     bias_attr=fluid.ParamAttr(name="cb"))
            L.assign(h, out)
        loss = L.mean(L.elementwise_mul(out, out))
        pg = fluid.backward.append_backward(loss)
        return [loss, "x@GRAD"] + [g for _, g in pg]
    return build


def cond_block_feeds(steps=2):
    rs = np.random.RandomState(5)
    return [{"x": rs.randn(6, 4).astype("float32")} for _ in range(steps)]


CASES["cond_block_true"] = (cond_block(True), cond_block_feeds)
CASES["cond_block_false"] = (cond_block(False), cond_block_feeds)
