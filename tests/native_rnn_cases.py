"""LoD recurrent programs for the C++ executor's lstm / gru kernels (ops_rnn.cc,
ops_rnn_gpu.hip): dynamic_lstm (peepholes, reverse, relu candidate -- the book
label_semantic_roles settings), dynamic_gru, trained end to end; the native engine must
follow the interpreter's trajectory with the recurrent ops run natively.
Reference: python/paddle/fluid/tests/book/test_label_semantic_roles.py (db_lstm),
operators/lstm_op.h, operators/gru_op.h."""
import numpy as np
import torch

import paddle_amd.fluid as fluid
from paddle_amd.framework import core

V, E, H = 40, 8, 6


def lstm_net(peep=True, rev=False, cand="tanh", cell="tanh", h0=False):
    def build():
        words = fluid.layers.data(name="words", shape=[1], lod_level=1, dtype="int64")
        label = fluid.layers.data(name="label", shape=[1], dtype="int64")
        emb = fluid.layers.embedding(input=words, size=[V, E])
        proj = fluid.layers.fc(input=emb, size=4 * H)
        init_h = init_c = None
        if h0:
            init_h = fluid.layers.data(name="h0", shape=[H], dtype="float32")
            init_c = fluid.layers.data(name="c0", shape=[H], dtype="float32")
            init_h.stop_gradient = init_c.stop_gradient = False
        hid, cell_ = fluid.layers.dynamic_lstm(input=proj, size=4 * H, h_0=init_h, c_0=init_c, use_peepholes=peep,
                                               is_reverse=rev, candidate_activation=cand, cell_activation=cell)
        last = fluid.layers.sequence_pool(hid, "last")
        cl = fluid.layers.sequence_pool(cell_, "max")
        logit = fluid.layers.fc(input=[last, cl], size=3, act="softmax")
        loss = fluid.layers.mean(fluid.layers.cross_entropy(input=logit, label=label))
        fluid.optimizer.SGD(learning_rate=0.5).minimize(loss)
        return [loss]
    return build


def gru_net(rev=False, h0=False):
    def build():
        words = fluid.layers.data(name="words", shape=[1], lod_level=1, dtype="int64")
        label = fluid.layers.data(name="label", shape=[1], dtype="int64")
        emb = fluid.layers.embedding(input=words, size=[V, E])
        proj = fluid.layers.fc(input=emb, size=3 * H)
        init_h = None
        if h0:
            init_h = fluid.layers.data(name="h0", shape=[H], dtype="float32")
            init_h.stop_gradient = False
        hid = fluid.layers.dynamic_gru(input=proj, size=H, is_reverse=rev, h_0=init_h)
        last = fluid.layers.sequence_pool(hid, "sum")
        logit = fluid.layers.fc(input=last, size=3, act="softmax")
        loss = fluid.layers.mean(fluid.layers.cross_entropy(input=logit, label=label))
        fluid.optimizer.Adam(learning_rate=0.02).minimize(loss)
        return [loss]
    return build


def feeds(steps=4, h0=False, c0=False):
    out = []
    for seed in range(steps):
        rs = np.random.RandomState(seed)
        lens = rs.randint(1, 9, 5).tolist()
        off = np.concatenate([[0], np.cumsum(lens)]).tolist()
        fd = {"words": core.LoDTensor(torch.from_numpy(rs.randint(0, V, (off[-1], 1)).astype("int64")), [off]),
              "label": core.LoDTensor(torch.from_numpy(rs.randint(0, 3, (len(lens), 1)).astype("int64")))}
        if h0:
            fd["h0"] = core.LoDTensor(torch.from_numpy(rs.randn(len(lens), H).astype("float32") * 0.5))
        if c0:
            fd["c0"] = core.LoDTensor(torch.from_numpy(rs.randn(len(lens), H).astype("float32") * 0.5))
        out.append(fd)
    return out


CASES = {
    "lstm_peep": (lstm_net(), {}),
    "lstm_rev_relu_srl": (lstm_net(rev=True, cand="relu", cell="sigmoid"), {}),
    "lstm_nopeep_h0": (lstm_net(peep=False, h0=True), {"h0": True, "c0": True}),
    "gru": (gru_net(), {}),
    "gru_rev_h0": (gru_net(rev=True, h0=True), {"h0": True}),
}


# ---------------------------------------------------------------------------------
# book label_semantic_roles (tests/book/test_label_semantic_roles.py db_lstm) at toy
# sizes: 8 LoD feature slots -> embeddings (one shared, frozen; is_sparse ones) -> fc
# -> sums -> a stack of dynamic_lstm alternating direction (relu candidate, sigmoid
# cell) -> linear_chain_crf cost with SGD on exponential_decay; crf_decoding fetched.
WD, LD, PD, MD = 30, 7, 6, 2  # word / label / predicate dicts, mark dict


def srl(depth=3, hidden=8, word_dim=4, mark_dim=3):
    def build():
        names = ["word", "verb", "ctx_n2", "ctx_n1", "ctx_0", "ctx_p1", "ctx_p2", "mark"]
        feats = {n: fluid.layers.data(name=n, shape=[1], dtype="int64", lod_level=1) for n in names}
        target = fluid.layers.data(name="target", shape=[1], dtype="int64", lod_level=1)
        pred_emb = fluid.layers.embedding(input=feats["verb"], size=[PD, word_dim], is_sparse=True,
                                          param_attr="vemb")
        mark_emb = fluid.layers.embedding(input=feats["mark"], size=[MD, mark_dim], is_sparse=True)
        embs = [fluid.layers.embedding(size=[WD, word_dim], input=feats[n],
                                       param_attr=fluid.ParamAttr(name="emb", trainable=False))
                for n in ("word", "ctx_n2", "ctx_n1", "ctx_0", "ctx_p1", "ctx_p2")]
        embs += [pred_emb, mark_emb]
        h0 = fluid.layers.sums(input=[fluid.layers.fc(input=e, size=hidden) for e in embs])
        lstm = fluid.layers.dynamic_lstm(input=fluid.layers.fc(h0, 4 * hidden), size=4 * hidden,
                                         candidate_activation="relu", gate_activation="sigmoid",
                                         cell_activation="sigmoid")[0]
        tmp = [h0, lstm]
        for i in range(1, depth):
            mix = fluid.layers.sums(input=[fluid.layers.fc(input=tmp[0], size=hidden),
                                           fluid.layers.fc(input=tmp[1], size=hidden)])
            lstm = fluid.layers.dynamic_lstm(input=fluid.layers.fc(mix, 4 * hidden), size=4 * hidden,
                                             candidate_activation="relu", gate_activation="sigmoid",
                                             cell_activation="sigmoid", is_reverse=(i % 2) == 1)[0]
            tmp = [mix, lstm]
        feature = fluid.layers.sums(input=[fluid.layers.fc(input=tmp[0], size=LD, act="tanh"),
                                           fluid.layers.fc(input=tmp[1], size=LD, act="tanh")])
        crf_cost = fluid.layers.linear_chain_crf(input=feature, label=target,
                                                 param_attr=fluid.ParamAttr(name="crfw", learning_rate=0.5))
        avg = fluid.layers.mean(crf_cost)
        fluid.optimizer.SGD(learning_rate=fluid.layers.exponential_decay(
            learning_rate=0.05, decay_steps=3, decay_rate=0.5, staircase=True)).minimize(avg)
        decode = fluid.layers.crf_decoding(input=feature, param_attr=fluid.ParamAttr(name="crfw"))
        return [avg, decode]
    return build


def srl_feeds(steps=4):
    out = []
    for seed in range(steps):
        rs = np.random.RandomState(100 + seed)
        lens = rs.randint(2, 8, 4).tolist()
        off = np.concatenate([[0], np.cumsum(lens)]).tolist()
        n = off[-1]

        def ids(hi):
            return core.LoDTensor(torch.from_numpy(rs.randint(0, hi, (n, 1)).astype("int64")), [off])
        fd = {k: ids(WD) for k in ("word", "ctx_n2", "ctx_n1", "ctx_0", "ctx_p1", "ctx_p2")}
        fd.update(verb=ids(PD), mark=ids(MD), target=ids(LD))
        out.append(fd)
    return out
