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
