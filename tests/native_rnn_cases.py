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


def lstmp_net(peep=True, rev=False, proj_act="tanh"):
    def build():
        words = fluid.layers.data(name="words", shape=[1], lod_level=1, dtype="int64")
        label = fluid.layers.data(name="label", shape=[1], dtype="int64")
        emb = fluid.layers.embedding(input=words, size=[V, E])
        proj = fluid.layers.fc(input=emb, size=4 * H)
        r, c = fluid.layers.dynamic_lstmp(input=proj, size=4 * H, proj_size=4, use_peepholes=peep, is_reverse=rev,
                                          proj_activation=proj_act)
        last = fluid.layers.sequence_pool(r, "last")
        cl = fluid.layers.sequence_pool(c, "average")
        logit = fluid.layers.fc(input=[last, cl], size=3, act="softmax")
        loss = fluid.layers.mean(fluid.layers.cross_entropy(input=logit, label=label))
        fluid.optimizer.SGD(learning_rate=0.5).minimize(loss)
        return [loss]
    return build


CASES = {
    "lstmp_peep": (lstmp_net(), {}),
    "lstmp_rev_nopeep_relu": (lstmp_net(peep=False, rev=True, proj_act="relu"), {}),
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


def srl(depth=3, hidden=8, word_dim=4, mark_dim=3, extra=False):
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
        dbg = [h0, lstm]
        for i in range(1, depth):
            mix = fluid.layers.sums(input=[fluid.layers.fc(input=tmp[0], size=hidden),
                                           fluid.layers.fc(input=tmp[1], size=hidden)])
            lstm = fluid.layers.dynamic_lstm(input=fluid.layers.fc(mix, 4 * hidden), size=4 * hidden,
                                             candidate_activation="relu", gate_activation="sigmoid",
                                             cell_activation="sigmoid", is_reverse=(i % 2) == 1)[0]
            tmp = [mix, lstm]
            dbg += [mix, lstm]
        feature = fluid.layers.sums(input=[fluid.layers.fc(input=tmp[0], size=LD, act="tanh"),
                                           fluid.layers.fc(input=tmp[1], size=LD, act="tanh")])
        crf_cost = fluid.layers.linear_chain_crf(input=feature, label=target,
                                                 param_attr=fluid.ParamAttr(name="crfw", learning_rate=0.5))
        avg = fluid.layers.mean(crf_cost)
        fluid.optimizer.SGD(learning_rate=fluid.layers.exponential_decay(
            learning_rate=0.05, decay_steps=3, decay_rate=0.5, staircase=True)).minimize(avg)
        decode = fluid.layers.crf_decoding(input=feature, param_attr=fluid.ParamAttr(name="crfw"))
        if extra:
            return [avg, decode, feature, crf_cost] + dbg
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


# ---------------------------------------------------------------------------------
# book machine_translation (tests/book/test_machine_translation.py) at toy sizes:
# training = LSTM encoder + DynamicRNN decoder, Adagrad with L2 decay; decoding =
# the While loop with topk + beam_search over tensor arrays + beam_search_decode.
MT_DICT, MT_WORD, MT_HID, MT_BEAM, MT_MAXLEN, MT_END = 20, 6, 8, 2, 4, 3


def _mt_encoder():
    src = fluid.layers.data(name="src_word_id", shape=[1], dtype="int64", lod_level=1)
    emb = fluid.layers.embedding(input=src, size=[MT_DICT, MT_WORD], param_attr=fluid.ParamAttr(name="vemb"))
    fc1 = fluid.layers.fc(input=emb, size=MT_HID * 4, act="tanh")
    hid, _ = fluid.layers.dynamic_lstm(input=fc1, size=MT_HID * 4)
    return fluid.layers.sequence_last_step(input=hid)


def mt_train():
    ctx = _mt_encoder()
    trg = fluid.layers.data(name="target_language_word", shape=[1], dtype="int64", lod_level=1)
    trg_emb = fluid.layers.embedding(input=trg, size=[MT_DICT, MT_WORD], param_attr=fluid.ParamAttr(name="vemb"))
    rnn = fluid.layers.DynamicRNN()
    with rnn.block():
        w = rnn.step_input(trg_emb)
        pre = rnn.memory(init=ctx)
        cur = fluid.layers.fc(input=[w, pre], size=MT_HID, act="tanh")
        score = fluid.layers.fc(input=cur, size=MT_DICT, act="softmax")
        rnn.update_memory(pre, cur)
        rnn.output(score)
    label = fluid.layers.data(name="target_language_next_word", shape=[1], dtype="int64", lod_level=1)
    avg = fluid.layers.mean(fluid.layers.cross_entropy(input=rnn(), label=label))
    fluid.optimizer.Adagrad(learning_rate=0.1, regularization=fluid.regularizer.L2DecayRegularizer(
        regularization_coeff=0.01)).minimize(avg)
    return [avg]


def mt_decode():
    pd = fluid.layers
    ctx = _mt_encoder()
    array_len = pd.fill_constant(shape=[1], dtype="int64", value=MT_MAXLEN)
    counter = pd.zeros(shape=[1], dtype="int64", force_cpu=True)
    state_array = pd.create_array("float32")
    pd.array_write(ctx, array=state_array, i=counter)
    ids_array, scores_array = pd.create_array("int64"), pd.create_array("float32")
    init_ids = pd.data(name="init_ids", shape=[1], dtype="int64", lod_level=2)
    init_scores = pd.data(name="init_scores", shape=[1], dtype="float32", lod_level=2)
    pd.array_write(init_ids, array=ids_array, i=counter)
    pd.array_write(init_scores, array=scores_array, i=counter)
    cond = pd.less_than(x=counter, y=array_len)
    loop = pd.While(cond=cond)
    with loop.block():
        pre_ids = pd.array_read(array=ids_array, i=counter)
        pre_state = pd.array_read(array=state_array, i=counter)
        pre_score = pd.array_read(array=scores_array, i=counter)
        pre_state_exp = pd.sequence_expand(pre_state, pre_score)
        pre_ids_emb = pd.embedding(input=pre_ids, size=[MT_DICT, MT_WORD], param_attr=fluid.ParamAttr(name="vemb"))
        cur = pd.fc(input=[pre_state_exp, pre_ids_emb], size=MT_HID, act="tanh")
        cur_lod = pd.lod_reset(x=cur, y=pre_score)
        score = pd.fc(input=cur_lod, size=MT_DICT, act="softmax")
        topk_scores, topk_idx = pd.topk(score, k=MT_BEAM)
        accu = pd.elementwise_add(x=pd.log(topk_scores), y=pd.reshape(pre_score, shape=[-1]), axis=0)
        sel_ids, sel_scores = pd.beam_search(pre_ids, pre_score, topk_idx, accu, MT_BEAM, end_id=MT_END, level=0)
        pd.increment(x=counter, value=1, in_place=True)
        pd.array_write(cur, array=state_array, i=counter)
        pd.array_write(sel_ids, array=ids_array, i=counter)
        pd.array_write(sel_scores, array=scores_array, i=counter)
        length_cond = pd.less_than(x=counter, y=array_len)
        finish_cond = pd.logical_not(pd.is_empty(x=sel_ids))
        pd.logical_and(x=length_cond, y=finish_cond, out=cond)
    tids, tscores = pd.beam_search_decode(ids=ids_array, scores=scores_array, beam_size=MT_BEAM, end_id=MT_END)
    return [tids, tscores]


def _mt_words(rs, n, lo=1, hi=6):
    lens = rs.randint(lo, hi, n).tolist()
    off = np.concatenate([[0], np.cumsum(lens)]).tolist()
    return core.LoDTensor(torch.from_numpy(rs.randint(0, MT_DICT, (off[-1], 1)).astype("int64")), [off]), off


def mt_train_feeds(steps=4):
    out = []
    for seed in range(steps):
        rs = np.random.RandomState(200 + seed)
        src, _ = _mt_words(rs, 3)
        trg, off = _mt_words(rs, 3)
        nxt = core.LoDTensor(torch.from_numpy(rs.randint(0, MT_DICT, (off[-1], 1)).astype("int64")), [off])
        out.append({"src_word_id": src, "target_language_word": trg, "target_language_next_word": nxt})
    return out


def mt_decode_feeds(steps=2):
    out = []
    for seed in range(steps):
        rs = np.random.RandomState(300 + seed)
        n = 2
        src, _ = _mt_words(rs, n)
        lod = [list(range(n + 1)), list(range(n + 1))]
        init_ids = core.LoDTensor(torch.zeros(n, 1, dtype=torch.int64), lod)
        init_scores = core.LoDTensor(torch.ones(n, 1, dtype=torch.float32), lod)
        out.append({"src_word_id": src, "init_ids": init_ids, "init_scores": init_scores})
    return out


# ---------------------------------------------------------------------------------
# sequence row-map ops (ops_seq.cc): a text-CNN (sequence_conv + pool, the book
# understand_sentiment conv net) plus pad / unpad / slice / erase / mask / enumerate
# on the same LoD batch, trained end to end.
def seq_ops_net():
    def build():
        words = fluid.layers.data(name="words", shape=[1], lod_level=1, dtype="int64")
        label = fluid.layers.data(name="label", shape=[1], dtype="int64")
        off = fluid.layers.data(name="off", shape=[1], dtype="int64", append_batch_size=False)
        ln = fluid.layers.data(name="len", shape=[1], dtype="int64", append_batch_size=False)
        kept = fluid.layers.sequence_erase(words, tokens=[3, 7])
        emb = fluid.layers.embedding(input=kept, size=[V, E])
        conv = fluid.nets.sequence_conv_pool(input=emb, num_filters=H, filter_size=3, act="tanh", pool_type="max")
        pad_v = fluid.layers.fill_constant(shape=[1], dtype="float32", value=0.0)
        padded, lens = fluid.layers.sequence_pad(emb, pad_v)
        back = fluid.layers.sequence_unpad(padded * 2.0, lens)
        sl = fluid.layers.sequence_slice(back, off, ln)
        pooled = fluid.layers.sequence_pool(sl, "sum")
        mask = fluid.layers.cast(fluid.layers.sequence_mask(lens, maxlen=6, dtype="float32"), "float32")
        enum = fluid.layers.sequence_enumerate(kept, win_size=2)
        enum.stop_gradient = True  # integer ids: no gradient path
        enum_emb = fluid.layers.sequence_pool(fluid.layers.embedding(
            input=fluid.layers.reshape(enum, [-1, 1]), size=[V, E]), "sum")
        logit = fluid.layers.fc(input=conv, size=3, act="softmax")
        # (compile-time shapes of the padded branch are not needed: reduce it to scalars)
        loss = fluid.layers.mean(fluid.layers.cross_entropy(input=logit, label=label)) + \
            fluid.layers.mean(pooled) * 0.05 + fluid.layers.mean(mask) * 0.01 + fluid.layers.mean(enum_emb) * 0.02
        fluid.optimizer.SGD(learning_rate=0.3).minimize(loss)
        return [loss]
    return build


def seq_ops_feeds(steps=4):
    out = []
    for seed in range(steps):
        rs = np.random.RandomState(400 + seed)
        lens = rs.randint(3, 8, 4).tolist()
        off = np.concatenate([[0], np.cumsum(lens)]).tolist()
        ids = rs.randint(0, V, (off[-1], 1)).astype("int64")
        ids[ids == 3] = 4  # keep every sequence non-empty after the erase of 3 / 7
        ids[ids == 7] = 8
        ids[off[0], 0] = 3   # one erasable token per batch
        fd = {"words": core.LoDTensor(torch.from_numpy(ids), [off]),
              "label": core.LoDTensor(torch.from_numpy(rs.randint(0, 3, (len(lens), 1)).astype("int64"))),
              "off": core.LoDTensor(torch.from_numpy(np.array([[1], [0], [1], [0]], dtype="int64"))),
              "len": core.LoDTensor(torch.from_numpy(np.array([[1], [2], [1], [2]], dtype="int64")))}
        out.append(fd)
    return out


# ---------------------------------------------------------------------------------
# StaticRNN (layers.StaticRNN: a fixed-length RNN over the time-major first dim; the
# reference's recurrent op, here unrolled at build time into the block) trained end
# to end -- tests/unittests/test_recurrent_op.py's RecurrentOpTest1 cell.
SR_T, SR_B, SR_D = 4, 3, 5


def static_rnn():
    def build():
        x = fluid.layers.data(name="x", shape=[SR_T, SR_B, SR_D], dtype="float32", append_batch_size=False)
        h0 = fluid.layers.data(name="h0", shape=[SR_B, SR_D], dtype="float32", append_batch_size=False)
        x.stop_gradient = h0.stop_gradient = False
        rnn = fluid.layers.StaticRNN()
        with rnn.step():
            h_pre = rnn.memory(init=h0)
            xt = rnn.step_input(x)
            h = fluid.layers.scale(fluid.layers.elementwise_add(
                fluid.layers.fc(xt, SR_D, bias_attr=False), fluid.layers.fc(h_pre, SR_D, bias_attr=False)), 0.5)
            h = fluid.layers.tanh(h)
            rnn.update_memory(h_pre, h)
            rnn.output(h)
        out = rnn()
        loss = fluid.layers.mean(fluid.layers.square(out))
        fluid.optimizer.Momentum(learning_rate=0.2, momentum=0.9).minimize(loss)
        return [loss]
    return build


def static_rnn_feeds(steps=4):
    out = []
    for seed in range(steps):
        rs = np.random.RandomState(500 + seed)
        out.append({"x": core.LoDTensor(torch.from_numpy(rs.randn(SR_T, SR_B, SR_D).astype("float32"))),
                    "h0": core.LoDTensor(torch.from_numpy(rs.randn(SR_B, SR_D).astype("float32")))})
    return out


LY_B = 3


def layout_net():
    """slice (multi-axis, negative start) / transpose / unstack / stack / expand /
    unsqueeze / squeeze / flatten between two fc layers: every layout op and its
    gradient on the C++ executor."""
    def build():
        x = fluid.layers.data(name="x", shape=[LY_B, 6, 8], dtype="float32", append_batch_size=False)
        h = fluid.layers.fc(x, 8, num_flatten_dims=2, bias_attr=False)
        a = fluid.layers.slice(h, axes=[1, 2], starts=[1, -6], ends=[5, 100])       # [B, 4, 6]
        t = fluid.layers.transpose(a, [0, 2, 1])                                    # [B, 6, 4]
        parts = fluid.layers.unstack(t, axis=1)                                     # 6 x [B, 4]
        s = fluid.layers.stack(parts[::2], axis=2)                                  # [B, 4, 3]
        e = fluid.layers.expand(s, [1, 1, 2])                                       # [B, 4, 6]
        q = fluid.layers.squeeze(fluid.layers.unsqueeze(e, [1]), [1])
        f = fluid.layers.flatten(q, axis=1)                                         # [B, 24]
        y = fluid.layers.fc(f, 5, bias_attr=False)
        loss = fluid.layers.mean(fluid.layers.square(y))
        fluid.optimizer.SGD(learning_rate=0.1).minimize(loss)
        return [loss, e]
    return build


def layout_feeds(steps=4):
    out = []
    for seed in range(steps):
        rs = np.random.RandomState(700 + seed)
        out.append({"x": core.LoDTensor(torch.from_numpy(rs.randn(LY_B, 6, 8).astype("float32")))})
    return out


UN_B, UN_D, UN_T = 4, 5, 3


def units_net():
    """gru_unit and lstm_unit unrolled over UN_T dense steps (the StaticRNN-free way
    the reference's unit tests drive them), trained with SGD."""
    def build():
        x = fluid.layers.data(name="x", shape=[UN_T, UN_B, UN_D], dtype="float32", append_batch_size=False)
        h = fluid.layers.data(name="h", shape=[UN_B, UN_D], dtype="float32", append_batch_size=False)
        c = fluid.layers.data(name="c", shape=[UN_B, UN_D], dtype="float32", append_batch_size=False)
        h.stop_gradient = c.stop_gradient = False
        hg, hl, cl = h, h, c
        for t in range(UN_T):
            xt = fluid.layers.reshape(fluid.layers.slice(x, axes=[0], starts=[t], ends=[t + 1]), [UN_B, UN_D])
            gin = fluid.layers.fc(xt, 3 * UN_D, bias_attr=False)
            hg, _, _ = fluid.layers.gru_unit(gin, hg, 3 * UN_D)
            hl, cl = fluid.layers.lstm_unit(xt, hl, cl, forget_bias=0.5)
        loss = fluid.layers.mean(fluid.layers.square(fluid.layers.elementwise_add(hg, hl)))
        fluid.optimizer.SGD(learning_rate=0.3).minimize(loss)
        return [loss]
    return build


def units_feeds(steps=4):
    out = []
    for seed in range(steps):
        rs = np.random.RandomState(900 + seed)
        out.append({k: core.LoDTensor(torch.from_numpy(rs.randn(*s).astype("float32")))
                    for k, s in (("x", (UN_T, UN_B, UN_D)), ("h", (UN_B, UN_D)), ("c", (UN_B, UN_D)))})
    return out


def vol_net():
    """conv3d (padding, stride, groups, bias) + max / avg (exclusive=False, ceil_mode)
    pool3d, trained with Momentum: the NCDHW ops and their grads on the C++ executor."""
    def build():
        x = fluid.layers.data(name="x", shape=[2, 5, 6, 8], dtype="float32")
        label = fluid.layers.data(name="label", shape=[1], dtype="int64")
        c1 = fluid.layers.conv3d(x, 4, 3, stride=[1, 2, 1], padding=1, act="relu")
        p1 = fluid.layers.pool3d(c1, 2, "max", pool_stride=2, ceil_mode=True)
        c2 = fluid.layers.conv3d(p1, 4, [1, 2, 2], padding=[0, 1, 0], groups=2, dilation=[1, 1, 2])
        p2 = fluid.layers.pool3d(c2, 2, "avg", pool_stride=1, pool_padding=1, exclusive=False)
        logit = fluid.layers.fc(input=p2, size=3, act="softmax")
        loss = fluid.layers.mean(fluid.layers.cross_entropy(input=logit, label=label))
        fluid.optimizer.Momentum(learning_rate=0.05, momentum=0.9).minimize(loss)
        return [loss]
    return build


def vol_feeds(steps=4):
    out = []
    for seed in range(steps):
        rs = np.random.RandomState(1100 + seed)
        out.append({"x": core.LoDTensor(torch.from_numpy(rs.randn(3, 2, 5, 6, 8).astype("float32"))),
                    "label": core.LoDTensor(torch.from_numpy(rs.randint(0, 3, (3, 1)).astype("int64")))})
    return out


LS_C = 6


def losses_net():
    """warpctc (norm_by_times), nce (custom negatives), hsigmoid and roi_pool heads
    summed into one loss, plus edit_distance between two id sequences; Momentum."""
    def build():
        feat = fluid.layers.data(name="feat", shape=[E], lod_level=1, dtype="float32")
        lab = fluid.layers.data(name="lab", shape=[1], lod_level=1, dtype="int64")
        logits = fluid.layers.fc(feat, LS_C)
        ctc = fluid.layers.mean(fluid.layers.warpctc(logits, lab, blank=0, norm_by_times=True))
        x = fluid.layers.data(name="x", shape=[E], dtype="float32")
        y = fluid.layers.data(name="y", shape=[1], dtype="int64")
        h = fluid.layers.fc(x, E, act="tanh")
        nce = fluid.layers.mean(fluid.layers.nce(h, y, num_total_classes=9, num_neg_samples=3))
        op = fluid.default_main_program().global_block().ops[-3]
        assert op.type == "nce", op.type
        op.set_attr("custom_neg_classes", [1, 4, 7])
        hs = fluid.layers.mean(fluid.layers.hsigmoid(h, y, num_classes=9))
        img = fluid.layers.data(name="img", shape=[2, 6, 7], dtype="float32")
        rois = fluid.layers.data(name="rois", shape=[4], lod_level=1, dtype="float32")
        fmap = fluid.layers.conv2d(img, 3, 3, padding=1)
        pooled = fluid.layers.roi_pool(fmap, rois, pooled_height=2, pooled_width=3, spatial_scale=0.5)
        rp = fluid.layers.mean(fluid.layers.square(fluid.layers.fc(pooled, 2)))
        loss = fluid.layers.sums([ctc, nce, hs, rp])
        fluid.optimizer.Momentum(learning_rate=0.05, momentum=0.9).minimize(loss)
        hyp = fluid.layers.data(name="hyp", shape=[1], lod_level=1, dtype="int64")
        dist, _ = fluid.layers.edit_distance(hyp, lab, normalized=True)
        return [loss, dist]
    return build


def losses_feeds(steps=4):
    out = []
    for seed in range(steps):
        rs = np.random.RandomState(1300 + seed)
        tl = [5, 3, 7]
        ll = [2, 1, 3]
        to = np.concatenate([[0], np.cumsum(tl)]).tolist()
        lo = np.concatenate([[0], np.cumsum(ll)]).tolist()
        hl = [3, 2, 2]
        ho = np.concatenate([[0], np.cumsum(hl)]).tolist()
        R = [2, 1]
        ro = np.concatenate([[0], np.cumsum(R)]).tolist()
        boxes = []
        for _ in range(sum(R)):
            x1, y1 = rs.randint(0, 8), rs.randint(0, 6)
            boxes.append([x1, y1, x1 + rs.randint(1, 6), y1 + rs.randint(1, 6)])
        out.append({
            "feat": core.LoDTensor(torch.from_numpy(rs.randn(to[-1], E).astype("float32")), [to]),
            "lab": core.LoDTensor(torch.from_numpy(rs.randint(1, LS_C, (lo[-1], 1)).astype("int64")), [lo]),
            "x": core.LoDTensor(torch.from_numpy(rs.randn(4, E).astype("float32"))),
            "y": core.LoDTensor(torch.from_numpy(rs.randint(0, 9, (4, 1)).astype("int64"))),
            "img": core.LoDTensor(torch.from_numpy(rs.randn(2, 2, 6, 7).astype("float32"))),
            "rois": core.LoDTensor(torch.from_numpy(np.array(boxes, dtype="float32")), [ro]),
            "hyp": core.LoDTensor(torch.from_numpy(rs.randint(1, LS_C, (ho[-1], 1)).astype("int64")), [ho]),
        })
    return out


# ---------------------------------------------------------------------------------
# The reference StaticRNN's op: `recurrent` over a hand-built step block (two time-major
# inputs, two linked states, a trainable initial state), its recurrent_grad, SGD.
RT, RB, RD, RH = 5, 3, 4, 6


def recurrent_net(reverse=False):
    def build():
        from paddle_amd.fluid.framework import VarType

        main = fluid.default_main_program()
        gb = main.global_block()
        x1 = fluid.layers.data(name="rx1", shape=[RT, RB, RD], dtype="float32", append_batch_size=False)
        x2 = fluid.layers.data(name="rx2", shape=[RT, RB, RH], dtype="float32", append_batch_size=False)
        x1.stop_gradient = False
        h0 = fluid.layers.create_parameter([RB, RH], "float32", name="rh0")
        c0 = fluid.layers.fill_constant([RB, RH], "float32", 0.5)
        w = fluid.layers.create_parameter([RD, RH], "float32", name="rw")
        u = fluid.layers.create_parameter([RH, RH], "float32", name="ru")
        sub = main.create_block()
        v = {}
        for n, shp in (("rx1", [RB, RD]), ("rx2", [RB, RH]), ("h_pre", [RB, RH]), ("c_pre", [RB, RH]), ("a", [RB, RH]),
                       ("b", [RB, RH]), ("s1", [RB, RH]), ("s2", [RB, RH]), ("h", [RB, RH]), ("c", [RB, RH]),
                       ("y", [RB, RH])):
            v[n] = sub.create_var(name=n, dtype="float32", shape=shp)
        sub.append_op(type="mul", inputs={"X": [v["rx1"]], "Y": [w]}, outputs={"Out": [v["a"]]})
        sub.append_op(type="mul", inputs={"X": [v["h_pre"]], "Y": [u]}, outputs={"Out": [v["b"]]})
        sub.append_op(type="elementwise_add", inputs={"X": [v["a"]], "Y": [v["b"]]}, outputs={"Out": [v["s1"]]})
        sub.append_op(type="elementwise_add", inputs={"X": [v["s1"]], "Y": [v["rx2"]]}, outputs={"Out": [v["s2"]]})
        sub.append_op(type="tanh", inputs={"X": [v["s2"]]}, outputs={"Out": [v["h"]]})
        sub.append_op(type="elementwise_mul", inputs={"X": [v["c_pre"]], "Y": [v["h"]]}, outputs={"Out": [v["c"]]})
        sub.append_op(type="elementwise_add", inputs={"X": [v["c"]], "Y": [v["h"]]}, outputs={"Out": [v["y"]]})
        main.rollback()
        out = gb.create_var(name="y", dtype="float32", shape=[RT, RB, RH])
        hs = gb.create_var(name="h", dtype="float32", shape=[RT, RB, RH])
        scopes = gb.create_var(name="rnn_scopes", type=VarType.STEP_SCOPES)
        gb.append_op(type="recurrent", inputs={"inputs": [x1, x2], "initial_states": [h0, c0], "parameters": [w, u]},
                     outputs={"outputs": [out, hs], "step_scopes": [scopes]},
                     attrs={"ex_states": ["h_pre", "c_pre"], "states": ["h", "c"], "sub_block": sub,
                            "reverse": reverse})
        loss = fluid.layers.mean(out * out) + fluid.layers.mean(hs)
        fluid.optimizer.SGD(learning_rate=0.1).minimize(loss)
        return [loss, out, "rx1@GRAD", "rh0@GRAD", "rw@GRAD", "ru@GRAD"]
    return build


def recurrent_feeds(steps):
    out = []
    for k in range(steps):
        rs = np.random.RandomState(300 + k)
        out.append({"rx1": rs.randn(RT, RB, RD).astype("float32"), "rx2": rs.randn(RT, RB, RH).astype("float32")})
    return out
