"""fluid.contrib decoders (reference: contrib/decoder/beam_search_decoder.py and its
book test high-level-api machine_translation): a TrainingDecoder seq2seq trains
through DynamicRNN/while_grad; a BeamSearchDecoder with the same StateCell
generates LoD sentences with beam_search / beam_search_decode."""
import numpy as np
import torch

import paddle_amd.fluid as fluid
from paddle_amd.fluid.contrib import BeamSearchDecoder, InitState, StateCell, TrainingDecoder
from paddle_amd.framework import core

V, E, H = 12, 8, 16


def _cell(context):
    cell = StateCell(inputs={"x": None}, states={"h": InitState(init=context, need_reorder=True)}, out_state="h")

    @cell.state_updater
    def updater(c):
        x, hp = c.get_input("x"), c.get_state("h")
        hn = fluid.layers.fc(input=[x, hp], size=H, act="tanh",
                             param_attr=[fluid.ParamAttr(name="cell_wx"), fluid.ParamAttr(name="cell_wh")],
                             bias_attr=fluid.ParamAttr(name="cell_b"))
        c.set_state("h", hn)

    return cell


def _encoder(src):
    emb = fluid.layers.embedding(src, size=[V, E], param_attr=fluid.ParamAttr(name="src_emb"))
    h = fluid.layers.fc(emb, size=H, act="tanh", param_attr=fluid.ParamAttr(name="enc_w"),
                        bias_attr=fluid.ParamAttr(name="enc_b"))
    return fluid.layers.sequence_pool(h, "last")


def _lod(seqs):
    off = [0]
    for s in seqs:
        off.append(off[-1] + len(s))
    arr = np.concatenate(seqs).reshape(-1, 1).astype("int64")
    return core.LoDTensor(torch.from_numpy(arr), [off])


def test_training_decoder_trains():
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 7
    with fluid.program_guard(main, startup):
        src = fluid.layers.data(name="src", shape=[1], dtype="int64", lod_level=1)
        trg = fluid.layers.data(name="trg", shape=[1], dtype="int64", lod_level=1)
        lbl = fluid.layers.data(name="lbl", shape=[1], dtype="int64", lod_level=1)
        context = _encoder(src)
        cell = _cell(context)
        trg_emb = fluid.layers.embedding(trg, size=[V, E], param_attr=fluid.ParamAttr(name="trg_emb"))
        dec = TrainingDecoder(cell)
        with dec.block():
            cur = dec.step_input(trg_emb)
            cell.compute_state(inputs={"x": cur})
            score = fluid.layers.fc(cell.get_state("h"), size=V, act="softmax",
                                    param_attr=fluid.ParamAttr(name="out_w"), bias_attr=fluid.ParamAttr(name="out_b"))
            cell.update_states()
            dec.output(score)
        pred = dec()
        loss = fluid.layers.mean(fluid.layers.cross_entropy(pred, lbl))
        fluid.optimizer.Adam(learning_rate=0.02).minimize(loss)
    rng = np.random.RandomState(0)
    srcs = [rng.randint(2, V, n) for n in (3, 5, 2, 4)]
    # successor task: next target token = current + 1 (learnable from the step input)
    trgs = [(s[0] + np.arange(len(s) + 1)) % (V - 2) + 2 for s in srcs]
    lbls = [(t - 2 + 1) % (V - 2) + 2 for t in trgs]
    exe = fluid.Executor(fluid.CPUPlace())
    with fluid.executor.scope_guard(core.Scope()):
        exe.run(startup)
        feed = {"src": _lod(srcs), "trg": _lod(trgs), "lbl": _lod(lbls)}
        ls = [float(np.asarray(exe.run(main, feed=feed, fetch_list=[loss])[0]).reshape(-1)[0]) for _ in range(60)]
    assert ls[-1] < 0.5 * ls[0], ls


def test_beam_search_decoder_generates():
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 7
    beam, max_len = 2, 4
    with fluid.program_guard(main, startup):
        src = fluid.layers.data(name="src", shape=[1], dtype="int64", lod_level=1)
        init_ids = fluid.layers.data(name="init_ids", shape=[1], dtype="int64", lod_level=2)
        init_scores = fluid.layers.data(name="init_scores", shape=[1], dtype="float32", lod_level=2)
        context = _encoder(src)
        cell = StateCell(inputs={"x": None}, states={"h": InitState(init=context)}, out_state="h")

        @cell.state_updater
        def updater(c):
            x, hp = c.get_input("x"), c.get_state("h")
            c.set_state("h", fluid.layers.fc(input=[x, hp], size=H, act="tanh"))

        dec = BeamSearchDecoder(cell, init_ids, init_scores, target_dict_dim=V, word_dim=E, topk_size=4,
                                sparse_emb=False, max_len=max_len, beam_size=beam, end_id=1)
        dec.decode()
        ids, scores = dec()
    srcs = [np.array([3, 4, 5]), np.array([6, 7])]
    n = len(srcs)
    lod2 = [list(range(n + 1)), list(range(n + 1))]
    exe = fluid.Executor(fluid.CPUPlace())
    with fluid.executor.scope_guard(core.Scope()):
        exe.run(startup)
        feed = {"src": _lod(srcs),
                "init_ids": core.LoDTensor(torch.zeros(n, 1, dtype=torch.int64), lod2),
                "init_scores": core.LoDTensor(torch.ones(n, 1, dtype=torch.float32), lod2)}
        out_ids, out_scores = exe.run(main, feed=feed, fetch_list=[ids, scores], return_numpy=False)
    lod = out_ids.lod()
    assert len(lod) == 2 and len(lod[0]) == n + 1          # per source: its hypotheses
    assert lod[1][-1] == out_ids.tensor.shape[0]            # per hypothesis: its tokens
    assert all(1 <= lod[0][i + 1] - lod[0][i] <= beam for i in range(n))
    lens = np.diff(lod[1])
    assert lens.min() >= 1 and lens.max() <= max_len + 1
    assert np.isfinite(out_scores.tensor.numpy()).all()
