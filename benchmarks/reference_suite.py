#!/usr/bin/env python3
"""The reference's own published benchmark rows, re-measured on one MI355X.

Rows (reference doc/fluid/new_docs/advanced_usage/benchmark.rst:111-119
-- "the unit is samples/s" -- models from benchmark/fluid/models/*.py; inference
rows from paddle/contrib/float16/float16_benchmark.md:21-44):

  vgg16          VGG-16 train, Flowers102 shape (224x224, 102 classes)    59.83 images/s
  stacked_lstm   IMDB sentiment: emb 512 -> fc tanh 512 -> LSTM 512 ->    1319.99 samples/s
                 last step -> fc 2 (benchmark/fluid/models/stacked_dynamic_lstm.py)
  seq2seq        wmt14 attention seq2seq, dict 30000, emb/enc/dec 512,    7147.89 samples/s
                 bi-LSTM encoder + LSTM decoder with additive attention
                 (benchmark/fluid/models/machine_translation.py)
  infer          ResNet-50 / VGG-16 ImageNet inference, batch 64,         67.93 / 178.95 ms (fp32)
                 fp32 and reduced precision                               33.20 / 60.23 ms (fp16)

All data is synthetic with the datasets' shapes (IMDB review lengths ~ lognormal,
mean ~230 words, cropped < 1500 like the reference; wmt14 sentence lengths ~ 5-80
tokens); weights are random-init.  ``stacked_lstm --impl fluid`` runs the
reference's Fluid program (DynamicRNN over LoD sequences, Adam) through this
framework's executor; ``--impl dygraph`` runs the same network on MIOpen's fused
LSTM.  Prints one JSON line per measurement.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BASE = {"vgg16": 59.83327, "stacked_lstm": 1319.99315, "seq2seq": 7147.89081,
        "infer_resnet50_fp32": 67.93, "infer_resnet50_lowp": 33.20,
        "infer_vgg16_fp32": 178.95, "infer_vgg16_lowp": 60.23}


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _timeit(step, steps, warmup):
    for _ in range(warmup):
        step()
    _sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    _sync()
    return (time.perf_counter() - t0) / steps, out


def _emit(d):
    print(json.dumps(d), flush=True)


# ------------------------------------------------------------------ VGG-16 train
def vgg16_bn_drop(num_classes=102, data_format="NHWC"):
    """The benchmark's network (benchmark/fluid/models/vgg.py:28-52): five groups of
    conv3x3+BN+ReLU (with the listed dropouts) and a 2x2 max-pool each, then
    dropout, fc 512, BN+ReLU, dropout, fc 512, fc num_classes; Adam."""
    from paddle_amd import nn

    layers, c = [], 3
    for nf, drops in ((64, [0.3, 0]), (128, [0.4, 0]), (256, [0.4, 0.4, 0]), (512, [0.4, 0.4, 0]),
                      (512, [0.4, 0.4, 0])):
        for d in drops:
            layers += [nn.Conv2D(c, nf, 3, padding=1, data_format=data_format),
                       nn.BatchNorm2D(nf, data_format=data_format), nn.ReLU()]
            if d:
                layers.append(nn.Dropout(d))
            c = nf
        layers.append(nn.MaxPool2D(2, 2, data_format=data_format))
    return nn.Sequential(*layers, nn.Flatten(), nn.Dropout(0.5), nn.Linear(512 * 7 * 7, 512),
                         nn.BatchNorm1D(512), nn.ReLU(), nn.Dropout(0.5), nn.Linear(512, 512),
                         nn.Linear(512, num_classes))


def bench_vgg16(a, dev):
    import paddle_amd as paddle
    from paddle_amd import nn

    paddle.seed(0)
    model = vgg16_bn_drop().to(dev)
    opt = paddle.optimizer.Adam(learning_rate=1e-3, parameters=model.parameters())
    model, opt = paddle.amp.decorate(model, opt, level="O2", dtype="bfloat16")
    B = a.batch or 64
    x = torch.randn(B, 224, 224, 3, device=dev, dtype=torch.bfloat16)
    y = torch.randint(0, 102, (B, 1), device=dev)
    loss_fn = nn.CrossEntropyLoss()

    def step():
        loss = loss_fn(model(x).float(), y)
        loss.backward()
        opt.step()
        opt.clear_grad(set_to_zero=False)
        return loss

    dt, loss = _timeit(step, a.steps, a.warmup)
    v = B / dt
    _emit({"bench": "vgg16_train", "model": "vgg16_bn_drop (reference benchmark net)", "value": round(v, 1),
           "unit": "images/s", "batch": B, "dtype": "bf16", "layout": "NHWC",
           "ms_per_step": round(dt * 1e3, 2), "baseline": BASE["vgg16"], "vs_baseline": round(v / BASE["vgg16"], 2),
           "loss": float(loss.detach())})


# ------------------------------------------------------------------ stacked LSTM (IMDB)
def _imdb_lengths(rng, n):
    return np.clip(rng.lognormal(5.25, 0.65, n), 10, 1499).astype(np.int64)


def bench_stacked_lstm_dygraph(a, dev):
    V, E, Hs = 5147, 512, 512
    B = a.batch or 32
    torch.manual_seed(0)
    emb = torch.nn.Embedding(V, E).to(dev)
    fc0 = torch.nn.Linear(E, Hs).to(dev)
    import paddle_amd as paddle

    lstm = paddle.nn.LSTM(Hs, Hs).to(dev)  # persistent gfx950 kernel on the GPU
    head = torch.nn.Linear(Hs, 2).to(dev)
    params = [*emb.parameters(), *fc0.parameters(), *lstm.parameters(), *head.parameters()]
    from paddle_amd.optimizer import Adam

    opt = Adam(learning_rate=1e-3, parameters=params)
    rng = np.random.RandomState(0)
    batches = []
    for _ in range(8):
        lens = torch.from_numpy(_imdb_lengths(rng, B))
        T = int(lens.max())
        lens = lens.to(dev)
        ids = torch.randint(0, V, (B, T), device=dev)
        lab = torch.randint(0, 2, (B,), device=dev)
        batches.append((ids, lens, lab))
    it = [0]

    def step():
        ids, lens, lab = batches[it[0] % len(batches)]
        it[0] += 1
        x = torch.tanh(fc0(emb(ids)))
        _, (h, _) = lstm(x, sequence_length=lens)  # h = hidden state at each sequence's last step
        loss = torch.nn.functional.cross_entropy(head(h[-1]), lab)
        loss.backward()
        opt.step()
        opt.clear_grad()
        return loss

    dt, loss = _timeit(step, a.steps, a.warmup)
    words = float(np.mean([b[1].float().mean().item() for b in batches]))
    v = B / dt
    _emit({"bench": "stacked_lstm_train", "impl": "dygraph paddle.nn.LSTM (persistent gfx950 kernel)", "value": round(v, 1),
           "unit": "samples/s", "words_per_s": round(v * words, 1), "avg_len": round(words, 1), "batch": B,
           "dtype": "fp32", "ms_per_step": round(dt * 1e3, 2), "baseline": BASE["stacked_lstm"],
           "vs_baseline": round(v / BASE["stacked_lstm"], 2), "loss": float(loss.detach())})


def stacked_lstm_program(V=5147, E=512, Hs=512):
    """The reference benchmark program (benchmark/fluid/models/stacked_dynamic_lstm.py):
    embedding -> fc tanh -> DynamicRNN LSTM written with fc/sums/elementwise ops ->
    sequence_pool last -> fc softmax -> cross entropy, Adam."""
    import paddle_amd.fluid as fluid

    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 1
    with fluid.program_guard(main, startup):
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
        fluid.optimizer.Adam(learning_rate=1e-3).minimize(loss)
    return main, startup, loss


def stacked_lstm_op_program(V=5147, E=512, Hs=512):
    """The same network with the recurrence as ONE Fluid op: fc -> dynamic_lstm (the
    reference's lstm op, no peepholes) instead of a DynamicRNN of fc/sums ops."""
    import paddle_amd.fluid as fluid

    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 1
    with fluid.program_guard(main, startup):
        words = fluid.layers.data(name="words", shape=[1], lod_level=1, dtype="int64")
        label = fluid.layers.data(name="label", shape=[1], dtype="int64")
        sent = fluid.layers.embedding(input=words, size=[V, E])
        sent = fluid.layers.fc(input=sent, size=Hs, act="tanh")
        proj = fluid.layers.fc(input=sent, size=4 * Hs)
        hidden, _ = fluid.layers.dynamic_lstm(input=proj, size=4 * Hs, use_peepholes=False)
        last = fluid.layers.sequence_pool(hidden, "last")
        logit = fluid.layers.fc(input=last, size=2, act="softmax")
        loss = fluid.layers.mean(fluid.layers.cross_entropy(input=logit, label=label))
        fluid.optimizer.Adam(learning_rate=1e-3).minimize(loss)
    return main, startup, loss


def bench_stacked_lstm_fluid(a, dev, lstm_op=False):
    import paddle_amd.fluid as fluid
    from paddle_amd.framework import core

    V, E, Hs = 5147, 512, 512
    B = a.batch or 32
    main, startup, loss = (stacked_lstm_op_program if lstm_op else stacked_lstm_program)(V, E, Hs)
    place = fluid.CUDAPlace(0) if dev.type == "cuda" else fluid.CPUPlace()
    exe = fluid.Executor(place)
    scope = core.Scope()
    rng = np.random.RandomState(0)
    feeds = []
    for _ in range(4):
        lens = _imdb_lengths(rng, B)
        if a.max_len:
            lens = np.minimum(lens, a.max_len)
        off = np.concatenate([[0], np.cumsum(lens)]).tolist()
        ids = torch.randint(0, V, (off[-1], 1), device=dev)
        lab = torch.randint(0, 2, (B, 1), device=dev)
        feeds.append(({"words": core.LoDTensor(ids, [off]), "label": core.LoDTensor(lab)}, float(lens.mean())))
    it = [0]
    with fluid.executor.scope_guard(scope):
        exe.run(startup)

        def step():
            fd, _ = feeds[it[0] % len(feeds)]
            it[0] += 1
            return exe.run(main, feed=fd, fetch_list=[loss], return_numpy=False)[0]

        dt, out = _timeit(step, a.steps, a.warmup)
    avg = float(np.mean([f[1] for f in feeds]))
    v = B / dt
    impl = ("fluid program, dynamic_lstm op (persistent kernel)" if lstm_op
            else "fluid DynamicRNN program of fc/sums ops (op-by-op executor)")
    _emit({"bench": "stacked_lstm_train", "impl": impl, "value": round(v, 1),
           "unit": "samples/s", "words_per_s": round(v * avg, 1), "avg_len": round(avg, 1), "batch": B,
           "dtype": "fp32", "ms_per_step": round(dt * 1e3, 2), "baseline": BASE["stacked_lstm"],
           "vs_baseline": round(v / BASE["stacked_lstm"], 2)})


# ------------------------------------------------------------------ seq2seq (wmt14)
class Seq2Seq(torch.nn.Module):
    """Reference machine_translation.py network: bi-LSTM encoder, decoder boot =
    tanh(fc(first step of the backward encoder)), additive attention
    score = w . tanh(enc_proj + fc(h)), LSTM step over [context, word, h], softmax
    over the 30000-word target dictionary.  The decoder recurrence runs on the
    fused attention-decoder kernels (ops/rnn.py::attention_lstm_decoder)."""

    def __init__(self, V=30000, E=512, H=512):
        super().__init__()
        import paddle_amd as paddle

        self.H = H
        self.src_emb = torch.nn.Embedding(V, E)
        self.trg_emb = torch.nn.Embedding(V, E)
        self.enc = paddle.nn.LSTM(E, H, direction="bidirect")   # persistent gfx950 kernel on the GPU
        self.enc_proj = torch.nn.Linear(2 * H, H, bias=False)
        self.boot = torch.nn.Linear(H, H)
        self.state_proj = torch.nn.Linear(H, H, bias=False)
        self.score = torch.nn.Linear(H, 1, bias=False)
        self.w_ctx_h = torch.nn.Parameter(torch.randn(2 * H + H, 4 * H) / (3 * H) ** 0.5)  # [ctx, h] -> gates
        self.y_gates = torch.nn.Linear(E, 4 * H)                                            # word -> gates (+ bias)
        self.out = torch.nn.Linear(H, V)

    def forward(self, src, slen, trg_in, trg_out, tmask):
        """slen: [B] device tensor of source lengths (no host sync: graph-capturable)."""
        from paddle_amd.ops import rnn

        x = self.src_emb(src)
        enc, _ = self.enc(x, sequence_length=slen)                # [B, Ts, 2H], padded rows zero
        ep = self.enc_proj(enc)                                   # [B, Ts, H]
        h0 = torch.tanh(self.boot(enc[:, 0, self.H:]))            # backward direction, first step
        c0 = torch.zeros_like(h0)
        Y = self.y_gates(self.trg_emb(trg_in)).transpose(0, 1)    # [Tt, B, 4H]
        hs = rnn.attention_lstm_decoder(enc, ep, slen, Y, h0, c0, self.state_proj.weight.t(),
                                        self.score.weight[0], self.w_ctx_h)
        from paddle_amd import ops

        logits = self.out(hs.transpose(0, 1))                     # [B, Tt, V]
        labels = torch.where(tmask > 0, trg_out, torch.full_like(trg_out, -100))
        # fused log-softmax + NLL over the 30000-word vocabulary (gradient written in place)
        return ops.softmax_cross_entropy(logits.flatten(0, 1), labels.flatten(), ignore_index=-100,
                                         inplace_grad=logits.is_cuda)


def bench_seq2seq(a, dev):
    """Lengths are bucketed to multiples of 16 and, on the GPU, each bucket's
    forward+backward is captured once as a HIP graph and replayed (the decoder's
    per-step attention is launch-bound: ~40 small kernels per target word)."""
    B = a.batch or 128
    torch.manual_seed(0)
    model = Seq2Seq().to(dev)
    from paddle_amd.optimizer import Adam

    params = list(model.parameters())
    opt = Adam(learning_rate=1e-3, parameters=params)
    rng = np.random.RandomState(0)
    bucket = lambda n: (n + 15) // 16 * 16  # noqa: E731
    batches = []
    for _ in range(4):
        sl = np.clip(rng.lognormal(3.2, 0.5, B), 5, 80).astype(np.int64)
        tl = np.clip((sl * rng.uniform(0.8, 1.2, B)).astype(np.int64), 5, 80)
        Ts, Tt = bucket(int(sl.max())), bucket(int(tl.max()))
        src = torch.randint(0, 30000, (B, Ts), device=dev)
        trg = torch.randint(0, 30000, (B, Tt + 1), device=dev)
        tmask = (torch.arange(Tt)[None] < torch.from_numpy(tl)[:, None]).float().to(dev)
        batches.append((src, torch.from_numpy(sl).to(dev), trg[:, :-1], trg[:, 1:], tmask, float(tl.mean())))
    it = [0]
    amp = a.dtype == "bf16"
    use_graph = dev.type == "cuda" and not a.no_graph
    graphs = {}  # (Ts, Tt) -> (graph, static inputs, static loss, grads)

    def fwd_bwd(src, sl, ti, to, tm):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp and dev.type == "cuda"):
            loss = model(src, sl, ti, to, tm)
        loss.backward()
        return loss

    def capture(inputs):
        static = [t.clone() for t in inputs]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                for p in params:
                    p.grad = None
                fwd_bwd(*static)
        torch.cuda.current_stream().wait_stream(s)
        for p in params:
            p.grad = None
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = fwd_bwd(*static)
        return g, static, loss, [p.grad for p in params]

    def step():
        src, sl, ti, to, tm, _ = batches[it[0] % len(batches)]
        it[0] += 1
        inputs = (src, sl, ti, to, tm)
        if use_graph:
            key = (src.shape[1], ti.shape[1])
            if key not in graphs:
                graphs[key] = capture(inputs)
            g, static, loss, grads = graphs[key]
            for d, x in zip(static, inputs):
                d.copy_(x)
            g.replay()
            for p, gr in zip(params, grads):
                p.grad = gr
        else:
            loss = fwd_bwd(*inputs)
        opt.step()
        if not use_graph:
            opt.clear_grad()
        return loss

    dt, loss = _timeit(step, a.steps, max(a.warmup, len(batches)))
    avg = float(np.mean([b[-1] for b in batches]))
    v = B / dt
    _emit({"bench": "seq2seq_train", "value": round(v, 1), "unit": "samples/s", "trg_words_per_s": round(v * avg, 1),
           "avg_trg_len": round(avg, 1), "batch": B, "dtype": a.dtype, "hip_graph": use_graph,
           "ms_per_step": round(dt * 1e3, 2), "baseline": BASE["seq2seq"],
           "vs_baseline": round(v / BASE["seq2seq"], 2), "loss": float(loss.detach())})


# ------------------------------------------------------------------ inference
def bench_infer(a, dev):
    import paddle_amd as paddle

    B = a.batch or 64
    for name in ("resnet50", "vgg16"):
        for prec in ("fp32", "lowp"):
            paddle.seed(0)
            fmt = "NHWC" if prec == "lowp" else "NCHW"
            kw = {"data_format": fmt} if name == "resnet50" else {"data_format": fmt}
            m = getattr(paddle.vision.models, name)(num_classes=1000, **kw).to(dev).eval()
            dt_ = torch.bfloat16 if prec == "lowp" else torch.float32
            m = m.to(dt_)
            shape = (B, 224, 224, 3) if fmt == "NHWC" else (B, 3, 224, 224)
            x = torch.randn(shape, device=dev, dtype=dt_)
            graph = None
            with torch.no_grad():
                run = lambda: m(x)  # noqa: E731
                if a.graph and dev.type == "cuda":
                    s = torch.cuda.Stream()
                    s.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(s):
                        for _ in range(3):
                            m(x)
                    torch.cuda.current_stream().wait_stream(s)
                    graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(graph):
                        m(x)
                    run = graph.replay
                dt, _ = _timeit(run, a.steps, a.warmup)
            key = f"infer_{name}_{prec}"
            _emit({"bench": key, "value": round(dt * 1e3, 3), "unit": "ms/batch", "batch": B,
                   "dtype": "bf16" if prec == "lowp" else "fp32", "layout": fmt, "hip_graph": graph is not None,
                   "higher_is_better": False, "baseline_ms": BASE[key],
                   "speedup_vs_baseline": round(BASE[key] / (dt * 1e3), 2)})
            del m, x, graph
            torch.cuda.empty_cache() if dev.type == "cuda" else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", nargs="+", choices=["vgg16", "stacked_lstm", "seq2seq", "infer"])
    ap.add_argument("--impl", default="both", choices=["both", "dygraph", "fluid", "fluid_lstm_op"])
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--graph", action="store_true", help="replay inference as a HIP graph")
    ap.add_argument("--no-graph", action="store_true", help="seq2seq: eager steps instead of HIP-graph replay")
    ap.add_argument("--max-len", type=int, default=0, help="cap IMDB lengths (fluid path smoke runs)")
    a = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    for w in a.which:
        if w == "vgg16":
            bench_vgg16(a, dev)
        elif w == "stacked_lstm":
            if a.impl in ("both", "dygraph"):
                bench_stacked_lstm_dygraph(a, dev)
            if a.impl in ("both", "fluid_lstm_op"):
                bench_stacked_lstm_fluid(a, dev, lstm_op=True)
            if a.impl == "fluid":
                bench_stacked_lstm_fluid(a, dev)
        elif w == "seq2seq":
            bench_seq2seq(a, dev)
        else:
            bench_infer(a, dev)


if __name__ == "__main__":
    main()
