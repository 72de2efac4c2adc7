"""The v1 trainer front end (reference paddle/legacy/trainer: TrainerMain.cpp:32
``paddle_trainer --config=... --job=train|test|time|checkgrad``, Trainer.cpp:265
train / :496 trainOnePass / :406 trainOneDataBatch) and the PyDataProvider2 bridge
(python/paddle/trainer/PyDataProvider2.py ``@provider``,
trainer_config_helpers/data_sources.py:158 ``define_py_data_sources2``).

The legacy C++ GradientMachine is replaced by the v1 DSL -> Fluid program path of
``paddle_amd.trainer_config_helpers``: ``python -m paddle_amd.trainer --config
conf.py`` parses the config, imports the data provider module it names, feeds the
files of its train / test lists through the ``@provider`` generator, batches them
with the config's ``settings(batch_size=...)`` and trains with the v2 trainer
(periodic cost logging, per-pass test, parameter tars per pass under
``--save_dir``).
"""
from __future__ import annotations

import argparse
import importlib
import os
import random
import sys
import time

from . import PyDataProvider2  # noqa: F401
from .PyDataProvider2 import provider  # noqa: F401


def _file_list(path):
    if not path:
        return []
    base = os.path.dirname(os.path.abspath(path))
    out = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line:
                out.append(line if os.path.isabs(line) else os.path.join(base, line))
    return out


def _reader(source, which, batch_size, shuffle_seed=None):
    """A v2 batch reader over one data source of the config (train or test)."""
    if source is None:
        return None
    mod_name, obj_name, args = source["module"], source["obj"], source.get("args") or {}
    files = _file_list(source["train_list" if which == "train" else "test_list"])
    if not files:
        return None
    mod = importlib.import_module(mod_name)
    prov = getattr(mod, obj_name)

    def read():
        settings = prov.make_settings(args, is_train=(which == "train"))
        order = list(files)
        if which == "train" and prov.should_shuffle and shuffle_seed is not None:
            random.Random(shuffle_seed).shuffle(order)
        batch = []
        for fn in order:
            for sample in prov.samples(settings, fn):
                batch.append(sample)
                if len(batch) == batch_size:
                    yield batch
                    batch = []
        if batch:
            yield batch

    return read, prov


def main(argv=None):
    ap = argparse.ArgumentParser(prog="paddle_trainer", description="v1 trainer front end on the Fluid engine")
    ap.add_argument("--config", required=True)
    ap.add_argument("--config_args", default="")
    ap.add_argument("--job", default="train", choices=["train", "test", "time", "checkgrad"])
    ap.add_argument("--checkgrad_eps", type=float, default=1e-3)
    ap.add_argument("--num_passes", type=int, default=1)
    ap.add_argument("--log_period", type=int, default=100)
    ap.add_argument("--save_dir", default="")
    ap.add_argument("--init_model_path", default="")
    ap.add_argument("--use_gpu", type=int, default=0)
    ap.add_argument("--trainer_count", type=int, default=1)
    ap.add_argument("--test_period", type=int, default=0, help="0: test at the end of every pass")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--local", type=int, default=1, help="0: remote updates on the parameter servers")
    ap.add_argument("--pservers", default="", help="host:port,... of distributed.pserver2 servers (--local=0)")
    ap.add_argument("--trainer_id", type=int, default=0)
    ap.add_argument("--log_stat", type=int, default=0, help="1: print / reset the timer statistics every log period")
    ap.add_argument("--op_stack_trace", type=int, default=0, help="1: operator stack in errors, SIGUSR1 dumps it")
    a = ap.parse_args(argv)

    from .. import v2
    from .. import trainer_config_helpers as tch

    v2._core.STATE["use_gpu"] = bool(a.use_gpu)
    conf = tch.parse_config(a.config, a.config_args)
    src = tch._CFG.get("data_sources")
    bs = conf.batch_size or 1
    train = _reader(src, "train", bs, shuffle_seed=a.seed)
    test = _reader(src, "test", bs)
    if train is None and a.job in ("train", "time", "checkgrad"):
        raise SystemExit("the config defines no training data (define_py_data_sources2 train_list)")
    prov = (train or test)[1]
    feeding = prov.feeding(conf.input_layer_names)
    if a.job == "checkgrad":
        return checkgrad(conf, train[0], prov.feeding(conf.input_layer_names), eps=a.checkgrad_eps, seed=a.seed)
    remote = {} if a.local else {"is_local": False, "pserver_spec": a.pservers, "trainer_id": a.trainer_id}
    trainer, params = conf.make_trainer(**remote)
    if a.init_model_path:
        with open(a.init_model_path, "rb") as f:
            params.init_from_tar(f)
    log = []
    from ..utils import stack_trace
    from ..utils.stat import global_stat

    if a.op_stack_trace:
        stack_trace.install()
    t_batch = [None]

    def handler(e):
        name = type(e).__name__
        if name == "BeginIteration":
            t_batch[0] = time.perf_counter()
        if name == "EndIteration" and t_batch[0] is not None:
            global_stat.add("trainBatch", time.perf_counter() - t_batch[0])
        if name == "EndIteration" and (e.batch_id + 1) % a.log_period == 0:
            print(f"Pass {e.pass_id}, Batch {e.batch_id + 1}, Cost {e.cost:.6f}, {e.metrics}", flush=True)
            if a.log_stat:
                global_stat.print_all_status()
                global_stat.reset()
        if name == "EndIteration":
            log.append(e.cost)
        if name == "EndPass":
            msg = f"Pass {e.pass_id} done, {e.metrics}"
            if test is not None:
                r = trainer.test(reader=test[0], feeding=feeding)
                msg += f"; Test cost {r.cost:.6f}, {r.metrics}"
            print(msg, flush=True)
            if a.save_dir:
                d = os.path.join(a.save_dir, f"pass-{e.pass_id:05d}")
                os.makedirs(d, exist_ok=True)
                with open(os.path.join(d, "params.tar"), "wb") as f:
                    params.to_tar(f)

    if a.job == "train":
        trainer.train(reader=train[0], num_passes=a.num_passes, event_handler=handler, feeding=feeding)
    elif a.job == "test":
        r = trainer.test(reader=(test or train)[0], feeding=feeding)
        print(f"Test cost {r.cost:.6f}, {r.metrics}", flush=True)
    else:  # time: throughput of the training step over one pass
        t0 = time.perf_counter()
        trainer.train(reader=train[0], num_passes=1, event_handler=handler, feeding=feeding)
        dt = time.perf_counter() - t0
        print(f"time: {len(log)} batches in {dt:.3f} s, {len(log) * bs / max(dt, 1e-9):.1f} samples/s", flush=True)
    return log


def checkgrad(conf, reader, feeding, eps=1e-3, seed=1):
    """``--job=checkgrad`` (Trainer.cpp checkGradient): on the first training batch,
    for every parameter compare the analytic directional derivative <dL/dp, d>
    (the program's backward) with the central difference (L(p + eps d) - L(p - eps d))
    / (2 eps) along a random unit direction d.  Prints one line per parameter and
    returns {name: relative difference}."""
    import numpy as np

    from .. import fluid
    from ..v2 import _core

    STATE = _core.STATE
    main = STATE["main"]
    fwd = main.clone(for_test=True)
    with _core.guard():
        pg = fluid.backward.append_backward(conf.cost)
    names = list(STATE["data"])
    order = sorted(feeding.items(), key=lambda kv: kv[1]) if isinstance(feeding, dict) else \
        [(n, i) for i, n in enumerate(feeding)]
    names = [n for n, _ in order] or names
    place = _core.place()
    feeder = fluid.DataFeeder(feed_list=[main.global_block().var(n) for n in names], place=place, program=main)
    batch = next(iter(reader()))
    feed = feeder.feed(batch)
    exe = fluid.Executor(place)
    scope = fluid.core.Scope()
    rs = np.random.RandomState(seed)
    out = {}
    with fluid.scope_guard(scope):
        exe.run(STATE["startup"])
        grads = exe.run(main, feed=feed, fetch_list=[g for _, g in pg])

        def loss():
            (v,) = exe.run(fwd, feed=feed, fetch_list=[conf.cost])
            return float(np.array(v, dtype=np.float64).ravel()[0])

        for (p, _), g in zip(pg, grads):
            t = scope.find_var(p.name).get_tensor()
            p0 = np.array(t.numpy(), dtype=np.float64)
            d = rs.randn(*p0.shape)
            d /= max(np.linalg.norm(d), 1e-12)
            analytic = float((np.array(g, dtype=np.float64) * d).sum())
            t.set((p0 + eps * d).astype(np.float32), place)
            lp = loss()
            t.set((p0 - eps * d).astype(np.float32), place)
            lm = loss()
            t.set(p0.astype(np.float32), place)
            numeric = (lp - lm) / (2 * eps)
            rel = abs(analytic - numeric) / max(abs(analytic), abs(numeric), 1e-8)
            out[p.name] = rel
            print(f"checkgrad {p.name}: analytic {analytic:.6e} numeric {numeric:.6e} rel diff {rel:.3e}",
                  flush=True)
    return out


if __name__ == "__main__":
    main(sys.argv[1:])
