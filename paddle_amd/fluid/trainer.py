"""High-level Trainer with events and checkpointing (python/paddle/fluid/trainer.py).

Checkpoint layout (trainer.py:558-606,1168-1236): ``checkpoint_dir/checkpoint_<serial>/``
with ``__model__/`` persistables, ``trainer_<id>/{epoch_id,step_id}`` and a ``_SUCCESS``
marker written last; resume picks the newest serial that has ``_SUCCESS``; only
trainer 0 writes persistables; ``max_num_checkpoints`` rotation.
"""
from __future__ import annotations

import os
import shutil

from ..framework import core
from . import io, unique_name
from .data_feeder import DataFeeder
from .executor import Executor, scope_guard
from .framework import Program, program_guard
from .parallel_executor import ParallelExecutor

SUCCESS_MARK_FILENAME = "_SUCCESS"
CHECKPOINT_PREFIX = "checkpoint"
MODEL_DIR = "__model__"
TRAINER_PREFIX = "trainer"
CHECKPOINT_SEPARATOR = "_"


class BeginEpochEvent:
    def __init__(self, epoch_id):
        self.epoch = epoch_id


class EndEpochEvent:
    def __init__(self, epoch_id):
        self.epoch = epoch_id


class BeginStepEvent:
    def __init__(self, epoch_id, step_id):
        self.epoch = epoch_id
        self.step = step_id
        self.fetch_metrics = True


class EndStepEvent:
    def __init__(self, epoch_id, step_id, metrics):
        self.epoch = epoch_id
        self.step = step_id
        self.metrics = metrics


class CheckpointConfig:
    def __init__(self, checkpoint_dir=None, max_num_checkpoints=3, epoch_interval=1, step_interval=10):
        self.checkpoint_dir = checkpoint_dir or os.getcwd()
        self.max_num_checkpoints = max_num_checkpoints
        self.epoch_interval = max(1, epoch_interval)
        self.step_interval = max(1, step_interval)
        self.epoch_id = 0
        self.step_id = 0
        self.load_serial = None
        self.pserver_id = None
        self.lookup_table_name = None


def _serial_dirs(checkpoint_dir):
    if not os.path.isdir(checkpoint_dir):
        return []
    out = []
    for d in os.listdir(checkpoint_dir):
        if d.startswith(CHECKPOINT_PREFIX + CHECKPOINT_SEPARATOR):
            try:
                out.append(int(d.split(CHECKPOINT_SEPARATOR)[-1]))
            except ValueError:
                pass
    return sorted(out)


def _get_latest_checkpoint_serial(checkpoint_dir):
    for s in reversed(_serial_dirs(checkpoint_dir)):
        if os.path.isfile(os.path.join(checkpoint_dir, f"{CHECKPOINT_PREFIX}_{s}", SUCCESS_MARK_FILENAME)):
            return s
    return -1


def save_checkpoint(executor, checkpoint_dir, trainer_id, main_program, trainer_args=None, max_num_checkpoints=3):
    serial = _get_latest_checkpoint_serial(checkpoint_dir) + 1
    cur = os.path.join(checkpoint_dir, f"{CHECKPOINT_PREFIX}_{serial}")
    os.makedirs(cur, exist_ok=True)
    tdir = os.path.join(cur, f"{TRAINER_PREFIX}_{trainer_id}")
    os.makedirs(tdir, exist_ok=True)
    for k, v in (trainer_args or {}).items():
        with open(os.path.join(tdir, k), "w") as f:
            f.write(str(v))
    if trainer_id == 0:
        io.save_persistables(executor, os.path.join(cur, MODEL_DIR), main_program)
        open(os.path.join(cur, SUCCESS_MARK_FILENAME), "w").close()
    _scroll_delete(checkpoint_dir, max_num_checkpoints)
    return serial


def _scroll_delete(checkpoint_dir, max_num_checkpoints=3):
    serials = _serial_dirs(checkpoint_dir)
    for s in serials[:-max_num_checkpoints] if max_num_checkpoints > 0 else []:
        shutil.rmtree(os.path.join(checkpoint_dir, f"{CHECKPOINT_PREFIX}_{s}"), ignore_errors=True)


def load_checkpoint(executor, checkpoint_dir, main_program, serial=None, trainer_id=0):
    if serial is None:
        serial = _get_latest_checkpoint_serial(checkpoint_dir)
    if serial < 0:
        return None
    cur = os.path.join(checkpoint_dir, f"{CHECKPOINT_PREFIX}_{serial}")
    io.load_persistables(executor, os.path.join(cur, MODEL_DIR), main_program)
    args = {}
    tdir = os.path.join(cur, f"{TRAINER_PREFIX}_{trainer_id}")
    if os.path.isdir(tdir):
        for k in os.listdir(tdir):
            with open(os.path.join(tdir, k)) as f:
                args[k] = f.read()
    return args


def clean_checkpoint(checkpoint_dir, delete_dir=False):
    for s in _serial_dirs(checkpoint_dir):
        shutil.rmtree(os.path.join(checkpoint_dir, f"{CHECKPOINT_PREFIX}_{s}"), ignore_errors=True)
    if delete_dir and os.path.isdir(checkpoint_dir) and not os.listdir(checkpoint_dir):
        os.rmdir(checkpoint_dir)


class Trainer:
    def __init__(self, train_func, optimizer_func, param_path=None, place=None, parallel=False,
                 checkpoint_config=None):
        self.__stop = False
        self.parallel = parallel
        self.checkpoint_cfg = checkpoint_config
        self.scope = core.Scope()
        self.startup_program = Program()
        self.train_program = Program()
        self.trainer_id = int(os.environ.get("PADDLE_TRAINER_ID", "0"))
        with program_guard(self.train_program, self.startup_program):
            with unique_name.guard():
                outs = train_func()
                self.train_func_outputs = outs if isinstance(outs, list) else [outs]
                self.test_program = self.train_program.clone(for_test=True)
                loss = self.train_func_outputs[0]
                optimizer = optimizer_func()
                optimizer.minimize(loss)
                self._dist_transpile_if_necessary()
        self.place = place or core.CPUPlace()
        with scope_guard(self.scope):
            exe = Executor(self.place)
            exe.run(self.startup_program)
            if self.checkpoint_cfg is not None:
                args = load_checkpoint(exe, self.checkpoint_cfg.checkpoint_dir, self.train_program,
                                       self.checkpoint_cfg.load_serial, self.trainer_id)
                if args:
                    self.checkpoint_cfg.epoch_id = int(args.get("epoch_id", 0))
                    self.checkpoint_cfg.step_id = int(args.get("step_id", 0))
            if param_path and os.path.isdir(param_path):
                io.load_persistables(exe, dirname=param_path, main_program=self.startup_program)

    # ------------------------------------------------------------------ cluster roles
    def _dist_transpile_if_necessary(self):
        """Environment-driven distribution (reference trainer.py:295-360).

        * ``PADDLE_TRAINER_IPS`` (+ ``PADDLE_PSERVER_PORT``, ``PADDLE_TRAINER_ID``,
          ``PADDLE_CURRENT_IP``): collective data parallelism -- the reference's NCCL2
          mode -- one process per trainer over ``torch.distributed`` (RCCL on the GPU),
          gradients synchronised by the ParallelExecutor's bucket all-reduce.
        * ``PADDLE_TRAINING_ROLE`` = TRAINER / PSERVER (+ ``PADDLE_PSERVER_IPS``,
          ``PADDLE_PSERVER_PORT``, ``PADDLE_TRAINERS``, ``PADDLE_CURRENT_IP``):
          DistributeTranspiler parameter-server training; a PSERVER's ``train``
          serves until every trainer has finished."""
        self.training_role = None
        self.nccl_mode = False
        ips = os.environ.get("PADDLE_TRAINER_IPS")
        if ips:
            from ..parallel import comm

            port = os.environ.get("PADDLE_PSERVER_PORT", "6174")
            ips = [ip for ip in ips.split(",") if ip]
            self.trainer_id = int(os.environ.get("PADDLE_TRAINER_ID", "0"))
            self.num_trainers = len(ips)
            os.environ.setdefault("MASTER_ADDR", ips[0])
            os.environ.setdefault("MASTER_PORT", port)
            os.environ.setdefault("RANK", str(self.trainer_id))
            os.environ.setdefault("WORLD_SIZE", str(self.num_trainers))
            if self.num_trainers > 1:
                comm.init_parallel_env()
            self.nccl_mode = True
            self.parallel = True
            return
        role = os.environ.get("PADDLE_TRAINING_ROLE")
        if not role:
            return
        from .transpiler.distribute_transpiler import DistributeTranspiler

        port = os.environ.get("PADDLE_PSERVER_PORT", "6174")
        eps = [f"{ip}:{port}" for ip in os.environ.get("PADDLE_PSERVER_IPS", "").split(",") if ip]
        trainers = int(os.environ.get("PADDLE_TRAINERS", "1"))
        current = os.environ.get("PADDLE_CURRENT_IP", "") + ":" + port
        self.trainer_id = int(os.environ.get("PADDLE_TRAINER_ID", "0"))
        t = DistributeTranspiler()
        t.transpile(self.trainer_id, program=self.train_program, pservers=",".join(eps), trainers=trainers,
                    startup_program=self.startup_program)
        if role == "PSERVER":
            if self.checkpoint_cfg is not None:
                self.checkpoint_cfg.pserver_id = eps.index(current)
            self.train_program, self.startup_program = t.get_pserver_programs(current)
        elif role == "TRAINER":
            self.train_program = t.get_trainer_program()
        else:
            raise ValueError("PADDLE_TRAINING_ROLE must be TRAINER or PSERVER")
        self.training_role = role

    def stop(self):
        self.__stop = True

    def train(self, num_epochs, event_handler, reader=None, feed_order=None):
        if self.training_role == "PSERVER":
            with scope_guard(self.scope):
                Executor(self.place).run(self.train_program)  # listen_and_serv until trainers finish
            return
        with scope_guard(self.scope):
            feed_vars = [self.train_program.global_block().var(n) for n in (feed_order or [])]
            feeder = DataFeeder(feed_list=feed_vars, place=self.place, program=self.train_program)
            exe = ParallelExecutor(use_cuda=isinstance(self.place, core.CUDAPlace),
                                   loss_name=self.train_func_outputs[0].name, main_program=self.train_program,
                                   scope=self.scope) if self.parallel else Executor(self.place)
            start_epoch = self.checkpoint_cfg.epoch_id if self.checkpoint_cfg else 0
            for epoch_id in range(start_epoch, num_epochs):
                event_handler(BeginEpochEvent(epoch_id))
                for step_id, data in enumerate(reader()):
                    if self.__stop:
                        return
                    begin = BeginStepEvent(epoch_id, step_id)
                    event_handler(begin)
                    fetch = self.train_func_outputs if begin.fetch_metrics else []
                    if self.parallel:
                        metrics = exe.run(fetch_list=[v.name for v in fetch], feed=feeder.feed(data))
                    else:
                        metrics = exe.run(self.train_program, feed=feeder.feed(data), fetch_list=fetch)
                    cfg = self.checkpoint_cfg
                    if cfg and step_id % cfg.step_interval == 0 and epoch_id % cfg.epoch_interval == 0:
                        save_checkpoint(Executor(self.place), cfg.checkpoint_dir, self.trainer_id,
                                        self.train_program, {"epoch_id": epoch_id, "step_id": step_id},
                                        cfg.max_num_checkpoints)
                    event_handler(EndStepEvent(epoch_id, step_id, metrics))
                event_handler(EndEpochEvent(epoch_id))
            if self.checkpoint_cfg:
                clean_checkpoint(self.checkpoint_cfg.checkpoint_dir)
            if self.training_role == "TRAINER" and hasattr(exe, "close"):
                exe.close()  # tells the pservers this trainer is done

    def test(self, reader, feed_order):
        with scope_guard(self.scope):
            feed_vars = [self.test_program.global_block().var(n) for n in feed_order]
            feeder = DataFeeder(feed_list=feed_vars, place=self.place, program=self.test_program)
            exe = Executor(self.place)
            accum = [0.0] * len(self.train_func_outputs)
            count = 0
            for data in reader():
                outs = exe.run(self.test_program, feed=feeder.feed(data), fetch_list=self.train_func_outputs)
                accum = [a + float(o.mean()) for a, o in zip(accum, outs)]
                count += 1
            return [a / max(1, count) for a in accum]

    def save_params(self, param_path):
        with scope_guard(self.scope):
            io.save_persistables(Executor(self.place), param_path, self.train_program)
