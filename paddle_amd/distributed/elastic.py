"""Failure detection, fault injection and restart-from-checkpoint.

The reference's only real fault tolerance is the Go master/pserver pair (task
re-dispatch, etcd snapshots; ported in :mod:`paddle_amd.distributed.master`); a
dead trainer in its NCCL mode simply hangs or aborts.  MI355X-native equivalents
for the collective (RCCL) world:

* :class:`Watchdog` -- a heartbeat thread.  Training loops call ``beat(step)``; if
  no beat arrives for ``timeout_s`` (a collective stuck on a dead peer, a hung
  kernel, a deadlocked data loader) it dumps every thread's stack and exits the
  process with :data:`EXIT_WATCHDOG`, so the launcher can tear the group down and
  restart it instead of hanging until the RCCL timeout.  Each poll also checks the
  framework RCCL communicators' asynchronous errors (``CommContextMap.check_health``:
  ncclCommGetAsyncError, then ncclCommAbort on all of them) and takes the same exit
  as soon as a peer has failed.
* :func:`maybe_inject_fault` -- ``PADDLE_FAULT_INJECT="rank:step[:kind]"``
  (kind = ``exit`` | ``raise`` | ``hang``) makes one rank fail at one step; it fires
  only in the first launch (``PADDLE_RESTART_COUNT`` == 0) so the restarted job
  runs clean.  Used by the tests; harmless when unset.
* :class:`CheckpointManager` -- serial-numbered checkpoint directories with a
  ``_SUCCESS`` marker written last, ``max_num_checkpoints`` rotation and
  ``latest()`` = newest complete checkpoint (reference trainer.py:1168-1236
  semantics, with ``.pdparams`` / ``.pdopt`` payloads).
* ``python -m paddle_amd.distributed.launch --max_restarts N`` restarts the whole
  process group after a failure (new rendezvous port, ``PADDLE_RESTART_COUNT``
  incremented); scripts resume from ``CheckpointManager.latest()``.
"""
from __future__ import annotations

import faulthandler
import os
import shutil
import sys
import threading
import time

EXIT_WATCHDOG = 86
EXIT_INJECTED = 87


class Watchdog:
    def __init__(self, timeout_s=600.0, name="train", on_timeout=None, poll_s=None):
        self.timeout_s = float(timeout_s)
        self.name = name
        self.on_timeout = on_timeout
        self._last = time.monotonic()
        self._step = -1
        self._stop = threading.Event()
        self._poll = poll_s or min(5.0, max(0.05, self.timeout_s / 10))
        self._t = threading.Thread(target=self._run, daemon=True, name=f"watchdog-{name}")
        self._t.start()

    def beat(self, step=None):
        self._last = time.monotonic()
        if step is not None:
            self._step = step

    def _comm_failed(self):
        """Poll the framework RCCL communicators' asynchronous errors (a dead peer):
        ``check_health`` aborts every communicator and raises -> True."""
        try:
            from ..parallel import rccl

            if rccl._MAP._comms:
                rccl._MAP.check_health()
        except Exception as e:  # noqa: BLE001 - RcclError, or a library that is gone
            sys.stderr.write(f"[watchdog:{self.name}] communicator failure: {e}\n")
            return True
        return False

    def _run(self):
        while not self._stop.wait(self._poll):
            if self._comm_failed():
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
                if self.on_timeout is not None:
                    self.on_timeout(self._step)
                    return
                os._exit(EXIT_WATCHDOG)
            idle = time.monotonic() - self._last
            if idle > self.timeout_s:
                sys.stderr.write(f"[watchdog:{self.name}] no progress for {idle:.1f}s after step {self._step} "
                                 f"(rank {os.environ.get('RANK', '0')}); dumping stacks and exiting\n")
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
                if self.on_timeout is not None:
                    self.on_timeout(self._step)
                    return
                os._exit(EXIT_WATCHDOG)

    def stop(self):
        self._stop.set()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()


def restart_count():
    return int(os.environ.get("PADDLE_RESTART_COUNT", "0"))


def maybe_inject_fault(step, rank=None):
    spec = os.environ.get("PADDLE_FAULT_INJECT")
    if not spec or restart_count() > 0:
        return
    parts = spec.split(":")
    frank, fstep = int(parts[0]), int(parts[1])
    kind = parts[2] if len(parts) > 2 else "exit"
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    if rank != frank or step != fstep:
        return
    sys.stderr.write(f"[fault-inject] rank {rank} step {step}: {kind}\n")
    sys.stderr.flush()
    if kind == "raise":
        raise RuntimeError(f"injected fault at step {step}")
    if kind == "hang":
        while True:
            time.sleep(3600)
    os._exit(EXIT_INJECTED)


class CheckpointManager:
    """``root/checkpoint_<serial>/{...payload..., _SUCCESS}`` with rotation."""

    PREFIX = "checkpoint_"

    def __init__(self, root, max_num_checkpoints=3):
        self.root = root
        self.max_num = max_num_checkpoints
        os.makedirs(root, exist_ok=True)

    def _serials(self, complete_only=True):
        out = []
        for d in os.listdir(self.root):
            if d.startswith(self.PREFIX):
                try:
                    s = int(d[len(self.PREFIX):])
                except ValueError:
                    continue
                if not complete_only or os.path.exists(os.path.join(self.root, d, "_SUCCESS")):
                    out.append(s)
        return sorted(out)

    def dir(self, serial):
        return os.path.join(self.root, f"{self.PREFIX}{serial}")

    def latest(self):
        s = self._serials()
        return (s[-1], self.dir(s[-1])) if s else (None, None)

    def save(self, step, payload: dict, rank=0):
        """Rank 0 writes ``payload`` (name -> state dict) as ``name.pdparams``; the
        ``_SUCCESS`` marker goes last so a crash mid-save leaves no 'latest'."""
        from .. import checkpoint as ckpt

        d = self.dir(step)
        if rank == 0:
            os.makedirs(d, exist_ok=True)
            for name, sd in payload.items():
                ckpt.save(sd, os.path.join(d, f"{name}.pdparams"))
            with open(os.path.join(d, "step"), "w") as f:
                f.write(str(step))
            with open(os.path.join(d, "_SUCCESS"), "w") as f:
                f.write("ok")
            self._rotate()
        return d

    def load(self, serial=None):
        from .. import checkpoint as ckpt

        if serial is None:
            serial, d = self.latest()
            if serial is None:
                return None, {}
        else:
            d = self.dir(serial)
        out = {}
        for fn in os.listdir(d):
            if fn.endswith(".pdparams"):
                out[fn[:-len(".pdparams")]] = ckpt.load(os.path.join(d, fn))
        return serial, out

    def _rotate(self):
        s = self._serials(complete_only=False)
        for old in s[:-self.max_num] if self.max_num and len(s) > self.max_num else []:
            shutil.rmtree(self.dir(old), ignore_errors=True)
