"""Elastic data-dispatch master (reference: go/master/service.go, client.go,
etcd_client.go, inmem_store.go -- the Go "master" of the fault-tolerant v2
trainer).

The dataset (RecordIO files) is cut into chunks, chunks are grouped into tasks and
trainers pull tasks one at a time:

  * ``get_task(pass_id)`` -> a task (or ``PassBefore`` / ``PassAfter`` /
    ``NoMoreAvailable`` / ``AllTaskFailed``); the task moves todo -> pending and a
    timer is armed;
  * ``task_finished(id)`` -> pending -> done; when todo and pending are empty the
    pass ends: done (+ failed) become the next pass's todo;
  * ``task_failed(id, epoch)`` or the timeout -> the task is re-queued, or moved to
    failed after ``failure_max`` failures (a stale epoch is ignored, so a late
    report from a trainer that timed out cannot fail the re-dispatched copy);
  * every state change is snapshotted to a :class:`Store` and a restarted master
    recovers from it (etcd in the reference; here an atomic-rename JSON file, or
    memory for tests); one master per store holds an exclusive lock (leader);
  * ``request_save_model(trainer, block_s)`` elects one trainer to save the model.

Transport: line-delimited JSON over TCP (one thread per connection), so any
trainer process -- on any node -- can pull work from it.
"""
from __future__ import annotations

import copy
import fcntl
import glob
import json
import os
import socket
import socketserver
import threading
import time


class PassBefore(Exception):
    pass


class PassAfter(Exception):
    pass


class NoMoreAvailable(Exception):
    pass


class AllTaskFailed(Exception):
    pass


_ERRORS = {c.__name__: c for c in (PassBefore, PassAfter, NoMoreAvailable, AllTaskFailed)}


# ------------------------------------------------------------------ stores
class InMemStore:
    def __init__(self):
        self._d = None
        self._lock = threading.Lock()

    def save(self, state: dict):
        with self._lock:
            self._d = json.dumps(state)

    def load(self):
        with self._lock:
            return json.loads(self._d) if self._d else None

    def acquire_leader(self):
        return True

    def release_leader(self):
        pass


class FileStore:
    """Snapshot file + exclusive lock file (the etcd key + election mutex)."""

    def __init__(self, path):
        self.path = path
        self._lockf = None

    def save(self, state: dict):
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(state, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, self.path)

    def load(self):
        if not os.path.exists(self.path):
            return None
        with open(self.path) as f:
            return json.load(f)

    def acquire_leader(self, timeout=10.0):
        self._lockf = open(self.path + ".lock", "w")
        t0 = time.time()
        while True:
            try:
                fcntl.flock(self._lockf, fcntl.LOCK_EX | fcntl.LOCK_NB)
                return True
            except OSError:
                if time.time() - t0 > timeout:
                    return False
                time.sleep(0.05)

    def release_leader(self):
        if self._lockf is not None:
            fcntl.flock(self._lockf, fcntl.LOCK_UN)
            self._lockf.close()
            self._lockf = None


# ------------------------------------------------------------------ dataset
def read_chunks(glob_paths, records_per_chunk=None):
    """A chunk = (path, first_record, n_records).  By default one chunk per RecordIO
    chunk boundary is approximated by ``records_per_chunk`` records (the native
    writer flushes a chunk every ``max_num_records``)."""
    from ..io.recordio import recordio_records

    out = []
    for pat in glob_paths:
        for path in sorted(glob.glob(pat)):
            n = sum(1 for _ in recordio_records(path))
            step = records_per_chunk or max(n, 1)
            for s in range(0, n, step):
                out.append({"path": path, "begin": s, "count": min(step, n - s)})
    return out


# ------------------------------------------------------------------ service
class MasterService:
    def __init__(self, store=None, chunks_per_task=1, timeout_s=20.0, failure_max=3):
        self.store = store or InMemStore()
        if not self.store.acquire_leader():
            raise RuntimeError("another master holds the store lock")
        self.chunks_per_task = chunks_per_task
        self.timeout_s = timeout_s
        self.failure_max = failure_max
        self._mu = threading.RLock()
        self._ready = threading.Event()
        self._timers = []
        self.saving_trainer = None
        self.saving_until = 0.0
        self.state = {"todo": [], "pending": {}, "done": [], "failed": [], "cur_pass": 0}
        st = self.store.load()
        if st is not None:                     # recover (service.go:166)
            self.state = st
            # re-arm timeouts of tasks that were pending when the previous master died
            for tid, t in list(self.state["pending"].items()):
                self._arm(int(tid), t["task"]["epoch"])
            self._ready.set()

    # ---------------------------------------------------------- internals
    def _snapshot(self):
        self.store.save(self.state)

    def _arm(self, task_id, epoch):
        tm = threading.Timer(self.timeout_s, self._check_timeout, (task_id, epoch))
        tm.daemon = True
        tm.start()
        self._timers.append(tm)

    def _check_timeout(self, task_id, epoch):
        with self._mu:
            t = self.state["pending"].get(str(task_id))
            if t is not None:
                self._process_failed(t, epoch)

    def _process_failed(self, t, epoch):
        if t["task"]["epoch"] != epoch:
            return
        self.state["pending"].pop(str(t["task"]["id"]), None)
        t["num_failure"] += 1
        if t["num_failure"] > self.failure_max:
            self.state["failed"].append(t)
        else:
            self.state["todo"].append(t)
        self._snapshot()

    # ---------------------------------------------------------- RPCs
    def set_dataset(self, glob_paths, records_per_chunk=None):
        with self._mu:
            if self._ready.is_set():
                return True
            chunks = read_chunks(glob_paths, records_per_chunk)
            tasks = []
            for i in range(0, len(chunks), self.chunks_per_task):
                tasks.append({"task": {"id": len(tasks), "epoch": 0, "chunks": chunks[i:i + self.chunks_per_task]},
                              "num_failure": 0})
            self.state["todo"] = tasks
            self._snapshot()
            self._ready.set()
            return True

    def get_task(self, pass_id):
        self._ready.wait()
        with self._mu:
            cur = self.state["cur_pass"]
            if pass_id < cur:
                raise PassBefore(f"pass {pass_id} < master pass {cur}")
            if pass_id > cur:
                raise PassAfter(f"pass {pass_id} > master pass {cur}")
            if not self.state["todo"]:
                if not self.state["done"] and not self.state["pending"]:
                    raise AllTaskFailed("all tasks failed")
                raise NoMoreAvailable("no more available task")
            t = self.state["todo"].pop(0)
            t["task"]["epoch"] += 1
            self.state["pending"][str(t["task"]["id"])] = t
            self._snapshot()
            self._arm(t["task"]["id"], t["task"]["epoch"])
            return copy.deepcopy(t["task"])

    def task_finished(self, task_id):
        self._ready.wait()
        with self._mu:
            t = self.state["pending"].pop(str(task_id), None)
            if t is None:
                return False
            t["num_failure"] = 0
            self.state["done"].append(t)
            if not self.state["todo"] and not self.state["pending"]:
                self.state["cur_pass"] += 1
                self.state["todo"] = self.state["done"] + self.state["failed"]
                self.state["done"], self.state["failed"] = [], []
            self._snapshot()
            return True

    def task_failed(self, task_id, epoch):
        self._ready.wait()
        with self._mu:
            t = self.state["pending"].get(str(task_id))
            if t is None:
                return False
            self._process_failed(t, epoch)
            return True

    def request_save_model(self, trainer_id, block_s=5.0):
        if not trainer_id:
            raise ValueError("trainer id is empty")
        with self._mu:
            now = time.time()
            if self.saving_trainer is None or now > self.saving_until or self.saving_trainer == trainer_id:
                self.saving_trainer, self.saving_until = trainer_id, now + block_s
                return True
            return False

    def status(self):
        with self._mu:
            s = self.state
            return {"todo": len(s["todo"]), "pending": len(s["pending"]), "done": len(s["done"]),
                    "failed": len(s["failed"]), "cur_pass": s["cur_pass"]}

    def shutdown(self):
        for t in self._timers:
            t.cancel()
        self.store.release_leader()


# ------------------------------------------------------------------ TCP transport
class _Handler(socketserver.StreamRequestHandler):
    def handle(self):
        svc = self.server.service
        for line in self.rfile:
            req = json.loads(line)
            try:
                res = {"ok": getattr(svc, req["method"])(*req.get("args", []))}
            except Exception as e:  # noqa: BLE001  (sent back to the client)
                res = {"err": type(e).__name__, "msg": str(e)}
            self.wfile.write((json.dumps(res) + "\n").encode())
            self.wfile.flush()


class _Server(socketserver.ThreadingMixIn, socketserver.TCPServer):
    daemon_threads = True
    allow_reuse_address = True


class MasterServer:
    """Serve a MasterService on ``host:port`` (port 0 = pick one)."""

    def __init__(self, service, host="127.0.0.1", port=0):
        self.service = service
        self._srv = _Server((host, port), _Handler)
        self._srv.service = service
        self.endpoint = f"{host}:{self._srv.server_address[1]}"
        self._t = threading.Thread(target=self._srv.serve_forever, daemon=True)
        self._t.start()

    def stop(self):
        self._srv.shutdown()
        self._srv.server_close()
        self.service.shutdown()


class MasterClient:
    """Trainer side (go/master/client.go): pulls tasks and streams their records."""

    _RPC = ("set_dataset", "get_task", "task_finished", "task_failed", "request_save_model", "status")

    def __init__(self, endpoint, timeout=30.0):
        host, port = endpoint.rsplit(":", 1)
        self._sock = socket.create_connection((host, int(port)), timeout=timeout)
        self._f = self._sock.makefile("rwb")
        self._lock = threading.Lock()

    def _call(self, method, *args):
        with self._lock:
            self._f.write((json.dumps({"method": method, "args": list(args)}) + "\n").encode())
            self._f.flush()
            res = json.loads(self._f.readline())
        if "err" in res:
            raise _ERRORS.get(res["err"], RuntimeError)(res["msg"])
        return res["ok"]

    def __getattr__(self, name):
        if name in self._RPC:
            return lambda *a: self._call(name, *a)
        raise AttributeError(name)

    def records(self, pass_id, on_task=None):
        """Yield every record of ``pass_id`` handed to this trainer; a task is
        reported finished once all its records were consumed."""
        from ..io.recordio import recordio_records

        while True:
            try:
                task = self.get_task(pass_id)
            except (NoMoreAvailable,):
                time.sleep(0.05)
                try:
                    st = self.status()
                except Exception:  # noqa: BLE001
                    return
                if st["cur_pass"] > pass_id or (st["todo"] == 0 and st["pending"] == 0):
                    return
                continue
            except (PassBefore, AllTaskFailed):
                return
            if on_task is not None:
                on_task(task)
            for ch in task["chunks"]:
                for i, rec in enumerate(recordio_records(ch["path"])):
                    if i < ch["begin"]:
                        continue
                    if i >= ch["begin"] + ch["count"]:
                        break
                    yield rec
            self.task_finished(task["id"])

    def close(self):
        try:
            self._f.close()
            self._sock.close()
        except OSError:
            pass
