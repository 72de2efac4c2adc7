"""Multi-process launcher: ``python -m paddle_amd.distributed.launch --nproc_per_node 8 train.py ...``.

Reference parity: ``python/paddle/distributed/launch.py`` (one process per GPU,
exporting PADDLE_TRAINER_ID / PADDLE_CURRENT_ENDPOINT / PADDLE_TRAINER_ENDPOINTS /
PADDLE_TRAINERS_NUM and CUDA_VISIBLE_DEVICES per child).

MI355X design: the launcher itself never touches the GPU (so it may start and
supervise children freely); each child gets ``LOCAL_RANK`` / ``RANK`` /
``WORLD_SIZE`` / ``MASTER_ADDR`` / ``MASTER_PORT`` (the TCP-store rendezvous
RCCL's ``init_process_group`` uses) plus the Paddle variable names, and sees ALL
GPUs of the node (HIP_VISIBLE_DEVICES is not narrowed, so RCCL can map the xGMI
topology; the child binds ``cuda:LOCAL_RANK``).  If any child fails the others are
terminated and the launcher exits with that child's code.
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time


def _parse(argv):
    ap = argparse.ArgumentParser(description="paddle_amd multi-process launcher")
    ap.add_argument("--nproc_per_node", "--gpus_per_node", type=int, default=None)
    ap.add_argument("--gpus", type=str, default=None, help="comma list of GPU ids (default: all)")
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--node_rank", type=int, default=0)
    ap.add_argument("--master_addr", "--ips", type=str, default="127.0.0.1")
    ap.add_argument("--master_port", "--started_port", type=int, default=29500)
    ap.add_argument("--log_dir", type=str, default=None)
    ap.add_argument("--max_restarts", type=int, default=0,
                    help="restart the whole process group up to N times after a failure (elastic)")
    ap.add_argument("script")
    ap.add_argument("script_args", nargs=argparse.REMAINDER)
    return ap.parse_args(argv)


def _count_gpus():
    # counting devices does not initialise HIP (safe in a launcher)
    try:
        import torch

        return max(1, torch.cuda.device_count())
    except Exception:  # noqa: BLE001
        return 1


def child_envs(nproc, nnodes=1, node_rank=0, master_addr="127.0.0.1", master_port=29500, gpus=None):
    world = nproc * nnodes
    eps = [f"{master_addr}:{master_port + i}" for i in range(world)]
    envs = []
    for local in range(nproc):
        rank = node_rank * nproc + local
        e = dict(os.environ)
        e.update(RANK=str(rank), LOCAL_RANK=str(gpus[local] if gpus else local), WORLD_SIZE=str(world),
                 LOCAL_WORLD_SIZE=str(nproc), MASTER_ADDR=master_addr, MASTER_PORT=str(master_port),
                 PADDLE_TRAINER_ID=str(rank), PADDLE_TRAINERS_NUM=str(world),
                 PADDLE_CURRENT_ENDPOINT=eps[rank], PADDLE_TRAINER_ENDPOINTS=",".join(eps),
                 FLAGS_selected_gpus=str(gpus[local] if gpus else local))
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        envs.append(e)
    return envs


def _run_group(a, envs, attempt):
    procs = []
    for i, e in enumerate(envs):
        e = dict(e, PADDLE_RESTART_COUNT=str(attempt))
        out = None
        if a.log_dir:
            os.makedirs(a.log_dir, exist_ok=True)
            out = open(os.path.join(a.log_dir, f"workerlog.{i}" + (f".restart{attempt}" if attempt else "")), "w")
        procs.append(subprocess.Popen([sys.executable, "-u", a.script] + a.script_args, env=e,
                                      stdout=out, stderr=subprocess.STDOUT if out else None))
    rc = 0
    try:
        alive = list(procs)
        while alive:
            for p in list(alive):
                r = p.poll()
                if r is None:
                    continue
                alive.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    # one rank died: the survivors would block in their next collective
                    for q in alive:
                        q.send_signal(signal.SIGTERM)
                    deadline = time.time() + 15
                    for q in alive:
                        try:
                            q.wait(max(0.1, deadline - time.time()))
                        except subprocess.TimeoutExpired:
                            q.kill()
            time.sleep(0.2)
    except KeyboardInterrupt:
        for p in procs:
            p.send_signal(signal.SIGTERM)
        return 130, True
    return rc, False


def launch(argv=None):
    a = _parse(argv if argv is not None else sys.argv[1:])
    gpus = [int(x) for x in a.gpus.split(",")] if a.gpus else None
    nproc = a.nproc_per_node or (len(gpus) if gpus else _count_gpus())
    rc = 0
    for attempt in range(a.max_restarts + 1):
        # a fresh rendezvous port per attempt (the old one may sit in TIME_WAIT)
        envs = child_envs(nproc, a.nnodes, a.node_rank, a.master_addr, a.master_port + 17 * attempt, gpus)
        rc, interrupted = _run_group(a, envs, attempt)
        if rc == 0 or interrupted:
            return rc
        sys.stderr.write(f"[launch] process group failed (rc={rc}); "
                         f"{'restarting' if attempt < a.max_restarts else 'giving up'} "
                         f"({attempt + 1}/{a.max_restarts + 1})\n")
    return rc


def spawn(func, args=(), nprocs=1, join=True, backend=None):
    """``paddle.distributed.spawn``: run ``func(*args)`` in ``nprocs`` processes with the
    rendezvous environment set (fork-free: multiprocessing ``spawn`` context)."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    envs = child_envs(nprocs, master_port=port)
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_spawn_entry, args=(envs[i], func, args, backend)) for i in range(nprocs)]
    for p in procs:
        p.start()
    if join:
        for p in procs:
            p.join()
        bad = [p.exitcode for p in procs if p.exitcode]
        if bad:
            raise RuntimeError(f"spawned process failed with exit code {bad[0]}")
    return procs


def _spawn_entry(env, func, args, backend):
    os.environ.update(env)
    from ..parallel.comm import init_parallel_env

    init_parallel_env(backend)
    func(*args)


if __name__ == "__main__":
    sys.exit(launch())
