"""Direct intra-node all-reduce over IPC-mapped peer buffers.

A ring all-reduce drives one outbound and one inbound xGMI link per GPU; on a
fully connected 8-GPU MI355X node each GPU has 7 links.  Here every rank exports
an uncached staging buffer and a signal array (hipIpcGetMemHandle), maps every
peer's (hipIpcOpenMemHandle, exchanged over the process group), and the
collective is three or four plain kernels on the caller's stream
(csrc/kernels/p2p.hip):

* one-shot (messages <= ``one_shot_bytes``): copy-in, barrier, every rank sums
  all P stagings into its output (reads the 7 peers concurrently), barrier;
* two-shot: copy-in, barrier, rank r reduces chunk r of all stagings into its own
  staging, barrier, every rank gathers the P reduced chunks, barrier;
* reduce-scatter (ZeRO gradient shards): copy-in, barrier, rank r sums chunk r of
  the P stagings straight into its shard, barrier;
* all-gather (ZeRO parameter shards): copy the shard into chunk r of the own
  staging, barrier, every rank reads the P chunks into its output, barrier.

The training path uses these under ``FLAGS_dp_comm=direct``
(parallel/sharding.py FlatShardedOptimizer, distributed/sharding.py ShardedStage3);
the framework RCCL communicators (parallel/rccl.py) stay the default.

Barriers are bounded spins on system-scope signals: a missing peer makes the op
fail (``DirectAllReduce.check``) instead of hanging the device.  Reference
counterpart: platform/nccl_helper.h + details/all_reduce_op_handle.cc, which
only ever call ncclAllReduce.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from ..ops import _native as N
from . import comm

_P = ctypes.c_void_p


def _env_int(name, default):
    import os

    v = os.environ.get(name, "")
    return int(v) if v.strip() else default


class DirectAllReduce:
    def __init__(self, group=None, max_bytes=None, one_shot_bytes=None, max_spins=None, extra_bytes=0):
        """``extra_bytes``: a second region of the registered staging allocation, after
        the ``max_bytes`` scratch area, handed out by :meth:`staging_tensor` -- a buffer
        placed there (the sharded optimizer's flat gradient) is reduce-scattered in
        place, without the copy-in pass.  Unset sizes come from the flags
        ``FLAGS_direct_max_bytes`` (scratch staging, default 64 MiB),
        ``FLAGS_direct_one_shot_bytes`` (one-shot / two-shot switch, default 1 MiB:
        below it the 7 concurrent peer reads of one-shot beat the extra barrier of
        two-shot) and ``FLAGS_direct_max_spins`` (barrier spin bound)."""
        max_bytes = _env_int("FLAGS_direct_max_bytes", 64 << 20) if max_bytes is None else max_bytes
        one_shot_bytes = _env_int("FLAGS_direct_one_shot_bytes", 1 << 20) if one_shot_bytes is None else one_shot_bytes
        max_spins = _env_int("FLAGS_direct_max_spins", 1 << 25) if max_spins is None else max_spins
        self.group = group
        self.world = comm.get_world_size(group)
        self.rank = comm.get_rank(group)
        if not 1 <= self.world <= 8:
            raise ValueError("DirectAllReduce: 1..8 ranks (one node)")
        self.max_bytes = (int(max_bytes) + 4095) // 4096 * 4096
        self.extra_bytes = (int(extra_bytes) + 4095) // 4096 * 4096
        self.one_shot_bytes = int(one_shot_bytes)
        self.max_spins = int(max_spins)
        self.device = torch.device("cuda", torch.cuda.current_device())
        lib = N.lib()
        self._own = []
        stage, sig = _P(), _P()
        N.check(lib.pa_p2p_alloc(ctypes.byref(stage), self.max_bytes + self.extra_bytes), "pa_p2p_alloc")
        self._own.append(stage.value)
        N.check(lib.pa_p2p_alloc(ctypes.byref(sig), 4096), "pa_p2p_alloc")
        self._own.append(sig.value)
        N.check(lib.pa_p2p_zero(sig, 4096), "pa_p2p_zero")
        torch.cuda.synchronize()
        hs = lib.pa_p2p_ipc_handle_size()
        h_stage, h_sig = ctypes.create_string_buffer(hs), ctypes.create_string_buffer(hs)
        N.check(lib.pa_p2p_ipc_handle(stage, h_stage), "pa_p2p_ipc_handle")
        N.check(lib.pa_p2p_ipc_handle(sig, h_sig), "pa_p2p_ipc_handle")
        allh = [None] * self.world
        dist.all_gather_object(allh, (h_stage.raw, h_sig.raw), group=group)
        self._opened = []
        stages, sigs = [], []
        for r, (hst, hsg) in enumerate(allh):
            if r == self.rank:
                stages.append(stage.value)
                sigs.append(sig.value)
                continue
            ps, pg = _P(), _P()
            N.check(lib.pa_p2p_ipc_open(ctypes.create_string_buffer(hst, hs), ctypes.byref(ps)), "pa_p2p_ipc_open")
            N.check(lib.pa_p2p_ipc_open(ctypes.create_string_buffer(hsg, hs), ctypes.byref(pg)), "pa_p2p_ipc_open")
            self._opened += [ps.value, pg.value]
            stages.append(ps.value)
            sigs.append(pg.value)
        self._stage = (_P * 8)(*stages)
        self._sig = (_P * 8)(*sigs)
        self._err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.epoch = 0
        comm.barrier(group)

    def staging_tensor(self, numel, dtype):
        """A tensor over the extra region of this rank's registered staging buffer
        (every rank places the same layout there).  Uncached device memory: stores
        reach HBM, so peers read it straight after a barrier."""
        es = torch.empty((), dtype=dtype).element_size()
        if numel * es > self.extra_bytes:
            raise ValueError(f"staging_tensor: {numel * es} bytes > the {self.extra_bytes}-byte extra region")
        base = self._stage[self.rank] + self.max_bytes

        class _Iface:  # zero-copy byte view (torch keeps this object alive with the tensor)
            __cuda_array_interface__ = {"shape": (int(numel * es),), "typestr": "|u1", "data": (base, False),
                                        "version": 3}

        t = torch.as_tensor(_Iface(), device=self.device).view(dtype)
        if t.data_ptr() != base:
            raise RuntimeError("staging_tensor: torch copied the buffer instead of viewing it")
        return t

    def _in_place(self, t):
        """Byte offset of ``t`` inside this rank's extra staging region, or None."""
        off = t.data_ptr() - self._stage[self.rank]
        n = t.numel() * t.element_size()
        if self.extra_bytes and off >= self.max_bytes and off + n <= self.max_bytes + self.extra_bytes:
            return off
        return None

    # ------------------------------------------------------------------ pieces
    def _barrier(self):
        self.epoch += 1
        N.call("pa_p2p_barrier", self._stage, self._sig, self.world, self.rank, ctypes.c_uint(self.epoch & 0xffffffff),
               self.max_spins, N.ptr(self._err), N.stream())

    def check(self):
        """Raises if any barrier timed out (synchronises the stream)."""
        e = int(self._err.item())
        if e:
            raise RuntimeError(f"DirectAllReduce: rank {self.rank} timed out waiting for peer {e - 1}")

    def supports(self, t):
        return (t.is_cuda and t.is_contiguous() and t.dtype in (torch.float32, torch.bfloat16)
                and t.numel() % 8 == 0 and t.numel() * t.element_size() <= self.max_bytes)

    # ------------------------------------------------------------------ collective
    def all_reduce(self, t, algo="auto"):
        """In-place sum over the group.  ``algo``: "one_shot", "two_shot" or "auto"."""
        if self.world == 1:
            return t
        if not self.supports(t):
            comm.all_reduce(t, group=self.group)
            return t
        nbytes = t.numel() * t.element_size()
        if algo == "auto":
            algo = "one_shot" if nbytes <= self.one_shot_bytes else "two_shot"
        dt = N.dt(t)
        n = t.numel()
        own = _P(self._stage[self.rank])
        N.call("pa_p2p_copy", own, N.ptr(t), nbytes, N.stream())
        self._barrier()
        if algo == "one_shot":
            N.call("pa_p2p_reduce", dt, self._stage, self._sig, self.world, self.rank, N.ptr(t), 0, n,
                   N.ptr(self._err), N.stream())
        else:
            chunk = (n + 8 * self.world - 1) // (8 * self.world) * 8
            b, e = min(n, self.rank * chunk), min(n, (self.rank + 1) * chunk)
            if e > b:
                N.call("pa_p2p_reduce", dt, self._stage, self._sig, self.world, self.rank, own, b, e,
                       N.ptr(self._err), N.stream())
            self._barrier()
            N.call("pa_p2p_gather", dt, self._stage, self._sig, self.world, self.rank, N.ptr(t), n, chunk,
                   N.ptr(self._err), N.stream())
        self._barrier()  # nobody refills its staging before every peer has read it
        return t

    def _dense_ok(self, *ts):
        return all(t.is_cuda and t.is_contiguous() and t.dtype in (torch.float32, torch.bfloat16) for t in ts)

    def reduce_scatter(self, out, inp):
        """out[:] = sum over ranks of inp[rank * L:(rank + 1) * L], L = out.numel()."""
        L = out.numel()
        n = inp.numel()
        if self.world == 1:
            out.copy_(inp)
            return out
        es = inp.element_size()
        off = self._in_place(inp) if self._dense_ok(inp) else None
        if (n != L * self.world or L % 8 or out.dtype != inp.dtype or (off is None and n * es > self.max_bytes)
                or not self._dense_ok(out, inp)):
            comm.reduce_scatter(out, inp, self.group)
            return out
        if off is None:
            stages = self._stage
            N.call("pa_p2p_copy", _P(self._stage[self.rank]), N.ptr(inp), n * es, N.stream())
        else:
            # the input already lives in the registered buffer at the same offset on
            # every rank: no copy-in pass
            stages = (_P * 8)(*[self._stage[r] + off if r < self.world else 0 for r in range(8)])
        self._barrier()
        b = self.rank * L
        # the kernel writes out[i] for absolute i in [b, b + L): shift the base
        N.call("pa_p2p_reduce", N.dt(inp), stages, self._sig, self.world, self.rank,
               _P(out.data_ptr() - b * es), b, b + L, N.ptr(self._err), N.stream())
        self._barrier()
        return out

    def all_gather(self, out, shard):
        """out[r * L:(r + 1) * L] = shard of rank r, L = shard.numel()."""
        L = shard.numel()
        n = out.numel()
        if self.world == 1:
            out.copy_(shard)
            return out
        es = shard.element_size()
        if (n != L * self.world or L % 8 or out.dtype != shard.dtype or n * es > self.max_bytes
                or not self._dense_ok(out, shard)):
            comm.all_gather(out, shard, self.group)
            return out
        N.call("pa_p2p_copy", _P(self._stage[self.rank] + self.rank * L * es), N.ptr(shard), L * es, N.stream())
        self._barrier()
        N.call("pa_p2p_gather", N.dt(out), self._stage, self._sig, self.world, self.rank, N.ptr(out), n, L,
               N.ptr(self._err), N.stream())
        self._barrier()
        return out

    def error_async(self):
        """Start copying the timeout flag to the host; ``poll_error`` reads it later
        (no stream synchronisation on the step path)."""
        if not hasattr(self, "_err_host"):
            self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._err_ev = None
        self._err_host.copy_(self._err, non_blocking=True)
        self._err_ev = torch.cuda.current_stream().record_event()

    def poll_error(self):
        """Raise if a barrier of an earlier step timed out (waits only for that copy)."""
        ev = getattr(self, "_err_ev", None)
        if ev is None:
            return
        ev.synchronize()
        e = int(self._err_host[0])
        if e:
            raise RuntimeError(f"direct collectives: rank {self.rank} timed out waiting for peer {e - 1}")

    def close(self):
        lib = N.lib()
        torch.cuda.synchronize()
        for p in self._opened:
            lib.pa_p2p_ipc_close(_P(p))
        self._opened = []
        comm.barrier(self.group)
        for p in self._own:
            lib.pa_p2p_free(_P(p))
        self._own = []
