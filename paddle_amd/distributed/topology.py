"""Hybrid-parallel process topology (Fleet ``HybridCommunicateGroup``).

North-star component (TP/PP/sharding/EP/CP are all absent from the
reference, whose only multi-device topology is the flat NCCL ring of
``NCCLContextMap`` -- paddle/fluid/platform/nccl_helper.h:81-123 -- with
``rank = trainer_id * ngpu + gpu_id``).

Ranks form a 5-D grid ``[dp, pp, sharding, sep, mp]`` (``mp`` fastest).  On an
MI355X node every GPU pair has its own xGMI link (fully connected, 7 links), so
the mp / sep groups -- the most bandwidth-hungry, latency-critical collectives --
sit on consecutive ranks (same node), and dp is the slowest axis (the only one
that ever needs to leave a node).  One ``torch.distributed`` group per axis slice
is created eagerly on every rank (process-group creation is collective).
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass

from ..parallel import comm

AXES = ("dp", "pp", "sharding", "sep", "mp")


@dataclass
class CommunicateTopology:
    dims: dict  # axis -> degree

    def __post_init__(self):
        for a in AXES:
            self.dims.setdefault(a, 1)
        self.shape = [self.dims[a] for a in AXES]
        self.world_size = 1
        for d in self.shape:
            self.world_size *= d

    def coord(self, rank):
        c = []
        for d in reversed(self.shape):
            c.append(rank % d)
            rank //= d
        return dict(zip(AXES, reversed(c)))

    def rank_of(self, **coord):
        r = 0
        for a, d in zip(AXES, self.shape):
            r = r * d + coord.get(a, 0)
        return r

    def axis_groups(self, axis):
        """All rank lists that vary only along ``axis`` (one list per slice)."""
        others = [a for a in AXES if a != axis]
        out = []
        for fixed in itertools.product(*[range(self.dims[a]) for a in others]):
            base = dict(zip(others, fixed))
            out.append([self.rank_of(**base, **{axis: i}) for i in range(self.dims[axis])])
        return out


class HybridCommunicateGroup:
    def __init__(self, topo: CommunicateTopology, rank: int | None = None):
        self.topo = topo
        self.global_rank = comm.get_rank() if rank is None else rank
        self.nranks = topo.world_size
        ws = comm.get_world_size()
        if comm.is_dist() and ws != topo.world_size:
            raise ValueError(f"hybrid degrees {topo.dims} need {topo.world_size} ranks, world is {ws}")
        self.coord = topo.coord(self.global_rank)
        self._groups, self._ranks = {}, {}
        for axis in AXES:
            for ranks in topo.axis_groups(axis):
                g = comm.new_group(ranks) if comm.is_dist() and len(ranks) > 1 else (
                    comm.SELF if comm.is_dist() else None)
                if self.global_rank in ranks:
                    self._groups[axis], self._ranks[axis] = g, ranks
        # data-parallel gradient reduction spans dp x sharding (sharding is a dp axis)
        for ranks in self._dp_sharding_slices():
            g = comm.new_group(ranks) if comm.is_dist() and len(ranks) > 1 else (
                comm.SELF if comm.is_dist() else None)
            if self.global_rank in ranks:
                self._groups["dp_sharding"], self._ranks["dp_sharding"] = g, ranks

    def _dp_sharding_slices(self):
        d = self.topo.dims
        out = []
        for pp, sep, mp in itertools.product(range(d["pp"]), range(d["sep"]), range(d["mp"])):
            out.append([self.topo.rank_of(dp=a, pp=pp, sharding=s, sep=sep, mp=mp)
                        for a in range(d["dp"]) for s in range(d["sharding"])])
        return out

    # --- Fleet-compatible accessors ------------------------------------------------
    def _deg(self, a):
        return self.topo.dims[a]

    def get_data_parallel_world_size(self):
        return self._deg("dp")

    def get_data_parallel_rank(self):
        return self.coord["dp"]

    def get_data_parallel_group(self):
        return self._groups["dp"]

    def get_model_parallel_world_size(self):
        return self._deg("mp")

    def get_model_parallel_rank(self):
        return self.coord["mp"]

    def get_model_parallel_group(self):
        return self._groups["mp"]

    def get_model_parallel_group_src_rank(self):
        return self._ranks["mp"][0]

    def get_pipe_parallel_world_size(self):
        return self._deg("pp")

    def get_stage_id(self):
        return self.coord["pp"]

    def get_pipe_parallel_group(self):
        return self._groups["pp"]

    def get_pipe_ranks(self):
        return self._ranks["pp"]

    def get_sharding_parallel_world_size(self):
        return self._deg("sharding")

    def get_sharding_parallel_rank(self):
        return self.coord["sharding"]

    def get_sharding_parallel_group(self):
        return self._groups["sharding"]

    def get_sep_parallel_world_size(self):
        return self._deg("sep")

    def get_sep_parallel_rank(self):
        return self.coord["sep"]

    def get_sep_parallel_group(self):
        return self._groups["sep"]

    def get_dp_sharding_group(self):
        return self._groups["dp_sharding"]

    def get_dp_sharding_world_size(self):
        return self._deg("dp") * self._deg("sharding")

    def is_first_stage(self):
        return self.coord["pp"] == 0

    def is_last_stage(self):
        return self.coord["pp"] == self._deg("pp") - 1

    def stage_rank(self, stage):
        """Global rank of pipeline stage ``stage`` in this rank's pp slice."""
        return self._ranks["pp"][stage]

    def parallel_mode(self):
        d = self.topo.dims
        parts = [f"{a}{d[a]}" for a in AXES if d[a] > 1]
        return "+".join(parts) or "single"
