"""paddle.distributed equivalent: process groups + collectives (RCCL over xGMI),
DataParallel, Fleet hybrid parallelism, group-sharded (ZeRO 1/2/3) training and
the multi-process launcher."""
from ..parallel.comm import (all_gather, all_reduce, all_to_all, barrier, broadcast, get_rank,  # noqa: F401
                             get_world_size, init_parallel_env, new_group, reduce_scatter)
from . import fleet  # noqa: F401
from .parallel import DataParallel  # noqa: F401
from .launch import spawn  # noqa: F401
from .sharding import ShardedStage3, group_sharded_parallel  # noqa: F401
from .topology import CommunicateTopology, HybridCommunicateGroup  # noqa: F401
