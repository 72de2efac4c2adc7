"""Fleet collective training API (hybrid parallel: dp / mp / pp / sharding / sep / ep)."""
from .base import DistributedStrategy, HybridParallelOptimizer, TensorParallel, fleet  # noqa: F401
from .context_parallel import (allgather_kv_attention, ring_attention, ulysses_attention,  # noqa: F401
                               zigzag_merge, zigzag_split)
from .moe import MoELayer, TopKGate  # noqa: F401
from .mp_layers import (ColumnParallelLinear, ParallelCrossEntropy, RowParallelLinear, TPGroup,  # noqa: F401
                        VocabParallelEmbedding, parallel_cross_entropy, vocab_parallel_embedding)
from .pipeline import LayerDesc, PipelineLayer, PipelineParallel, SharedLayerDesc  # noqa: F401

init = fleet.init
distributed_model = fleet.distributed_model
distributed_optimizer = fleet.distributed_optimizer
get_hybrid_communicate_group = fleet.get_hybrid_communicate_group
worker_index = fleet.worker_index
worker_num = fleet.worker_num
is_first_worker = fleet.is_first_worker
barrier_worker = fleet.barrier_worker


class meta_parallel:  # namespace mirror of paddle.distributed.fleet.meta_parallel
    ColumnParallelLinear = ColumnParallelLinear
    RowParallelLinear = RowParallelLinear
    VocabParallelEmbedding = VocabParallelEmbedding
    ParallelCrossEntropy = ParallelCrossEntropy
    LayerDesc = LayerDesc
    SharedLayerDesc = SharedLayerDesc
    PipelineLayer = PipelineLayer
    PipelineParallel = PipelineParallel
    TensorParallel = TensorParallel
