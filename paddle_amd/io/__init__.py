"""paddle.io: datasets, samplers, the DataLoader, and RecordIO tensor files."""
from .dataloader import (BatchSampler, ChainDataset, ComposeDataset, DataLoader, Dataset,  # noqa: F401
                         DistributedBatchSampler, IterableDataset, RandomSampler, Sampler, SequenceSampler,
                         Subset, TensorDataset, WeightedRandomSampler, default_collate_fn, get_worker_info,
                         random_split)
from .recordio import Compressor, RecordIOWriter, recordio_iter, recordio_records  # noqa: F401
