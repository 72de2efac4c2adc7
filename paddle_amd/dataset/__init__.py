"""paddle.dataset: synthetic stand-ins with the reference's reader signatures.

There is no network in this environment, so the dataset modules generate
deterministic synthetic samples of the right shapes/dtypes (documented as such);
the reader API (train()/test() returning sample iterators) matches
python/paddle/dataset/*.
"""
from . import cifar, flowers, imdb, imikolov, mnist, movielens, uci_housing, wmt14, wmt16, conll05  # noqa: F401
