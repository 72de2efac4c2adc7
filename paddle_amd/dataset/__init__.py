"""paddle.dataset: the reference's dataset readers (python/paddle/dataset/*).

There is no network: each module parses its files from the cache directory
(``common.DATA_HOME``: ``PADDLE_DATA_HOME`` or ``~/.cache/paddle/dataset``) when
they are present -- mnist (IDX), uci_housing (text), imikolov (PTB tgz), imdb
(aclImdb tgz), cifar (binary releases), movielens (ml-1m zip) -- and otherwise
serves deterministic synthetic samples of the same shapes with a one-time
warning.  conll05, wmt14, wmt16 and flowers are synthetic only.
"""
from . import common  # noqa: F401
from . import cifar, flowers, imdb, imikolov, mnist, movielens, uci_housing, wmt14, wmt16, conll05  # noqa: F401
