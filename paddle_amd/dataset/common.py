"""Dataset cache + helpers (reference python/paddle/dataset/common.py).

There is no network here: ``download`` never fetches.  It resolves the file a
dataset module needs inside ``DATA_HOME/<module>/`` (``PADDLE_DATA_HOME`` or
``~/.cache/paddle/dataset``, the reference's location), checks its md5 when one is
given, and returns the path -- or ``None`` when the file is absent, in which case
the module serves deterministic synthetic samples of the same shapes and says so
once (``synthetic_notice``).
"""
from __future__ import annotations

import glob
import hashlib
import os
import warnings

DATA_HOME = os.path.expanduser(os.environ.get("PADDLE_DATA_HOME", "~/.cache/paddle/dataset"))
_NOTICED = set()


def md5file(fname):
    h = hashlib.md5()
    with open(fname, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def download(url, module_name, md5sum=None, save_name=None):
    """Path of the cached file for ``url`` (no fetching), or None if absent."""
    path = os.path.join(DATA_HOME, module_name, save_name or url.split("/")[-1])
    if not os.path.exists(path):
        return None
    if md5sum and os.environ.get("PADDLE_DATASET_CHECK_MD5", "1") == "1" and md5file(path) != md5sum:
        raise RuntimeError(f"{path}: md5 mismatch (expected {md5sum}); remove it or set PADDLE_DATASET_CHECK_MD5=0")
    return path


def synthetic_notice(module_name, what):
    if module_name not in _NOTICED:
        _NOTICED.add(module_name)
        warnings.warn(f"paddle.dataset.{module_name}: {what} not found under {DATA_HOME}/{module_name}; "
                      "serving deterministic synthetic samples of the same shapes", stacklevel=3)


def split(reader, line_count, suffix="%05d.txt", dumper=None):
    """Write the samples of ``reader`` into files of ``line_count`` samples each
    (``dumper(samples, file)``; default: one ``repr`` line per sample -- no pickle)."""
    if dumper is None:
        def dumper(lines, f):
            for ln in lines:
                f.write((repr(ln) + "\n").encode())
    lines, idx = [], 0
    for i, d in enumerate(reader()):
        lines.append(d)
        if len(lines) == line_count:
            with open(suffix % idx, "wb") as f:
                dumper(lines, f)
            lines, idx = [], idx + 1
    if lines:
        with open(suffix % idx, "wb") as f:
            dumper(lines, f)


def cluster_files_reader(files_pattern, trainer_count, trainer_id, loader):
    """Reader over the files matching ``files_pattern`` assigned to this trainer
    (file i goes to trainer i % trainer_count); ``loader(file) -> iterable``."""
    def reader():
        files = sorted(glob.glob(files_pattern))
        for i, fn in enumerate(files):
            if i % trainer_count == trainer_id:
                with open(fn, "rb") as f:
                    for s in loader(f):
                        yield s
    return reader
