"""v2 parameters (reference v2/parameters.py): a name -> ndarray view of the v2
session's scope, with the v2 tar format -- one member per parameter holding a
16-byte header (uint32 version 0, uint32 value size 4, uint64 element count) and
the raw float32 values, plus ``<name>.protobuf`` describing it.  (The reference
stores a binary ParameterConfig proto there; this facade writes its text form
``name: ... dims: ...``, which ``from_tar`` reads back for the shape.)"""
from __future__ import annotations

import io
import struct
import tarfile

import numpy as np

from .. import fluid
from ._core import STATE, executor


def _param_names():
    return [p.name for p in STATE["main"].global_block().all_parameters()]


def create(layers):
    """Initialise the parameters of the topology ending at ``layers`` (runs the
    startup program in the v2 scope)."""
    with fluid.scope_guard(STATE["scope"]):
        executor().run(STATE["startup"])
    return Parameters(bound=True)


class Parameters:
    def __init__(self, bound=False):
        self._bound = bound
        self._local = {}  # name -> ndarray for unbound (from_tar) parameter sets

    def _tensor(self, name):
        v = STATE["scope"].find_var(name)
        if v is None:
            raise KeyError(name)
        return v.get_tensor()

    def keys(self):
        return _param_names() if self._bound else list(self._local)

    names = keys

    def has_key(self, key):
        return key in self.keys()

    __contains__ = has_key

    def __iter__(self):
        return iter(self.keys())

    def __len__(self):
        return len(self.keys())

    def __getitem__(self, key):
        if not self._bound:
            return self._local[key]
        return np.array(self._tensor(key)).copy()

    get = __getitem__

    def get_shape(self, key):
        return tuple(self[key].shape)

    def __setitem__(self, key, value):
        value = np.asarray(value, dtype="float32")
        if not self._bound:
            self._local[key] = value
            return
        t = self._tensor(key)
        cur = np.array(t)
        if cur.size != value.size:
            raise ValueError(f"parameter {key}: {value.size} values for shape {cur.shape}")
        from ._core import place

        t.set(value.reshape(cur.shape), place())

    set = __setitem__

    def snapshot(self):
        return {k: self[k] for k in self.keys()}

    def restore(self, snap):
        for k, v in snap.items():
            if self.has_key(k):
                self[k] = v

    def serialize(self, name, f):
        a = self[name].astype("float32").ravel()
        f.write(struct.pack("IIQ", 0, 4, a.size))
        f.write(a.tobytes())

    def deserialize(self, name, f):
        _, _, n = struct.unpack("IIQ", f.read(16))
        a = np.frombuffer(f.read(4 * n), dtype="float32")
        self[name] = a.reshape(self.get_shape(name)) if self.has_key(name) and self._bound else a

    def to_tar(self, f):
        tar = tarfile.TarFile(fileobj=f, mode="w")
        for name in self.keys():
            buf = io.BytesIO()
            self.serialize(name, buf)
            info = tarfile.TarInfo(name=name)
            info.size = buf.tell()
            buf.seek(0)
            tar.addfile(info, buf)
            conf = f"name: \"{name}\"\n" + "".join(f"dims: {d}\n" for d in self.get_shape(name))
            cb = conf.encode()
            ci = tarfile.TarInfo(name=name + ".protobuf")
            ci.size = len(cb)
            tar.addfile(ci, io.BytesIO(cb))
        tar.close()

    @staticmethod
    def from_tar(f):
        p = Parameters(bound=False)
        tar = tarfile.TarFile(fileobj=f, mode="r")
        shapes = {}
        for m in tar.getmembers():
            if m.name.endswith(".protobuf"):
                txt = tar.extractfile(m).read().decode()
                shapes[m.name[: -len(".protobuf")]] = tuple(int(line.split(":")[1]) for line in txt.splitlines()
                                                             if line.startswith("dims:"))
        for m in tar.getmembers():
            if not m.name.endswith(".protobuf"):
                buf = tar.extractfile(m)
                _, _, n = struct.unpack("IIQ", buf.read(16))
                a = np.frombuffer(buf.read(4 * n), dtype="float32").copy()
                p._local[m.name] = a.reshape(shapes.get(m.name, (n,)))
        return p

    def init_from_tar(self, f, exclude_params=()):
        src = Parameters.from_tar(f)
        for k in src.keys():
            if k in exclude_params or not self.has_key(k):
                continue
            self[k] = src[k].reshape(self.get_shape(k))
