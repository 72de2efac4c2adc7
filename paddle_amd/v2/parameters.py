"""v2 parameters (reference v2/parameters.py): a name -> ndarray view of the v2
session's scope, with the v2 tar format -- one member per parameter holding a
16-byte header (uint32 version 0, uint32 value size 4, uint64 element count) and
the raw float32 values, plus ``<name>.protobuf`` holding the parameter's binary
``ParameterConfig`` message (reference proto/ParameterConfig.proto:34-83; written
at reference v2/parameters.py:350, read at :378).  The proto2 wire format is
encoded and decoded here directly (no generated protobuf module): ``name`` (1),
``size`` (2) and the repeated ``dims`` (9, packed or not) are interpreted, every
other field is skipped by its wire type."""
from __future__ import annotations

import io
import struct
import tarfile

import numpy as np

from .. import fluid
from ._core import STATE, executor


def _varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if not v:
            out.append(b)
            return bytes(out)
        out.append(b | 0x80)


def encode_parameter_config(name: str, dims) -> bytes:
    """ParameterConfig{name, size, dims} in proto2 wire format (dims unpacked, the
    proto2 default for ``repeated uint64``)."""
    nb = name.encode()
    size = 1
    for d in dims:
        size *= int(d)
    out = bytearray(b"\x0a" + _varint(len(nb)) + nb)  # field 1, length-delimited
    out += b"\x10" + _varint(size)  # field 2, varint
    for d in dims:
        out += b"\x48" + _varint(int(d))  # field 9, varint
    return bytes(out)


def _read_varint(buf: bytes, pos: int, end: int):
    v = shift = 0
    while True:
        if pos >= end or shift > 63:
            raise ValueError("ParameterConfig: truncated varint")
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, pos
        shift += 7


def decode_parameter_config(buf: bytes) -> dict:
    """Parse a binary ParameterConfig into {"name", "size", "dims"}; raises
    ValueError on a truncated or malformed message."""
    pos, n = 0, len(buf)
    out = {"name": None, "size": None, "dims": []}
    while pos < n:
        key, pos = _read_varint(buf, pos, n)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _read_varint(buf, pos, n)
            if field == 2:
                out["size"] = v
            elif field == 9:
                out["dims"].append(v)
        elif wt == 2:
            ln, pos = _read_varint(buf, pos, n)
            if pos + ln > n:
                raise ValueError("ParameterConfig: truncated field")
            if field == 1:
                out["name"] = bytes(buf[pos:pos + ln]).decode()
            elif field == 9:  # packed dims
                sp = pos
                while sp < pos + ln:
                    v, sp = _read_varint(buf, sp, pos + ln)
                    out["dims"].append(v)
            pos += ln
        elif wt in (1, 5):
            pos += 8 if wt == 1 else 4
            if pos > n:
                raise ValueError("ParameterConfig: truncated fixed field")
        else:
            raise ValueError(f"ParameterConfig: unsupported wire type {wt}")
    if out["name"] is None or out["size"] is None:
        raise ValueError("ParameterConfig: missing required name / size")
    return out


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
            cb = encode_parameter_config(name, self.get_shape(name))
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
                conf = decode_parameter_config(tar.extractfile(m).read())
                shapes[m.name[: -len(".protobuf")]] = tuple(conf["dims"]) or (conf["size"],)
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
