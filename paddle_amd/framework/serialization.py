"""LoDTensor / SelectedRows binary stream format (the reference's checkpoint format).

Bit-compatible with framework/lod_tensor.cc:251-304 (SerializeToStream /
DeserializeFromStream), tensor_util.cc TensorToStream, selected_rows.cc:66-115:

  LoDTensor := u32 version(0) | u64 lod_level | lod_level x (u64 nbytes | u64[] offsets)
               | Tensor
  Tensor    := u32 version(0) | i32 desc_size | VarType.TensorDesc proto | raw LE data
  SelectedRows := u32 version(0) | u64 nrows | i64[] rows | i64 height | Tensor

The native runtime (csrc/runtime/lod_tensor_io.cc) implements the same format in
C++ for large checkpoints (streaming, no Python copies); this module is the
reference implementation both are tested against.
"""
from __future__ import annotations

import io
import struct

import numpy as np
import torch

from . import core
from .proto import VarTypePB

_NP = {0: np.bool_, 1: np.int16, 2: np.int32, 3: np.int64, 4: np.float16, 5: np.float32, 6: np.float64,
       20: np.uint8, 21: np.int8, 19: np.uint64}


def tensor_to_bytes(t: torch.Tensor) -> bytes:
    vt = core.convert_dtype(t.dtype)
    desc = VarTypePB.TensorDesc(data_type=vt, dims=list(t.shape))
    db = desc.SerializeToString()
    tc = t.detach().contiguous().cpu()
    if tc.dtype == torch.bfloat16:
        raw = tc.view(torch.int16).numpy().tobytes()
    else:
        raw = tc.numpy().tobytes()
    return struct.pack("<Ii", 0, len(db)) + db + raw


def write_tensor(f, t):
    f.write(tensor_to_bytes(t))


def read_tensor(f, device="cpu") -> torch.Tensor:
    ver, dsz = struct.unpack("<Ii", f.read(8))
    if ver != 0:
        raise ValueError(f"unsupported tensor version {ver}")
    desc = VarTypePB.TensorDesc.FromString(f.read(dsz))
    dims = list(desc.dims)
    n = int(np.prod(dims)) if dims else 1
    vt = desc.data_type
    if vt == core.VT.BF16:
        a = np.frombuffer(f.read(n * 2), dtype=np.int16).copy()
        t = torch.from_numpy(a).view(torch.bfloat16)
    else:
        dt = np.dtype(_NP[vt])
        a = np.frombuffer(f.read(n * dt.itemsize), dtype=dt).copy()
        t = torch.from_numpy(a)
    return t.reshape(dims).to(device)


def write_lod_tensor(f, lt: core.LoDTensor):
    lod = lt.lod()
    f.write(struct.pack("<IQ", 0, len(lod)))
    for lvl in lod:
        f.write(struct.pack("<Q", len(lvl) * 8))
        f.write(np.asarray(lvl, dtype=np.uint64).tobytes())
    write_tensor(f, lt.tensor)


def read_lod_tensor(f, device="cpu") -> core.LoDTensor:
    ver, nl = struct.unpack("<IQ", f.read(12))
    if ver != 0:
        raise ValueError(f"unsupported LoDTensor version {ver}")
    lod = []
    for _ in range(nl):
        (nb,) = struct.unpack("<Q", f.read(8))
        lod.append(np.frombuffer(f.read(nb), dtype=np.uint64).astype(np.int64).tolist())
    t = read_tensor(f, device)
    return core.LoDTensor(t, lod)


def write_selected_rows(f, sr: core.SelectedRows):
    rows = sr.rows()
    f.write(struct.pack("<IQ", 0, len(rows)))
    f.write(np.asarray(rows, dtype=np.int64).tobytes())
    f.write(struct.pack("<q", sr.height()))
    write_tensor(f, sr.get_tensor().tensor)


def read_selected_rows(f, device="cpu") -> core.SelectedRows:
    ver, n = struct.unpack("<IQ", f.read(12))
    rows = np.frombuffer(f.read(n * 8), dtype=np.int64).tolist()
    (h,) = struct.unpack("<q", f.read(8))
    t = read_tensor(f, device)
    return core.SelectedRows(rows, h, t)


def lod_tensor_to_bytes(lt) -> bytes:
    b = io.BytesIO()
    write_lod_tensor(b, lt)
    return b.getvalue()


def lod_tensor_from_bytes(data, device="cpu"):
    return read_lod_tensor(io.BytesIO(data), device)
