"""Program IR schema, wire-compatible with the reference's ``framework.proto``
(paddle/fluid/framework/framework.proto:19-183): same package, message names,
field numbers and enum values, so ``__model__`` files and checkpoints written by
the reference parse here and vice versa.  Additions (north star): VarType.BF16=22,
FP8_E4M3=23, FP8_E5M2=24.

The schema is assembled at import time with ``descriptor_pb2`` (no protoc step).
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto
OPT, REQ, REP = _F.LABEL_OPTIONAL, _F.LABEL_REQUIRED, _F.LABEL_REPEATED
T_STR, T_I32, T_I64, T_F32, T_BOOL, T_MSG, T_ENUM = (_F.TYPE_STRING, _F.TYPE_INT32, _F.TYPE_INT64,
                                                     _F.TYPE_FLOAT, _F.TYPE_BOOL, _F.TYPE_MESSAGE,
                                                     _F.TYPE_ENUM)
PKG = "paddle.framework.proto"

ATTR_TYPES = ["INT", "FLOAT", "STRING", "INTS", "FLOATS", "STRINGS", "BOOLEAN", "BOOLEANS", "BLOCK",
              "LONG", "BLOCKS"]
VAR_TYPES = [("BOOL", 0), ("INT16", 1), ("INT32", 2), ("INT64", 3), ("FP16", 4), ("FP32", 5), ("FP64", 6),
             ("LOD_TENSOR", 7), ("SELECTED_ROWS", 8), ("FEED_MINIBATCH", 9), ("FETCH_LIST", 10),
             ("STEP_SCOPES", 11), ("LOD_RANK_TABLE", 12), ("LOD_TENSOR_ARRAY", 13), ("PLACE_LIST", 14),
             ("READER", 15), ("CHANNEL", 16), ("RAW", 17), ("TUPLE", 18), ("SIZE_T", 19), ("UINT8", 20),
             ("INT8", 21), ("BF16", 22), ("FP8_E4M3", 23), ("FP8_E5M2", 24)]


def _field(msg, name, num, label, ftype, type_name=None, default=None):
    f = msg.field.add(name=name, number=num, label=label, type=ftype)
    if type_name:
        f.type_name = type_name
    if default is not None:
        f.default_value = default
    return f


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="paddle_amd_framework.proto", package=PKG, syntax="proto2")
    e = fd.enum_type.add(name="AttrType")
    for i, n in enumerate(ATTR_TYPES):
        e.value.add(name=n, number=i)

    op = fd.message_type.add(name="OpDesc")
    a = op.nested_type.add(name="Attr")
    _field(a, "name", 1, REQ, T_STR)
    _field(a, "type", 2, REQ, T_ENUM, f".{PKG}.AttrType")
    _field(a, "i", 3, OPT, T_I32)
    _field(a, "f", 4, OPT, T_F32)
    _field(a, "s", 5, OPT, T_STR)
    _field(a, "ints", 6, REP, T_I32)
    _field(a, "floats", 7, REP, T_F32)
    _field(a, "strings", 8, REP, T_STR)
    _field(a, "b", 10, OPT, T_BOOL)
    _field(a, "bools", 11, REP, T_BOOL)
    _field(a, "block_idx", 12, OPT, T_I32)
    _field(a, "l", 13, OPT, T_I64)
    _field(a, "blocks_idx", 14, REP, T_I32)
    v = op.nested_type.add(name="Var")
    _field(v, "parameter", 1, REQ, T_STR)
    _field(v, "arguments", 2, REP, T_STR)
    _field(op, "inputs", 1, REP, T_MSG, f".{PKG}.OpDesc.Var")
    _field(op, "outputs", 2, REP, T_MSG, f".{PKG}.OpDesc.Var")
    _field(op, "type", 3, REQ, T_STR)
    _field(op, "attrs", 4, REP, T_MSG, f".{PKG}.OpDesc.Attr")
    _field(op, "is_target", 5, OPT, T_BOOL, default="false")

    pr = fd.message_type.add(name="OpProto")
    pv = pr.nested_type.add(name="Var")
    _field(pv, "name", 1, REQ, T_STR)
    _field(pv, "comment", 2, REQ, T_STR)
    _field(pv, "duplicable", 3, OPT, T_BOOL, default="false")
    _field(pv, "intermediate", 4, OPT, T_BOOL, default="false")
    _field(pv, "dispensable", 5, OPT, T_BOOL, default="false")
    _field(pv, "reuse", 6, OPT, T_STR)
    pa = pr.nested_type.add(name="Attr")
    _field(pa, "name", 1, REQ, T_STR)
    _field(pa, "type", 2, REQ, T_ENUM, f".{PKG}.AttrType")
    _field(pa, "comment", 3, REQ, T_STR)
    _field(pa, "generated", 4, OPT, T_BOOL, default="false")
    _field(pr, "type", 1, REQ, T_STR)
    _field(pr, "inputs", 2, REP, T_MSG, f".{PKG}.OpProto.Var")
    _field(pr, "outputs", 3, REP, T_MSG, f".{PKG}.OpProto.Var")
    _field(pr, "attrs", 4, REP, T_MSG, f".{PKG}.OpProto.Attr")
    _field(pr, "comment", 5, REQ, T_STR)

    vt = fd.message_type.add(name="VarType")
    te = vt.enum_type.add(name="Type")
    for n, i in VAR_TYPES:
        te.value.add(name=n, number=i)
    T = f".{PKG}.VarType.Type"
    td = vt.nested_type.add(name="TensorDesc")
    _field(td, "data_type", 1, REQ, T_ENUM, T)
    _field(td, "dims", 2, REP, T_I64)
    ld = vt.nested_type.add(name="LoDTensorDesc")
    _field(ld, "tensor", 1, REQ, T_MSG, f".{PKG}.VarType.TensorDesc")
    _field(ld, "lod_level", 2, OPT, T_I32, default="0")
    la = vt.nested_type.add(name="LoDTensorArrayDesc")
    _field(la, "tensor", 1, REQ, T_MSG, f".{PKG}.VarType.TensorDesc")
    _field(la, "lod_level", 2, OPT, T_I32, default="0")
    rd = vt.nested_type.add(name="ReaderDesc")
    _field(rd, "lod_tensor", 1, REP, T_MSG, f".{PKG}.VarType.LoDTensorDesc")
    cd = vt.nested_type.add(name="ChannelDesc")
    _field(cd, "data_type", 1, REQ, T_ENUM, T)
    _field(cd, "capacity", 2, REQ, T_I64)
    tu = vt.nested_type.add(name="Tuple")
    _field(tu, "element_type", 1, REP, T_ENUM, T)
    _field(vt, "type", 1, REQ, T_ENUM, T)
    _field(vt, "selected_rows", 2, OPT, T_MSG, f".{PKG}.VarType.TensorDesc")
    _field(vt, "lod_tensor", 3, OPT, T_MSG, f".{PKG}.VarType.LoDTensorDesc")
    _field(vt, "tensor_array", 4, OPT, T_MSG, f".{PKG}.VarType.LoDTensorArrayDesc")
    _field(vt, "reader", 5, OPT, T_MSG, f".{PKG}.VarType.ReaderDesc")
    _field(vt, "channel", 6, OPT, T_MSG, f".{PKG}.VarType.ChannelDesc")
    _field(vt, "tuple", 7, OPT, T_MSG, f".{PKG}.VarType.Tuple")

    vd = fd.message_type.add(name="VarDesc")
    _field(vd, "name", 1, REQ, T_STR)
    _field(vd, "type", 2, REQ, T_MSG, f".{PKG}.VarType")
    _field(vd, "persistable", 3, OPT, T_BOOL, default="false")

    bd = fd.message_type.add(name="BlockDesc")
    _field(bd, "idx", 1, REQ, T_I32)
    _field(bd, "parent_idx", 2, REQ, T_I32)
    _field(bd, "vars", 3, REP, T_MSG, f".{PKG}.VarDesc")
    _field(bd, "ops", 4, REP, T_MSG, f".{PKG}.OpDesc")
    _field(bd, "forward_block_idx", 5, OPT, T_I32, default="-1")

    pd = fd.message_type.add(name="ProgramDesc")
    _field(pd, "blocks", 1, REP, T_MSG, f".{PKG}.BlockDesc")

    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    names = ["OpDesc", "OpProto", "VarType", "VarDesc", "BlockDesc", "ProgramDesc"]
    out = {}
    for n in names:
        d = pool.FindMessageTypeByName(f"{PKG}.{n}")
        out[n] = message_factory.GetMessageClass(d)
    out["AttrType"] = pool.FindEnumTypeByName(f"{PKG}.AttrType")
    return out


_M = _build()
OpDescPB = _M["OpDesc"]
OpProtoPB = _M["OpProto"]
VarTypePB = _M["VarType"]
VarDescPB = _M["VarDesc"]
BlockDescPB = _M["BlockDesc"]
ProgramDescPB = _M["ProgramDesc"]


class AttrType:
    INT, FLOAT, STRING, INTS, FLOATS, STRINGS, BOOLEAN, BOOLEANS, BLOCK, LONG, BLOCKS = range(11)


class VarTypeEnum:
    """Mirror of ``core.VarDesc.VarType`` in the reference Python API."""


for _n, _i in VAR_TYPES:
    setattr(VarTypeEnum, _n, _i)
