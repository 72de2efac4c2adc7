"""Untrusted-input hardening of the native runtime.

* LoDTensor stream reader (csrc/runtime/lod_tensor_io.cc): truncated and
  malformed checkpoint files must raise IOError, never read or write past the
  caller's arrays (reference format: framework/lod_tensor.cc:251-304).
* Pserver RPC (csrc/runtime/rpc.cc): an oversized or garbage frame must close
  only that connection; the server keeps serving well-formed clients.
"""
import socket
import struct

import numpy as np
import pytest

from paddle_amd import runtime

pytestmark = pytest.mark.skipif(not runtime.available(), reason="native runtime not built")


def _good(tmp_path):
    p = str(tmp_path / "ok.bin")
    arr = np.arange(12, dtype=np.float32).reshape(3, 4)
    runtime.write_lod_tensors(p, [(arr, [[0, 1, 3]], 5)])
    return open(p, "rb").read()


def _desc(dims, dtype=5):
    d = bytes([0x08, dtype])
    for x in dims:
        v, b = x, bytearray()
        while v >= 0x80:
            b.append((v & 0x7F) | 0x80)
            v >>= 7
        b.append(v)
        d += bytes([0x10]) + bytes(b)
    return d


def _stream(lod_levels, dims, payload=b"", dtype=5, desc=None):
    out = struct.pack("<IQ", 0, len(lod_levels))
    for lv in lod_levels:
        out += struct.pack("<Q", 8 * len(lv)) + struct.pack(f"<{len(lv)}Q", *lv)
    d = desc if desc is not None else _desc(dims, dtype)
    out += struct.pack("<Ii", 0, len(d)) + d + payload
    return out


def _read(tmp_path, data):
    p = tmp_path / "bad.bin"
    p.write_bytes(data)
    return runtime.read_lod_tensors(str(p))


def test_roundtrip_still_works(tmp_path):
    (a, lod, vt), = _read(tmp_path, _good(tmp_path))
    assert a.shape == (3, 4) and lod == [[0, 1, 3]] and vt == 5


@pytest.mark.parametrize("cut", [3, 10, 20, 30, 40])
def test_truncated_streams_raise(tmp_path, cut):
    data = _good(tmp_path)
    with pytest.raises(IOError):
        _read(tmp_path, data[:cut] if cut < len(data) - 8 else data[:-8])


def test_too_many_lod_levels(tmp_path):
    with pytest.raises(IOError, match="lod_level"):
        _read(tmp_path, _stream([[0, 1]] * 17, [1]))


def test_too_many_dims(tmp_path):
    with pytest.raises(IOError, match="rank exceeds"):
        _read(tmp_path, _stream([], [1] * 17, b"\0" * 4))


def test_negative_and_huge_desc_size(tmp_path):
    for dsz in (-5, 1 << 30):
        data = struct.pack("<IQ", 0, 0) + struct.pack("<Ii", 0, dsz) + b"\x08\x05"
        with pytest.raises(IOError):
            _read(tmp_path, data)


def test_packed_dims_past_end(tmp_path):
    desc = bytes([0x08, 5, 0x12, 50, 3, 4])  # packed field claims 50 bytes, has 2
    with pytest.raises(IOError, match="packed"):
        _read(tmp_path, _stream([], [], desc=desc))


def test_declared_size_beyond_file(tmp_path):
    with pytest.raises(IOError):
        _read(tmp_path, _stream([], [1 << 20, 1 << 10], b"\0" * 64))


def test_unknown_dtype(tmp_path):
    with pytest.raises(IOError):
        _read(tmp_path, _stream([], [2], b"\0" * 8, dtype=31))


def test_rpc_server_survives_bad_frames():
    import torch

    from paddle_amd.distributed.ps.rpc import RPCClient, RPCServer, var_to_bytes

    srv = RPCServer(0, 1, host="127.0.0.1")
    ep = f"127.0.0.1:{srv.port}"
    try:
        # oversized name / payload lengths: the server must drop the connection
        for hdr in (struct.pack("<IBIQ", 0x50415250, 0, 1 << 31, 0),
                    struct.pack("<IBIQ", 0x50415250, 0, 4, 1 << 62),
                    b"\xff" * 17):
            s = socket.create_connection(("127.0.0.1", srv.port), timeout=5)
            s.sendall(hdr)
            s.settimeout(5)
            try:
                got = s.recv(64)
            except (ConnectionResetError, socket.timeout):
                got = b""
            assert got == b""  # closed, no reply
            s.close()
        # a well-formed client is still served
        RPCClient()._send(ep, "w@GRAD", var_to_bytes(torch.ones(4)))
        got = srv.pop_all()
        assert got and got[0][0] == "w@GRAD"
    finally:
        srv.stop()
