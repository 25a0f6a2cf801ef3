"""Wire format between fractional pods and the node's pod server.

One message = an 8-byte header (two big-endian uint32: JSON length, payload
length), a UTF-8 JSON object, then an opaque payload (raw little-endian
tensor bytes: an input image, returned detections).  Requests carry ``op``;
replies carry ``ok`` and, on failure, ``error``.  Pure stdlib + numpy: a
client pod never imports torch or opens the GPU -- its kernels run in the
server's HIP context, which is the point of the server (see server.py).
"""
from __future__ import annotations

import json
import socket
import struct

import numpy as np

_HDR = struct.Struct(">II")
MAX_JSON = 1 << 20
MAX_PAYLOAD = 1 << 30


class ProtocolError(RuntimeError):
    pass


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed the connection")
        got += k
    return bytes(buf)


def send_msg(sock: socket.socket, obj: dict, payload: bytes | memoryview = b"") -> None:
    js = json.dumps(obj, separators=(",", ":")).encode()
    sock.sendall(_HDR.pack(len(js), len(payload)) + js)
    if len(payload):
        sock.sendall(payload)


def recv_msg(sock: socket.socket) -> tuple[dict, bytes]:
    nj, npay = _HDR.unpack(_recv_exact(sock, _HDR.size))
    if nj > MAX_JSON or npay > MAX_PAYLOAD:
        raise ProtocolError(f"message too large ({nj} B header, {npay} B payload)")
    obj = json.loads(_recv_exact(sock, nj))
    if not isinstance(obj, dict):
        raise ProtocolError("message is not a JSON object")
    return obj, _recv_exact(sock, npay) if npay else b""


def pack_arrays(arrays: list[np.ndarray]) -> tuple[list[dict], bytes]:
    """float32 arrays -> (descriptors, one payload)."""
    descs, parts, off = [], [], 0
    for a in arrays:
        a = np.ascontiguousarray(a, dtype=np.float32)
        descs.append({"shape": list(a.shape), "offset": off, "nbytes": a.nbytes})
        parts.append(a.tobytes())
        off += a.nbytes
    return descs, b"".join(parts)


def unpack_arrays(descs: list[dict], payload: bytes) -> list[np.ndarray]:
    out = []
    for d in descs:
        end = d["offset"] + d["nbytes"]
        if end > len(payload):
            raise ProtocolError("payload shorter than its descriptors")
        out.append(np.frombuffer(payload[d["offset"]:end], dtype=np.float32).reshape(d["shape"]))
    return out


__all__ = ["send_msg", "recv_msg", "pack_arrays", "unpack_arrays", "ProtocolError"]
