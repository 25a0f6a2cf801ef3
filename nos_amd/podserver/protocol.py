"""Wire format between fractional pods and the node's pod server.

One message = a 12-byte header (big-endian uint32 JSON length, uint64
payload length), a UTF-8 JSON object, then an opaque payload (raw
little-endian tensor bytes: a tenant's weights, an input image, returned
detections).  A receiver bounds the payload per message (``payload_limit``):
the pod server allows a register request as many weight bytes as the
tenant's memory slice holds -- tens of GB on a 288 GB GPU -- and other
requests ``MAX_PAYLOAD``; an oversized payload is read and dropped so the
connection stays in step and the sender gets an error reply, not a reset.  Requests carry ``op``;
replies carry ``ok`` and, on failure, ``error``.  Pure stdlib + numpy: a
client pod never imports torch or opens the GPU -- its kernels run in the
server's HIP context, which is the point of the server (see server.py).
"""
from __future__ import annotations

import json
import socket
import struct
import time

import numpy as np

_HDR = struct.Struct(">IQ")
MAX_JSON = 1 << 20
MAX_PAYLOAD = 1 << 30
_DRAIN = 1 << 24


class ProtocolError(RuntimeError):
    pass


class PayloadTooLarge(ProtocolError):
    """The payload was over the receiver's limit; it has been read and
    dropped, so the connection can carry the error reply."""


def _recv_exact(sock: socket.socket, n: int, deadline: float | None = None) -> bytearray:
    """``n`` bytes; with a ``deadline`` (time.monotonic()) the whole read must
    end by then -- a trickle of bytes does not reset it -- else TimeoutError
    (an OSError), the socket's own timeout restored either way."""
    buf = bytearray(n)  # returned as is: no second copy of a multi-GB payload
    view = memoryview(buf)
    got = 0
    old = sock.gettimeout() if deadline is not None else None
    try:
        while got < n:
            if deadline is not None:
                left = deadline - time.monotonic()
                if left <= 0:
                    raise TimeoutError(f"payload not received in time ({got} of {n} B)")
                sock.settimeout(left)
            k = sock.recv_into(view[got:], n - got)
            if k == 0:
                raise ConnectionError("peer closed the connection")
            got += k
    finally:
        if deadline is not None:
            sock.settimeout(old)
    return buf


def _drain(sock: socket.socket, n: int) -> None:
    buf = bytearray(min(n, _DRAIN))
    view = memoryview(buf)
    while n:
        k = sock.recv_into(view[:min(n, len(buf))])
        if k == 0:
            raise ConnectionError("peer closed the connection")
        n -= k


def send_msg(sock: socket.socket, obj: dict, payload: bytes | memoryview = b"") -> None:
    js = json.dumps(obj, separators=(",", ":")).encode()
    sock.sendall(_HDR.pack(len(js), len(payload)) + js)
    if len(payload):
        sock.sendall(payload)


def recv_msg(sock: socket.socket, payload_limit=None, payload_timeout=None) -> tuple[dict, bytes | bytearray]:
    """(JSON object, payload).  ``payload_limit(obj, npay) -> int`` bounds
    the payload of this message (default ``MAX_PAYLOAD``); it sees the
    announced payload size before a byte of it is read, so a receiver can
    reserve (or refuse) what the payload is for first.  An oversized JSON
    header desynchronises nothing that can be trusted: ConnectionError.
    ``payload_timeout(obj, npay) -> seconds | None``: a deadline for the
    payload once its header has arrived (TimeoutError, an OSError, past it):
    a sender that announces a payload and stalls cannot hold what the
    receiver reserved for it."""
    nj, npay = _HDR.unpack(_recv_exact(sock, _HDR.size))
    if nj > MAX_JSON:
        raise ConnectionError(f"message header too large ({nj} B)")
    obj = json.loads(_recv_exact(sock, nj))
    limit = MAX_PAYLOAD if payload_limit is None or not isinstance(obj, dict) else int(payload_limit(obj, npay))
    if npay > limit:
        _drain(sock, npay)
        raise PayloadTooLarge(f"payload of {npay} B is over this request's limit of {limit} B")
    if not isinstance(obj, dict):
        _drain(sock, npay)
        raise ProtocolError("message is not a JSON object")
    if not npay:
        return obj, b""
    t = payload_timeout(obj, npay) if payload_timeout is not None else None
    return obj, _recv_exact(sock, npay, None if t is None else time.monotonic() + float(t))


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


__all__ = ["send_msg", "recv_msg", "pack_arrays", "unpack_arrays", "ProtocolError", "PayloadTooLarge", "MAX_PAYLOAD"]
