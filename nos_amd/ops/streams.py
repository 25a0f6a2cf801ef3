"""CU-masked HIP streams -- in-process enforcement of cumask slices.

A cumask slice (the MPS analogue of the reference, ``pkg/gpu/slicing``) is a
set of compute units of one GPU.  Pods get it through the device plugin as
``ROC_GLOBAL_CU_MASK`` (process-wide); in-process tenants and the gpuagent's
probes get the same hardware mechanism per queue via
``hipExtStreamCreateWithCUMask``, wrapped here as a ``torch.cuda.ExternalStream``
so graphs and torch ops run on it.
"""
from __future__ import annotations

import ctypes
from typing import Iterable

import torch

from . import _lib


def mask_words(cus: Iterable[int], num_cus: int) -> list[int]:
    """Bit list -> 32-bit words (bit i = logical CU i)."""
    words = [0] * ((num_cus + 31) // 32)
    for c in cus:
        if not 0 <= c < num_cus:
            raise ValueError(f"CU {c} out of range [0, {num_cus})")
        words[c // 32] |= 1 << (c % 32)
    return words


def words_to_cus(words: Iterable[int]) -> list[int]:
    out = []
    for wi, w in enumerate(words):
        for b in range(32):
            if (w >> b) & 1:
                out.append(32 * wi + b)
    return out


def mask_hex(cus: Iterable[int], num_cus: int) -> str:
    """ROC_GLOBAL_CU_MASK syntax: one hex number, most significant word first."""
    words = mask_words(cus, num_cus)
    v = 0
    for i, w in enumerate(words):
        v |= w << (32 * i)
    return hex(v)


class CUMaskedStream:
    """Owns a hipStream_t created with a CU mask; ``.torch`` is the torch view."""

    def __init__(self, cus: Iterable[int] | None, num_cus: int, device: int | None = None):
        L = _lib.lib()
        self.cus = sorted(set(cus)) if cus is not None else None
        self.num_cus = num_cus
        dev = torch.cuda.current_device() if device is None else device
        with torch.cuda.device(dev):
            handle = ctypes.c_void_p()
            if self.cus is None:
                rc = L.nos_stream_create_cumask(None, 0, ctypes.byref(handle))
            else:
                w = mask_words(self.cus, num_cus)
                arr = (ctypes.c_uint * len(w))(*w)
                rc = L.nos_stream_create_cumask(arr, len(w), ctypes.byref(handle))
            _lib.check(rc, "hipExtStreamCreateWithCUMask")
        self.handle = handle.value
        self.device = dev
        self.torch = torch.cuda.ExternalStream(self.handle, device=torch.device("cuda", dev))

    def get_mask(self) -> list[int]:
        n = (self.num_cus + 31) // 32
        arr = (ctypes.c_uint * n)()
        _lib.check(_lib.lib().nos_stream_get_cumask(self.handle, n, arr), "hipExtStreamGetCUMask")
        return words_to_cus(list(arr))

    def synchronize(self) -> None:
        _lib.check(_lib.lib().nos_stream_sync(self.handle), "hipStreamSynchronize")

    def close(self) -> None:
        if self.handle:
            _lib.lib().nos_stream_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - interpreter shutdown ordering
        try:
            self.close()
        except Exception:
            pass


def device_info(dev: int = 0) -> dict:
    L = _lib.lib()
    n = ctypes.c_int()
    mem = ctypes.c_longlong()
    clk = ctypes.c_int()
    arch = ctypes.create_string_buffer(64)
    _lib.check(L.nos_device_info(dev, ctypes.byref(n), ctypes.byref(mem), ctypes.byref(clk), arch, 64),
               "hipGetDeviceProperties")
    return {"num_cus": n.value, "total_mem": mem.value, "clock_khz": clk.value,
            "arch": arch.value.decode()}
