"""Fractional pod side of the pod server (server.py): stdlib + numpy only.

A pod scheduled onto a pod-server slice gets, from the device plugin,
``NOS_AMD_POD_SERVER`` (the GPU's server socket, under a host directory the
container mounts) and ``NOS_AMD_MEMORY_LIMIT_GB`` (its slice), optionally
``NOS_AMD_POD_CU_MASK``, and no ``/dev/kfd`` or render node.  The container
never opens the GPU.  It registers its model once, then sends inference
requests.  This is the role MPS clients play in the reference: their CUDA
calls go to the MPS server, which runs them in the server's context.
"""
from __future__ import annotations

import os
import socket
import time

import numpy as np

from ..api.constants import ENV_POD_CU_MASK, ENV_POD_SERVER
from . import protocol as P


class PodServerError(RuntimeError):
    pass


class PodClient:
    def __init__(self, path: str | os.PathLike, connect_timeout_s: float = 60.0):
        deadline = time.monotonic() + connect_timeout_s
        while True:  # the server's socket appears once it accepts (server.start)
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            try:
                s.connect(str(path))
                break
            except (FileNotFoundError, ConnectionRefusedError):
                s.close()
                if time.monotonic() > deadline:
                    raise PodServerError(f"no pod server at {path} after {connect_timeout_s} s")
                time.sleep(0.1)
        self.sock = s
        self.path = str(path)
        self.tenant: int | None = None
        self.info: dict = {}

    @classmethod
    def from_env(cls, env: dict | None = None, **kw) -> "PodClient":
        env = os.environ if env is None else env
        path = env.get(ENV_POD_SERVER)
        if not path:
            raise PodServerError(f"{ENV_POD_SERVER} is not set: this pod was not allocated a pod-server slice")
        return cls(path, **kw)

    def _call(self, req: dict, payload: bytes = b"") -> tuple[dict, bytes]:
        P.send_msg(self.sock, req, payload)
        rep, data = P.recv_msg(self.sock)
        if not rep.get("ok"):
            raise PodServerError(rep.get("error", "pod server error"))
        return rep, data

    def register(self, pod: str, dtype: str = "fp32", seed: int = 0, memory_limit_gb: float | None = None,
                 cu_mask: str | None = None, env: dict | None = None) -> dict:
        """Build the pod's model in the server; the slice comes from the device
        plugin's env unless given."""
        env = os.environ if env is None else env
        if memory_limit_gb is None and env.get("NOS_AMD_MEMORY_LIMIT_GB"):
            memory_limit_gb = float(env["NOS_AMD_MEMORY_LIMIT_GB"])
        rep, _ = self._call({"op": "register", "pod": pod, "dtype": dtype, "seed": seed,
                             "memory_limit_gb": memory_limit_gb, "cu_mask": cu_mask or env.get(ENV_POD_CU_MASK)})
        self.tenant = rep["tenant"]
        self.info = rep
        return rep

    def infer(self, x: np.ndarray | None = None, outputs: bool = False) -> tuple[list[np.ndarray], dict]:
        """One inference on the pod's model; ``x`` replaces the resident input
        (float32, the model's input shape)."""
        payload = b"" if x is None else np.ascontiguousarray(x, dtype=np.float32).tobytes()
        rep, data = self._call({"op": "infer", "outputs": outputs}, payload)
        return (P.unpack_arrays(rep["outputs"], data) if outputs else []), rep

    def stats(self) -> dict:
        return self._call({"op": "stats"})[0]

    def close(self) -> None:
        if self.sock is None:
            return
        try:
            self._call({"op": "close"})
        except (OSError, PodServerError, ConnectionError):
            pass
        self.sock.close()
        self.sock = None


__all__ = ["PodClient", "PodServerError", "ENV_POD_SERVER", "ENV_POD_CU_MASK"]
